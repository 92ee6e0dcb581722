"""Run the fused INT4 GEMM for one shape a few times (target for rocprofv3 --pmc): MFMA utilisation."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--group", type=int, default=-2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variant", type=int, default=0, help="iwq_w4a16_gemm flags variant")
    ap.add_argument("--ref", action="store_true", help="run F.linear(x, W_deq) (hipBLASLt) instead")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels
    w = torch.empty(a.n, a.k, dtype=torch.float16, device="cuda")
    kernels.fill_synthetic(w, 7)
    r = kernels.quantize_minmax(w, 4, a.group, False, 0, want_codes=True)
    x = (torch.randn(a.m, a.k, device="cuda") * 0.5).half()
    fl = kernels.gemm_variant_flags(a.variant)
    for _ in range(a.reps):
        if a.ref:
            torch.nn.functional.linear(x, r.out)
        else:
            kernels.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, a.group, a.n, flags=fl)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

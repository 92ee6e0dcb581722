"""Runner for PMC passes over the quant_dim = 1 column kernel (k_column_reg): INT4 g = 128 asym on
[11008, 4096] fp16, --reps cold calls over distinct copies, eager.

    rocprofv3 --pmc ... -- python3 tools/col_run.py [--reps 8] [--group 128]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--group", type=int, default=128)
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    ws = []
    for c in range(a.reps):
        t = torch.empty(11008, 4096, dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, 200 + c)
        ws.append(t)
    outs = [torch.empty_like(t) for t in ws]
    for w, o in zip(ws, outs):
        K.quantize_minmax(w, 4, a.group, False, 1, out=o)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()

"""Host-side cost per call of the decode forward (eager, no graph): kernels.w4a16_gemm and
QuantLinear(fused_forward='auto').forward at M = 1 vs F.linear on the fp16 weight.  Times N
back-to-back calls on the host (device work is queued, then synchronised outside the timing)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def host_us(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    from iron_weight_only_quant_amd import kernels as K
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    N, Kd = 4096, 4096
    lin = torch.nn.Linear(Kd, N, bias=False).half().cuda()
    q = QuantLinear.from_linear(lin, w_bit=4, w_group_size=128, symmetric=False, fused_forward="auto")
    x = torch.randn(1, 1, Kd, dtype=torch.float16, device="cuda")
    w = torch.randn(N, Kd, dtype=torch.float16, device="cuda")
    rec = {"F_linear_us": host_us(lambda: torch.nn.functional.linear(x, w)),
           "w4a16_gemm_us": host_us(lambda: K.w4a16_gemm(x, q.qweight_tiled, q.scales, q.zeros, 4, 128, N,
                                                           tiled=True)),
           "quantlinear_auto_forward_us": host_us(lambda: q(x))}
    print(json.dumps({k: round(v, 2) for k, v in rec.items()}), flush=True)


if __name__ == "__main__":
    main()

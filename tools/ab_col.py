"""A/B the quant_dim=1 column kernel block shapes (flags variant 0 = default, 1 = 8x32, 2 = 32x8, 3 = 16x16) on a
cold rotation of [rows, cols] weights (INT4, g=128 down the columns), graph-replayed device time."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.bench_formats import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=11008)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--variants", default="", help="comma list (default: every block shape of the group)")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    ws = []
    for c in range(a.copies):
        t = torch.empty(a.rows, a.cols, dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, 7 + c)
        ws.append(t)
    outs = [torch.empty_like(t) for t in ws]
    n = a.rows * a.cols
    algo = 4 * n + 4 * (n // a.group)
    ref = K.quantize_minmax(ws[0], 4, a.group, False, 1).out
    import time
    t_end = time.time() + 1.0  # clock ramp: ~1 s of untimed launches before the first timing
    while time.time() < t_end:
        for w, o in zip(ws, outs):
            K.quantize_minmax(w, 4, a.group, False, 1, out=o)
    torch.cuda.synchronize()
    vs = [int(t) for t in a.variants.split(",")] if a.variants else ((0, 1, 2, 3, 4) if a.group in (32, 64) else (0, 1, 2, 3))
    for v in vs:
        flags = K.gemm_variant_flags(v)
        r = K.quantize_minmax(ws[0], 4, a.group, False, 1, flags=flags).out
        assert torch.equal(r.view(torch.int16), ref.view(torch.int16)), v

        def run(flags=flags):
            for w, o in zip(ws, outs):
                K.quantize_minmax(w, 4, a.group, False, 1, out=o, flags=flags)
        t = timed(run, 2) / len(ws)
        print(json.dumps({"variant": v, "shape": [a.rows, a.cols], "group": a.group, "us": round(t * 1e6, 2),
                          "frac_of_8TBps": round(algo / t / 8e12, 3)}), flush=True)


if __name__ == "__main__":
    main()

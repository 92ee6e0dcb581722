"""A/B the k_group tuning variants (and the copy probes) on ONE weight tensor per launch
(QuantLinear-style per-layer use) instead of the whole model: graph-replayed device time per launch.

--copies N (default 24) rotates the launches over N distinct resident tensors of the shape, so a
replay streams >= 1 GB and the 256 MB MALL holds none of it (cold, as when quantize_model walks a
model's layers); --copies 1 re-runs one tensor (MALL-warm for shapes under ~128 MB)."""
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
    ap.add_argument("--copies", type=int, default=24)
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,8,100,102")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    plans = []
    for c in range(a.copies):
        w = torch.empty(a.rows, a.cols, dtype=torch.float16, device="cuda")
        K.fill_synthetic(w, 3 + c)
        plans.append(K.BatchPlan([w], 4, 128, False, outs=[torch.empty_like(w)]))
    n = a.rows * a.cols
    algo = 4 * n + 4 * (n // 128)
    for v in [int(t) for t in a.variants.split(",")]:
        def run(v=v):
            for p in plans:
                p.run(variant=v)
        t = timed(run, 4) / len(plans)
        print(json.dumps({"variant": v, "shape": [a.rows, a.cols], "copies": a.copies, "us": round(t * 1e6, 2),
                          "achieved_GBps": round(algo / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()

"""A/B two builds of libiwq.so in separate processes on the same box (a kernel change that touches a
shared helper cannot be kept beside the old code as a variant).  One process per (library, round):

    python tools/ab_lib.py --lib iron_weight_only_quant_amd/_lib/libiwq_base.so --tag base

prints one JSON line: the whole-model headline launch (k_group batched over all 224 Llama-2-7B
weights, HIP-event kernel time, best of 3 x 10 launches after a 1 s clock ramp) and bench.py's cold
single-call shapes (hipGraph replay over 32 distinct instances per shape).  Alternate the libraries
over several rounds and compare medians."""
import argparse
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--tag", required=True)
    a = ap.parse_args()
    from iron_weight_only_quant_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from iron_weight_only_quant_amd import kernels
    weights, names, _ = bench.make_weights("llama2-7b", 0, 1)
    plan = kernels.BatchPlan(weights, 4, 128, False)
    bench.clock_ramp(plan, 1.0)
    st = torch.cuda.current_stream()
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            plan.run(st)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        best = ms if best is None else min(best, ms)
    alg = plan.numel * 4 + plan.numel // 128 * 4
    args = types.SimpleNamespace(bits=4, group=128, symmetric=False)
    shapes = bench.per_shape(plan, names, 1, args)
    rec = {"tag": a.tag, "lib": os.path.basename(a.lib), "model_ms": round(best, 4),
           "model_frac": round(alg / (best / 1e3) / 1e9 / 8000.0, 4),
           "shapes_us": {k: v["us_per_call"] for k, v in shapes.items()},
           "shapes_frac": {k: v["frac"] for k, v in shapes.items()}}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

"""Is the out-of-place placement effect absolute (where the outputs live) or relative (where they live
against the inputs)?  A 2 x 2 of input sets {A = bench.make_weights, B = copies of A allocated later}
and output sets {per-tensor torch.empty_like (default), one flat arena}, plus in place on A and on B,
the read-only probe (103) on A and B and the write-only probe (104) on both output sets.  Kernel time
per arm: HIP events, best of 3 x 10 launches, arms interleaved over --rounds, after a 1 s ramp.
    IWQ_AB=1 python tools/ab_placement.py --variants 0,100,118 --out gpurun_out/x.jsonl"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="0,100,118")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    from iron_weight_only_quant_amd import kernels
    A, _, _ = bench.make_weights("llama2-7b", 0, 1)
    numel = sum(w.numel() for w in A)
    alg = numel * 4 + numel // 128 * 4
    arena = torch.empty(numel * 2, dtype=torch.uint8, device="cuda")
    outs_arena, off = [], 0
    for w in A:
        nb = w.numel() * 2
        outs_arena.append(arena[off:off + nb].view(torch.float16).view(w.shape))
        off += nb
    outs_def = [torch.empty_like(w) for w in A]
    B = [w.clone() for w in A]
    A2 = [w.clone() for w in A]  # in place on copies: A stays the input of the other arms
    B2 = [w.clone() for w in A]
    plans = {"A->default": kernels.BatchPlan(A, 4, 128, False, outs=outs_def),
             "A->arena": kernels.BatchPlan(A, 4, 128, False, outs=outs_arena),
             "B->default": kernels.BatchPlan(B, 4, 128, False, outs=outs_def),
             "B->arena": kernels.BatchPlan(B, 4, 128, False, outs=outs_arena),
             "A2 in place": kernels.BatchPlan(A2, 4, 128, False, outs=A2),
             "B2 in place": kernels.BatchPlan(B2, 4, 128, False, outs=B2)}
    variants = [int(v) for v in a.variants.split(",")]
    probes = [("A read-only", plans["A->default"], 103), ("B read-only", plans["B->default"], 103),
              ("default write-only", plans["A->default"], 104), ("arena write-only", plans["A->arena"], 104)]
    st = torch.cuda.current_stream()
    fh = open(a.out, "a") if a.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if fh:
            fh.write(line + "\n")
            fh.flush()

    def best_ms(plan, v):
        best = None
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(10):
                plan.run(st, variant=v)
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            best = ms if best is None else min(best, ms)
        return best

    bench.clock_ramp(plans["A->default"], 1.0)
    for rnd in range(a.rounds):
        for k, plan in plans.items():
            for v in variants:
                ms = best_ms(plan, v)
                b = alg if v == 0 else numel * 4
                emit({"round": rnd, "arm": k, "variant": v, "ms": round(ms, 4), "GBps": round(b / ms / 1e6, 1),
                      "frac": round(b / ms / 1e6 / 8000, 4)})
        for k, plan, v in probes:
            ms = best_ms(plan, v)
            emit({"round": rnd, "arm": k, "variant": v, "ms": round(ms, 4), "GBps": round(numel * 2 / ms / 1e6, 1),
                  "frac": round(numel * 2 / ms / 1e6 / 8000, 4)})


if __name__ == "__main__":
    main()

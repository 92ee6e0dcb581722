"""Whole-model throughput per weight format: all 224 Llama-2-7B Linear weights (12.95 GB fp16,
synthetic, resident) in ONE batched launch per step — the quantize_model path — for INT4 g128
(kernels.BatchPlan) and the FP formats / approximate decode / grid (kernels.FpBatchPlan).

Prints one JSON line per format: ms per model, weights GB/s (fp16 input bytes / time), algorithmic
HBM bytes (read w + write deq + scales/zeros) / time and its fraction of 8 TB/s.  HIP events on the
launch stream over `--steps` back-to-back launches after a 1 s clock ramp.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--model", default="llama2-7b")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import _lib as L
    from iron_weight_only_quant_amd import kernels as K
    from iron_weight_only_quant_amd import shard
    ws = []
    for i, (_, (r, c)) in enumerate(shard.model_linear_shapes(a.model)):
        t = torch.empty((r, c), dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, seed=i)
        ws.append(t)
    outs = [torch.empty_like(w) for w in ws]
    numel = sum(w.numel() for w in ws)
    g = 128
    cases = [
        ("int4_g128_asym", lambda: K.BatchPlan(ws, 4, g, False, outs=outs), 4),
        ("fp8_e4m3_g128_sym", lambda: K.FpBatchPlan(ws, L.IWQ_CODEC_FP, 4, 3, g, True, outs=outs), 2),
        ("fp8_e4m3_g128_asym", lambda: K.FpBatchPlan(ws, L.IWQ_CODEC_FP, 4, 3, g, False, outs=outs), 4),
        ("fp6_e3m2_g128_asym", lambda: K.FpBatchPlan(ws, L.IWQ_CODEC_FP, 3, 2, g, False, outs=outs), 4),
        ("fp4_e2m1_g128_asym", lambda: K.FpBatchPlan(ws, L.IWQ_CODEC_FP, 2, 1, g, False, outs=outs), 4),
        ("approx_fp8_g128", lambda: K.FpBatchPlan(ws, L.IWQ_CODEC_APX, 4, 3, g, True, 12, 15, 1, outs=outs), 2),
        ("fp4_grid_g128", lambda: K.FpBatchPlan(ws, L.IWQ_CODEC_GRID, 2, 1, g, True, outs=outs), 2),
    ]
    st = torch.cuda.current_stream()
    for name, mk, pbytes in cases:
        plan = mk()
        plan.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 1.0:
            for _ in range(10):
                plan.run()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            plan.run()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        algo = numel * 4 + (numel // g) * pbytes
        print(json.dumps({"format": name, "model": a.model, "numel": numel, "ms": round(ms, 4),
                          "weights_GBps": round(numel * 2 / ms / 1e6, 1), "algo_bytes": algo,
                          "achieved_GBps": round(algo / ms / 1e6, 1), "frac_of_8TBps": round(algo / ms / 8e9, 4)}),
              flush=True)
        del plan


if __name__ == "__main__":
    main()

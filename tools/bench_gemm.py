"""Config 3 measurement: fused INT4 dequant->GEMM forward (kernels.w4a16_gemm, MFMA) vs the
reference forward F.linear(x, W_deq) (hipBLASLt on the fp16 dequantized weight), Llama-2-7B shapes.

Prints one JSON line per (shape, M) with TFLOP/s of both, the fraction of the 2.5 PF dense fp16
MFMA peak (MI355X_MICROARCH.md) and the weight bytes each reads.  Timing: HIP events around R
back-to-back calls on the current stream, median of 5 rounds, interleaved (rule 24).
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_TFLOPS = 2500.0
SHAPES = [("q_proj", 4096, 4096), ("gate_proj", 11008, 4096), ("down_proj", 4096, 11008)]


def timed_graph(fn, reps, rounds=5):
    """Device time per call: `reps` calls captured in one hipGraph, replayed (no host launch cost)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    out = []
    st = torch.cuda.current_stream()
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    out.sort()
    return out[len(out) // 2]


def timed(fn, reps, rounds=5):
    st = torch.cuda.current_stream()
    out = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    out.sort()
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="8192,16,1")
    ap.add_argument("--group", type=int, default=-2)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels
    for name, N, K in SHAPES:
        w = torch.empty(N, K, dtype=torch.float16, device="cuda")
        kernels.fill_synthetic(w, 7)
        r = kernels.quantize_minmax(w, 4, a.group, False, 0, want_codes=True)
        for M in [int(m) for m in a.m.split(",")]:
            x = (torch.randn(M, K, device="cuda") * 0.5).half()
            fused = lambda: kernels.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, a.group, N)
            ref = lambda: torch.nn.functional.linear(x, r.out)
            fused(); ref(); torch.cuda.synchronize()
            err = float((fused().float() - ref().float()).abs().max())
            reps = a.reps if M >= 1024 else a.reps * 20
            if M >= 1024:
                t_f = timed(fused, reps)
                t_r = timed(ref, reps)
            else:  # decode: launch-bound from Python, so time device work via hipGraph replay
                t_f = timed_graph(fused, 50)
                t_r = timed_graph(ref, 50)
            flops = 2.0 * M * N * K
            rec = {"shape": name, "M": M, "N": N, "K": K, "group": a.group,
                   "fused_ms": round(t_f, 4), "fused_tflops": round(flops / t_f / 1e9, 1),
                   "fused_frac_peak": round(flops / t_f / 1e9 / PEAK_TFLOPS, 4),
                   "hipblaslt_fp16_ms": round(t_r, 4), "hipblaslt_tflops": round(flops / t_r / 1e9, 1),
                   "speedup_vs_F_linear": round(t_r / t_f, 3),
                   "weight_bytes_fused": int(r.codes.numel() + r.scales.numel() * 4),
                   "weight_bytes_fp16": int(N * K * 2), "max_abs_diff_vs_F_linear": err}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

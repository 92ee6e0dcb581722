"""Config 3 measurement: fused INT4 dequant->GEMM forward (kernels.w4a16_gemm, MFMA) vs the
reference forward F.linear(x, W_deq) (hipBLASLt on the fp16 dequantized weight), Llama-2-7B shapes,
plus the packed-only alternative dequant-once (iwq_dequant_packed) + hipBLASLt.

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
    ap.add_argument("--variants", default="0", help="decode-kernel variants to time for M <= 16 (IWQ_FLAG_VARIANT)")
    ap.add_argument("--shapes", default="q_proj,gate_proj,down_proj")
    ap.add_argument("--warm-seconds", type=float, default=1.5,
                    help="untimed MFMA load before the first measurement (clock ramp)")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels
    import time
    xw = torch.randn(8192, 4096, device="cuda").half()
    ww = torch.randn(4096, 4096, device="cuda").half()
    t_end = time.time() + a.warm_seconds
    while time.time() < t_end:
        for _ in range(20):
            torch.nn.functional.linear(xw, ww)
        torch.cuda.synchronize()
    del xw, ww
    shapes = SHAPES + [("70b_gate", 28672, 8192), ("70b_down", 8192, 28672)]
    for name, N, K in [t for t in shapes if t[0] in a.shapes.split(",")]:
        w = torch.empty(N, K, dtype=torch.float16, device="cuda")
        kernels.fill_synthetic(w, 7)
        r = kernels.quantize_minmax(w, 4, a.group, False, 0, want_codes=True)
        for M in [int(m) for m in a.m.split(",")]:
            x = (torch.randn(M, K, device="cuda") * 0.5).half()
            ref = lambda: torch.nn.functional.linear(x, r.out)
            ref()
            t_r = timed(ref, a.reps) if M >= 1024 else timed_graph(ref, 50)
            # packed-only prefill alternative: dequantize once (iwq_dequant_packed) + hipBLASLt
            dq = lambda: torch.nn.functional.linear(
                x, kernels.dequant_packed(r.codes, r.scales, r.zeros, 4, a.group, N, K))
            dq()
            t_dq = timed(dq, a.reps) if M >= 1024 else timed_graph(dq, 50)
            deq_only = lambda: kernels.dequant_packed(r.codes, r.scales, r.zeros, 4, a.group, N, K)
            t_deq = timed_graph(deq_only, 20)
            for v in [int(t) for t in a.variants.split(",")]:
                fl = kernels.gemm_variant_flags(v)
                fused = lambda: kernels.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, a.group, N, flags=fl)
                fused(); torch.cuda.synchronize()
                err = float((fused().float() - ref().float()).abs().max())
                # decode: launch-bound from Python, so time device work via hipGraph replay
                t_f = timed(fused, a.reps) if M >= 1024 else timed_graph(fused, 50)
                flops = 2.0 * M * N * K
                wbytes = int(r.codes.numel() + r.scales.numel() * 2 + (r.zeros.numel() * 2 if r.zeros is not None else 0))
                t_tiled = None
                if M <= 16:
                    tiled = kernels.tile_codes(r.codes, N, K)
                    ft = lambda: kernels.w4a16_gemm(x, tiled, r.scales, r.zeros, 4, a.group, N, flags=fl, tiled=True)
                    ft()
                    t_tiled = timed_graph(ft, 50)
                rec = {"shape": name, "M": M, "N": N, "K": K, "group": a.group, "variant": v,
                       "tiled_ms": round(t_tiled, 4) if t_tiled else None,
                       "tiled_weight_GBps": round(int(r.codes.numel() + r.scales.numel() * 2 + (r.zeros.numel() * 2 if r.zeros is not None else 0)) / t_tiled / 1e6, 1) if t_tiled else None,
                       "fused_ms": round(t_f, 4), "fused_tflops": round(flops / t_f / 1e9, 1),
                       "fused_frac_peak": round(flops / t_f / 1e9 / PEAK_TFLOPS, 4),
                       "fused_weight_GBps": round(wbytes / t_f / 1e6, 1),
                       "hipblaslt_fp16_ms": round(t_r, 4), "hipblaslt_tflops": round(flops / t_r / 1e9, 1),
                       "speedup_vs_F_linear": round(t_r / t_f, 3),
                       "dequant_plus_hipblaslt_ms": round(t_dq, 4), "dequant_only_ms": round(t_deq, 4),
                       "dequant_GBps": round((wbytes + N * K * 2) / t_deq / 1e6, 1),
                       "weight_bytes_fused": wbytes,
                       "weight_bytes_fp16": int(N * K * 2), "max_abs_diff_vs_F_linear": err}
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

"""Throughput of every weight-format path on one Llama-2-7B gate_proj weight ([11008, 4096] fp16,
resident in HBM): INT (pseudo_quantize_tensor / QuantLinear modes), FP8/FP6/FP4 (config 5), the E2M1
grid, BFP and the approximate / double-approximate decodes; and the "unpack" paths (packed FP / grid
codes -> fp16, iwq_dequant_fp_packed) and the grid's "pack" (fp4_grid with codes).

Prints one JSON line per path: weights GB/s (fp16 input bytes / time), algorithmic HBM bytes per call
(read weight + write dequant + scales/zeros [+ codes]), achieved GB/s and the fraction of 8 TB/s.
Timing: R calls captured in one hipGraph and replayed, HIP events around the replay, median of 5
rounds — device time per call without the Python wrapper's host cost (which exceeds the device
time of a single 90 MB tensor).  The calls rotate over --copies distinct resident weights (default
16 = 1.4 GB of input per replay), so the 256 MB MALL holds none of a call's bytes (cold, as when
quantize_model walks a model's layers); --copies 1 re-runs one MALL-warm tensor.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8.0e12


def timed(fn, reps, rounds=5):
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
    st = torch.cuda.current_stream()
    out = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps * 1e-3)
    out.sort()
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=11008)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=2, help="passes over the copies per graph")
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--only", default="", help="comma list of path names to run")
    ap.add_argument("--lib", default="", help="A/B: load this libiwq.so build instead of the tree's")
    ap.add_argument("--tag", default="", help="A/B: label added to every line")
    a = ap.parse_args()
    if a.lib:
        from iron_weight_only_quant_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    from iron_weight_only_quant_amd import kernels as K
    R, C = a.rows, a.cols
    n = R * C
    ws = []
    for c in range(a.copies):
        t = torch.empty(R, C, dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, 1 + c)
        ws.append(t)
    outs = [torch.empty_like(t) for t in ws]
    g = 128
    G = n // g
    cases = [
        ("int4_g128_asym", lambda w, out: K.quantize_minmax(w, 4, g, False, 0, out=out), 4 * n + 4 * G),
        ("int4_g128_asym_codes", lambda w, out: K.quantize_minmax(w, 4, g, False, 0, out=out, want_codes=True),
         4 * n + 4 * G + n // 2),
        ("int8_perchannel_asym", lambda w, out: K.quantize_minmax(w, 8, -2, False, 0, out=out), 4 * n + 4 * R),
        ("int4_g128_quant_dim1", lambda w, out: K.quantize_minmax(w, 4, g, False, 1, out=out), 4 * n + 4 * G),
        ("int4_per_tensor", lambda w, out: K.quantize_minmax(w, 4, -1, False, 0, out=out), 4 * n + 4),
        ("fp8_e4m3_g128_sym", lambda w, out: K.quantize_fp(w, 4, 3, g, True, 0, out=out), 4 * n + 2 * G),
        ("fp8_e4m3_g128_asym", lambda w, out: K.quantize_fp(w, 4, 3, g, False, 0, out=out), 4 * n + 4 * G),
        ("fp6_e3m2_g128_asym", lambda w, out: K.quantize_fp(w, 3, 2, g, False, 0, out=out), 4 * n + 4 * G),
        ("fp4_e2m1_g128_asym", lambda w, out: K.quantize_fp(w, 2, 1, g, False, 0, out=out), 4 * n + 4 * G),
        ("fp8_e4m3_g128_asym_codes", lambda w, out: K.quantize_fp(w, 4, 3, g, False, 0, out=out, want_codes=True),
         5 * n + 4 * G),
        ("fp4_e2m1_g128_asym_codes", lambda w, out: K.quantize_fp(w, 2, 1, g, False, 0, out=out, want_codes=True),
         4.5 * n + 4 * G),
        ("fp4_grid_g128", lambda w, out: K.fp4_grid(w, g), 4 * n + 2 * G),
        ("bfp_w4_g128", lambda w, out: K.quantize_bfp(w, 4, g, out=out), 4 * n),
        ("bfp_w8_g32", lambda w, out: K.quantize_bfp(w, 8, 32, out=out), 4 * n),
        ("approx_fp8_g128", lambda w, out: K.quantize_fp_approx(w, 4, 3, g, 0, 12, 15, 1, False, out=out), 4 * n + 2 * G),
        # double: one pass (k_apx_double_lut, g in {32, 64, 128}): read w, write dequant + scales
        ("approx_fp8_g128_double", lambda w, out: K.quantize_fp_approx(w, 4, 3, g, 0, 12, 15, 1, True, out=out),
         4 * n + 2 * G),
    ]
    # packed inputs of the unpack paths: codes + scales (+ zeros) of every copy
    packs = {}

    def packed(fmt):
        if fmt not in packs:
            if fmt == "grid":
                packs[fmt] = [K.fp4_grid(w, g, want_codes=True) for w in ws]
            else:
                e, m, sym = fmt
                packs[fmt] = [K.quantize_fp(w, e, m, g, sym, 0, want_codes=True) for w in ws]
        return packs[fmt]
    unpack = [
        ("fp4_grid_g128_codes (pack)", lambda i, w, out: K.fp4_grid(w, g, want_codes=True), 4 * n + 2 * G + n // 2),
        ("unpack_fp8_e4m3_g128_sym", ("e4m3s", (4, 3, True)), 3 * n + 2 * G),
        ("unpack_fp8_e4m3_g128_asym", ("e4m3a", (4, 3, False)), 3 * n + 4 * G),
        ("unpack_fp6_e3m2_g128_asym", ("e3m2a", (3, 2, False)), 3 * n + 4 * G),
        ("unpack_fp4_e2m1_g128_asym", ("e2m1a", (2, 1, False)), 2.5 * n + 4 * G),
        ("unpack_fp4_grid_g128", ("grid", "grid"), 2.5 * n + 2 * G),
    ]
    for name, spec, algo in unpack:
        if callable(spec):
            cases.append((name, spec, algo))
            continue
        fmt = spec[1]
        e, m = (2, 1) if fmt == "grid" else fmt[:2]

        def f1(i, w, out, fmt=fmt, e=e, m=m):
            r = packed(fmt)[i]
            K.dequant_fp_packed(r.codes, r.scales, r.zeros, e, m, g, R, C, out=out)
        cases.append((name, f1, algo))
    only = set(a.only.split(",")) if a.only else None
    for name, f1, algo in cases:
        if only is not None and name not in only:
            continue
        if f1.__code__.co_argcount == 2:
            f1 = (lambda f: (lambda i, w, out: f(w, out)))(f1)

        def fn(f1=f1):
            for i, (w, out) in enumerate(zip(ws, outs)):
                f1(i, w, out)
        fn()
        torch.cuda.synchronize()
        t = timed(fn, a.reps) / len(ws)
        print(json.dumps({**({"tag": a.tag} if a.tag else {}), "path": name, "shape": [R, C], "copies": len(ws), "ms": round(t * 1e3, 4),
                          "weights_GBps": round(2 * n / t / 1e9, 1), "algo_bytes": int(algo),
                          "achieved_GBps": round(algo / t / 1e9, 1), "frac_of_8TBps": round(algo / t / PEAK, 3)}),
              flush=True)


if __name__ == "__main__":
    main()

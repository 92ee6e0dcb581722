"""Where the fixed cost of a short streaming kernel goes (decode GEMV, single-call quantize).

A cold decode GEMV call costs ~t0 + bytes / BW with t0 ~ 2.5 us (BENCH fused_forward M = 1: 8.4 MB
in 4.2 us, 22.5 MB in 6.5 us).  Each arm below is a hipGraph of CALLS dependent launches (per-call
device time = replay time / CALLS, median of 5 replays), so the inter-kernel boundary is included:
  fill16       a one-wave fill of 16 halves: the graph's per-kernel floor
  gemv K=<k>   the default M = 1 GEMV on [N, K] tile-layout codes, cold (distinct copies) / warm
  probe        (IWQ_AB=1) A/B variants given by --variants on q_proj, cold
  quant <r>x<c> pseudo_quantize_tensor's device path, cold
One JSON line per arm."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def graph_us(calls, rounds=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for c in calls:
            c()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for c in calls:
            c()
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
        out.append(e0.elapsed_time(e1) * 1e3 / len(calls))
    del g
    return sorted(out)[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=128)
    ap.add_argument("--variants", default="")
    ap.add_argument("--group", type=int, default=-2)
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    dev = "cuda"
    y16 = torch.empty(16, dtype=torch.float16, device=dev)
    print(json.dumps({"arm": "fill16", "us": round(graph_us([lambda: y16.fill_(1.0)] * a.calls), 3)}), flush=True)

    def gemv_arm(N, Kd, warm=False, variant=0, tag=""):
        w = torch.empty(N, Kd, dtype=torch.float16, device=dev)
        K.fill_synthetic(w, 7)
        r = K.quantize_minmax(w, 4, a.group, False, 0, want_codes=True)
        tiled = K.tile_codes(r.codes, N, Kd)
        ncopy = 1 if warm else max(2, min(a.calls, int((1 << 30) // tiled.numel())))
        copies = [tiled] + [tiled.clone() for _ in range(ncopy - 1)]
        x = torch.randn(1, Kd, device=dev).half()
        y = torch.empty(1, N, dtype=torch.float16, device=dev)
        fl = K.gemm_variant_flags(variant)
        calls = [(lambda c=copies[i % ncopy]: K.w4a16_gemm(x, c, r.scales, r.zeros, 4, a.group, N, tiled=True,
                                                           out=y, flags=fl)) for i in range(a.calls)]
        us = graph_us(calls)
        nb = tiled.numel() + r.scales.numel() * 2 + (r.zeros.numel() * 2 if r.zeros is not None else 0)
        print(json.dumps({"arm": f"gemv{tag}", "N": N, "K": Kd, "warm": warm, "variant": variant, "copies": ncopy,
                          "us": round(us, 3), "bytes": nb, "GBps": round(nb / us / 1e3, 1)}), flush=True)
        del copies, tiled, w, r
        torch.cuda.empty_cache()

    for N, Kd in ((4096, 128), (4096, 512), (4096, 1024), (4096, 2048), (4096, 4096), (256, 4096), (1024, 4096),
                  (11008, 4096), (4096, 11008)):
        gemv_arm(N, Kd)
    gemv_arm(4096, 4096, warm=True)
    gemv_arm(11008, 4096, warm=True)
    for v in [int(v) for v in a.variants.split(",") if v]:
        gemv_arm(4096, 4096, variant=v, tag="_variant")

    for rows, cols in ((64, 4096), (512, 4096), (2048, 4096), (4096, 4096)):
        n = max(2, min(a.calls, int((1 << 30) // (rows * cols * 4))))
        ws = [torch.empty(rows, cols, dtype=torch.float16, device=dev) for _ in range(n)]
        for i, w in enumerate(ws):
            K.fill_synthetic(w, 100 + i)
        outs = [torch.empty_like(w) for w in ws]
        calls = [(lambda i=i % n: K.quantize_minmax(ws[i], 4, 128, False, 0, out=outs[i])) for i in range(a.calls)]
        us = graph_us(calls)
        nb = rows * cols * 4 + rows * cols // 128 * 4
        print(json.dumps({"arm": "quant", "shape": f"{rows}x{cols}", "copies": n, "us": round(us, 3),
                          "GBps": round(nb / us / 1e3, 1)}), flush=True)
        del ws, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

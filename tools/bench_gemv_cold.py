"""Decode GEMV (kernels.w4a16_gemm, M <= 16) timed COLD: every call reads a different resident copy
of the packed weight (rotation over >= --rot-bytes of codes, default 1 GiB), so the 256 MB MALL
holds none of a call's codes -- what a real token step sees (a 7B/70B INT4 model is 3.5/35 GB of
codes, each layer read once per token).  tools/bench_gemm.py re-runs ONE weight, which is
MALL-warm for every Llama shape (<= 118 MB of codes).

One JSON line per (shape, M, layout, variant): device time per call from a hipGraph of the whole
rotation, median of 5 replays; packed-weight bytes / time.  Also the row-major hipBLASLt reference
F.linear(x, W_deq) on rotated fp16 weights.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"q_proj": (4096, 4096), "gate_proj": (11008, 4096), "down_proj": (4096, 11008),
          "70b_gate": (28672, 8192), "70b_down": (8192, 28672), "70b_q": (8192, 8192),
          "qkv_fused": (12288, 4096), "gate_up_fused": (22016, 4096)}


def graph_time(calls, rounds=5):
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
        out.append(e0.elapsed_time(e1) / len(calls))
    out.sort()
    del g
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="q_proj,gate_proj,down_proj,70b_gate,70b_down")
    ap.add_argument("--m", default="1,4,16")
    ap.add_argument("--group", type=int, default=-2)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--layouts", default="tiled,row")
    ap.add_argument("--rot-bytes", type=float, default=float(1 << 30))
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--lib", default="", help="A/B: load this libiwq.so build instead of the tree's")
    ap.add_argument("--tag", default="", help="A/B: label added to every line")
    a = ap.parse_args()
    if a.lib:
        from iron_weight_only_quant_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    from iron_weight_only_quant_amd import kernels
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        w = torch.empty(N, K, dtype=torch.float16, device="cuda")
        kernels.fill_synthetic(w, 7)
        r = kernels.quantize_minmax(w, 4, a.group, False, 0, want_codes=True)
        cbytes = r.codes.numel()
        copies = max(4, int(a.rot_bytes // cbytes) + 1)
        rows = [r.codes.clone() for _ in range(copies)]
        tiles = [kernels.tile_codes(c, N, K) for c in rows] if "tiled" in a.layouts else []
        wbytes = int(cbytes + r.scales.numel() * 2 + (r.zeros.numel() * 2 if r.zeros is not None else 0))
        ref_w = None
        if not a.no_ref:
            nref = max(2, int(a.rot_bytes // (N * K * 2)) + 1)
            ref_w = [r.out.clone() for _ in range(nref)]
        for M in [int(m) for m in a.m.split(",")]:
            x = (torch.randn(M, K, device="cuda") * 0.5).half()
            y = torch.empty(M, N, dtype=torch.float16, device="cuda")
            want = torch.nn.functional.linear(x, r.out).float()
            t_ref = None
            if ref_w is not None:
                t_ref = graph_time([(lambda wt=wt: torch.nn.functional.linear(x, wt)) for wt in ref_w])
            for layout in a.layouts.split(","):
                srcs = tiles if layout == "tiled" else rows
                y0 = None
                for v in [int(t) for t in a.variants.split(",")]:
                    fl = kernels.gemm_variant_flags(v)
                    # the batched decode's K-split needs zero counters: one zeroed workspace serves every
                    # call of the graph (they run in order on one stream and each leaves it zeroed)
                    wsb = kernels.gemm_workspace_bytes(M, N, K, a.group, fl) if M <= 16 else 0
                    zws = torch.zeros(wsb, dtype=torch.uint8, device="cuda") if wsb else None
                    mk = lambda c: (lambda: kernels.w4a16_gemm(x, c, r.scales, r.zeros, 4, a.group, N, flags=fl,
                                                               tiled=(layout == "tiled"), out=y,
                                                               zeroed_workspace=zws))
                    mk(srcs[0])()
                    torch.cuda.synchronize()
                    err = float((y.float() - want).abs().max())
                    if y0 is None:
                        y0 = y.clone()
                    same = bool(torch.equal(y.view(torch.int16), y0.view(torch.int16)))
                    t = graph_time([mk(c) for c in srcs])
                    rec = {"shape": name, "N": N, "K": K, "M": M, "group": a.group, "layout": layout,
                           "variant": v, "copies": len(srcs), "us": round(t * 1e3, 2),
                           "weight_GBps": round(wbytes / t / 1e6, 1),
                           "frac_of_8TBps": round(wbytes / t / 1e6 / 8000, 3),
                           "hipblaslt_fp16_us": round(t_ref * 1e3, 2) if t_ref else None,
                           "speedup_vs_F_linear": round(t_ref / t, 3) if t_ref else None,
                           "max_abs_diff_vs_F_linear": err, "bits_equal_first_variant": same}
                    if a.tag:
                        rec["tag"] = a.tag
                    print(json.dumps(rec), flush=True)
        del rows, tiles, ref_w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

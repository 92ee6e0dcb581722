"""Where should QuantLinear(fused_forward="auto") take the packed-code kernels?  COLD A/B of the
reference forward F.linear(x, W_deq) (hipBLASLt on the resident fp16 weight) against the fused
forward kernels.w4a16_gemm on the packed codes (tiled codes at M <= 16, as "auto" keeps them), per
Llama-2-7B shape, per M, per channel and g128.  Cold: each timed pass walks C distinct weight copies
(>= 1 GB of fp16, so the 256 MB MALL holds none of them), as a model forward touches each layer's
weight once; per-call time = pass time / C, median of rounds, arms interleaved in rotating order.
Each pass is captured in a hipGraph and replayed, so the time is DEVICE time (--eager: eager calls,
which at small M measure the host launch cost instead).  One JSON line per (group, shape, M).
--packed: the packed-only forward instead (PackedLinear / kernels.w4a16_linear, no fp16 weight held):
the fused kernels against dequant-once (iwq_dequant_packed) + F.linear, cold over >= --gb of CODES."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"q_proj": (4096, 4096), "gate_proj": (11008, 4096), "down_proj": (4096, 11008),
          "qkv_proj": (12288, 4096), "gate_up_proj": (22016, 4096)}  # the last two: fused-projection probes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,8,16,24,32,48,64,96,128,192,255")
    ap.add_argument("--groups", default="-2,128")
    ap.add_argument("--shapes", default="q_proj,gate_proj,down_proj")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--gb", type=float, default=1.2)
    ap.add_argument("--eager", action="store_true", help="time eager calls (host launch cost included)")
    ap.add_argument("--packed", action="store_true", help="fused vs dequant-once + F.linear (packed-only weights)")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels
    for group in [int(g) for g in a.groups.split(",")]:
        for name in a.shapes.split(","):
            N, K = SHAPES[name]
            copies = max(4, int(a.gb * 1e9 / (N * K * (0.5 if a.packed else 2))) + 1)
            ws, cs, ts, ss, zs = [], [], [], [], []
            for c in range(copies):
                w = torch.empty(N, K, dtype=torch.float16, device="cuda")
                kernels.fill_synthetic(w, 100 + c)
                r = kernels.quantize_minmax(w, 4, group, False, 0, out=w, want_codes=True)
                ws.append(None if a.packed else w)
                cs.append(r.codes)
                ts.append(kernels.tile_codes(r.codes, N, K))
                ss.append(r.scales)
                zs.append(r.zeros)
            for M in [int(m) for m in a.ms.split(",")]:
                x = (torch.randn(M, K, device="cuda") * 0.5).half()
                y = torch.empty(M, N, dtype=torch.float16, device="cuda")

                def ref():
                    for c in range(copies):
                        if a.packed:  # kernels.w4a16_linear above FUSED_MAX_M
                            torch.nn.functional.linear(x, kernels.dequant_packed(cs[c], ss[c], zs[c], 4, group, N, K))
                        else:
                            torch.nn.functional.linear(x, ws[c])

                def fused():
                    tiled = M <= kernels.GEMV_MAX_M
                    for c in range(copies):
                        kernels.w4a16_gemm(x, ts[c] if tiled else cs[c], ss[c], zs[c], 4, group, N, None,
                                           tiled=tiled, out=y)
                arms = {"hipblaslt": ref, "fused": fused}
                for f in arms.values():
                    f()
                torch.cuda.synchronize()
                if not a.eager:  # device time: each pass captured once, replayed (no host launch cost)
                    graphs = {}
                    for k, f in arms.items():
                        s = torch.cuda.Stream()
                        s.wait_stream(torch.cuda.current_stream())
                        with torch.cuda.stream(s):
                            f()
                        torch.cuda.current_stream().wait_stream(s)
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g):
                            f()
                        graphs[k] = g
                    arms = {k: g.replay for k, g in graphs.items()}
                    for f in arms.values():
                        f()
                    torch.cuda.synchronize()
                times = {k: [] for k in arms}
                keys = list(arms)
                for rd in range(a.rounds):
                    for k in keys[rd % 2:] + keys[:rd % 2]:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        arms[k]()
                        e1.record()
                        torch.cuda.synchronize()
                        times[k].append(e0.elapsed_time(e1) * 1e3 / copies)
                med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
                print(json.dumps({"mode": ("packed-" if a.packed else "") + ("eager" if a.eager else "graph"), "group": group, "shape": name, "M": M, "copies": copies,
                                  "hipblaslt_us": round(med["hipblaslt"], 2), "fused_us": round(med["fused"], 2),
                                  "fused_speedup": round(med["hipblaslt"] / med["fused"], 3)}), flush=True)
            del ws, cs, ts, ss, zs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

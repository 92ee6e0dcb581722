"""Cold single-call replay of pseudo_quantize_tensor's device path per Llama-2-7B shape (bench.py
per_shape's method: CALLS calls on distinct resident weights captured in one hipGraph), for a
rocprofv3 --kernel-trace run that splits each call into kernel time and the inter-kernel boundary
(tools/trace_gaps.py reads the trace).  Prints the event-timed us per call per shape too.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/single_trace.py
    python3 tools/trace_gaps.py OUT"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096,4096x11008,11008x4096")
    ap.add_argument("--calls", type=int, default=32)
    ap.add_argument("--replays", type=int, default=5)
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--inplace", action="store_true", help="write the dequantized weight over the input")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    fl = K.gemm_variant_flags(a.variant)
    for shp in a.shapes.split(","):
        r, c = (int(v) for v in shp.split("x"))
        ws = [torch.empty(r, c, dtype=torch.float16, device="cuda") for _ in range(a.calls)]
        outs = ws if a.inplace else [torch.empty_like(w) for w in ws]
        for i, w in enumerate(ws):
            K.fill_synthetic(w, 100 + i)
        fns = [(lambda i=i: K.quantize_minmax(ws[i], a.bits, a.group, False, 0, out=outs[i], flags=fl))
               for i in range(a.calls)]
        for f in fns:
            f()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for f in fns:
                f()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for f in fns:
                f()
        g.replay()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        ts = []
        for _ in range(a.replays):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            g.replay()
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / a.calls)
        ts.sort()
        n = r * c
        alg = n * 4 + (n // a.group) * 4
        us = ts[len(ts) // 2]
        print(json.dumps({"shape": shp, "variant": a.variant, "inplace": a.inplace, "us_per_call": round(us, 2),
                          "frac": round(alg / (us * 1e-6) / 8e12, 4)}), flush=True)
        del g, ws, outs, fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Per-tensor (w_group_size = -1) quantization by storage dtype, cold single calls: the one-pass
kernel (variant 8, forced; the default takes it from 32 MiB, 16 MiB for bf16) against the reduce +
apply pair (variant 6), fp16 / bf16 / fp32;
arms "0z" / "8z": on a caller-zeroed workspace (IWQ_FLAG_WS_ZEROED: no zeroing launch,
what eager calls get from the per-stream cache).
Per call device time from a hipGraph over distinct resident copies (>= 1 GiB per replay), median of 5
replays; algorithmic bytes = read + write of the weight (+ the scale / zero).  One JSON line per arm.

    python tools/bench_tensor_dt.py [--shapes 4096x4096,11008x4096] [--dtypes float16,bfloat16,float32]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.gemv_floor import graph_us  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096,11008x4096")
    ap.add_argument("--dtypes", default="float16,bfloat16,float32")
    ap.add_argument("--variants", default="0,0z,8z,6")
    ap.add_argument("--bits", type=int, default=4)
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    for shp in a.shapes.split(","):
        rows, cols = (int(v) for v in shp.split("x"))
        for dn in a.dtypes.split(","):
            dt = getattr(torch, dn)
            eb = torch.tensor([], dtype=dt).element_size()
            n = max(2, min(32, int((1 << 30) // (rows * cols * eb * 2))))
            ws = [torch.empty(rows, cols, dtype=dt, device="cuda") for _ in range(n)]
            for i, w in enumerate(ws):
                K.fill_synthetic(w, 300 + i)
            outs = [torch.empty_like(w) for w in ws]
            wsb = int(K.L.load().iwq_workspace_bytes(rows, cols, -1, 0))
            zw = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
            for v in a.variants.split(","):
                fl = K.gemm_variant_flags(int(v.rstrip("z")))
                kw = {"zeroed_workspace": zw} if v.endswith("z") else {}
                calls = [(lambda i=i: K.quantize_minmax(ws[i], a.bits, -1, False, 0, out=outs[i], flags=fl, **kw))
                         for i in range(n)]
                us = graph_us(calls)
                alg = rows * cols * eb * 2 + 2 * eb
                print(json.dumps({"shape": shp, "dtype": dn, "variant": v, "copies": n, "us": round(us, 2),
                                  "alg_GBps": round(alg / us / 1e3, 1),
                                  "frac_of_8TBps": round(alg / us / 1e3 / 8000, 4)}), flush=True)
            del ws, outs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

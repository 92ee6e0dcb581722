"""A/B two builds of libiwq.so on the quant_dim = 1 column kernel, in separate processes on one box:

    python tools/ab_col_lib.py --lib iron_weight_only_quant_amd/_lib/libiwq_base.so --tag base

prints one JSON line per group (INT4 asym, [11008, 4096] fp16, cold rotation over 16 copies,
hipGraph replay, median of 5 rounds after a 1 s clock ramp).  Alternate the libraries over rounds."""
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
    ap.add_argument("--lib", required=True)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--groups", default="128,64,32")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    from iron_weight_only_quant_amd import kernels as K
    from tools.bench_formats import timed
    ws = []
    for c in range(16):
        t = torch.empty(11008, 4096, dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, 7 + c)
        ws.append(t)
    outs = [torch.empty_like(t) for t in ws]
    n = 11008 * 4096
    for g in (int(x) for x in a.groups.split(",")):
        t_end = time.time() + 1.0
        while time.time() < t_end:
            for w, o in zip(ws, outs):
                K.quantize_minmax(w, 4, g, False, 1, out=o)
        torch.cuda.synchronize()
        i = [0]

        def call():
            K.quantize_minmax(ws[i[0] % 16], 4, g, False, 1, out=outs[i[0] % 16])
            i[0] += 1
        us = timed(call, 16) * 1e6
        alg = 4 * n + 4 * (n // g)
        print(json.dumps({"tag": a.tag, "group": g, "us": round(us, 2),
                          "frac_of_8TBps": round(alg / us / 1e3 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()

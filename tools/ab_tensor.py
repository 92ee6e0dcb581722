"""A/B the per-tensor (q_group_size = -1) kernel-pair variants (iwq_minmax.hip launch_tensor_t) on
single weights, COLD: the calls rotate over --copies distinct resident tensors (>= 1 GB per replay),
so only what the reduce pass itself left in the MALL can help the apply pass.  One JSON line per
(shape, variant): graph-replayed device time per call, algorithmic 4 B/elem rate."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.bench_formats import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="11008x4096,4096x4096")
    ap.add_argument("--variants", default="0,2,3")
    ap.add_argument("--rot-bytes", type=float, default=float(1 << 30))
    ap.add_argument("--codes", action="store_true")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    for shp in a.shapes.split(","):
        rows, cols = (int(t) for t in shp.split("x"))
        n = rows * cols
        copies = max(2, int(a.rot_bytes // (4 * n)) + 1)
        ws, outs = [], []
        for c in range(copies):
            w = torch.empty(rows, cols, dtype=torch.float16, device="cuda")
            K.fill_synthetic(w, 11 + c)
            ws.append(w)
            outs.append(torch.empty_like(w))
        ref = K.quantize_minmax(ws[0], 4, -1, False, want_codes=a.codes)
        for v in [int(t) for t in a.variants.split(",")]:
            fl = (v & 0xFF) << 16
            r = K.quantize_minmax(ws[0], 4, -1, False, want_codes=a.codes, flags=fl)
            same = torch.equal(r.out.view(torch.int16), ref.out.view(torch.int16)) and \
                torch.equal(r.scales.view(torch.int16), ref.scales.view(torch.int16))

            def run(v=v):
                for w, o in zip(ws, outs):
                    K.quantize_minmax(w, 4, -1, False, out=o, want_codes=a.codes, flags=fl)
            t = timed(run, 2) / copies
            print(json.dumps({"path": "int4_per_tensor" + ("_codes" if a.codes else ""), "variant": v,
                              "shape": [rows, cols], "copies": copies, "us": round(t * 1e6, 2),
                              "achieved_GBps": round(4 * n / t / 1e9, 1),
                              "frac_of_8TBps": round(4 * n / t / 8e12, 3), "identical_to_v0": same}), flush=True)
        del ws, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""In-process A/B of the FP pack kernels' forms (A/B library, IWQ_AB=1): bench.py's formats rows
(pack = fake-quant + codes on [11008, 4096] fp16, g128, cold over 16 resident copies, hipGraph
replays) for each variant in --variants, interleaved over --rounds; every variant's output, codes,
scales and zeros are checked bit for bit against variant 0 first.
    IWQ_AB=1 python tools/ab_fp_variants.py --formats 2:1:asym,4:3:asym --variants 0,1,2"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--formats", default="2:1:asym,4:3:asym,4:3:sym")
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rows", type=int, default=11008)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    from iron_weight_only_quant_amd import kernels as K
    rows, cols, g = a.rows, a.cols, 128
    n, G = rows * cols, rows * cols // 128
    ws = []
    for c in range(a.copies):
        t = torch.empty(rows, cols, dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, 100 + c)
        ws.append(t)
    outs = [torch.empty_like(t) for t in ws]
    fh = open(a.out, "a") if a.out else None
    variants = [int(v) for v in a.variants.split(",")]
    for spec in a.formats.split(","):
        e, m, kind = spec.split(":")
        e, m, sym = int(e), int(m), kind == "sym"
        cb = n if 1 + e + m > 4 else n // 2
        alg = 4 * n + cb + 2 * G * (1 if sym else 2)
        ref = K.quantize_fp(ws[0], e, m, g, sym, 0, want_codes=True)
        torch.cuda.synchronize()
        for v in variants:
            r = K.quantize_fp(ws[0], e, m, g, sym, 0, want_codes=True, flags=v << 16)
            torch.cuda.synchronize()
            same = (torch.equal(r.out.view(torch.int16), ref.out.view(torch.int16)) and torch.equal(r.codes, ref.codes)
                    and torch.equal(r.scales.view(torch.int16), ref.scales.view(torch.int16))
                    and (sym or torch.equal(r.zeros.view(torch.int16), ref.zeros.view(torch.int16))))
            assert same, f"variant {v} differs on E{e}M{m} {kind}"
        for rnd in range(a.rounds):
            for v in variants:
                calls = [(lambda w=w, o=o, v=v: K.quantize_fp(w, e, m, g, sym, 0, out=o, want_codes=True, flags=v << 16))
                         for w, o in zip(ws, outs)]
                t = bench._graph_ms(calls) / 1e3
                rec = {"fmt": f"E{e}M{m}_{kind}", "variant": v, "round": rnd, "us": round(t * 1e6, 2),
                       "frac": round(alg / t / 1e9 / 8000, 4)}
                line = json.dumps(rec)
                print(line, flush=True)
                if fh:
                    fh.write(line + "\n")


if __name__ == "__main__":
    main()

"""Runner for PMC passes over the FP pack kernels (BASELINE configs[4], bench.py formats rows):
FP8 E4M3 g128 sym / asym and FP4 E2M1 g128 asym pack (fake-quant + codes) on [11008, 4096] fp16,
REPS calls each over distinct copies (cold), eager.  Kernel names tell the arms apart
(k_fp_group_lut<CODEC, G, SYM, GS, BATCHED, CODES>).

    rocprofv3 --pmc ... -- python3 tools/fp_pack_run.py [--reps 8]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--arms", default="e4m3_sym,e4m3_asym,e2m1_asym")
    a = ap.parse_args()
    from iron_weight_only_quant_amd import kernels as K
    ws = []
    for c in range(a.reps):
        t = torch.empty(11008, 4096, dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, 100 + c)
        ws.append(t)
    outs = [torch.empty_like(t) for t in ws]
    arms = {"e4m3_sym": (4, 3, True), "e4m3_asym": (4, 3, False), "e2m1_asym": (2, 1, False)}
    for name in a.arms.split(","):
        e, m, sym = arms[name]
        for w, o in zip(ws, outs):
            K.quantize_fp(w, e, m, 128, sym, 0, out=o, want_codes=True)
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()

"""A/B of the double-approximate decode kernel variants (iwq_fp.hip k_apx_double_lut, flags bits 16..23):
cold (16 distinct 11008x4096 fp16 weights per pass), interleaved, median of rounds; bit-identity vs v0
for real variants (diagnostic ones are reported but not compared)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from iron_weight_only_quant_amd import kernels as K  # noqa: E402

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,2,3,1").split(",")]
diag = {1}
rows, cols, copies, g = 11008, 4096, 16, 128
ws = []
for c in range(copies):
    w = torch.empty(rows, cols, dtype=torch.float16, device="cuda")
    K.fill_synthetic(w, 300 + c)
    ws.append(w)
outs = [torch.empty_like(w) for w in ws]
ref = K.quantize_fp_approx(ws[0], 4, 3, g, 0, 12, 15, 1, True).out.clone()


def run(v):
    for w, o in zip(ws, outs):
        K.quantize_fp_approx(w, 4, 3, g, 0, 12, 15, 1, True, out=o, flags=K.gemm_variant_flags(v))


for v in variants:
    run(v)
torch.cuda.synchronize()
times = {v: [] for v in variants}
for r in range(9):
    for v in variants[r % len(variants):] + variants[:r % len(variants)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(v)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) * 1e3 / copies)
for v in variants:
    run(v)
    same = None if v in diag else bool(torch.equal(outs[0].view(torch.int16), ref.view(torch.int16)))
    t = sorted(times[v])[len(times[v]) // 2]
    print(json.dumps({"variant": v, "us": round(t, 2), "GBps": round(rows * cols * 4 / t / 1e3, 1),
                      "identical_to_v0": same}), flush=True)

"""In-process A/B of the headline batched launch (Llama-2-7B, INT4 g=128 asym) over memory layouts
and store policies, on the same box, interleaved rounds (cdna_hip_programming.md §5.4 rule 24):

  oop      out-of-place, every weight and output its own allocation (bench.py default)
  inplace  dequantized weights written over the inputs (QuantLinear.quantize_weight semantics)
  adj      out-of-place, input i and output i adjacent in one allocation ([in0|out0|in1|out1|...])
  v<N>     oop with kernel variant N (iwq_minmax.hip launch_variant)

Prints one JSON line per arm: median / min ms per launch and achieved GB/s (4.03 B/elem)."""
import argparse
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="oop,inplace,adj,v13,v14")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    from iron_weight_only_quant_amd import kernels, shard
    try:
        smi = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True, timeout=30).stdout
        print(json.dumps({"rocm_smi_clocks": [l for l in smi.splitlines() if "clk" in l.lower()][:12]}), flush=True)
    except Exception as e:  # informational only
        print(json.dumps({"rocm_smi_error": str(e)}), flush=True)
    shapes = shard.model_linear_shapes("llama2-7b")
    ws = []
    for i, (_, (r, c)) in enumerate(shapes):
        t = torch.empty((r, c), dtype=torch.float16, device="cuda")
        kernels.fill_synthetic(t, seed=i)
        ws.append(t)
    numel = sum(w.numel() for w in ws)
    arms = args.arms.split(",")
    plans = {}
    for a in arms:
        if a == "oop" or a.startswith("v"):
            if "oop" not in plans:
                plans["oop"] = kernels.BatchPlan(ws, 4, 128, False)
            plans[a] = plans["oop"]
        elif a == "inplace":
            ws2 = [w.clone() for w in ws]
            plans[a] = kernels.BatchPlan(ws2, 4, 128, False, outs=ws2)
        elif a == "adj":
            flat = torch.empty(2 * numel, dtype=torch.float16, device="cuda")
            ins, outs, off = [], [], 0
            for w in ws:
                n = w.numel()
                iv = flat[off: off + n].view(w.shape)
                iv.copy_(w)
                ins.append(iv)
                outs.append(flat[off + n: off + 2 * n].view(w.shape))
                off += 2 * n
            plans[a] = kernels.BatchPlan(ins, 4, 128, False, outs=outs)
    stream = torch.cuda.current_stream()
    var = {a: (int(a[1:]) if a.startswith("v") else 0) for a in arms}
    # clock ramp ~1 s
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for a in arms:
            plans[a].run(stream, variant=var[a])
        torch.cuda.synchronize()
    times = {a: [] for a in arms}
    for _ in range(args.rounds):
        for a in arms:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.steps):
                plans[a].run(stream, variant=var[a])
            e1.record(stream)
            torch.cuda.synchronize()
            times[a].append(e0.elapsed_time(e1) / args.steps)
    alg = numel * 4 + (numel // 128) * 4
    for a in arms:
        t = sorted(times[a])
        med = t[len(t) // 2]
        print(json.dumps({"arm": a, "ms": round(med, 4), "ms_min": round(t[0], 4),
                          "GBps": round(alg / med / 1e6, 1), "frac": round(alg / med / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()

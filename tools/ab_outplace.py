"""Where the out-of-place outputs of the whole-model launch live, A/B (box-dependent out-of-place
penalty vs in place): the 224 Llama-2-7B weights quantized INT4 g128 by one batched launch into
  default   torch.empty_like per weight (what BatchPlan allocates)
  inplace   the weights themselves
  arena+S   one flat buffer, weight i's output at a running offset + i * S bytes of skew
HIP-event kernel time, best of 3 x 10 launches after a 1 s ramp; arms interleaved over --rounds."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--skews", default="0,4096,65536,1052672")
    a = ap.parse_args()
    import bench
    from iron_weight_only_quant_amd import kernels
    weights, names, _ = bench.make_weights("llama2-7b", 0, 1)
    numel = sum(w.numel() for w in weights)
    alg = numel * 4 + numel // 128 * 4
    arms = {"default": None, "inplace": weights}
    arenas = []
    for sk in (int(x) for x in a.skews.split(",")):
        total = sum(w.numel() * 2 for w in weights) + sk * len(weights) + 4096
        buf = torch.empty(total, dtype=torch.uint8, device="cuda")
        arenas.append(buf)
        outs, off = [], 0
        for w in weights:
            nb = w.numel() * 2
            outs.append(buf[off:off + nb].view(torch.float16).view(w.shape))
            off += (nb + sk + 255) // 256 * 256
        arms[f"arena+{sk}"] = outs
    plans = {k: kernels.BatchPlan(weights, 4, 128, False, outs=v) for k, v in arms.items()}
    bench.clock_ramp(plans["default"], 1.0)
    st = torch.cuda.current_stream()
    for rnd in range(a.rounds):
        for k, plan in plans.items():
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10):
                    plan.run(st)
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                best = ms if best is None else min(best, ms)
            print(json.dumps({"round": rnd, "arm": k, "ms": round(best, 4),
                              "frac": round(alg / (best * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()

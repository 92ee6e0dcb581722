"""End-to-end quantize_model wall time on a Llama-2-7B-shaped module tree (224 nn.Linear on one
GPU, synthetic fp16 weights): the drop-in call the reference's main.py makes (quant_wrapper.py:44-82),
host work included (module swap, buffers), batched (one launch per format) vs per layer.

Prints one JSON line per (format, mode): wall ms from the call to a device sync, and the kernel-only
share measured separately (bench_model_formats.py)."""
import argparse
import gc
import json
import os
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(model_name):
    from iron_weight_only_quant_amd import kernels as K
    from iron_weight_only_quant_amd import shard
    root = torch.nn.Module()
    for i, (name, (r, c)) in enumerate(shard.model_linear_shapes(model_name)):
        parent = root
        parts = name.split(".")
        for p in parts[:-1]:
            if not hasattr(parent, p):
                parent.add_module(p, torch.nn.Module())
            parent = getattr(parent, p)
        lin = torch.nn.Linear(c, r, bias=False, device="meta")
        lin.weight = torch.nn.Parameter(torch.empty(r, c, dtype=torch.float16, device="cuda"), requires_grad=False)
        K.fill_synthetic(lin.weight.data, seed=i)
        parent.add_module(parts[-1], lin)
    torch.cuda.synchronize()
    return root


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--formats", default="int,fp8")
    a = ap.parse_args()
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    for fmt in a.formats.split(","):
        for batched in (True, False):
            for rep in range(2):  # rep 0 includes the first launch of each kernel (code-object load)
                m = build(a.model)
                args = SimpleNamespace(w_bit=4 if fmt == "int" else 8, a_bit=16, w_group_size=128,
                                       w_symmetric=False, w_format=fmt, quant_dim=0)
                torch.cuda.synchronize()
                gc.collect()  # no collector pause left over from the previous model inside the timing
                t0 = time.perf_counter()
                quantize_model(m, args, batched=batched, verbose=False)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                print(json.dumps({"model": a.model, "format": fmt, "batched": batched, "rep": rep,
                                  "host_ms": round((t1 - t0) * 1e3, 2), "wall_ms": round((t2 - t0) * 1e3, 2)}),
                      flush=True)
                del m
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

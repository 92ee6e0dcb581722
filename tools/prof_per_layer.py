"""Host-side profile of the per-layer drop-in path (QuantLinear.from_linear -> quantize_weight ->
kernels.quantize_minmax) over a Llama-2-7B-shaped module tree: cProfile of quantize_model(batched=False)."""
import cProfile
import gc
import os
import pstats
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.bench_quantize_model import build  # noqa: E402


def main():
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    args = SimpleNamespace(w_bit=4, a_bit=16, w_group_size=128, w_symmetric=False, w_format="int", quant_dim=0)
    for rep in range(3):
        m = build("llama2-7b")
        torch.cuda.synchronize()
        gc.collect()
        pr = cProfile.Profile() if rep == 2 else None
        t0 = time.perf_counter()
        if pr:
            pr.enable()
        quantize_model(m, args, batched=False, verbose=False)
        if pr:
            pr.disable()
        torch.cuda.synchronize()
        print(f"rep {rep}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
        del m
        torch.cuda.empty_cache()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()

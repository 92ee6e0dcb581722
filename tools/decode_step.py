"""Decode-step linear time of a Llama-2-7B-shaped model: the 7 projections of each of 32 decoder layers
(q, k, v, o, gate, up: [.., 4096] in; down: [.., 11008] in) at M decode rows, QuantLinear(fused_forward=
"auto") 4-bit, unfused vs fuse_projections (one GEMV for q/k/v and one for gate/up), against the
reference forward (F.linear on the fp16 weights).  Each step is captured in a hipGraph and replayed,
so the times are device times; the 32 layers' weights are distinct (cold, as in a real decode step).
One JSON line per (group, M)."""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"q_proj": (4096, 4096), "k_proj": (4096, 4096), "v_proj": (4096, 4096), "o_proj": (4096, 4096),
          "gate_proj": (11008, 4096), "up_proj": (11008, 4096), "down_proj": (4096, 11008)}


class Layer(nn.Module):
    def __init__(self):
        super().__init__()
        for n, (o, i) in SHAPES.items():
            setattr(self, n, nn.Linear(i, o, bias=False, dtype=torch.float16, device="cuda"))

    def forward(self, x, h):
        return (self.q_proj(x), self.k_proj(x), self.v_proj(x), self.o_proj(x), self.gate_proj(x), self.up_proj(x),
                self.down_proj(h))


def step_time(model, x, h, rounds=7):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(2):
            model(x, h)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), torch.no_grad():
        model(x, h)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


class Model(nn.Module):
    def __init__(self, n):
        super().__init__()
        self.layers = nn.ModuleList(Layer() for _ in range(n))

    def forward(self, x, h):
        for layer in self.layers:
            layer(x, h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--ms", default="1,4,16")
    ap.add_argument("--groups", default="128,-2")
    a = ap.parse_args()
    from types import SimpleNamespace

    from iron_weight_only_quant_amd import kernels
    from iron_weight_only_quant_amd.fused_proj import fuse_projections, unfuse_projections
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    for group in [int(g) for g in a.groups.split(",")]:
        model = Model(a.layers)
        for i, lin in enumerate(m for m in model.modules() if isinstance(m, nn.Linear)):
            kernels.fill_synthetic(lin.weight.data, 1000 + i)
        ms = [int(m) for m in a.ms.split(",")]
        xs = {M: (torch.randn(M, 4096, device="cuda") * 0.5).half() for M in ms}
        hs = {M: (torch.randn(M, 11008, device="cuda") * 0.5).half() for M in ms}
        ref = {M: step_time(model, xs[M], hs[M]) for M in ms}  # fp16 weights: the reference forward
        quantize_model(model, SimpleNamespace(w_bit=4, a_bit=16, w_group_size=group, w_symmetric=False,
                                              w_format="int", quant_dim=0, fused_forward="auto"), verbose=False)
        unf = {M: step_time(model, xs[M], hs[M]) for M in ms}
        n = fuse_projections(model)
        fus = {M: step_time(model, xs[M], hs[M]) for M in ms}
        unfuse_projections(model)
        wbytes = sum(o * i for o, i in SHAPES.values()) * a.layers
        for M in ms:
            print(json.dumps({"group": group, "M": M, "layers": a.layers, "fused_groups": n,
                              "fp16_F_linear_us": round(ref[M], 1), "packed_us": round(unf[M], 1),
                              "packed_fused_proj_us": round(fus[M], 1),
                              "speedup_vs_F_linear": round(ref[M] / fus[M], 2),
                              "fusion_gain": round(unf[M] / fus[M], 3),
                              "packed_weight_TBps": round(wbytes * 0.5 / fus[M] / 1e6, 2)}), flush=True)
        del model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

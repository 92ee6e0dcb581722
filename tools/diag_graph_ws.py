"""Diagnostic: per-tensor one-pass calls (variant 8) captured in a hipGraph on a capture-allocated
workspace (zeroed by the captured memset), replayed on changing inputs: bits vs the oracle and the
workspace's hand-off words after each replay."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from iron_weight_only_quant_amd import kernels as K  # noqa: E402
from oracle import iwq_oracle as O  # noqa: E402
from oracle.synth import synth  # noqa: E402


def closure_ws(r):
    for c in r.retry.__closure__:
        v = c.cell_contents
        if isinstance(v, torch.Tensor) and v.dtype == torch.uint8 and v.numel() >= 4096:
            return v


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    shape = (1024, 2048)
    dev = [torch.empty(shape, dtype=torch.float16, device="cuda") for _ in range(n)]
    outs = [torch.empty_like(d) for d in dev]
    fl = K.gemm_variant_flags(8)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    res = []
    with torch.cuda.stream(s):
        for d, o in zip(dev, outs):
            K.quantize_minmax(d, 4, -1, False, 0, out=o, flags=fl)
        with torch.cuda.graph(g, stream=s):
            for d, o in zip(dev, outs):
                res.append(K.quantize_minmax(d, 4, -1, False, 0, out=o, flags=fl))
    torch.cuda.current_stream().wait_stream(s)
    wss = [closure_ws(r) for r in res]
    print("ws ptrs", [hex(w.data_ptr()) for w in wss], "flags", [hex(r.nan_flag.data_ptr()) for r in res], flush=True)
    for rnd in range(4):
        xs = [synth(200 + n * rnd + i, shape, "float16") * np.float16(1 + 5 * i) for i in range(n)]
        for d, x in zip(dev, xs):
            d.copy_(torch.from_numpy(x).cuda())
        torch.cuda.synchronize()
        pre = [w[:2080].view(torch.int64).cpu().numpy().copy() for w in wss]
        g.replay()
        torch.cuda.synchronize()
        for i, (x, o, r, w) in enumerate(zip(xs, outs, res, wss)):
            exp = O.quantlinear_int(x, 4, -1, False, 0, "float16")
            ok = np.array_equal(o.cpu().numpy().view(np.uint16), exp.dequant.view(np.uint16))
            post = w[:2080].view(torch.int64).cpu().numpy()
            print(f"rnd {rnd} call {i}: ok={ok} flag={int(r.nan_flag.item())} pre_nonzero={int((pre[i] != 0).sum())} "
                  f"post_nonzero={int((post != 0).sum())} pre_head={[hex(int(v)) for v in pre[i][:3]]} "
                  f"pre_tail={[hex(int(v)) for v in pre[i][254:260]]}", flush=True)


if __name__ == "__main__":
    main()

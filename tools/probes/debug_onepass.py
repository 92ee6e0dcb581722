"""Debug: per-tensor one-pass determinism on 4096x4096 (workspace granules inspected after each call)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from iron_weight_only_quant_amd import _lib as L, kernels as K  # noqa: E402

lib = L.load()
for rows, cols, nbits in ((4096, 4096, 4), (11008, 4096, 4), (4096, 4096, 8), (2048, 4096, 4)):
    x = torch.empty(rows, cols, dtype=torch.float16, device="cuda")
    K.fill_synthetic(x, 0)
    outs = []
    for it in range(6):
        out = torch.empty_like(x)
        sc = torch.empty(1, dtype=torch.float16, device="cuda")
        zr = torch.empty(1, dtype=torch.float16, device="cuda")
        ws = torch.full((32768,), 0x5A, dtype=torch.uint8, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        st = lib.iwq_quantize_minmax(L.ptr(x), rows, cols, cols, 0, nbits, -1, 0, 0, L.ptr(out), cols, None,
                                     L.ptr(sc), L.ptr(zr), L.ptr(ws), ws.numel(), L.ptr(flag), 0,
                                     L.stream_handle(x.device))
        torch.cuda.synchronize()
        g = ws[:2048].cpu().numpy().view(np.uint64)
        tags = (g >> 32)
        keys = g & 0xFFFFFFFF
        mn = (keys & 0xFFFF).astype(np.uint16).view(np.int16)
        mx = (keys >> 16).astype(np.uint16).view(np.int16)
        ntag1 = int((tags == 1).sum())
        print(rows, cols, nbits, "it", it, "st", st, "flag", int(flag.item()), "scale", sc.item(), "zero", zr.item(),
              "granules tag1", ntag1, "min", int(mn[tags == 1].min()), "max", int(mx[tags == 1].max()), flush=True)
        outs.append(out)
    for o in outs[1:]:
        d = (o.view(torch.int16) != outs[0].view(torch.int16))
        n = int(d.sum())
        if n:
            idx = d.nonzero()[:5].tolist()
            print("  DIFF count", n, "first", idx, [(float(outs[0][i, j]), float(o[i, j])) for i, j in idx], flush=True)
    r6 = K.quantize_minmax(x, nbits, -1, False, 0, flags=K.gemm_variant_flags(6))
    print("  vs pair:", int((r6.out.view(torch.int16) != outs[0].view(torch.int16)).sum()), "scale", r6.scales.item(),
          "zero", r6.zeros.item(), flush=True)

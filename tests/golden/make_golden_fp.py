"""Golden fixtures for the FP weight formats, produced FROM THE REFERENCE ITSELF (run only in the
build container; imports /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fp.py

Produces tests/golden/fp_small.npz (data only):
  * exhaustive encode tables: quant_linear._float_to_fp over every finite fp16 value, for E4M3,
    E3M2, E2M1 and E5M2 (configure_fp_formats), and the 256-entry _fp_to_float decode tables
  * torch.floor(torch.log2(x)) and floor(log2(x) + 1) over every positive finite fp16 value
  * QuantLinear FP4/FP6/FP8 branches (quant_linear.py:724-883): sym/asym x groups x quant_dim
  * fp4_quantize_cpu.quantize_fp16_to_fp4_e1m2 (the E2M1 "grid"), groups 32/128/per-tensor
  * SHA-256 of the reference outputs at 4096x4096 (oracle/synth.py seed 0) for FP8/FP4 g=128
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

import fp4_quantize_cpu  # noqa: E402  (reference)
import quant_linear  # noqa: E402  (reference)

from oracle.synth import synth  # noqa: E402

FORMATS = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e5m2": (5, 2)}


def all_finite_fp16():
    b = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    x = b.view(np.float16)
    return x[np.isfinite(x)]


def ref_ql_fp(x16, fmt_name, which, **kw):
    """Run QuantLinear.from_linear with weight_format=which ('fp4'|'fp6'|'fp8') under format fmt."""
    e, m = FORMATS[fmt_name]
    if which == "fp8":
        quant_linear.configure_fp_formats(fp8_exp_bits=e, fp8_mantissa_bits=m)
    elif which == "fp6":
        quant_linear.configure_fp_formats(fp6_exp_bits=e, fp6_mantissa_bits=m)
    else:
        quant_linear.configure_fp_formats(fp4_exp_bits=e, fp4_mantissa_bits=m)
    try:
        w = torch.from_numpy(np.ascontiguousarray(x16)).clone()
        lin = torch.nn.Linear(w.shape[1], w.shape[0], bias=False)
        lin.weight.data = w
        q = quant_linear.QuantLinear.from_linear(lin, weight_format=which, **kw)
        z = q.zeros
        return q.weight.data.numpy().copy(), q.scales.numpy().copy(), (None if z is None else z.numpy().copy())
    finally:
        quant_linear.configure_fp_formats()


def main():
    d = {}
    xs = all_finite_fp16()
    d["in/all_fp16"] = xs
    xt = torch.from_numpy(xs.copy())
    for name, (e, m) in FORMATS.items():
        bias = 2 ** (e - 1) - 1
        codes = quant_linear._float_to_fp(xt, e, m, bias)
        d[f"enc/{name}"] = codes.numpy().astype(np.uint8)
        dec = quant_linear._fp_to_float(torch.arange(256, dtype=torch.int32), e, m, bias)
        d[f"dec/{name}"] = dec.numpy().astype(np.float32)
    pos = xs[(xs > 0)]
    pt = torch.from_numpy(pos.copy())
    d["in/pos_fp16"] = pos
    d["log2/floor"] = torch.floor(torch.log2(pt)).numpy().astype(np.float32)
    d["log2/floor_plus1"] = torch.floor(torch.log2(pt) + 1).numpy().astype(np.float32)

    shp = (48, 256)
    x = synth(300, shp, "float16")
    # a few exact zeros and a one-sided row for the codec paths
    x[3, :] = np.abs(x[3, :])
    x[5, ::5] = 0.0
    d["in/fp_a"] = x
    for which, fmts in (("fp8", ("e4m3", "e5m2")), ("fp6", ("e3m2",)), ("fp4", ("e2m1",))):
        for fmt in fmts:
            for sym in (False, True):
                for qd in (0, 1):
                    for g in ((32, 128, -1, -2) if qd == 0 else (16, -1, -2)):
                        key = f"ql/{which}/{fmt}/{int(sym)}/{g}/{qd}"
                        try:
                            deq, s, z = ref_ql_fp(x, fmt, which, w_bit=8, w_group_size=g, symmetric=sym,
                                                  quant_dim=qd)
                        except RuntimeError:  # fp_max not representable in fp16 (E5M2: 114688)
                            d[key + "/error"] = np.zeros(1, np.uint8)
                            continue
                        d[key + "/deq"] = deq
                        d[key + "/scales"] = s
                        if z is not None:
                            d[key + "/zeros"] = z
    for g, pt_ in ((128, False), (32, False), (-1, True), (256, False)):
        out = fp4_quantize_cpu.quantize_fp16_to_fp4_e1m2(torch.from_numpy(x.copy()), group_size=g, per_tensor=pt_)
        d[f"grid/{g}/{int(pt_)}"] = out.numpy()
    big = synth(0, (4096, 4096), "float16")
    for which, fmt, sym in (("fp8", "e4m3", True), ("fp8", "e4m3", False), ("fp4", "e2m1", False)):
        deq, s, z = ref_ql_fp(big, fmt, which, w_bit=8, w_group_size=128, symmetric=sym)
        d[f"sha/{which}/{fmt}/{int(sym)}"] = np.frombuffer(hashlib.sha256(deq.tobytes()).digest(), np.uint8)
    out = fp4_quantize_cpu.quantize_fp16_to_fp4_e1m2(torch.from_numpy(big.copy()), group_size=128)
    d["sha/grid/128"] = np.frombuffer(hashlib.sha256(out.numpy().tobytes()).digest(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "fp_small.npz"), **d)
    print("fp fixtures:", len(d), "arrays")


if __name__ == "__main__":
    main()

"""Golden fixtures for the BFP and approximate / double-approximate FP weight formats, produced FROM
THE REFERENCE ITSELF (run only in the build container; imports /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_approx.py

Produces tests/golden/approx_small.npz (data only):
  * aligned-decode tables: quant_linear._fp_decode_aligned over every code of E4M3 / E3M2 / E2M1 /
    E1M2, several (hi_align_start, hi_align_exp_field, tail_pad_bits) settings
  * double-approximate decode of code quads: every E2M1 quad (65,536), 40,000 random E3M2 and
    E4M3 quads plus all E4M3 quads mixing a chosen exponent pair (covers the int8 wrap cases)
  * QuantLinear end to end: BFP (w_bit x group x quant_dim, fp16 / fp32 / bf16 weights, edge rows),
    approximate FP8 / FP6 / FP4 (E2M1 and E1M2), single and double, several groups / quant_dim
  * SHA-256 of reference outputs at 4096x4096 (oracle/synth.py seed 0)
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

import quant_linear  # noqa: E402  (reference)

from oracle.synth import synth  # noqa: E402

FORMATS = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e1m2": (1, 2)}
ALIGN_PARAMS = {
    "e4m3": [(12, 15, 1), (10, 14, 0), (12, 15, -1), (8, 15, 2)],
    "e3m2": [(4, 7, 2), (3, 6, 1), (4, 7, -1)],
    "e2m1": [(1, 1, 0), (1, 3, 1), (2, 3, 0), (1, 2, -1)],
    "e1m2": [(1, 1, 0), (1, 1, 1), (0, 1, -1)],
}
DOUBLE_PARAMS = {
    "e2m1": [(1, 1, 0), (2, 3, 1), (1, 2, -1)],
    "e3m2": [(4, 7, 2), (3, 6, -1)],
    "e4m3": [(12, 15, 1), (10, 15, 0), (12, 15, -1)],
}


def sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def ref_ql(w, **kw):
    lin = torch.nn.Linear(w.shape[1], w.shape[0], bias=False)
    lin.weight.data = w.clone()
    q = quant_linear.QuantLinear.from_linear(lin, **kw)
    return q


def set_fmt(which, e, m):
    quant_linear.configure_fp_formats(**{f"{which}_exp_bits": e, f"{which}_mantissa_bits": m})


def quads_e4m3(rng):
    """Random quads + all quads whose exponents are drawn from pairs that hit shifts 0..14."""
    r = rng.integers(0, 256, size=(4, 40000)).astype(np.uint8)
    ex = np.array([0, 1, 7, 8, 12, 15], dtype=np.int64)
    cols = []
    for a in ex:
        for b in ex:
            for s in range(4):
                c = np.zeros((4, 16), dtype=np.int64)
                c[:, :] = (a << 3) | (np.arange(16) & 7)
                c[s, :] = (b << 3) | ((np.arange(16) * 3) & 7)
                c[:, 8:] |= 0x80 * ((np.arange(4)[:, None] + s) % 2)
                cols.append(c)
    return np.concatenate([r] + [c.astype(np.uint8) for c in cols], axis=1)


def edge_rows(shape):
    x = synth(400, shape, "float16")
    f16 = np.float16
    x[0, :] = 0.0
    x[1, :] = -0.0
    x[2, :] = np.float16(6e-8) * (np.arange(shape[1]) % 7 - 3)                # subnormals
    x[3, : shape[1] // 2] = np.float16(65504.0)
    x[4, 5] = np.inf
    x[5, 7] = -np.inf
    x[6, 9] = np.nan
    x[7, :] = (np.arange(shape[1]) % 2 * 2 - 1).astype(f16) * f16(1e-4)
    x[8, ::3] = f16(3.0e4)
    x[9, :] = f16(1.0)
    return x


def main():
    d = {}
    # ---- aligned decode tables
    for name, (e, m) in FORMATS.items():
        bias = 2 ** (e - 1) - 1
        codes = torch.arange(1 << (1 + e + m), dtype=torch.int32)
        for (hs, hf, tp) in ALIGN_PARAMS[name]:
            v = quant_linear._fp_decode_aligned(codes, hs, hf, tp, e, m, bias, align_subnorm_exp_as_one=True,
                                                limit_align_exp_to_field=True, decode_dtype=torch.float16)
            d[f"adec/{name}/{hs}/{hf}/{tp}"] = v.numpy().astype(np.float32)
    # ---- double-approximate quads
    rng = np.random.default_rng(7)
    quads = {
        "e2m1": np.array(np.meshgrid(*[np.arange(16)] * 4, indexing="ij")).reshape(4, -1).astype(np.uint8),
        "e3m2": rng.integers(0, 64, size=(4, 40000)).astype(np.uint8),
        "e4m3": quads_e4m3(rng),
    }
    for name, q in quads.items():
        e, m = FORMATS[name]
        bias = 2 ** (e - 1) - 1
        d[f"dq_in/{name}"] = q
        for (hs, hf, tp) in DOUBLE_PARAMS[name]:
            v = quant_linear.fp_decode_aligned_double_approx(torch.from_numpy(q.copy()), hs, hf, tp, e, m, bias,
                                                              align_subnorm_exp_as_one=True, handle_max_outlier=True,
                                                              decode_dtype=torch.float16)
            d[f"dq/{name}/{hs}/{hf}/{tp}"] = v.numpy()
    # ---- BFP end to end
    shp = (32, 256)
    x = synth(401, shp, "float16")
    xe = edge_rows(shp)
    d["in/bfp_a"] = x
    d["in/bfp_edge"] = xe
    for tag, src in (("a", x), ("edge", xe)):
        for wb in (1, 2, 3, 4, 5, 8, 12, 13, 16):
            for qd in (0, 1):
                for g in ((8, 32, 128) if qd == 0 else (16,)):
                    q = ref_ql(torch.from_numpy(src.copy()), w_bit=wb, w_group_size=g, weight_format="bfp",
                               quant_dim=qd)
                    d[f"bfp/{tag}/{wb}/{g}/{qd}"] = q.weight.data.numpy().copy()
    xf = synth(402, (16, 128), "float32") * np.float32(3.0)
    xf[0, 3] = np.float32(1e-9)
    xf[1, :] = np.float32(7e4)   # beyond fp16 range: .to(float16) -> inf
    d["in/bfp_f32"] = xf
    xb = torch.from_numpy(xf.copy()).to(torch.bfloat16)
    d["in/bfp_bf16_bits"] = xb.view(torch.int16).numpy().view(np.uint16)
    for wb in (3, 4, 8):
        q = ref_ql(torch.from_numpy(xf.copy()), w_bit=wb, w_group_size=32, weight_format="bfp")
        d[f"bfp/f32/{wb}"] = q.weight.data.numpy().copy()
        q = ref_ql(xb.clone(), w_bit=wb, w_group_size=32, weight_format="bfp")
        d[f"bfp/bf16/{wb}"] = q.weight.data.view(torch.int16).numpy().view(np.uint16).copy()
    # ---- approximate end to end
    xa = synth(403, (32, 256), "float16")
    xa[2, :] = np.abs(xa[2, :])
    xa[4, ::4] = 0.0
    xa[6, 1] = -0.0
    d["in/apx_a"] = xa
    cases = [("fp8", "e4m3", dict(fp8_hi_align_start=12, fp8_hi_align_exp_field=15, fp8_tail_pad_bits=1)),
             ("fp8", "e4m3", dict(fp8_hi_align_start=10, fp8_hi_align_exp_field=15, fp8_tail_pad_bits=0)),
             ("fp6", "e3m2", dict(fp6_hi_align_start=4, fp6_hi_align_exp_field=7, fp6_tail_pad_bits=2)),
             ("fp6", "e3m2", dict(fp6_hi_align_start=3, fp6_hi_align_exp_field=6, fp6_tail_pad_bits=-1)),
             ("fp4", "e2m1", dict(fp4_hi_align_start=1, fp4_hi_align_exp_field=1, fp4_tail_pad_bits=0)),
             ("fp4", "e2m1", dict(fp4_hi_align_start=1, fp4_hi_align_exp_field=3, fp4_tail_pad_bits=1)),
             ("fp4", "e1m2", dict(fp4_hi_align_start=1, fp4_hi_align_exp_field=1, fp4_tail_pad_bits=0))]
    for ci, (which, fmt, params) in enumerate(cases):
        e, m = FORMATS[fmt]
        set_fmt(which, e, m)
        try:
            for dbl in (False, True):
                for qd in (0, 1):
                    for g in ((32, 128) if qd == 0 else (16,)):
                        q = ref_ql(torch.from_numpy(xa.copy()), w_bit=8, w_group_size=g, weight_format=which,
                                   approximate=True, double_approximate=dbl, quant_dim=qd, **params)
                        key = f"apx/{ci}/{int(dbl)}/{g}/{qd}"
                        d[key + "/deq"] = q.weight.data.numpy().copy()
                        d[key + "/scales"] = q.scales.numpy().copy()
        finally:
            quant_linear.configure_fp_formats()
    d["apx_cases"] = np.array([f"{w}|{f}|" + ",".join(f"{k}={v}" for k, v in p.items()) for w, f, p in cases])
    # ---- large SHA
    big = synth(0, (4096, 4096), "float16")
    q = ref_ql(torch.from_numpy(big.copy()), w_bit=4, w_group_size=128, weight_format="bfp")
    d["sha/bfp/4/128"] = sha(q.weight.data.numpy())
    for dbl in (False, True):
        q = ref_ql(torch.from_numpy(big.copy()), w_bit=8, w_group_size=128, weight_format="fp8", approximate=True,
                   double_approximate=dbl)
        d[f"sha/apx/fp8/{int(dbl)}"] = sha(q.weight.data.numpy())
    np.savez_compressed(os.path.join(HERE, "approx_small.npz"), **d)
    print("approx fixtures:", len(d), "arrays")


if __name__ == "__main__":
    main()

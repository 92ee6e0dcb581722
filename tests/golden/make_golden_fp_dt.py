"""Golden fixtures for the FP weight formats on bf16 and fp32 weights, produced FROM THE REFERENCE
ITSELF (run only in the build container; imports /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fp_dt.py

The reference's FP4/FP6/FP8 branches (quant_linear.py:724-883) and quantize_weight_approximate
(:470-632) run in the weight's own dtype: scales, (w - zeros) / scales, the clamp and the torch.log2
of _float_to_fp (:139) round to bf16 / fp32, the decoded value is cast to the dtype and multiplied
by the dtype's scales, while the stored scales / zeros buffers are .half() -- and the zero point is
added back from that fp16 buffer.  E5M2's fp_max (114688) is representable in bf16 / fp32, so that
format works there (it raises on fp16).

Produces tests/golden/fp_dt.npz (data only), for dtype in (bfloat16, float32):
  * enc/<dtype>/<fmt>: _float_to_fp over a code-exhaustive input set -- every finite bf16 in
    [-fp_max, fp_max]; for fp32 every binade's log2 threshold (tools/gen_fp_tables_dt.py), its
    predecessor and random values -- (inputs in/enc/<dtype>/<fmt>)
  * ql/<dtype>/<which>/<fmt>/<sym>/<g>/<qd>: QuantLinear FP branches, weight bits + fp16 scales/zeros
  * apx/<dtype>/<case>/<double>/<g>/<qd>: quantize_weight_approximate, weight bits + fp16 scales
bf16 arrays hold bit patterns (uint16).
"""
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

FORMATS = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e5m2": (5, 2)}
TD = {"bfloat16": torch.bfloat16, "float32": torch.float32}


def to_np(t):
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    return t.numpy().copy()


def from_np(a, dtype):
    if dtype == "bfloat16":
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).clone()
    return torch.from_numpy(np.ascontiguousarray(a)).clone()


def set_fmt(which, e, m):
    quant_linear.configure_fp_formats(**{f"{which}_exp_bits": e, f"{which}_mantissa_bits": m})


def ref_ql(w, **kw):
    lin = torch.nn.Linear(w.shape[1], w.shape[0], bias=False)
    lin.weight.data = w.clone()
    return quant_linear.QuantLinear.from_linear(lin, **kw)


def fp_max(e, m):
    bias = 2 ** (e - 1) - 1
    return (1.0 + (2 ** m - 1) / 2 ** m) * 2.0 ** ((1 << e) - 1 - bias)


def enc_inputs(dtype, e, m, rng):
    fm = fp_max(e, m)
    if dtype == "bfloat16":
        b = np.arange(65536, dtype=np.uint32).astype(np.uint16)
        x = (b.astype(np.uint32) << 16).view(np.float32)
        keep = np.isfinite(x) & (np.abs(x) <= fm)
        return b[keep]
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import gen_fp_tables_dt as G
    thr = [t for t in G.fp32_table() if t != 0xFFFFFFFF]
    t = np.array(thr, dtype=np.uint32)
    cand = np.concatenate([t, t - 1, t + 1, rng.integers(1, 0x7F800000, 20000, dtype=np.uint64).astype(np.uint32)])
    x = cand.view(np.float32)
    x = x[np.isfinite(x) & (np.abs(x) <= fm)]
    return np.concatenate([x, -x]).astype(np.float32)


def main():
    d = {}
    rng = np.random.default_rng(11)
    for dtype in TD:
        # ---- encoder over code-exhaustive inputs
        for name, (e, m) in FORMATS.items():
            xin = enc_inputs(dtype, e, m, rng)
            d[f"in/enc/{dtype}/{name}"] = xin
            bias = 2 ** (e - 1) - 1
            d[f"enc/{dtype}/{name}"] = quant_linear._float_to_fp(from_np(xin, dtype), e, m, bias).numpy().astype(np.uint8)
        # ---- QuantLinear FP branches
        x = synth(310, (48, 256), dtype)
        xf = (x.astype(np.uint32) << 16).view(np.float32) if dtype == "bfloat16" else x.astype(np.float32)
        xf = xf.copy()
        xf[3, :] = np.abs(xf[3, :])
        xf[5, ::5] = 0.0
        xf[7, 11] = -0.0
        xf[9, :] = 0.015625  # a constant row
        xf[11, 3] = 3.0e-38  # tiny (fp32 range)
        # bf16: back to bit patterns (the edits are bf16 values except the tiny one, rounded RNE)
        x = to_np(torch.from_numpy(xf).to(torch.bfloat16)) if dtype == "bfloat16" else xf
        d[f"in/fp/{dtype}"] = x
        for which, fmts in (("fp8", ("e4m3", "e5m2")), ("fp6", ("e3m2",)), ("fp4", ("e2m1",))):
            for fmt in fmts:
                e, m = FORMATS[fmt]
                set_fmt(which, e, m)
                try:
                    for sym in (False, True):
                        for qd in (0, 1):
                            for g in ((32, 128, -1, -2) if qd == 0 else (16, -1, -2)):
                                q = ref_ql(from_np(x, dtype), w_bit=8, w_group_size=g, symmetric=sym, quant_dim=qd,
                                           weight_format=which)
                                key = f"ql/{dtype}/{which}/{fmt}/{int(sym)}/{g}/{qd}"
                                d[key + "/deq"] = to_np(q.weight.data)
                                d[key + "/scales"] = to_np(q.scales)
                                if q.zeros is not None:
                                    d[key + "/zeros"] = to_np(q.zeros)
                finally:
                    quant_linear.configure_fp_formats()
        # ---- approximate single / double
        cases = [("fp8", "e4m3", dict(fp8_hi_align_start=12, fp8_hi_align_exp_field=15, fp8_tail_pad_bits=1)),
                 ("fp6", "e3m2", dict(fp6_hi_align_start=4, fp6_hi_align_exp_field=7, fp6_tail_pad_bits=2)),
                 ("fp4", "e2m1", dict(fp4_hi_align_start=1, fp4_hi_align_exp_field=1, fp4_tail_pad_bits=0)),
                 ("fp4", "e1m2", dict(fp4_hi_align_start=1, fp4_hi_align_exp_field=1, fp4_tail_pad_bits=0))]
        for ci, (which, fmt, params) in enumerate(cases):
            e, m = (1, 2) if fmt == "e1m2" else FORMATS[fmt]
            set_fmt(which, e, m)
            try:
                for dbl in (False, True):
                    for qd in (0, 1):
                        for g in ((32, 128) if qd == 0 else (16,)):
                            q = ref_ql(from_np(x, dtype), w_bit=8, w_group_size=g, weight_format=which,
                                       approximate=True, double_approximate=dbl, quant_dim=qd, **params)
                            key = f"apx/{dtype}/{ci}/{int(dbl)}/{g}/{qd}"
                            d[key + "/deq"] = to_np(q.weight.data)
                            d[key + "/scales"] = to_np(q.scales)
            finally:
                quant_linear.configure_fp_formats()
        d["apx_cases"] = np.array([f"{w}|{f}|" + ",".join(f"{k}={v}" for k, v in p.items()) for w, f, p in cases])
        print("done", dtype, flush=True)
    np.savez_compressed(os.path.join(HERE, "fp_dt.npz"), **d)
    print("fp dtype fixtures:", len(d), "arrays")


if __name__ == "__main__":
    main()

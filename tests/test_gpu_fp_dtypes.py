"""FP4/FP6/FP8 weight formats and the approximate decodes on bf16 / fp32 weights (round 4,
csrc/iwq_fpdt.hip) against the REFERENCE's own outputs (tests/golden/make_golden_fp_dt.py: the
reference's QuantLinear run on bf16 / fp32 weights), bit-exact: the encoder over every finite bf16
in [-fp_max, fp_max] and over fp32 values at every binade's torch.log2 threshold, then QuantLinear
FP branches (sym / asym, groups 32 / 128 / per-tensor / per-channel, quant_dim 0 / 1, E4M3 / E5M2 /
E3M2 / E2M1) and quantize_weight_approximate (single / double).  bf16 fixtures hold bit patterns."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
FORMATS = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e5m2": (5, 2)}
APX_CASES = [("fp8", "e4m3", (12, 15, 1)), ("fp6", "e3m2", (4, 7, 2)), ("fp4", "e2m1", (1, 1, 0)),
             ("fp4", "e1m2", (1, 1, 0))]
TD = {"bfloat16": torch.bfloat16, "float32": torch.float32}


@pytest.fixture(scope="module")
def Z():
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fp_dt.npz"))


def to_dev(a, dtype):
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16) if dtype == "bfloat16" \
        else torch.from_numpy(np.ascontiguousarray(a))
    return t.to(DEV)


def raw(t):
    t = t.detach().contiguous().cpu()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy().view(np.uint32)


def h16(t):
    assert t.dtype == torch.float16
    return t.detach().contiguous().cpu().numpy().view(np.uint16).reshape(-1)


def fp_max(e, m):
    bias = 2 ** (e - 1) - 1
    return (1.0 + (2 ** m - 1) / 2 ** m) * 2.0 ** ((1 << e) - 1 - bias)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
@pytest.mark.parametrize("fmt", list(FORMATS))
def test_fp_dtype_encoder_exhaustive(Z, dtype, fmt):
    """Rows of 128 whose first element is fp_max (sym scale exactly 1, so t = w): the packed codes
    of every other element equal the reference's _float_to_fp in that dtype."""
    from iron_weight_only_quant_amd import kernels as K
    e, m = FORMATS[fmt]
    xin = Z[f"in/enc/{dtype}/{fmt}"]
    exp = Z[f"enc/{dtype}/{fmt}"]
    n = len(xin)
    rows = (n + 126) // 127
    vals = np.zeros(rows * 127, dtype=xin.dtype)
    vals[:n] = xin
    fm = np.float32(fp_max(e, m))
    head = np.full((rows, 1), (fm.view(np.uint32) >> 16).astype(np.uint16) if dtype == "bfloat16" else fm,
                   dtype=xin.dtype)
    w = np.concatenate([head, vals.reshape(rows, 127)], axis=1)
    r = K.quantize_fp(to_dev(w, dtype), e, m, 128, True, 0, want_codes=True)
    assert bool((r.scales == 1.0).all())
    codes = r.codes.cpu().numpy()
    if 1 + e + m <= 4:  # nibbles, low = even column
        codes = np.stack([codes & 0xF, codes >> 4], axis=-1).reshape(-1)
    codes = codes.reshape(rows, 128)[:, 1:].reshape(-1)[:n]
    bad = np.nonzero(codes != exp)[0]
    assert len(bad) == 0, (len(bad), xin[bad[:5]], codes[bad[:5]], exp[bad[:5]])


def _ql(x, dtype, **kw):
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    w = to_dev(x, dtype)
    lin = torch.nn.Linear(w.shape[1], w.shape[0], bias=False, device=DEV, dtype=TD[dtype])
    lin.weight.data.copy_(w)
    return QuantLinear.from_linear(lin, **kw)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_fp_dtype_quantlinear_vs_reference(Z, dtype):
    from iron_weight_only_quant_amd import quant_linear as QL
    x = Z[f"in/fp/{dtype}"]
    for which, fmts in (("fp8", ("e4m3", "e5m2")), ("fp6", ("e3m2",)), ("fp4", ("e2m1",))):
        for fmt in fmts:
            e, m = FORMATS[fmt]
            QL.configure_fp_formats(**{f"{which}_exp_bits": e, f"{which}_mantissa_bits": m})
            try:
                for sym in (0, 1):
                    for qd in (0, 1):
                        for g in ((32, 128, -1, -2) if qd == 0 else (16, -1, -2)):
                            key = f"ql/{dtype}/{which}/{fmt}/{sym}/{g}/{qd}"
                            q = _ql(x, dtype, w_bit=8, w_group_size=g, symmetric=bool(sym), quant_dim=qd,
                                    weight_format=which)
                            assert q.weight.dtype == TD[dtype] and q.scales.dtype == torch.float16
                            exp = np.ascontiguousarray(Z[key + "/deq"])
                            exp = exp.view(np.uint16) if dtype == "bfloat16" else exp.view(np.uint32)
                            got = raw(q.weight.data)
                            bad = np.argwhere(got != exp)
                            assert len(bad) == 0, (key, len(bad), bad[:3])
                            assert np.array_equal(h16(q.scales), Z[key + "/scales"].view(np.uint16).reshape(-1)), key
                            assert (q.zeros is None) == (key + "/zeros" not in Z), key
                            if q.zeros is not None:
                                assert np.array_equal(h16(q.zeros), Z[key + "/zeros"].view(np.uint16).reshape(-1)), key
            finally:
                QL.configure_fp_formats()


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_fp_dtype_approximate_vs_reference(Z, dtype):
    from iron_weight_only_quant_amd import quant_linear as QL
    x = Z[f"in/fp/{dtype}"]
    for ci, (which, fmt, (hs, hf, tp)) in enumerate(APX_CASES):
        e, m = (1, 2) if fmt == "e1m2" else FORMATS[fmt]
        QL.configure_fp_formats(**{f"{which}_exp_bits": e, f"{which}_mantissa_bits": m})
        try:
            for dbl in (0, 1):
                for qd in (0, 1):
                    for g in ((32, 128) if qd == 0 else (16,)):
                        key = f"apx/{dtype}/{ci}/{dbl}/{g}/{qd}"
                        q = _ql(x, dtype, w_bit=8, w_group_size=g, weight_format=which, approximate=True,
                                double_approximate=bool(dbl), quant_dim=qd,
                                **{f"{which}_hi_align_start": hs, f"{which}_hi_align_exp_field": hf,
                                   f"{which}_tail_pad_bits": tp})
                        exp = np.ascontiguousarray(Z[key + "/deq"])
                        exp = exp.view(np.uint16) if dtype == "bfloat16" else exp.view(np.uint32)
                        bad = np.argwhere(raw(q.weight.data) != exp)
                        assert len(bad) == 0, (key, len(bad), bad[:3])
                        assert np.array_equal(h16(q.scales), Z[key + "/scales"].view(np.uint16).reshape(-1)), key
        finally:
            QL.configure_fp_formats()

"""Pin the FP-format CPU oracle (oracle/fp_codec.py) against golden vectors produced by the
reference itself (tests/golden/make_golden_fp.py).  CPU only, bit-exact."""
import hashlib
import os

import numpy as np
import pytest

from oracle import fp_codec as C
from oracle.synth import synth

from .golden_util import GOLD, bits_equal

FORMATS = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e5m2": (5, 2)}
WHICH_DEFAULT = {"fp8": "e4m3", "fp6": "e3m2", "fp4": "e2m1"}


@pytest.fixture(scope="module")
def d():
    return np.load(os.path.join(GOLD, "fp_small.npz"))


def test_log2_quirk_tables(d):
    pos = d["in/pos_fp16"]
    fl = np.floor(C.log2_fp16(pos).astype(np.float64))
    assert np.array_equal(fl, d["log2/floor"].astype(np.float64))
    fl1 = np.floor(C.R(C.log2_fp16(pos).astype(np.float64) + 1))
    assert np.array_equal(fl1, d["log2/floor_plus1"].astype(np.float64))
    assert int((fl != np.floor(np.log2(pos.astype(np.float64)))).sum()) == 94


@pytest.mark.parametrize("fmt", list(FORMATS))
def test_exhaustive_encode_decode(d, fmt):
    e, m = FORMATS[fmt]
    bias = 2 ** (e - 1) - 1
    xs = d["in/all_fp16"]
    assert np.array_equal(C.float_to_fp(xs, e, m, bias), d[f"enc/{fmt}"])
    dec = C.fp_to_float(np.arange(256), e, m, bias)
    assert bits_equal(dec, d[f"dec/{fmt}"])


def test_quantlinear_fp_branches(d):
    x = d["in/fp_a"]
    n = 0
    for key in d.files:
        if not key.startswith("ql/"):
            continue
        parts = key.split("/")
        _, which, fmt, sym, g, qd, kind = parts
        if kind not in ("deq", "error"):
            continue
        e, m = FORMATS[fmt]
        kw = dict(w_group_size=int(g), symmetric=bool(int(sym)), quant_dim=int(qd))
        if kind == "error":
            with pytest.raises(RuntimeError):
                C.quantlinear_fp(x, e, m, **kw)
            continue
        base = key[:-4]
        deq, s, z, _ = C.quantlinear_fp(x, e, m, **kw)
        assert bits_equal(deq, d[key]), key
        assert bits_equal(s, d[base + "/scales"]), key
        if base + "/zeros" in d.files:
            assert bits_equal(z, d[base + "/zeros"]), key
        n += 1
    assert n >= 40


def test_fp4_grid(d):
    x = d["in/fp_a"]
    for g, pt in ((128, False), (32, False), (-1, True), (256, False)):
        out = C.fp4_e2m1_grid(x, group_size=g, per_tensor=pt)
        assert bits_equal(out, d[f"grid/{g}/{int(pt)}"], nan_equal=True), (g, pt)


def test_large_sha(d):
    big = synth(0, (4096, 4096), "float16")
    for which, fmt, sym in (("fp8", "e4m3", True), ("fp8", "e4m3", False), ("fp4", "e2m1", False)):
        e, m = FORMATS[fmt]
        deq, _, _, _ = C.quantlinear_fp(big, e, m, w_group_size=128, symmetric=sym)
        assert hashlib.sha256(deq.tobytes()).digest() == d[f"sha/{which}/{fmt}/{int(sym)}"].tobytes(), (which, sym)
    out = C.fp4_e2m1_grid(big, group_size=128)
    assert hashlib.sha256(out.tobytes()).digest() == d["sha/grid/128"].tobytes()


# ---------------------------------------------------------------------------------------------
# bf16 / fp32 weights (round 4): the FP branches and the approximate decodes run in the weight's
# dtype; oracle/fp_codec_dt.py pinned to the reference's own outputs (make_golden_fp_dt.py)
FORMATS_DT = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e5m2": (5, 2)}
APX_DT_CASES = [("fp8", "e4m3", (12, 15, 1)), ("fp6", "e3m2", (4, 7, 2)), ("fp4", "e2m1", (1, 1, 0)),
                ("fp4", "e1m2", (1, 1, 0))]


def _fpdt():
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fp_dt.npz"))


def _raw(a, dtype):
    return np.ascontiguousarray(a).view(np.uint16 if dtype == "bfloat16" else np.uint32)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_fp_dtype_oracle_encode(dtype):
    """_float_to_fp in bf16 / fp32: every finite bf16 in [-fp_max, fp_max]; for fp32 every binade's
    torch.log2 threshold, its neighbours and random values (incl. |x| < 2^-128, where the int8
    exponent wraps)."""
    from oracle import fp_codec_dt as D
    Z = _fpdt()
    dt = D.Dt(dtype)
    for name, (e, m) in FORMATS_DT.items():
        got = D.float_to_fp_t(dt.from_input(Z[f"in/enc/{dtype}/{name}"]), e, m, 2 ** (e - 1) - 1, dt)
        assert np.array_equal(got, Z[f"enc/{dtype}/{name}"]), name


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_fp_dtype_oracle_quantlinear(dtype):
    from oracle import fp_codec_dt as D
    Z = _fpdt()
    x = Z[f"in/fp/{dtype}"]
    for which, fmts in (("fp8", ("e4m3", "e5m2")), ("fp6", ("e3m2",)), ("fp4", ("e2m1",))):
        for fmt in fmts:
            e, m = FORMATS_DT[fmt]
            for sym in (0, 1):
                for qd in (0, 1):
                    for g in ((32, 128, -1, -2) if qd == 0 else (16, -1, -2)):
                        key = f"ql/{dtype}/{which}/{fmt}/{sym}/{g}/{qd}"
                        deq, s, z = D.quantlinear_fp_t(x, e, m, g, bool(sym), qd, dtype)
                        assert np.array_equal(_raw(deq, dtype), _raw(Z[key + "/deq"], dtype)), key
                        assert np.array_equal(s.view(np.uint16), Z[key + "/scales"].view(np.uint16)), key
                        assert (z is None) == (key + "/zeros" not in Z), key
                        if z is not None:
                            assert np.array_equal(z.view(np.uint16), Z[key + "/zeros"].view(np.uint16)), key
    for ci, (which, fmt, (hs, hf, tp)) in enumerate(APX_DT_CASES):
        e, m = (1, 2) if fmt == "e1m2" else FORMATS_DT[fmt]
        for dbl in (0, 1):
            for qd in (0, 1):
                for g in ((32, 128) if qd == 0 else (16,)):
                    key = f"apx/{dtype}/{ci}/{dbl}/{g}/{qd}"
                    deq, s = D.quantlinear_approx_t(x, e, m, g, qd, hs, hf, tp, bool(dbl), dtype,
                                                    is_fp4=(which == "fp4"))
                    assert np.array_equal(_raw(deq, dtype), _raw(Z[key + "/deq"], dtype)), key
                    assert np.array_equal(s.view(np.uint16), Z[key + "/scales"].view(np.uint16)), key

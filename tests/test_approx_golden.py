"""Pin the BFP / approximate-FP CPU oracle (oracle/approx_codec.py) against golden vectors produced
by the reference itself (tests/golden/make_golden_approx.py).  CPU only, bit-exact."""
import os

import numpy as np
import pytest

from oracle import approx_codec as A
from oracle.iwq_oracle import bf16_bits_to_f32, f32_to_bf16_bits
from oracle.synth import synth

from .golden_util import GOLD, bits_equal, sha

FORMATS = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e1m2": (1, 2)}


@pytest.fixture(scope="module")
def d():
    return np.load(os.path.join(GOLD, "approx_small.npz"))


def _keys(d, prefix):
    return [k for k in d.files if k.startswith(prefix)]


def test_aligned_decode_tables(d):
    ks = _keys(d, "adec/")
    assert len(ks) == 14
    for k in ks:
        _, name, hs, hf, tp = k.split("/")
        e, m = FORMATS[name]
        bias = 2 ** (e - 1) - 1
        v = A.fp_decode_aligned(np.arange(1 << (1 + e + m)), int(hs), int(hf), int(tp), e, m, bias)
        assert bits_equal(v, d[k]), k


def test_double_approx_quads(d):
    ks = _keys(d, "dq/")
    assert len(ks) == 8
    for k in ks:
        _, name, hs, hf, tp = k.split("/")
        e, m = FORMATS[name]
        bias = 2 ** (e - 1) - 1
        v = A.fp_decode_aligned_double_approx(d[f"dq_in/{name}"], int(hs), int(hf), int(tp), e, m, bias)
        assert bits_equal(v, d[k]), k
    # the E4M3 set exercises the int8 wrap of a rounding shift by exactly 8 (mantissa -> -1)
    v = d["dq/e4m3/12/15/1"].astype(np.float32)
    q = d["dq_in/e4m3"]
    assert (v[q != 0] == 0).any()


def test_bfp_end_to_end(d):
    ks = [k for k in _keys(d, "bfp/") if k.split("/")[1] in ("a", "edge")]
    assert len(ks) == 2 * 9 * 4
    for k in ks:
        _, tag, wb, g, qd = k.split("/")
        src = d["in/bfp_a"] if tag == "a" else d["in/bfp_edge"]
        out = A.bfp_quantize(src, int(wb), int(g), int(qd))
        assert bits_equal(out, d[k]), k


def test_bfp_fp32_bf16(d):
    xf = d["in/bfp_f32"]
    xb = bf16_bits_to_f32(d["in/bfp_bf16_bits"])
    for wb in (3, 4, 8):
        assert bits_equal(A.bfp_quantize(xf, wb, 32, dtype="float32"), d[f"bfp/f32/{wb}"]), wb
        got = f32_to_bf16_bits(A.bfp_quantize(xb, wb, 32, dtype="bfloat16"))
        assert np.array_equal(got, d[f"bfp/bf16/{wb}"]), wb


def test_bfp_errors():
    x = synth(1, (4, 64), "float16")
    with pytest.raises(ValueError):
        A.bfp_quantize(x, 4, -1)
    with pytest.raises(AssertionError):
        A.bfp_quantize(x, 4, 48)
    with pytest.raises(ValueError):
        A.bfp_quantize(x, 0, 32)   # min(w_bit-1, 11) < 0: negative shift count, like the reference


def test_approximate_end_to_end(d):
    cases = [str(c) for c in d["apx_cases"]]
    xa = d["in/apx_a"]
    n = 0
    for ci, c in enumerate(cases):
        which, fmt, params = c.split("|")
        p = dict(kv.split("=") for kv in params.split(","))
        hs, hf, tp = (int(p[f"{which}_hi_align_start"]), int(p[f"{which}_hi_align_exp_field"]),
                      int(p[f"{which}_tail_pad_bits"]))
        e, m = FORMATS[fmt]
        for k in _keys(d, f"apx/{ci}/"):
            if not k.endswith("/deq"):
                continue
            _, _, dbl, g, qd, _ = k.split("/")
            deq, s = A.quantlinear_approx(xa, e, m, int(g), int(qd), hs, hf, tp, bool(int(dbl)), which == "fp4")
            assert bits_equal(deq, d[k]), k
            assert bits_equal(s, d[k[:-4] + "/scales"]), k
            n += 1
    assert n == len(cases) * 6


def test_approximate_errors():
    x = synth(2, (4, 64), "float16")
    with pytest.raises(ValueError):
        A.quantlinear_approx(x, 4, 3, -2)
    with pytest.raises(UnboundLocalError):
        A.quantlinear_approx(x, 3, 0, 32, is_fp4=True)   # FP4 with 3 exponent bits: reference leaves decoded unbound


def test_large_sha(d):
    big = synth(0, (4096, 4096), "float16")
    assert sha(A.bfp_quantize(big, 4, 128)) == bytes(d["sha/bfp/4/128"]).hex()
    for dbl in (0, 1):
        deq, _ = A.quantlinear_approx(big, 4, 3, 128, 0, 12, 15, 1, bool(dbl))
        assert sha(deq) == bytes(d[f"sha/apx/fp8/{dbl}"]).hex(), dbl

"""GPU parity for the research weight formats — BFP (quant_linear.py:648-723) and the approximate /
double-approximate aligned FP decodes (:470-632, :237-363) — through the C-ABI, bit-exact against
the reference's fixtures (tests/golden/approx_small.npz) and the pinned CPU oracle."""
import os

import numpy as np
import pytest
import torch

from oracle import approx_codec as A
from oracle import fp_codec as C
from oracle.iwq_oracle import bf16_bits_to_f32
from oracle.synth import synth

from .golden_util import GOLD, bits_equal, sha

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
FLAG_SETS = (0, 1)  # fast kernels, IWQ_FLAG_FORCE_GENERIC
FORMATS = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e1m2": (1, 2)}


@pytest.fixture(scope="module")
def K():
    from iron_weight_only_quant_amd import kernels
    return kernels


@pytest.fixture(scope="module")
def AD():
    return np.load(os.path.join(GOLD, "approx_small.npz"))


def dev16(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def np16(t):
    return t.detach().contiguous().cpu().numpy()


# ------------------------------------------------------------------------------------------- BFP
@pytest.mark.parametrize("flags", FLAG_SETS)
def test_bfp_golden(K, AD, flags):
    n = 0
    for k in AD.files:
        parts = k.split("/")
        if parts[0] != "bfp" or parts[1] not in ("a", "edge"):
            continue
        _, tag, wb, g, qd = parts
        x = dev16(AD["in/bfp_a"] if tag == "a" else AD["in/bfp_edge"])
        out = K.quantize_bfp(x, int(wb), int(g), int(qd), flags=flags)
        assert bits_equal(np16(out), AD[k]), k
        n += 1
    assert n == 72


def test_bfp_fp32_bf16_golden(K, AD):
    xf = torch.from_numpy(AD["in/bfp_f32"].copy()).to(DEV)
    xb = torch.from_numpy(AD["in/bfp_bf16_bits"].view(np.int16).copy()).view(torch.bfloat16).to(DEV)
    for wb in (3, 4, 8):
        for flags in FLAG_SETS:
            got = K.quantize_bfp(xf, wb, 32, flags=flags)
            assert bits_equal(np16(got), AD[f"bfp/f32/{wb}"]), (wb, flags)
            got = K.quantize_bfp(xb, wb, 32, flags=flags).view(torch.int16).cpu().numpy().view(np.uint16)
            assert np.array_equal(got, AD[f"bfp/bf16/{wb}"]), (wb, flags)


def test_bfp_quantlinear_inplace_and_strided(K):
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    x = synth(77, (96, 384), "float16")
    for wb, g, qd in ((4, 128, 0), (8, 32, 0), (5, 96, 0), (3, 48, 1)):
        exp = A.bfp_quantize(x, wb, g, qd)
        w = dev16(x)
        lin = torch.nn.Linear(384, 96, bias=False).to(DEV)
        lin.weight.data = w
        q = QuantLinear.from_linear(lin, w_bit=wb, w_group_size=g, weight_format="bfp", quant_dim=qd)
        assert q.weight.data_ptr() == w.data_ptr()
        assert bits_equal(np16(w), exp), (wb, g, qd)
        assert q.scales is None and q.zeros is None and bool(q.quantized)
    # a row-strided view (ld > cols)
    big = dev16(synth(78, (64, 512), "float16"))
    view = big[:, :256]
    out = K.quantize_bfp(view, 4, 64)
    assert bits_equal(np16(out), A.bfp_quantize(np16(view), 4, 64))


def test_bfp_errors(K):
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    x = dev16(synth(3, (8, 64), "float16"))
    with pytest.raises(ValueError):
        K.quantize_bfp(x, 4, -1)
    with pytest.raises(AssertionError):
        K.quantize_bfp(x, 4, 48)
    with pytest.raises(ValueError):
        K.quantize_bfp(x, 0, 32)
    lin = torch.nn.Linear(64, 8, bias=False).half().to(DEV)
    with pytest.raises(ValueError):
        QuantLinear.from_linear(lin, w_bit=4, w_group_size=-2, weight_format="bfp")


def test_bfp_large_sha(K, AD):
    x = torch.empty(4096, 4096, dtype=torch.float16, device=DEV)
    K.fill_synthetic(x, 0)
    assert sha(np16(K.quantize_bfp(x, 4, 128))) == bytes(AD["sha/bfp/4/128"]).hex()


# ----------------------------------------------------------------------------------- approximate
def _cases(AD):
    out = []
    for ci, c in enumerate(str(c) for c in AD["apx_cases"]):
        which, fmt, params = c.split("|")
        p = dict(kv.split("=") for kv in params.split(","))
        out.append((ci, which, fmt, int(p[f"{which}_hi_align_start"]), int(p[f"{which}_hi_align_exp_field"]),
                    int(p[f"{which}_tail_pad_bits"])))
    return out


def _ab_built():
    try:
        from iron_weight_only_quant_amd import _lib
        return _lib.ab_built()
    except OSError:
        return False


# + the double-approximate kernel's A/B forms (IWQ_AB library only): 2 (DPP / permlane exchange),
# 3 (the round-2 kernel)
@pytest.mark.parametrize("flags", FLAG_SETS + ((2 << 16, 3 << 16) if _ab_built() else ()))
def test_approx_golden_kernel(K, AD, flags):
    x = dev16(AD["in/apx_a"])
    n = 0
    for ci, which, fmt, hs, hf, tp in _cases(AD):
        e, m = FORMATS[fmt]
        for k in AD.files:
            if not (k.startswith(f"apx/{ci}/") and k.endswith("/deq")):
                continue
            _, _, dbl, g, qd, _ = k.split("/")
            double = bool(int(dbl)) and not (which == "fp4" and e == 1)
            r = K.quantize_fp_approx(x, e, m, int(g), int(qd), hs, hf, tp, double, flags=flags)
            assert bits_equal(np16(r.out), AD[k]), (k, flags)
            assert bits_equal(np16(r.scales), AD[k[:-4] + "/scales"].reshape(-1)), k
            n += 1
    assert n == 42


def test_approx_quantlinear_face(AD):
    from iron_weight_only_quant_amd import quant_linear as QL
    xa = AD["in/apx_a"]
    for ci, which, fmt, hs, hf, tp in _cases(AD):
        e, m = FORMATS[fmt]
        QL.configure_fp_formats(**{f"{which}_exp_bits": e, f"{which}_mantissa_bits": m})
        try:
            for dbl in (0, 1):
                key = f"apx/{ci}/{dbl}/32/0"
                w = dev16(xa)
                lin = torch.nn.Linear(256, 32, bias=False).to(DEV)
                lin.weight.data = w
                kw = {f"{which}_hi_align_start": hs, f"{which}_hi_align_exp_field": hf, f"{which}_tail_pad_bits": tp}
                q = QL.QuantLinear.from_linear(lin, w_bit=8, w_group_size=32, weight_format=which, approximate=True,
                                               double_approximate=bool(dbl), **kw)
                assert bits_equal(np16(w), AD[key + "/deq"]), key
                assert bits_equal(np16(q.scales), AD[key + "/scales"]), key
                assert q.zeros is None and q.approximate
        finally:
            QL.configure_fp_formats()


@pytest.mark.parametrize("double", [False, True])
def test_approx_e4m3_every_code(K, double):
    """Every finite fp16 in [-480, 480] in rows whose absmax is 480 (scale exactly 1): every E4M3 code
    goes through the aligned / double-approximate decoders; compared with the pinned oracle."""
    e, m = 4, 3
    bias, fp_max = C.fp_params(e, m)
    xs = np.arange(65536, dtype=np.uint32).astype(np.uint16).view(np.float16)
    xs = xs[np.isfinite(xs) & (np.abs(xs.astype(np.float32)) <= fp_max)]
    per = 127
    n = (len(xs) + per - 1) // per
    vals = np.concatenate([xs, np.zeros(n * per - len(xs), np.float16)]).reshape(n, per)
    rows = np.concatenate([np.full((n, 1), fp_max, np.float16), vals], axis=1)
    rows = rows[: n - n % 4]
    exp, _ = A.quantlinear_approx(rows, e, m, 128, 0, 12, 15, 1, double)
    for flags in FLAG_SETS:
        r = K.quantize_fp_approx(dev16(rows), e, m, 128, 0, 12, 15, 1, double, flags=flags)
        assert bool(torch.all(r.scales == 1))
        assert bits_equal(np16(r.out), exp), flags


def test_approx_generic_quads_and_transposed(K):
    """G % 4 != 0 (quads wrap across in-group positions) and quant_dim 1, vs the oracle."""
    for shape, g, qd in (((3, 64), 64, 0), ((5, 96), 32, 0), ((64, 6), 32, 1), ((128, 40), 64, 1)):
        x = synth(90 + g, shape, "float16")
        for double in (False, True):
            exp, s = A.quantlinear_approx(x, 3, 2, g, qd, 4, 7, 2, double)
            for flags in FLAG_SETS:
                r = K.quantize_fp_approx(dev16(x), 3, 2, g, qd, 4, 7, 2, double, flags=flags)
                assert bits_equal(np16(r.out), exp), (shape, g, qd, double, flags)
                assert bits_equal(np16(r.scales), s.reshape(-1)), (shape, g, qd)


def test_approx_errors(K):
    from iron_weight_only_quant_amd import quant_linear as QL
    x = dev16(synth(4, (8, 64), "float16"))
    with pytest.raises(ValueError):
        K.quantize_fp_approx(x, 4, 3, -2)
    with pytest.raises(AssertionError):
        K.quantize_fp_approx(x, 4, 3, 48)
    with pytest.raises(ValueError):
        K.quantize_fp_approx(dev16(synth(5, (3, 6), "float16")), 4, 3, 2, 0, double_approx=True)
    lin = torch.nn.Linear(64, 8, bias=False).half().to(DEV)
    with pytest.raises(NotImplementedError):
        QL.QuantLinear.from_linear(lin, w_group_size=32, weight_format="int", approximate=True)
    QL.configure_fp_formats(fp4_exp_bits=3, fp4_mantissa_bits=0)
    try:
        with pytest.raises(UnboundLocalError):
            QL.QuantLinear.from_linear(lin, w_group_size=32, weight_format="fp4", approximate=True)
    finally:
        QL.configure_fp_formats()


@pytest.mark.parametrize("double", [0, 1])
def test_approx_large_sha(K, AD, double):
    x = torch.empty(4096, 4096, dtype=torch.float16, device=DEV)
    K.fill_synthetic(x, 0)
    r = K.quantize_fp_approx(x, 4, 3, 128, 0, 12, 15, 1, bool(double))
    assert sha(np16(r.out)) == bytes(AD[f"sha/apx/fp8/{double}"]).hex()


def test_quantize_model_research_formats():
    """quantize_model with w_format bfp / approximate fp8: every replaced layer equals the oracle."""
    from types import SimpleNamespace
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    for fmt, extra in (("bfp", {}), ("fp8", {"approximate": True, "double_approximate": True})):
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(256, 128), torch.nn.ReLU(), torch.nn.Linear(128, 256)).half().to(DEV)
        orig = [np16(model[0].weight), np16(model[2].weight)]
        args = SimpleNamespace(w_bit=4, a_bit=16, w_group_size=64, w_symmetric=False, w_format=fmt, quant_dim=0,
                               **extra)
        quantize_model(model, args, verbose=False)
        for i, w0 in zip((0, 2), orig):
            if fmt == "bfp":
                exp = A.bfp_quantize(w0, 4, 64)
            else:
                exp, _ = A.quantlinear_approx(w0, 4, 3, 64, 0, 12, 15, 1, True)
            assert bits_equal(np16(model[i].weight), exp), (fmt, i)

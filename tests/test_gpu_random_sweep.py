"""Seeded random parity sweep (GPU): many small configurations of every quantization path, each
checked bit-exactly against the pinned CPU oracle — shapes, group modes, bit widths, symmetry,
quant_dim, storage dtypes, value scales (tiny / huge / mixed zeros), both kernel families
(specialised and IWQ_FLAG_FORCE_GENERIC).  Sized to run in seconds."""
import numpy as np
import pytest
import torch

from oracle import approx_codec as A
from oracle import fp_codec as C
from oracle import iwq_oracle as O
from oracle.synth import synth

from .golden_util import bits_equal

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _input(rng, shape, dtype):
    x = synth(int(rng.integers(1 << 30)), shape, "float32").astype(np.float64)
    scale = float(rng.choice([1.0, 1e-3, 50.0, 3e-6]))
    x = x * scale
    if rng.random() < 0.3:
        x[rng.random(shape) < 0.2] = 0.0
    if rng.random() < 0.2:
        x[int(rng.integers(shape[0]))] = float(rng.normal()) * scale  # a constant row
    x32 = x.astype(np.float32)
    if dtype == "float16":
        return x32.astype(np.float16)
    if dtype == "bfloat16":
        return O.f32_to_bf16_bits(x32)
    return x32


def _dev(a, dtype):
    a = np.ascontiguousarray(a)
    if dtype == "bfloat16":
        return torch.from_numpy(a.view(np.int16)).view(torch.bfloat16).to(DEV)
    return torch.from_numpy(a).to(DEV)


def _np(t):
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


@pytest.mark.parametrize("seed", range(12))
def test_int_random_sweep(seed):
    from iron_weight_only_quant_amd import kernels as K
    rng = np.random.default_rng(1000 + seed)
    for _ in range(16):
        dtype = str(rng.choice(["float16", "float16", "bfloat16", "float32"]))
        qd = int(rng.integers(2))
        group = int(rng.choice([8, 16, 32, 64, 128, 256, 512, 24, 96, -1, -2]))
        bits = int(rng.choice([2, 3, 4, 5, 8]))
        sym = bool(rng.integers(2))
        if sym and bits < 2:
            continue
        g = group if group > 0 else 8
        vr = int(rng.integers(1, 40))
        vc = g * int(rng.integers(1, 5)) if group > 0 else 8 * int(rng.integers(1, 60))
        rows, cols = (vc, vr) if qd == 1 else (vr, vc)
        if cols % 2:
            cols += 1 if group <= 0 or qd == 1 else 0
        if (qd == 0 and group > 0 and cols % group) or (qd == 1 and group > 0 and rows % group):
            continue
        x = _input(rng, (rows, cols), dtype)
        ref = O.quantlinear_int(x, bits, group, sym, qd, dtype)
        want_codes = bits <= 8 and cols % 2 == 0
        for flags in (0, 1):
            r = K.quantize_minmax(_dev(x, dtype), bits, group, sym, qd, want_codes=want_codes, flags=flags)
            cfg = (dtype, rows, cols, group, bits, sym, qd, flags)
            assert bits_equal(_np(r.out), ref.dequant, nan_equal=True), cfg
            assert bits_equal(_np(r.scales), ref.scales.reshape(-1), nan_equal=True), cfg
            if want_codes:
                assert np.array_equal(r.codes.cpu().numpy().reshape(-1),
                                      O.pack_codes(ref.codes, bits).reshape(-1)), cfg


@pytest.mark.parametrize("seed", range(6))
def test_fp_random_sweep(seed):
    from iron_weight_only_quant_amd import kernels as K
    rng = np.random.default_rng(2000 + seed)
    fmts = [(4, 3), (3, 2), (2, 1), (1, 2), (2, 3), (3, 3), (4, 2), (1, 1), (2, 2)]
    for _ in range(10):
        e, m = fmts[int(rng.integers(len(fmts)))]
        qd = int(rng.integers(2))
        group = int(rng.choice([16, 32, 64, 128, -1, -2]))
        sym = bool(rng.integers(2))
        g = group if group > 0 else 16
        vr, vc = int(rng.integers(1, 30)), g * int(rng.integers(1, 4))
        rows, cols = (vc, vr) if qd == 1 else (vr, vc)
        if 1 + e + m <= 4 and cols % 2:
            continue
        x = _input(rng, (rows, cols), "float16")
        deq, s, z, codes = C.quantlinear_fp(x, e, m, group, sym, qd)
        for flags in (0, 1):
            r = K.quantize_fp(_dev(x, "float16"), e, m, group, sym, qd, want_codes=True, flags=flags)
            cfg = (e, m, rows, cols, group, sym, qd, flags)
            assert bits_equal(_np(r.out), deq, nan_equal=True), cfg
            assert bits_equal(_np(r.scales), s.reshape(-1), nan_equal=True), cfg
            cb = r.codes.cpu().numpy().reshape(-1)
            if 1 + e + m <= 4:
                cb = np.stack([cb & 0xF, cb >> 4], axis=1).reshape(-1)
            assert np.array_equal(cb, codes.reshape(-1)), cfg


@pytest.mark.parametrize("seed", range(6))
def test_bfp_approx_random_sweep(seed):
    from iron_weight_only_quant_amd import kernels as K
    rng = np.random.default_rng(3000 + seed)
    for _ in range(8):
        dtype = str(rng.choice(["float16", "bfloat16", "float32"]))
        qd = int(rng.integers(2))
        group = int(rng.choice([8, 16, 32, 64, 128, 48]))
        wb = int(rng.integers(1, 14))
        vr, vc = int(rng.integers(1, 20)), group * int(rng.integers(1, 4))
        rows, cols = (vc, vr) if qd == 1 else (vr, vc)
        x = _input(rng, (rows, cols), dtype)
        src = O.bf16_bits_to_f32(x) if dtype == "bfloat16" else x
        exp = A.bfp_quantize(src, wb, group, qd, dtype=dtype)
        got = _np(K.quantize_bfp(_dev(x, dtype), wb, group, qd))
        if dtype == "bfloat16":
            exp = O.f32_to_bf16_bits(exp)
            assert np.array_equal(got, exp), (dtype, rows, cols, group, wb, qd)
        else:
            assert bits_equal(got, exp, nan_equal=True), (dtype, rows, cols, group, wb, qd)
    for _ in range(8):
        e, m, hs, hf, tp = [(4, 3, 12, 15, 1), (4, 3, 10, 14, 0), (3, 2, 4, 7, 2), (3, 2, 3, 6, -1),
                            (2, 1, 1, 1, 0), (2, 1, 1, 3, 1)][int(rng.integers(6))]
        qd = int(rng.integers(2))
        group = int(rng.choice([16, 32, 64]))
        dbl = bool(rng.integers(2))
        vr, vc = 4 * int(rng.integers(1, 8)), group * int(rng.integers(1, 3))
        rows, cols = (vc, vr) if qd == 1 else (vr, vc)
        if 1 + e + m <= 4 and cols % 2:
            continue
        x = _input(rng, (rows, cols), "float16")
        exp, s = A.quantlinear_approx(x, e, m, group, qd, hs, hf, tp, dbl)
        for flags in (0, 1):
            r = K.quantize_fp_approx(_dev(x, "float16"), e, m, group, qd, hs, hf, tp, dbl, flags=flags)
            cfg = (e, m, hs, hf, tp, rows, cols, group, qd, dbl, flags)
            assert bits_equal(_np(r.out), exp, nan_equal=True), cfg
            assert bits_equal(_np(r.scales), s.reshape(-1), nan_equal=True), cfg

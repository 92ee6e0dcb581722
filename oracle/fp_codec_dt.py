"""CPU oracle for the FP weight formats on bf16 and fp32 weights (round 4).

TEST INFRASTRUCTURE ONLY (tests/).  Restates, in the weight's own dtype T:
  _float_to_fp                  quant_linear.py:126-163   (torch.log2 in T: RN_T(log2 x))
  FP4/FP6/FP8 branches          quant_linear.py:724-883   (scales / (w - zeros) / clamp in T;
                                stored scales / zeros .half(); zero point added back from the fp16 buffer)
  quantize_weight_approximate   quant_linear.py:470-632   (decode_dtype = T; RN_T(decoded * scales))
Every T elementwise op is evaluated in float and rounded to T (ATen's opmath); for fp32 that is one
correctly rounded op, for bf16 RN_bf16(RN_f32(op)).  Pinned against reference-generated fixtures
(tests/golden/make_golden_fp_dt.py) in tests/test_fp_golden.py.
bf16 arrays are bit patterns (uint16) at the boundary.
"""
import numpy as np

from . import approx_codec as A
from .fp_codec import fp_params, fp_to_float


def bf16_to_f64(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def f32_to_bf16_bits(x32):
    """float32 -> bf16 bits, round to nearest even (NaN stays NaN)."""
    u = np.asarray(x32, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32)
    nan = np.isnan(np.asarray(x32, dtype=np.float32))
    return np.where(nan, (u >> 16) | 0x40, r).astype(np.uint16)


class Dt:
    """Rounding of one ATen op in dtype T (float64 in -> float64 holding a T value)."""

    def __init__(self, name):
        assert name in ("bfloat16", "float32")
        self.name = name

    def R(self, x):
        with np.errstate(over="ignore", invalid="ignore"):
            x32 = np.asarray(x, dtype=np.float64).astype(np.float32)
            if self.name == "float32":
                return x32.astype(np.float64)
            return bf16_to_f64(f32_to_bf16_bits(x32))

    def from_input(self, a):
        return bf16_to_f64(a) if self.name == "bfloat16" else np.asarray(a, dtype=np.float32).astype(np.float64)

    def to_output(self, x):
        x32 = np.asarray(x, dtype=np.float64).astype(np.float32)
        return f32_to_bf16_bits(x32) if self.name == "bfloat16" else x32


def floor_log2_t(xa, dt):
    """floor(torch.log2(x)) for positive T values: floor(RN_T(log2 x)) (x > 0)."""
    with np.errstate(divide="ignore"):
        return np.floor(dt.R(np.log2(xa)))


def float_to_fp_t(t, exp_bits, mant_bits, exp_bias, dt):
    """quant_linear.py:126-163 on T values (float64 holding T values) -> uint8 codes."""
    x = np.asarray(t, dtype=np.float64)
    sign = (x < 0).astype(np.int64)
    xa = np.abs(x)
    zero = xa == 0
    safe = np.where(zero, dt.R(1e-8), xa)
    min_normal = 1 - exp_bias
    e = floor_log2_t(safe, dt)
    e = np.where(np.isfinite(e), e, 0).astype(np.int64)
    # .to(torch.int8) (:139) wraps: |x| < 2^-128 (log2 <= -129) lands on a large positive exponent
    e = ((e + 128) & 0xFF) - 128
    is_sub = e < min_normal
    e_cl = np.clip(e, min_normal, (1 << exp_bits) - 1 - exp_bias)
    ms = 1 << mant_bits
    # T / fp32 tensor -> fp32 (exact here)
    m_norm = np.clip(np.rint((safe / np.exp2(e_cl.astype(np.float64)) - 1.0) * ms), 0, ms - 1).astype(np.int64)
    # T / 0-dim fp32 tensor -> T: RN_T(x / 2^(1-bias)) * 2^M (RN_T), round
    m_sub = np.clip(np.rint(dt.R(dt.R(safe / 2.0 ** min_normal) * ms)), 0, ms - 1).astype(np.int64)
    exp_field = np.where(is_sub, 0, e_cl + exp_bias)
    mant = np.where(is_sub, m_sub, m_norm)
    code = (sign << (exp_bits + mant_bits)) | (exp_field << mant_bits) | mant
    return (np.where(zero, 0, code) & 0xFF).astype(np.uint8)


def _grouped(w, group, quant_dim):
    wq = w.T if quant_dim == 1 else w
    qshape = wq.shape
    if group > 0:
        assert qshape[-1] % group == 0
        g = np.ascontiguousarray(wq).reshape(-1, group)
    elif group == -1:
        g = np.ascontiguousarray(wq).reshape(1, -1)
    elif group == -2:
        g = np.ascontiguousarray(wq).reshape(qshape[0], -1)
    else:
        raise ValueError("Invalid w_group_size")
    return g, qshape


def _half(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32).astype(np.float16)


def quantlinear_fp_t(weight, exp_bits, mant_bits, w_group_size, symmetric, quant_dim, dtype):
    """FP4/FP6/FP8 branches on a bf16 (bits) / fp32 weight.  Returns (dequant in the weight's
    representation, scales fp16 [G,1], zeros fp16 [G,1] or None)."""
    dt = Dt(dtype)
    bias, fp_max = fp_params(exp_bits, mant_bits)
    w = dt.from_input(weight)
    g, qshape = _grouped(w, w_group_size, quant_dim)
    eps = dt.R(1e-5)
    fpm = dt.R(fp_max)
    with np.errstate(all="ignore"):
        if symmetric:
            am = np.abs(g).max(axis=1, keepdims=True)
            am = np.where(am < eps, eps, am)
            s = dt.R(am / fp_max)
            s = np.where(s < eps, eps, s)
            z16 = None
            t = dt.R(g / s)
        else:
            mx = g.max(axis=1, keepdims=True)
            mn = g.min(axis=1, keepdims=True)
            mid = dt.R(dt.R(mx + mn) * 0.5)
            span = dt.R(dt.R(mx - mn) * 0.5)
            span = np.where(span < eps, eps, span)
            s = dt.R(span / fp_max)
            s = np.where(s < eps, eps, s)
            t = dt.R(dt.R(g - mid) / s)
            z16 = _half(mid)
        t = np.where(t < -fpm, -fpm, np.where(t > fpm, fpm, t))
        codes = float_to_fp_t(t, exp_bits, mant_bits, bias, dt)
        deq = dt.R(dt.R(fp_to_float(codes, exp_bits, mant_bits, bias).astype(np.float64)) * s)
        if z16 is not None:
            deq = dt.R(deq + dt.R(z16.astype(np.float64)))
    deq = deq.reshape(qshape)
    if quant_dim == 1:
        deq = np.ascontiguousarray(deq.T)
    return dt.to_output(deq), _half(s), (None if z16 is None else z16)


def quantlinear_approx_t(weight, exp_bits, mant_bits, w_group_size, quant_dim, hi_align_start, hi_align_exp_field,
                         tail_pad_bits, double_approximate, dtype, is_fp4=False):
    """quantize_weight_approximate on a bf16 (bits) / fp32 weight -> (dequant, scales fp16 [G,1])."""
    if w_group_size <= 0:
        raise ValueError("approximate needs w_group_size > 0")
    dt = Dt(dtype)
    bias, fp_max = fp_params(exp_bits, mant_bits)
    w = dt.from_input(weight)
    g, qshape = _grouped(w, w_group_size, quant_dim)
    eps = dt.R(1e-5)
    fpm = dt.R(fp_max)
    with np.errstate(all="ignore"):
        am = np.abs(g).max(axis=1, keepdims=True)
        am = np.where(am < eps, eps, am)
        s = dt.R(am / fp_max)
        s = np.where(s < eps, eps, s)
        t = dt.R(g / s)
        t = np.where(t < -fpm, -fpm, np.where(t > fpm, fpm, t))
    codes = float_to_fp_t(t, exp_bits, mant_bits, bias, dt)
    if double_approximate and not (is_fp4 and exp_bits == 1):
        dec = A.fp_decode_aligned_double_approx(codes, hi_align_start, hi_align_exp_field, tail_pad_bits, exp_bits,
                                                mant_bits, bias).astype(np.float64)
    else:
        dec = A.fp_decode_aligned(codes, hi_align_start, hi_align_exp_field, tail_pad_bits, exp_bits, mant_bits,
                                  bias).astype(np.float64)
    with np.errstate(all="ignore"):
        deq = dt.R(dt.R(dec) * s).reshape(qshape)
    if quant_dim == 1:
        deq = np.ascontiguousarray(deq.T)
    return dt.to_output(deq), _half(s)

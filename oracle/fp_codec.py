"""CPU oracle for the FP weight formats: numpy restatement of the reference's FP4/FP6/FP8 codec
and of fp4_quantize_cpu.py's E2M1 "grid" quantizer.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).  Restates:
  _float_to_fp            quant_linear.py:126-163   (encode, with subnormals, no mantissa carry)
  _fp_to_float            quant_linear.py:213-235   (decode)
  FP4/FP6/FP8 branches    quant_linear.py:724-883   (sym absmax / asym mid-span scaling)
  quantize_fp16_to_fp4_e1m2 + _fp_scale   fp4_quantize_cpu.py:37-72
fp16 storage only (the reference runs fp16 models).  Every fp16 elementwise op is evaluated in
float and rounded RNE to fp16, like ATen.  torch.log2 on fp16 = RN16(log2(x)) — reproduced with a
float64 log2 rounded to fp16 (checked equal to torch on all 31743 positive finite fp16 inputs;
94 inputs land one binade up, e.g. 255.875 -> 2^8: the "log2 quirk").  Pinned against
reference-generated fixtures in tests/test_fp_golden.py.
"""
import numpy as np

F16 = np.float16


def R(x):
    """Round float32/64 -> fp16 -> float64 (one ATen fp16 op's output rounding)."""
    with np.errstate(over="ignore", invalid="ignore"):
        return np.asarray(x).astype(np.float32).astype(F16).astype(np.float64)


def fp_params(exp_bits, mant_bits):
    bias = 2 ** (exp_bits - 1) - 1
    fp_max = (1.0 + (2 ** mant_bits - 1) / 2 ** mant_bits) * 2.0 ** ((1 << exp_bits) - 1 - bias)
    return bias, fp_max


def log2_fp16(x16):
    """torch.log2 on an fp16 tensor: RN16(log2(x)) (x > 0); -inf at 0."""
    x = np.asarray(x16, dtype=F16).astype(np.float64)
    with np.errstate(divide="ignore"):
        return np.log2(x).astype(F16)


def float_to_fp(x16, exp_bits, mant_bits, exp_bias):
    """quant_linear.py:126-163 on an fp16 array -> uint8 codes."""
    x = np.asarray(x16, dtype=F16)
    sign = (x < 0).astype(np.uint16)
    x_abs = np.abs(x)
    zero = x_abs == 0
    x_abs_safe = np.where(zero, F16(1e-8), x_abs)                     # fp16(1e-8) == 0
    max_exp_field = (1 << exp_bits) - 1
    min_normal_exp = 1 - exp_bias
    with np.errstate(invalid="ignore"):
        e = np.floor(log2_fp16(x_abs_safe).astype(np.float64))         # floor(RN16(log2)) (-inf at 0)
    e = np.where(np.isfinite(e), e, 0).astype(np.int64)                 # value irrelevant: zero-masked below
    is_sub = e < min_normal_exp
    e_cl = np.clip(e, min_normal_exp, max_exp_field - exp_bias)
    exp_unb = (e_cl + exp_bias).astype(np.uint16)
    ms = 1 << mant_bits
    xa = x_abs_safe.astype(np.float64)
    # fp16 / fp32 tensor -> fp32 arithmetic (exact here): ((x / 2^e) - 1) * 2^M, round half-even
    m_norm = np.rint((xa / np.exp2(e_cl.astype(np.float64)) - 1.0) * ms)
    m_norm = np.clip(m_norm, 0, ms - 1).astype(np.uint16)
    # fp16 / 0-dim fp32 tensor -> fp16 arithmetic: RN16(x / 2^(1-bias)) * 2^M (RN16), round
    m_sub = np.rint(R(R(xa / 2.0 ** min_normal_exp) * ms))
    m_sub = np.clip(m_sub, 0, ms - 1).astype(np.uint16)
    exp_field = np.where(is_sub, 0, exp_unb).astype(np.uint16)
    mant_field = np.where(is_sub, m_sub, m_norm).astype(np.uint16)
    code = (sign << (exp_bits + mant_bits)) | (exp_field << mant_bits) | mant_field
    code = np.where(zero, 0, code)
    return (code & 0xFF).astype(np.uint8)


def fp_to_float(code, exp_bits, mant_bits, exp_bias):
    """quant_linear.py:213-235: uint8 codes -> float32 values (exact)."""
    c = np.asarray(code).astype(np.int64) & 0xFF
    sign = (c >> (exp_bits + mant_bits)) & 1
    raw_exp = (c >> mant_bits) & ((1 << exp_bits) - 1)
    mant = (c & ((1 << mant_bits) - 1)).astype(np.float64)
    v_norm = (1.0 + mant / (1 << mant_bits)) * np.exp2((raw_exp - exp_bias).astype(np.float64))
    v_sub = (mant / (1 << mant_bits)) * 2.0 ** (1 - exp_bias)
    v = np.where(raw_exp == 0, v_sub, v_norm)
    v = np.where(sign == 1, -v, v)
    v = np.where(c == 0, 0.0, v)
    return v.astype(np.float32)


def quantlinear_fp(weight16, exp_bits, mant_bits, w_group_size=128, symmetric=False, quant_dim=0):
    """FP4/FP6/FP8 branches of QuantLinear.quantize_weight (quant_linear.py:724-883), fp16 weight.

    Returns (dequant fp16 [out,in], scales fp16 [G,1], zeros fp16 [G,1] or None, codes uint8 in the
    weight layout)."""
    bias, fp_max = fp_params(exp_bits, mant_bits)
    if not np.isfinite(R(fp_max)):
        # torch.clamp(fp16, min=-fp_max, max=fp_max) converts the bounds to half (quant_linear.py:747/801/852)
        raise RuntimeError("value cannot be converted to type c10::Half without overflow")
    w = np.asarray(weight16, dtype=F16)
    wq = w.T if quant_dim == 1 else w
    qshape = wq.shape
    if w_group_size > 0:
        assert qshape[-1] % w_group_size == 0
        g = np.ascontiguousarray(wq).reshape(-1, w_group_size)
    elif w_group_size == -1:
        g = np.ascontiguousarray(wq).reshape(1, -1)
    elif w_group_size == -2:
        g = np.ascontiguousarray(wq).reshape(qshape[0], -1)
    else:
        raise ValueError("Invalid w_group_size")
    W = g.astype(np.float64)
    eps = R(1e-5)
    with np.errstate(all="ignore"):
        if symmetric:
            am = np.abs(W).max(axis=1, keepdims=True)
            am = np.where(am < eps, eps, am)
            s = R(am / np.float32(fp_max))
            s = np.where(s < eps, eps, s)
            z = None
            t = R(W / s)
        else:
            mx = W.max(axis=1, keepdims=True)
            mn = W.min(axis=1, keepdims=True)
            mid = R(R(mx + mn) * 0.5)
            span = R(R(mx - mn) * 0.5)
            span = np.where(span < eps, eps, span)
            s = R(span / np.float32(fp_max))
            s = np.where(s < eps, eps, s)
            z = mid
            t = R(R(W - z) / s)
        fpm = R(fp_max)
        t = np.where(t < -fpm, -fpm, np.where(t > fpm, fpm, t))
        codes = float_to_fp(t.astype(F16), exp_bits, mant_bits, bias)
        deq = R(R(fp_to_float(codes, exp_bits, mant_bits, bias)) * s)
        if z is not None:
            deq = R(deq + z)
    deq = deq.astype(F16).reshape(qshape)
    codes = codes.reshape(qshape)
    if quant_dim == 1:
        deq, codes = np.ascontiguousarray(deq.T), np.ascontiguousarray(codes.T)
    return deq, s.astype(F16), (None if z is None else z.astype(F16)), codes


def fp4_e2m1_grid(tensor16, group_size=128, per_tensor=False):
    """fp4_quantize_cpu.quantize_fp16_to_fp4_e1m2 (:47-72) with _fp_scale (:37-44).

    NB: like the reference it returns the GROUPED shape [-1, group_size] (no reshape back)."""
    t = np.asarray(tensor16, dtype=F16)
    if t.ndim != 2:
        raise ValueError("Expected a 2D tensor of shape [out_features, in_features].")
    if group_size > 0:
        if t.shape[1] % group_size != 0:
            raise ValueError("in_features must be divisible by group_size.")
        t = t.reshape(-1, group_size)
    if per_tensor:
        t = t.reshape(1, -1)
    M, E = 1, 2
    bias = 2 ** (E - 1) - 1
    max_float = (2 - 2 ** (-M)) * 2 ** (2 ** E - 1 - bias)
    x = t.astype(np.float64)
    with np.errstate(all="ignore"):
        max_val = np.abs(x).max(axis=1, keepdims=True)
        max_val = np.where(max_val < 1e-8, R(1e-8), max_val)          # clamp(min=1e-8): fp16(1e-8) == 0
        S = R(max_val / max_float)
        u = R(x / S)
        u = np.where(u < -max_float, -max_float, np.where(u > max_float, max_float, u))
        l = log2_fp16(np.abs(u).astype(F16)).astype(np.float64)        # -inf at 0
        ls = np.floor(R(l + bias))
        ls = np.where(ls < 1.0, 1.0, ls)                                # clamp(min=1.0); NaN kept
        sc = R(np.exp2(ls - M - bias))
        q = np.rint(R(u / sc))
        q = R(q * sc)
        out = R(q * S)
    return out.astype(F16)

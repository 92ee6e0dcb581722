"""CPU oracle for the research weight formats: block floating point (BFP) and the "approximate" /
"double-approximate" aligned FP decodes.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).  Restates:
  _rounding_rshift                     quant_linear.py:112-123
  _fp_decode_aligned                   quant_linear.py:237-285
  fp_decode_aligned_double_approx      quant_linear.py:288-363
  QuantLinear.quantize_weight_approximate   quant_linear.py:470-632
  QuantLinear.quantize_weight BFP branch    quant_linear.py:648-723
Integer semantics follow ATen exactly, including int8 wrap-around in the double-approximate path
(its tensors are int8): x << b is 0 for b >= width, x >> b is x >> (width-1) for b >= width, and
int8 additions wrap.  fp16 ops round RNE per op (ATen).  Pinned by reference-generated fixtures
(tests/golden/make_golden_approx.py -> approx_small.npz, tests/test_approx_golden.py).
"""
import numpy as np

from .fp_codec import R, float_to_fp, fp_params

F16 = np.float16


# ---------------------------------------------------------------------------------------------
# ATen integer shift semantics
def _lshift(a, b, width):
    a = np.asarray(a, dtype=np.int64)
    b = np.broadcast_to(np.asarray(b, dtype=np.int64), a.shape)
    mask = (1 << width) - 1
    r = (a << np.clip(b, 0, width - 1)) & mask
    r = np.where((b < 0) | (b >= width), 0, r)
    return _wrap(r, width)


def _rshift(a, b, width):
    a = _wrap(np.asarray(a, dtype=np.int64), width)
    b = np.broadcast_to(np.asarray(b, dtype=np.int64), a.shape)
    return np.where((b < 0) | (b >= width), a >> (width - 1), a >> np.clip(b, 0, width - 1))


def _wrap(x, width):
    x = np.asarray(x, dtype=np.int64) & ((1 << width) - 1)
    return np.where(x >= (1 << (width - 1)), x - (1 << width), x)


def rounding_rshift(val, shift, width=32):
    """quant_linear.py:112-123: (val + (1 << (shift-1) if shift > 0 else 0)) >> shift in intN."""
    val = _wrap(val, width)
    shift = np.broadcast_to(np.asarray(shift, dtype=np.int64), val.shape)
    off = np.where(shift > 0, _lshift(np.ones_like(val), shift - 1, width), 0)
    return _rshift(_wrap(val + off, width), shift, width)


# ---------------------------------------------------------------------------------------------
def bfp_quantize(weight, w_bit, w_group_size, quant_dim=0, dtype="float16"):
    """BFP branch of QuantLinear.quantize_weight (quant_linear.py:648-723).

    weight: float16 array, or float32 array holding float32 / bfloat16 values (`dtype` names which).
    Group = w_group_size consecutive elements of the (transposed when quant_dim == 1) weight, taken
    to fp16 (RNE); shared exponent = the group's max 5-bit fp16 exponent field; mantissas (leading 1
    added for normals; a subnormal's exponent field counts as 0) truncated by the exponent
    difference, then round-half-up to min(w_bit-1, 11) bits and saturated; dequant =
    mant * 2^(e_max - 15 - (bits-1)) * sign, exact in fp32, rounded once to `dtype`."""
    from .iwq_oracle import bf16_bits_to_f32, f32_to_bf16_bits
    if w_group_size <= 0:
        raise ValueError("BFP needs w_group_size > 0")
    w = np.asarray(weight)
    wq = w.T if quant_dim == 1 else w
    qshape = wq.shape
    assert qshape[-1] % w_group_size == 0
    g = np.ascontiguousarray(wq).reshape(-1, w_group_size)
    with np.errstate(over="ignore"):
        h = g if g.dtype == F16 else g.astype(np.float32).astype(F16)  # .to(torch.float16), RNE
    bits = h.view(np.uint16).astype(np.int64)
    sign = (bits >> 15) & 1
    exp = (bits >> 10) & 0x1F
    mant = bits & 0x3FF
    mwl = (np.where(exp == 0, 0, 1) << 10) | mant
    eb = exp.max(axis=1, keepdims=True)
    aligned = mwl >> np.clip(eb - exp, 0, None)                              # shift <= 31: plain
    tmb = min(w_bit - 1, 11)
    sd = max(0, 11 - tmb)
    rounded = rounding_rshift(aligned, sd) if sd > 0 else aligned
    rounded = np.minimum(rounded, (1 << tmb) - 1)                            # ValueError if w_bit < 1
    val = rounded.astype(np.float64) * np.exp2((eb - 15).astype(np.float64) - (tmb - 1))
    val = np.where(sign == 1, -val, val).astype(np.float32)                  # exact in fp32
    if dtype == "float16":
        with np.errstate(over="ignore"):
            out = val.astype(F16)
    elif dtype == "bfloat16":
        out = bf16_bits_to_f32(f32_to_bf16_bits(val))
    else:
        out = val
    out = out.reshape(qshape)
    return np.ascontiguousarray(out.T) if quant_dim == 1 else out


# ---------------------------------------------------------------------------------------------
def fp_decode_aligned(code, hi_align_start, hi_align_exp_field, tail_pad_bits, exp_bits, mant_bits, exp_bias,
                      align_subnorm_exp_as_one=True, limit_align_exp_to_field=True):
    """quant_linear.py:237-285 with decode_dtype = float16 (the only caller's setting): float32 out.

    Codes whose (aligned) exponent lies in [hi_align_start, hi_align_exp_field] are re-expressed at
    exponent hi_align_exp_field (mantissa padded by tail_pad_bits, rounding right shift by the
    difference); the others decode normally (subnormals included)."""
    c = np.asarray(code).astype(np.int64) & 0xFF
    zero = c == 0
    sign = (c >> (exp_bits + mant_bits)) & 1
    ef = (c >> mant_bits) & ((1 << exp_bits) - 1)
    mf = c & ((1 << mant_bits) - 1)
    ae = np.where(ef == 0, 1, ef) if align_subnorm_exp_as_one else ef
    lead = np.where(ef == 0, 0, 1)
    mfull = _wrap((lead << mant_bits) | mf, 32)
    if tail_pad_bits >= 0:
        mpad = _lshift(mfull, tail_pad_bits, 32)
    else:
        mpad = rounding_rshift(mfull, -tail_pad_bits)
    eu = np.where(ef == 0, 1 - exp_bias, ef - exp_bias)
    # fp16 arithmetic: RN16(RN16(mant / 2^M) * RN16(2^e))
    v_norm = R(R(mfull.astype(np.float64) / 2.0 ** mant_bits) * R(np.exp2(eu.astype(np.float64))))
    hi = ae >= hi_align_start
    if limit_align_exp_to_field:
        hi = hi & (ae <= hi_align_exp_field)
    sh = np.clip(hi_align_exp_field - ae, 0, None)
    mal = rounding_rshift(mpad, sh)
    hu = hi_align_exp_field - exp_bias
    v_hi = (mal.astype(np.float64) / 2.0 ** (mant_bits + tail_pad_bits) * 2.0 ** hu).astype(np.float32)
    v = np.where(hi, v_hi, v_norm.astype(np.float32)).astype(np.float32)
    v = np.where(sign == 1, -v, v)
    return np.where(zero, np.float32(0), v).astype(np.float32)


def fp_decode_aligned_double_approx(code, hi_align_start, hi_align_exp_field, tail_pad_bits, exp_bits, mant_bits,
                                    exp_bias, align_subnorm_exp_as_one=True, handle_max_outlier=True):
    """quant_linear.py:288-363 with decode_dtype = float16: fp16 out, same shape as `code` (2-D).

    Quads = 4 consecutive elements of code.T flattened row-major (for a [G, g] grouped code matrix:
    4 consecutive groups at the same in-group position).  A quad with <= 1 exponent outlier
    (outside [hi_align_start, hi_align_exp_field]) aligns to hi_align_exp_field, otherwise to its
    max exponent; with handle_max_outlier a max-exponent outlier forces the max exponent field.
    All integer tensors are int8 (wrap-around emulated)."""
    c2 = np.asarray(code)
    if c2.ndim != 2:
        raise ValueError("double approx decode expects a 2-D code matrix")
    ct = (c2.astype(np.int64) & 0xFF).T
    zero = ct == 0
    W = 8
    sign = _wrap((ct >> (exp_bits + mant_bits)) & 1, W)
    ef = _wrap((ct >> mant_bits) & ((1 << exp_bits) - 1), W)
    mf = _wrap(ct & ((1 << mant_bits) - 1), W)
    ae = np.where(ef == 0, 1, ef) if align_subnorm_exp_as_one else ef
    lead = np.where(ef == 0, 0, 1)
    mfull = _wrap(_lshift(lead, mant_bits, W) | mf, W)
    if tail_pad_bits >= 0:
        mpad = _lshift(mfull, tail_pad_bits, W)
    else:
        mpad = rounding_rshift(mfull, -tail_pad_bits, W)
    fe, fm, fs, fz = ae.reshape(-1), mpad.reshape(-1), sign.reshape(-1), zero.reshape(-1)
    if fe.size % 4 != 0:
        raise ValueError("double approx requires total elements divisible by 4")
    eg, mg, sg, zg = fe.reshape(-1, 4), fm.reshape(-1, 4), fs.reshape(-1, 4), fz.reshape(-1, 4)
    out_m = (eg < hi_align_start) | (eg > hi_align_exp_field)
    cnt = out_m.sum(axis=1, keepdims=True)
    gmax = eg.max(axis=1, keepdims=True)
    tgt = np.where(cnt <= 1, _wrap(hi_align_exp_field, W), gmax)
    if handle_max_outlier:
        mx = (1 << exp_bits) - 1
        has = ((eg == mx) & out_m).any(axis=1, keepdims=True)
        tgt = np.where(has, _wrap(mx, W), tgt)
    sh = _wrap(tgt - eg, W)
    shr = np.clip(sh, 0, None)
    shl = np.clip(-sh, 0, None)
    mr = rounding_rshift(mg, shr, W)
    ml = _lshift(mg, shl, W)
    cap = (((1 << (mant_bits + 1)) - 1) << tail_pad_bits) if tail_pad_bits >= 0 else \
        (((1 << (mant_bits + 1)) - 1) >> (-tail_pad_bits))
    ml = np.minimum(ml, _wrap(cap, W))
    mal = np.where(sh >= 0, mr, ml)
    hu = _wrap(tgt - exp_bias, W).astype(np.float64)
    # fp16 arithmetic: RN16(RN16(mant / 2^(M+tail)) * RN16(2^hu))
    v = R(R(mal.astype(np.float64) / 2.0 ** (mant_bits + tail_pad_bits)) * R(np.exp2(hu)))
    v = np.where(sg == 1, -v, v)
    v = np.where(zg, 0.0, v)
    return v.astype(F16).reshape(ct.shape).T


# ---------------------------------------------------------------------------------------------
def quantlinear_approx(weight16, exp_bits, mant_bits, w_group_size, quant_dim=0, hi_align_start=12,
                       hi_align_exp_field=15, tail_pad_bits=1, double_approximate=False, is_fp4=False):
    """QuantLinear.quantize_weight_approximate (quant_linear.py:470-632) on an fp16 weight.

    Codes: symmetric absmax FP scaling (identical to the sym FP branch's codes); decode with the
    aligned (or double-approximate) decoder; dequant = RN16(decoded * scale).  FP4 with 1 exponent
    bit always uses the single-aligned decoder (:494-506); FP4 with an exponent width other than 1
    or 2 leaves `decoded` unbound in the reference (UnboundLocalError), mirrored here.
    Returns (dequant fp16 [out, in], scales fp16 [G, 1])."""
    if w_group_size <= 0:
        raise ValueError("approximate needs w_group_size > 0")
    bias, fp_max = fp_params(exp_bits, mant_bits)
    w = np.asarray(weight16, dtype=F16)
    wq = w.T if quant_dim == 1 else w
    qshape = wq.shape
    assert qshape[-1] % w_group_size == 0
    g = np.ascontiguousarray(wq).reshape(-1, w_group_size)
    if is_fp4 and exp_bits not in (1, 2):
        raise UnboundLocalError("cannot access local variable 'decoded' where it is not associated with a value")
    W = g.astype(np.float64)
    eps = R(1e-5)
    with np.errstate(all="ignore"):
        am = np.abs(W).max(axis=1, keepdims=True)
        am = np.where(am < eps, eps, am)
        s = R(am / np.float32(fp_max))
        s = np.where(s < eps, eps, s)
        fpm = R(fp_max)
        if not np.isfinite(fpm):
            raise RuntimeError("value cannot be converted to type c10::Half without overflow")
        t = R(W / s)
        t = np.where(t < -fpm, -fpm, np.where(t > fpm, fpm, t))
    codes = float_to_fp(t.astype(F16), exp_bits, mant_bits, bias)
    if double_approximate and not (is_fp4 and exp_bits == 1):
        dec = fp_decode_aligned_double_approx(codes, hi_align_start, hi_align_exp_field, tail_pad_bits, exp_bits,
                                              mant_bits, bias).astype(np.float64)
    else:
        dec = R(fp_decode_aligned(codes, hi_align_start, hi_align_exp_field, tail_pad_bits, exp_bits, mant_bits,
                                  bias))
    with np.errstate(all="ignore"):
        deq = R(dec * s).astype(F16).reshape(qshape)
    if quant_dim == 1:
        deq = np.ascontiguousarray(deq.T)
    return deq, s.astype(F16)

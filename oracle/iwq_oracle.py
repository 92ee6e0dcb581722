"""CPU oracle: numpy restatement of the reference's min-max weight quantizer.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker.  The product
path (iron_weight_only_quant_amd) never routes through it.

What it restates (file:line in /root/reference):
  * quant_funcs.pseudo_quantize_tensor          quant_funcs.py:4-46
  * QuantLinear.quantize_weight, INT branch      quant_linear.py:885-956
    (group modes -1 / -2 / >0 at :896-906, quant_dim=1 transpose at :640-647)

Arithmetic model (SURVEY.md §7 "Hard parts", §8c): PyTorch evaluates every
16-bit elementwise op in fp32 and rounds the result RNE to the storage dtype;
torch.round is half-to-even; amax/amin are exact.  We compute in float32 numpy
arrays and round to the storage dtype after every op the reference performs as
a separate tensor op.  Signed zeros: ATen's amax/amin pick an order-dependent
zero when a group holds both +0 and -0; this oracle (and the HIP kernels) use
the total order -0 < +0.  That only changes the sign bit of a stored zero-point
of such a group (never a code or a dequantized value).

Pinning: checked bit-exactly against golden vectors produced by the reference
itself (tests/golden/make_golden.py, run in the survey container) in
tests/test_oracle_golden.py.
"""
import numpy as np

# ----------------------------------------------------------------------------
# storage formats
# ----------------------------------------------------------------------------


def f32_to_bf16_bits(x):
    """RNE float32 -> bfloat16 bit patterns (uint16); NaN stays NaN."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    lsb = (u >> np.uint64(16)) & np.uint64(1)
    r = ((u + np.uint64(0x7FFF) + lsb) >> np.uint64(16)).astype(np.uint32)
    nan = np.isnan(x)
    r = np.where(nan, (u >> np.uint64(16)).astype(np.uint32) | np.uint32(0x40), r)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


class _Fmt:
    """A 16/32-bit storage format: conversion to/from f32 and the per-op rounding R()."""

    def __init__(self, name):
        self.name = name
        if name not in ("float16", "bfloat16", "float32"):
            raise ValueError(f"unsupported dtype {name}")

    def to_f32(self, a):
        if self.name == "float16":
            return np.asarray(a, dtype=np.float16).astype(np.float32)
        if self.name == "bfloat16":
            return bf16_bits_to_f32(a)
        return np.asarray(a, dtype=np.float32).copy()

    def store(self, x):
        x = np.asarray(x, dtype=np.float32)
        if self.name == "float16":
            return x.astype(np.float16)
        if self.name == "bfloat16":
            return f32_to_bf16_bits(x)
        return x.copy()

    def R(self, x):
        """Round an f32 array to the storage dtype and back (one ATen op's output rounding)."""
        return self.to_f32(self.store(x))

    def bits(self, a):
        """Raw integer bit patterns of a storage array (for min/max keys)."""
        if self.name == "float16":
            return np.asarray(a, dtype=np.float16).view(np.int16).astype(np.int64), 16
        if self.name == "bfloat16":
            return np.asarray(a, dtype=np.uint16).view(np.int16).astype(np.int64), 16
        return np.asarray(a, dtype=np.float32).view(np.int32).astype(np.int64), 32


def _key(bits, nb):
    # sign-magnitude -> two's complement order key; involution.  -0 < +0, NaNs sort outside +-inf.
    mag = (1 << (nb - 1)) - 1
    return np.where(bits < 0, bits ^ mag, bits)


def _group_minmax(fmt, g_store):
    """Exact per-row (min, max) of a [G, L] storage array, total order -0 < +0."""
    b, nb = fmt.bits(g_store)
    k = _key(b, nb)
    kmin = _key(k.min(axis=1, keepdims=True), nb)
    kmax = _key(k.max(axis=1, keepdims=True), nb)
    if nb == 16:
        kmin = kmin.astype(np.int16)
        kmax = kmax.astype(np.int16)
        if fmt.name == "float16":
            return kmin.view(np.float16).astype(np.float32), kmax.view(np.float16).astype(np.float32)
        return bf16_bits_to_f32(kmin.view(np.uint16)), bf16_bits_to_f32(kmax.view(np.uint16))
    return kmin.astype(np.int32).view(np.float32), kmax.astype(np.int32).view(np.float32)


def _clamp(x, lo, hi):
    """torch.clamp semantics: NaN propagates, an in-range value (incl. -0) is kept."""
    return np.where(x < lo, lo, np.where(x > hi, hi, x)).astype(np.float32)


def _quant_groups(fmt, g_store, n_bits, symmetric, sym_adds_zero=True):
    """Quantize a [G, L] storage array of groups.

    Returns (dequant_f32 [G,L], scales_f32 [G,1], zeros_f32 [G,1] or None, codes int64 [G,L]).
    Arithmetic follows quant_funcs.py:16-38 == quant_linear.py:909-947.
    """
    R = fmt.R
    W = fmt.to_f32(g_store).reshape(g_store.shape)
    eps = R(np.float32(1e-5))
    with np.errstate(all="ignore"):
        if not symmetric:
            mn, mx = _group_minmax(fmt, g_store)                           # amin/amax (:17-18 / :917-918)
            max_int = np.float32(2 ** n_bits - 1)
            rng = R(mx - mn)
            rng = np.where(rng < eps, eps, rng).astype(np.float32)         # .clamp(min=1e-5)
            s = R(rng / max_int)                                           # / max_int (:21 / :921)
            z = _clamp(-np.rint(R(mn / s)), np.float32(0), R(max_int))     # (:22 / :922)
            t = R(W / s)                                                   # tensor / scales
            r = np.rint(t)                                                 # torch.round (half-even)
            a = R(r + z)                                                   # + zeros
            c = _clamp(a, np.float32(0), R(max_int))                       # clamp(min_int, max_int)
            d = R(c - z)                                                   # - zeros
            out = R(d * s)                                                 # * scales
            codes = c
            zeros = z
        else:
            absb = np.abs(W)
            # abs().amax(): magnitudes of the storage values, exact
            am = absb.max(axis=1, keepdims=True).astype(np.float32)
            am = np.where(np.isnan(absb).any(axis=1, keepdims=True), np.float32(np.nan), am)
            am = np.where(am < eps, eps, am).astype(np.float32)            # clamp(min=1e-5)
            max_int = np.float32(2 ** (n_bits - 1) - 1)
            min_int = np.float32(-(2 ** (n_bits - 1)))
            s = R(am / max_int)                                            # (:28 / :914)
            t = R(W / s)
            r = np.rint(t)
            if sym_adds_zero:
                r = R(r + np.float32(0))      # "+ zeros" with zeros = python 0 (:37 / :936) -> -0 becomes +0
            c = _clamp(r, R(min_int), R(max_int))
            out = R(c * s)                    # (c - 0) * s  == c * s  for the +0-normalized c
            codes = c + np.float32(2 ** (n_bits - 1))   # offset-binary code (build's packed format)
            zeros = None
    codes = np.where(np.isfinite(codes), codes, -1).astype(np.int64)
    return out.astype(np.float32), s.astype(np.float32), (None if zeros is None else zeros.astype(np.float32)), codes


# ----------------------------------------------------------------------------
# public restatements
# ----------------------------------------------------------------------------

class OracleResult:
    def __init__(self, dequant, scales, zeros, codes, nan):
        self.dequant = dequant      # storage dtype, same shape as input
        self.scales = scales        # storage dtype [G,1]
        self.zeros = zeros          # storage dtype [G,1] or None
        self.codes = codes          # int64, same shape as the grouped view, reshaped to the weight layout
        self.nan = nan              # True if the dequantized output holds a NaN


def pseudo_quantize_tensor(tensor, n_bits=8, zero_point=True, q_group_size=-1, per_tensor=False,
                           dtype="float16"):
    """Restates quant_funcs.pseudo_quantize_tensor (quant_funcs.py:4-46).

    Raises AssertionError exactly where the reference does (:11, :15, :40)."""
    fmt = _Fmt(dtype)
    a = np.asarray(tensor)
    org_shape = a.shape
    g = a
    if q_group_size > 0:
        assert org_shape[-1] % q_group_size == 0
        g = a.reshape(-1, q_group_size)
    if per_tensor:
        g = g.reshape(1, -1)
    assert g.ndim == 2
    out, s, z, codes = _quant_groups(fmt, np.ascontiguousarray(g), n_bits, not zero_point, sym_adds_zero=True)
    nan = bool(np.isnan(out).any())
    assert not nan
    return OracleResult(fmt.store(out).reshape(org_shape), fmt.store(s),
                        None if z is None else fmt.store(z), codes.reshape(org_shape), nan)


def quantlinear_int(weight, w_bit=4, w_group_size=128, symmetric=True, quant_dim=0, dtype="float16"):
    """Restates QuantLinear.quantize_weight INT branch (quant_linear.py:885-956) incl. quant_dim (:640-647).

    Returns OracleResult; dequant has the weight's [out, in] layout; codes too.
    w_bit >= 16 -> returns None (layer left unquantized, :887-892)."""
    fmt = _Fmt(dtype)
    w = np.asarray(weight)
    assert w.ndim == 2
    if w_bit >= 16:
        return None
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
    out, s, z, codes = _quant_groups(fmt, g, w_bit, symmetric, sym_adds_zero=True)
    deq = fmt.store(out).reshape(qshape)
    codes = codes.reshape(qshape)
    if quant_dim == 1:
        deq = np.ascontiguousarray(deq.T)
        codes = np.ascontiguousarray(codes.T)
    nan = bool(np.isnan(out).any())
    return OracleResult(deq, fmt.store(s), None if z is None else fmt.store(z), codes, nan)


def pack_codes(codes, n_bits):
    """The build's packed layout (include/iwq.h): n_bits<=4 -> two codes per byte, low nibble = even
    column; 4<n_bits<=8 -> one byte per code.  codes: [rows, cols] int."""
    c = np.asarray(codes).astype(np.int64)
    if n_bits <= 4:
        assert c.shape[-1] % 2 == 0
        lo = c[..., 0::2] & 0xF
        hi = c[..., 1::2] & 0xF
        return (lo | (hi << 4)).astype(np.uint8)
    return (c & 0xFF).astype(np.uint8)

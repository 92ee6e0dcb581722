// iwq_fp.cuh — FP weight formats of the reference, bit-exact on gfx950 (fp16 storage).
//
//   encode  quant_linear._float_to_fp   quant_linear.py:126-163
//   decode  quant_linear._fp_to_float   quant_linear.py:213-235
//   FP4/FP6/FP8 branches of QuantLinear.quantize_weight   quant_linear.py:724-883
//   E2M1 "grid" quantizer  fp4_quantize_cpu.py:37-72
//
// The reference codec is neither IEEE nor OCP (E4M3 max is 480; a mantissa that rounds past the
// top of its binade is clamped, not carried; the exponent comes from an fp16 torch.log2, which
// rounds up for the top few mantissas of 40 binades).  CDNA4's v_cvt_*fp8/fp4 therefore cannot be
// used for the encode: it is integer/ALU code here, with the log2 behaviour as per-binade
// thresholds (iwq_fp_tables.h) and every arithmetic step exact in fp32.
#pragma once
#include "iwq_common.cuh"
#include "iwq_fp_tables.h"

namespace iwq {

struct FpSpec {
  int E, M, bias;    // exponent / mantissa bits, bias = 2^(E-1) - 1
  int emin, emax;    // min normal unbiased exponent (1 - bias), max ((2^E - 1) - bias)
  float fp_max;      // (1 + (2^M - 1)/2^M) * 2^emax  (python float in the reference)
  float fp_max16;    // RN16(fp_max): torch.clamp converts its bounds to half
  float rmax;        // RN32(1/fp_max): corrected division when fp_max is an fp16 value
  int fpmax_is_f16;  // fp_max exactly representable in fp16
  int hs, hf, tp;    // approximate decodes: hi_align_start, hi_align_exp_field, tail_pad_bits
  // fast-path constants (fp_roundtrip_fast), all formats that pass fp_spec have E <= 4
  uint32_t sh;        // 10 - M: fp16 mantissa bits dropped
  uint32_t rne_bias;  // 2^(sh-1) - 1
  uint32_t mmax;      // 2^M - 1
  uint32_t fpmax_bits, emin_bits;  // fp16 bits of fp_max and of 2^emin
  float sub_c;        // 2^(23 + emin - M): (x + c) - c rounds x to the FP subnormal grid (RNE)
  float sub_max;      // (2^M - 1) * 2^(emin - M): largest FP subnormal (no carry into the normals)
  float sub_inv;      // 2^(M - emin)
  float sub_c16;      // 2^(10 + emin - M): fp16 form of sub_c
};

// The log2 threshold tables live in LDS during a kernel (a per-lane index into __constant__ memory
// would be one vector-memory load per element): kernels call stage_log2_tables() once.
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
struct Log2Tabs {
  lds_u16* up;   // kLog2UpThresh
  lds_u16* p1;   // kLog2P1UpThresh
  lds_u16* up7;  // kLog2UpThresh with "none" (0xFFFF) as 0x7FFF: u - thr is then a valid int16
};
// all threads of the block must call it (contains a barrier); `buf` = a __shared__ uint16_t[120]
__device__ __forceinline__ Log2Tabs stage_log2_tables(uint16_t* buf) {
  if (threadIdx.x < 40) {
    const uint16_t u = kLog2UpThresh[threadIdx.x];
    buf[threadIdx.x] = u;
    buf[40 + threadIdx.x] = kLog2P1UpThresh[threadIdx.x];
    buf[80 + threadIdx.x] = u == 0xFFFFu ? (uint16_t)0x7FFFu : u;
  }
  __syncthreads();
  return Log2Tabs{(lds_u16*)buf, (lds_u16*)buf + 40, (lds_u16*)buf + 80};
}

// floor(RN16(log2 x)) for a positive fp16 magnitude (bit pattern, 1..0x7BFF)
__device__ __forceinline__ int fp16_floor_log2_torch(uint32_t mag, lds_u16* thresh) {
  const int ef = (int)(mag >> 10);
  const int e_true = ef > 0 ? ef - 15 : (31 - __builtin_clz(mag)) - 24;
  return e_true + (mag >= (uint32_t)thresh[e_true + 24] ? 1 : 0);
}

// _float_to_fp on an fp16 value (bit pattern).  NaN inputs (only reachable when the group's scale
// is NaN, where every output is NaN anyway) encode as 0.
__device__ __forceinline__ uint32_t fp_encode(uint32_t b, const FpSpec& f, const Log2Tabs& tb) {
  const uint32_t mag = b & 0x7FFFu;
  if (mag == 0 || mag > 0x7C00u) return 0;                // zero_mask (:132,:161); NaN
  const uint32_t sign = b >> 15;                          // x < 0 (:130)
  const int e = fp16_floor_log2_torch(mag < 0x7C00u ? mag : 0x7BFFu, tb.up);
  const float xa = (float)__builtin_bit_cast(_Float16, (uint16_t)mag);
  const float ms = (float)(1u << f.M);
  uint32_t exp_field, mant;
  if (e >= f.emin) {                                      // normal path (:145-149)
    const int ec = e < f.emax ? e : f.emax;
    float m = __builtin_rintf((__builtin_ldexpf(xa, -ec) - 1.0f) * ms);   // exact in fp32
    m = m < 0.0f ? 0.0f : (m > ms - 1.0f ? ms - 1.0f : m);               // no carry
    exp_field = (uint32_t)(ec + f.bias);
    mant = (uint32_t)m;
  } else {                                                // subnormal path (:152-154), fp16 ops exact
    float m = __builtin_rintf(__builtin_ldexpf(xa, -f.emin) * ms);
    m = m > ms - 1.0f ? ms - 1.0f : m;
    exp_field = 0;
    mant = (uint32_t)m;
  }
  return ((sign << (f.E + f.M)) | (exp_field << f.M) | mant) & 0xFFu;
}

// _fp_to_float: exact value in fp32 (code 0 -> +0; sign-only code -> -0)
__device__ __forceinline__ float fp_decode(uint32_t code, const FpSpec& f) {
  if (code == 0) return 0.0f;
  const uint32_t sign = (code >> (f.E + f.M)) & 1u;
  const int raw_exp = (int)((code >> f.M) & ((1u << f.E) - 1u));
  const int mant = (int)(code & ((1u << f.M) - 1u));
  const float v = raw_exp == 0 ? __builtin_ldexpf((float)mant, f.emin - f.M)
                               : __builtin_ldexpf((float)((1 << f.M) + mant), raw_exp - f.bias - f.M);
  return sign ? -v : v;
}

// Fast path of _float_to_fp + _fp_to_float for a finite fp16 t already clamped to +-fp_max:
// integer / fp32 bit work on t's fp16 pattern instead of the log2 / ldexp chain.  Returns the fp16
// bits of the decoded value (exact in fp16 for E <= 4) and, with WANT_CODE, the code.
//  normal FP range: RNE of the 10-bit fp16 mantissa to M bits, saturated at 2^M - 1 (no carry);
//    the torch.log2 quirk (mantissa >= per-binade threshold -> exponent + 1) gives exactly
//    2^(e+1) with mantissa 0 — the value a carry would give; capped at fp_max
//  FP subnormal range (exponent < emin after the quirk): RNE of x to multiples of 2^(emin-M) by
//    one fp32 add/sub pair, saturated below 2^emin
template <bool WANT_CODE>
__device__ __forceinline__ uint32_t fp_roundtrip_fast(uint32_t tb, float ta, const FpSpec& f, lds_u16* up_e16,
                                                      uint32_t& code) {
  const uint32_t u = tb & 0x7FFFu;
  const uint32_t e16 = u >> 10;
  const uint32_t fr = u & 0x3FFu;
  uint32_t q = (fr + f.rne_bias + ((fr >> f.sh) & 1u)) >> f.sh;
  q = q < f.mmax ? q : f.mmax;
  uint32_t r = (e16 << 10) | (q << f.sh);
  r = u >= (uint32_t)up_e16[e16] ? (e16 + 1u) << 10 : r;
  r = r < f.fpmax_bits ? r : f.fpmax_bits;
  float ys = opaque(ta + f.sub_c) - f.sub_c;
  ys = ys < f.sub_max ? ys : f.sub_max;
  const bool normal = r >= f.emin_bits;
  const uint32_t mag = normal ? r : (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)ys);
  if constexpr (WANT_CODE) {
    const uint32_t ef = normal ? (mag >> 10) - 15u + (uint32_t)f.bias : 0u;
    const uint32_t m = normal ? (mag >> f.sh) & f.mmax : (uint32_t)(ys * f.sub_inv);
    code = u == 0 ? 0u : ((((tb >> 15) & 1u) << (f.E + f.M)) | (ef << f.M) | m);
  }
  return u == 0 ? 0u : (mag | (tb & 0x8000u));
}

// Packed-pair form of fp_roundtrip_fast: two fp16 t (bits in one dword, finite, clamped) -> the two
// decoded fp16 values, all integer steps on 16-bit halves (v_pk_*_u16, bitwise selects), the FP
// subnormal grid in fp16 arithmetic: (|t| + C) - C with C = 2^(10 + emin - M) rounds |t| < 2^emin to
// multiples of 2^(emin - M) (RNE) because the fp16 spacing in [C, 2C) is exactly that.
__device__ __forceinline__ uint32_t pk_lt_mask(u16x2 a, u16x2 b) {  // 0xFFFF per half where a < b
  // valid when |a - b| < 2^15 (all callers); (a - b) >> 15 = 1 iff a < b
  const u16x2 lt = (a - b) >> (u16x2)15;
  return __builtin_bit_cast(uint32_t, (u16x2)0 - lt);
}
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {  // mask ? a : b
  return (mask & a) | (~mask & b);
}
__device__ __forceinline__ uint32_t fp_roundtrip_pk(uint32_t tpair, const FpSpec& f, const Log2Tabs& tabs,
                                                    h2 c16, h2 submax16) {
  const u16x2 tb = __builtin_bit_cast(u16x2, tpair);
  const u16x2 u = tb & (u16x2)0x7FFF;
  const u16x2 e16 = u >> (u16x2)10;
  const u16x2 fr = u & (u16x2)0x3FF;
  const u16x2 sh = (u16x2)(uint16_t)f.sh;
  u16x2 q = (fr + (u16x2)(uint16_t)f.rne_bias + ((fr >> sh) & (u16x2)1)) >> sh;
  q = __builtin_elementwise_min(q, (u16x2)(uint16_t)f.mmax);
  const uint32_t rn = __builtin_bit_cast(uint32_t, (u16x2)((e16 << (u16x2)10) | (q << sh)));
  const u16x2 thr = {tabs.up7[e16.x + 9], tabs.up7[e16.y + 9]};
  const uint32_t rup = __builtin_bit_cast(uint32_t, (u16x2)((e16 + (u16x2)1) << (u16x2)10));
  uint32_t r = bfi(pk_lt_mask(u, thr), rn, rup);                        // u < thr: RNE result, else 2^(e+1)
  r = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, r),
                                                             (u16x2)(uint16_t)f.fpmax_bits));
  const h2 ta = __builtin_bit_cast(h2, __builtin_bit_cast(uint32_t, u));
  const uint32_t rs = __builtin_bit_cast(uint32_t, pk_min((ta + c16) - c16, submax16));
  const uint32_t mag = bfi(pk_lt_mask(__builtin_bit_cast(u16x2, r), (u16x2)(uint16_t)f.emin_bits), rs, r);
  const u16x2 nz = (u + (u16x2)0x7FFF) >> (u16x2)15;                    // 1 where t != 0
  const uint32_t nzm = __builtin_bit_cast(uint32_t, (u16x2)0 - nz);
  return (mag | (tpair & 0x80008000u)) & nzm;
}

// code of one element from its decoded fp16 magnitude bits (see fp_roundtrip_fast)
__device__ __forceinline__ uint32_t fp_code_from_mag(uint32_t mag, uint32_t tb, const FpSpec& f) {
  const uint32_t u = tb & 0x7FFFu;
  const bool normal = mag >= f.emin_bits;
  const uint32_t ef = normal ? (mag >> 10) - 15u + (uint32_t)f.bias : 0u;
  const uint32_t m = normal ? (mag >> f.sh) & f.mmax
                            : (uint32_t)((float)__builtin_bit_cast(_Float16, (uint16_t)mag) * f.sub_inv);
  return u == 0 ? 0u : ((((tb >> 15) & 1u) << (f.E + f.M)) | (ef << f.M) | m);
}

struct FpParams {
  float s;    // scales (fp16 value)
  float rs;   // RN32(1/s)
  float z;    // zeros = mid point (asymmetric) / 0
  bool fast;  // finite group: corrected divisions are exact
};

__device__ __forceinline__ float f16r(float x) { return (float)(_Float16)opaque(x); }

// quotient of fp16 values x / y rounded to fp16: corrected division when allowed, else IEEE
__device__ __forceinline__ float div16(float x, float y, float ry, bool fast) {
  return fast ? (float)(_Float16)div_f16vals(x, y, ry) : f16r(x / y);
}

// sym (:744-747 etc.): max_val = absmax.clamp(1e-5); scales = (max_val / fp_max).clamp(1e-5)
__device__ __forceinline__ FpParams fp_params_sym(float am, const FpSpec& f) {
  FpParams p;
  const float eps = (float)(_Float16)1e-5f;
  const bool fin = am <= 65504.0f;  // false for NaN / inf
  float m = am < eps ? eps : am;
  float s = div16(m, f.fp_max, f.rmax, fin && f.fpmax_is_f16);
  s = s < eps ? eps : s;
  p.s = s;
  p.z = 0.0f;
  p.rs = rcp_f16val(s);
  p.fast = fin;
  return p;
}

// asym (:749-755): mid = (max + min) * 0.5; span = ((max - min) * 0.5).clamp(1e-5);
// scales = (span / fp_max).clamp(1e-5); zeros = mid
__device__ __forceinline__ FpParams fp_params_asym(float mn, float mx, const FpSpec& f) {
  FpParams p;
  const float eps = (float)(_Float16)1e-5f;
  const float mid = f16r(f16r(mx + mn) * 0.5f);
  float span = f16r(f16r(mx - mn) * 0.5f);
  const bool fin = span <= 65504.0f && mid == mid && mid <= 65504.0f && mid >= -65504.0f;
  span = span < eps ? eps : span;
  float s = div16(span, f.fp_max, f.rmax, fin && f.fpmax_is_f16);
  s = s < eps ? eps : s;
  p.s = s;
  p.z = mid;
  p.rs = rcp_f16val(s);
  p.fast = fin;
  return p;
}

// one element of the FP branches: returns the dequantized value (fp32 holding an fp16 value)
template <bool SYM, bool WANT_CODE = true>
__device__ __forceinline__ float fp_quant_elem(float w, const FpParams& p, const FpSpec& f, uint32_t& code,
                                               const Log2Tabs& tabs) {
  if (p.fast) {  // finite group: corrected division, med3 clamp, bit-level codec, native fp16 mul/add
    const float q = SYM ? div_f16vals(w, p.s, p.rs) : div_f16vals(f16r(w - p.z), p.s, p.rs);
    const float t = __builtin_amdgcn_fmed3f((float)(_Float16)q, -f.fp_max16, f.fp_max16);
    const uint32_t tb = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)t);
    const uint32_t d = fp_roundtrip_fast<WANT_CODE>(tb, __builtin_fabsf(t), f, tabs.up + 9, code);
    _Float16 y = __builtin_bit_cast(_Float16, (uint16_t)d) * (_Float16)p.s;  // RN16(exact product)
    if constexpr (!SYM) y = y + (_Float16)p.z;   // RN16(exact sum) == RN16(RN32(sum)) (24 >= 2*11+2)
    return (float)y;
  }
  float t;
  if constexpr (SYM) t = div16(w, p.s, p.rs, p.fast);                    // W / scales
  else t = div16(f16r(w - p.z), p.s, p.rs, p.fast);                      // (W - zeros) / scales
  t = clamp_nan(t, -f.fp_max16, f.fp_max16);                             // clamp(-fp_max, fp_max)
  const uint32_t tb = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)t);
  code = fp_encode(tb, f, tabs);
  float y = f16r(f16r(fp_decode(code, f)) * p.s);                        // .to(fp16) * scales
  if constexpr (!SYM) y = f16r(y + p.z);                                  // + zeros
  if (t != t) y = t;                                                      // NaN scale: NaN out
  return y;
}

// Two elements of the FP branches at once (finite group): corrected fp32 divisions as a float2
// (v_pk_mul/fma_f32), pair conversion, packed clamp, the packed codec, packed fp16 dequant.
template <bool SYM, bool WANT_CODE>
__device__ __forceinline__ uint32_t fp_quant_pair_fast(uint32_t wpair, const FpParams& p, const FpSpec& f,
                                                       const Log2Tabs& tabs, uint32_t& c0, uint32_t& c1) {
  const h2 s16 = h2{(_Float16)p.s, (_Float16)p.s};
  const h2 z16 = h2{(_Float16)p.z, (_Float16)p.z};
  h2 d = __builtin_bit_cast(h2, wpair);
  if constexpr (!SYM) d = d - z16;                              // RN16(w - z): fp16 sub == ATen's fp32-then-round
  const f2 df = {(float)d.x, (float)d.y};
  const f2 rs2 = {p.rs, p.rs}, s2 = {p.s, p.s};
  f2 q0 = df * rs2;
  f2 e = __builtin_elementwise_fma(-q0, s2, df);
  f2 q1 = __builtin_elementwise_fma(e, rs2, q0);
  asm volatile("" : "+v"(q1));                                   // keep the fp32 rounding (no fma_mix)
  h2 t = __builtin_convertvector(q1, h2);                        // RN16(d / s)
  const h2 fm = h2{(_Float16)f.fp_max16, (_Float16)f.fp_max16};
  t = pk_max(pk_min(t, fm), -fm);
  const uint32_t tb = __builtin_bit_cast(uint32_t, t);
  const h2 c16 = h2{(_Float16)f.sub_c16, (_Float16)f.sub_c16};
  const h2 sm16 = h2{(_Float16)f.sub_max, (_Float16)f.sub_max};
  const uint32_t dec = fp_roundtrip_pk(tb, f, tabs, c16, sm16);
  if constexpr (WANT_CODE) {
    c0 = fp_code_from_mag(dec & 0x7FFFu, tb & 0xFFFFu, f);
    c1 = fp_code_from_mag((dec >> 16) & 0x7FFFu, tb >> 16, f);
  }
  h2 y = __builtin_bit_cast(h2, dec) * s16;                     // RN16(exact product)
  if constexpr (!SYM) y = y + z16;
  return __builtin_bit_cast(uint32_t, y);
}

// ---------------------------------------------------------------------------------------------
// "approximate" decodes (quant_linear.py:112-123, :237-363).  Integer steps follow ATen's shift
// semantics: x << b == 0 and x >> b == x >> (width-1) once b >= width; the double-approximate
// decoder's tensors are int8, so its adds and shifts wrap at 8 bits (w8).
__device__ __forceinline__ int w8(int x) { return (int)(int8_t)(uint8_t)(x & 0xFF); }
__device__ __forceinline__ int lsh8(int a, int b) { return (b < 0 || b >= 8) ? 0 : w8(a << b); }
__device__ __forceinline__ int rsh8(int a, int b) { return (b < 0 || b >= 8) ? (a >> 7) : (a >> b); }
__device__ __forceinline__ int rrsh8(int v, int s) { return rsh8(w8(v + (s > 0 ? lsh8(1, s - 1) : 0)), s); }
__device__ __forceinline__ int lsh32(int a, int b) { return (b < 0 || b >= 32) ? 0 : (int)((uint32_t)a << b); }
__device__ __forceinline__ int rsh32(int a, int b) { return (b < 0 || b >= 32) ? (a >> 31) : (a >> b); }
__device__ __forceinline__ int rrsh32(int v, int s) {
  return rsh32((int)((uint32_t)v + (uint32_t)(s > 0 ? lsh32(1, s - 1) : 0)), s);
}

// _fp_decode_aligned (quant_linear.py:237-285) as every caller uses it (align_subnorm_exp_as_one,
// limit_align_exp_to_field, decode_dtype fp16): codes whose aligned exponent is in [hs, hf] are
// re-expressed at exponent hf (mantissa padded by tp bits, rounding right shift by hf - exp), the
// others decode normally.  Exact value in fp32; code 0 -> +0, sign-only code -> -0.
__device__ __forceinline__ float fp_decode_aligned(uint32_t code, const FpSpec& f) {
  code &= 0xFFu;
  if (code == 0) return 0.0f;
  const uint32_t sign = (code >> (f.E + f.M)) & 1u;
  const int ef = (int)((code >> f.M) & ((1u << f.E) - 1u));
  const int mf = (int)(code & ((1u << f.M) - 1u));
  const int ae = ef == 0 ? 1 : ef;
  const int mfull = ((ef != 0 ? 1 : 0) << f.M) | mf;
  float v;
  if (ae >= f.hs && ae <= f.hf) {
    const int mpad = f.tp >= 0 ? lsh32(mfull, f.tp) : rrsh32(mfull, -f.tp);
    const int mal = rrsh32(mpad, f.hf - ae);                 // hf - ae >= 0 here
    v = __builtin_ldexpf((float)mal, (f.hf - f.bias) - f.M - f.tp);
  } else {
    // fp16 ops RN16(mant / 2^M) * RN16(2^e): exact for every format that passes fp_spec
    v = __builtin_ldexpf((float)mfull, (ef == 0 ? 1 - f.bias : ef - f.bias) - f.M);
  }
  return sign ? -v : v;
}

// one element of quantize_weight_approximate (:470-632), single-aligned decode: symmetric absmax
// codes exactly as the FP branch, then RN16(RN16(decode_aligned(code)) * scales)
__device__ __forceinline__ float fp_apx_elem(float w, const FpParams& p, const FpSpec& f, uint32_t& code,
                                             const Log2Tabs& tabs) {
  float t = div16(w, p.s, p.rs, p.fast);
  t = clamp_nan(t, -f.fp_max16, f.fp_max16);
  const uint32_t tb = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)t);
  if (p.fast) fp_roundtrip_fast<true>(tb, __builtin_fabsf(t), f, tabs.up + 9, code);
  else code = fp_encode(tb, f, tabs);
  const float y = f16r(f16r(fp_decode_aligned(code, f)) * p.s);
  return t != t ? t : y;
}

// fp_decode_aligned_double_approx (quant_linear.py:288-363) on one quad of codes (4 consecutive
// elements of the transposed grouped code matrix), int8 arithmetic; fp16 values out.
__device__ __forceinline__ void fp_decode_double4(const uint32_t (&code)[4], const FpSpec& f, float (&out)[4]) {
  int ae[4], mpad[4], sg[4];
  bool zero[4];
  int cnt = 0, gmax = -128;
  bool has_max = false;
  const int maxv = (1 << f.E) - 1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t c = code[k] & 0xFFu;
    zero[k] = c == 0;
    sg[k] = w8((int)((c >> (f.E + f.M)) & 1u));
    const int ef = w8((int)((c >> f.M) & ((1u << f.E) - 1u)));
    const int mf = w8((int)(c & ((1u << f.M) - 1u)));
    ae[k] = ef == 0 ? 1 : ef;
    const int mfull = w8(lsh8(ef == 0 ? 0 : 1, f.M) | mf);
    mpad[k] = f.tp >= 0 ? lsh8(mfull, f.tp) : rrsh8(mfull, -f.tp);
    const bool outl = ae[k] < f.hs || ae[k] > f.hf;
    cnt += outl ? 1 : 0;
    gmax = ae[k] > gmax ? ae[k] : gmax;
    has_max |= outl && ae[k] == maxv;
  }
  int tgt = cnt <= 1 ? w8(f.hf) : gmax;
  if (has_max) tgt = w8(maxv);
  const int capr = ((1 << (f.M + 1)) - 1);
  const int cap = w8(f.tp >= 0 ? (capr << f.tp) : (capr >> (-f.tp)));
  const float scale_m = (float)(_Float16)__builtin_ldexpf(1.0f, -(f.M + f.tp));
  const float p2 = (float)(_Float16)__builtin_ldexpf(1.0f, w8(tgt - f.bias));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int sh = w8(tgt - ae[k]);
    const int shr = sh > 0 ? sh : 0;
    const int nsh = w8(-sh);
    const int shl = nsh > 0 ? nsh : 0;
    const int mr = rrsh8(mpad[k], shr);
    int ml = lsh8(mpad[k], shl);
    ml = ml > cap ? cap : ml;
    const int mal = sh >= 0 ? mr : ml;
    float v = f16r(f16r((float)mal * scale_m) * p2);   // fp16 ops: mant / 2^(M+tail) * 2^(tgt-bias)
    v = sg[k] == 1 ? -v : v;
    out[k] = zero[k] ? 0.0f : v;
  }
}

// fp4_quantize_cpu._fp_scale element (:37-44) with S = RN16(max(absmax, fp16(1e-8)) / 6)
// code (optional): the E2M1 code of q (sign | exponent field | mantissa; |q| in {0, .5, 1, 1.5, 2,
// 3, 4, 6} -> 0..7), so that decode(code) * S (iwq_dequant_fp_packed) reproduces the output
__device__ __forceinline__ float grid_elem(float x, float S, float rS, bool fast, const Log2Tabs& tabs,
                                           uint32_t* code = nullptr) {
  float u = (fast && S > 0.0f) ? (float)(_Float16)div_f16vals(x, S, rS) : f16r(x / S);
  u = clamp_nan(u, -6.0f, 6.0f);
  if (u != u) {
    if (code) *code = 0;
    return u;
  }
  const uint32_t mag = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)u) & 0x7FFFu;
  // ls = clamp(floor(log2|u| + 1), 1): |u| == 0 -> -inf -> 1
  int ls = mag == 0 ? 1 : fp16_floor_log2_torch(mag, tabs.p1) + 1;
  ls = ls < 1 ? 1 : ls;
  const float sc = __builtin_ldexpf(1.0f, ls - 2);                        // 2^(ls - M - bias)
  const float q = __builtin_rintf(u / sc) * sc;                           // exact (power-of-two scale)
  if (code) {
    const int i2 = (int)(__builtin_fabsf(q) * 2.0f);                      // 0 1 2 3 4 6 8 12
    const uint32_t e = i2 <= 4 ? (uint32_t)i2 : (i2 == 6 ? 5u : (i2 == 8 ? 6u : 7u));
    *code = (__builtin_signbit(q) ? 8u : 0u) | e;
  }
  return f16r(f16r(q) * S);
}

}  // namespace iwq

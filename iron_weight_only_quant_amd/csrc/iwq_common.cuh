// iwq_common.cuh — device-side building blocks for the gfx950 min-max quantizer.
//
// Numerics contract (SURVEY.md §7 "Hard parts", §8a): the reference evaluates
//   quant_funcs.py:16-38  /  quant_linear.py:909-947
// as a chain of ATen ops on 16-bit tensors; each op computes in fp32 and rounds RNE to the
// storage dtype.  Every function below that is marked "R()" reproduces one such rounding.
// Compiled with -ffp-contract=off and IEEE fp32 division (no fast-math).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace iwq {

enum : int { DT_F16 = 0, DT_BF16 = 1, DT_F32 = 2 };

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;

// ---------------------------------------------------------------------------------------------
// storage formats
// ---------------------------------------------------------------------------------------------
template <int DT>
struct Fmt;

template <>
struct Fmt<DT_F16> {
  static constexpr int BYTES = 2;
  static constexpr int NB = 16;  // bits of the storage word
  __device__ __forceinline__ static float to_f(uint32_t b) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)b);
  }
  __device__ __forceinline__ static uint32_t from_f(float x) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)x);  // v_cvt_f16_f32, RNE
  }
  __device__ __forceinline__ static float R(float x) { return (float)(_Float16)x; }
};

template <>
struct Fmt<DT_BF16> {
  static constexpr int BYTES = 2;
  static constexpr int NB = 16;
  __device__ __forceinline__ static float to_f(uint32_t b) { return __builtin_bit_cast(float, (uint32_t)(b << 16)); }
  __device__ __forceinline__ static uint32_t from_f(float x) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x);  // v_cvt_pk_bf16_f32, RNE, NaN-preserving
  }
  __device__ __forceinline__ static float R(float x) { return to_f(from_f(x)); }
};

template <>
struct Fmt<DT_F32> {
  static constexpr int BYTES = 4;
  static constexpr int NB = 32;
  __device__ __forceinline__ static float to_f(uint32_t b) { return __builtin_bit_cast(float, b); }
  __device__ __forceinline__ static uint32_t from_f(float x) { return __builtin_bit_cast(uint32_t, x); }
  __device__ __forceinline__ static float R(float x) { return x; }
};

// ---------------------------------------------------------------------------------------------
// order keys: sign-magnitude bits -> two's-complement order.  An involution; -0 < +0; +NaN sorts
// above +inf and -NaN below -inf, so a NaN anywhere in a group always reaches min or max and
// poisons the range exactly like ATen's NaN-propagating amax/amin (quant_funcs.py:17-18).
// ---------------------------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ int32_t key_of(uint32_t b) {
  if constexpr (Fmt<DT>::NB == 16) {
    int32_t s = (int32_t)(int16_t)(uint16_t)b;
    return s ^ ((s >> 31) & 0x7FFF);
  } else {
    int32_t s = (int32_t)b;
    return s ^ ((s >> 31) & 0x7FFFFFFF);
  }
}
template <int DT>
__device__ __forceinline__ uint32_t bits_of_key(int32_t k) {
  if constexpr (Fmt<DT>::NB == 16) {
    int32_t s = k ^ ((k >> 31) & 0x7FFF);
    return (uint32_t)(uint16_t)s;
  } else {
    return (uint32_t)(k ^ ((k >> 31) & 0x7FFFFFFF));
  }
}
// magnitude key for the symmetric (abs().amax(), quant_funcs.py:24) path; NaN > inf.
template <int DT>
__device__ __forceinline__ int32_t mag_key(uint32_t b) {
  if constexpr (Fmt<DT>::NB == 16) return (int32_t)(b & 0x7FFFu);
  else return (int32_t)(b & 0x7FFFFFFFu);
}

// torch.clamp: NaN propagates, in-range values (incl. -0) are returned unchanged.
__device__ __forceinline__ float clamp_nan(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

// ---------------------------------------------------------------------------------------------
// per-group parameters
// ---------------------------------------------------------------------------------------------
struct GroupParams {
  float s;    // scale (storage-rounded)
  float rs;   // RN(1/s) (fp32), for the reciprocal-corrected division
  float z;    // zero point (storage-rounded; 0 for symmetric)
  float lo;   // min_int (storage-rounded)
  float hi;   // max_int (storage-rounded)
  bool fast;  // the fast elementwise path is exact for this group (see quant_fast)
};

// zero_point=True branch: quant_funcs.py:17-22 == quant_linear.py:917-922
template <int DT>
__device__ __forceinline__ GroupParams params_asym(float mn, float mx, int n_bits) {
  using F = Fmt<DT>;
  GroupParams p;
  const float max_int = (float)((1u << n_bits) - 1u);
  const float eps = F::R(1e-5f);
  float rng = F::R(mx - mn);                  // max_val - min_val
  rng = rng < eps ? eps : rng;                // .clamp(min=1e-5)   (NaN kept)
  p.s = F::R(rng / max_int);                  // / max_int
  float zq = F::R(mn / p.s);                  // min_val / scales
  p.hi = F::R(max_int);
  p.lo = 0.0f;
  p.z = clamp_nan(-__builtin_rintf(zq), 0.0f, p.hi);   // (-round(.)).clamp_(0, max_int); -0 kept
  p.rs = 1.0f / p.s;
  p.fast = (DT == DT_F16) && (n_bits <= 10) && (p.s > 0.0f) && (p.s <= 3.0e38f) &&
           (p.z == p.z) && (p.z <= 65504.0f);
  return p;
}

// zero_point=False branch: quant_funcs.py:24-29 == quant_linear.py:910-915
template <int DT>
__device__ __forceinline__ GroupParams params_sym(float amax, int n_bits) {
  using F = Fmt<DT>;
  GroupParams p;
  const float max_int = (float)((1u << (n_bits - 1)) - 1u);
  const float eps = F::R(1e-5f);
  float m = amax < eps ? eps : amax;          // .clamp(min=1e-5)
  p.s = F::R(m / max_int);                    // max_val / max_int
  p.z = 0.0f;
  p.hi = F::R(max_int);
  p.lo = F::R(-(float)(1u << (n_bits - 1)));
  p.rs = 1.0f / p.s;
  p.fast = (DT == DT_F16) && (n_bits <= 10) && (p.s > 0.0f) && (p.s <= 3.0e38f);
  return p;
}

// ---------------------------------------------------------------------------------------------
// elementwise quantize->dequantize
// ---------------------------------------------------------------------------------------------
// Exact path: literally the reference op chain, each op rounded to the storage dtype.
// Handles NaN/inf/zero scales exactly as ATen does.  c_out receives the clamped integer value.
template <int DT, bool SYM>
__device__ __forceinline__ float quant_exact(float w, const GroupParams& p, float& c_out) {
  using F = Fmt<DT>;
  float t = F::R(w / p.s);               // tensor / scales
  float r = __builtin_rintf(t);          // torch.round (half to even)
  float a = F::R(r + p.z);               // + zeros   (symmetric: python 0 -> normalises -0 to +0)
  float c = clamp_nan(a, p.lo, p.hi);    // clamp(min_int, max_int)
  c_out = c;
  if constexpr (SYM) {
    return F::R(c * p.s);                // (q - 0) * scales
  } else {
    float d = F::R(c - p.z);             // - zeros
    return F::R(d * p.s);                // * scales
  }
}

// Fast path (fp16 storage, finite positive scale, finite zero point, n_bits <= 10):
//  * w/s via Markstein's reciprocal correction: q0 = RN(w*rs), e = fma(-q0, s, w) (exact),
//    q1 = RN(e*rs + q0) == RN32(w/s) for rs = RN32(1/s).  Then RN16 of it equals RN16 of the IEEE
//    fp32 quotient.  Verified exhaustively over all fp16 (w, s) pairs by iwq_selftest_division.
//  * r + z needs no rounding: integers below 2^11 are exact in fp16 and anything larger is
//    clamped to max_int <= 1023 either way; the clamp is a single v_med3_f32 (no NaN can occur).
//  * (c - z) is exact (small integers).
template <bool SYM>
__device__ __forceinline__ float quant_fast_f16(float w, const GroupParams& p, float& c_out) {
  float q0 = w * p.rs;
  float e = __builtin_fmaf(-q0, p.s, w);
  float q1 = __builtin_fmaf(e, p.rs, q0);
  float t = (float)(_Float16)q1;
  float r = __builtin_rintf(t);
  float a = r + p.z;                       // symmetric: z == +0 -> normalises -0 like "+ 0"
  float c = __builtin_amdgcn_fmed3f(a, p.lo, p.hi);
  c_out = c;
  if constexpr (SYM) {
    return c * p.s;                        // caller rounds to fp16 on store
  } else {
    return (c - p.z) * p.s;
  }
}

// ---------------------------------------------------------------------------------------------
// cross-lane reductions (wave64)
// ---------------------------------------------------------------------------------------------
// DPP controls (gfx9): quad_perm [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E, row_half_mirror 0x141,
// row_mirror 0x140.  Combined in this order they all-reduce over aligned groups of 2/4/8/16 lanes.
template <int CTRL>
__device__ __forceinline__ int32_t dpp(int32_t x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}

// All-reduce min and max over aligned groups of N lanes (N power of two, 1..64).
template <int N>
__device__ __forceinline__ void group_minmax(int32_t& mn, int32_t& mx) {
  if constexpr (N >= 2) { mn = min(mn, dpp<0xB1>(mn)); mx = max(mx, dpp<0xB1>(mx)); }
  if constexpr (N >= 4) { mn = min(mn, dpp<0x4E>(mn)); mx = max(mx, dpp<0x4E>(mx)); }
  if constexpr (N >= 8) { mn = min(mn, dpp<0x141>(mn)); mx = max(mx, dpp<0x141>(mx)); }
  if constexpr (N >= 16) { mn = min(mn, dpp<0x140>(mn)); mx = max(mx, dpp<0x140>(mx)); }
  if constexpr (N >= 32) { mn = min(mn, __shfl_xor(mn, 16)); mx = max(mx, __shfl_xor(mx, 16)); }
  if constexpr (N >= 64) { mn = min(mn, __shfl_xor(mn, 32)); mx = max(mx, __shfl_xor(mx, 32)); }
}
template <int N>
__device__ __forceinline__ void group_max(int32_t& mx) {
  if constexpr (N >= 2) mx = max(mx, dpp<0xB1>(mx));
  if constexpr (N >= 4) mx = max(mx, dpp<0x4E>(mx));
  if constexpr (N >= 8) mx = max(mx, dpp<0x141>(mx));
  if constexpr (N >= 16) mx = max(mx, dpp<0x140>(mx));
  if constexpr (N >= 32) mx = max(mx, __shfl_xor(mx, 16));
  if constexpr (N >= 64) mx = max(mx, __shfl_xor(mx, 32));
}

// ---------------------------------------------------------------------------------------------
// 8-element vectors: 16 B (16-bit dtypes) or 32 B (fp32) per lane
// ---------------------------------------------------------------------------------------------
template <int DT>
struct Vec8 {
  static constexpr int WORDS = Fmt<DT>::BYTES * 8 / 4;  // 4 or 8 dwords
  uint32_t u[WORDS];
  __device__ __forceinline__ uint32_t get(int i) const {
    if constexpr (Fmt<DT>::NB == 16) return (u[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
    else return u[i];
  }
  __device__ __forceinline__ void set(int i, uint32_t b) {
    if constexpr (Fmt<DT>::NB == 16) {
      if (i & 1) u[i >> 1] = (u[i >> 1] & 0xFFFFu) | (b << 16);
      else u[i >> 1] = (u[i >> 1] & 0xFFFF0000u) | (b & 0xFFFFu);
    } else {
      u[i] = b;
    }
  }
  __device__ __forceinline__ void load(const void* p) {
    const u32x4* q = reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int k = 0; k < WORDS / 4; ++k) {
      u32x4 v = __builtin_nontemporal_load(q + k);
      u[4 * k + 0] = v.x; u[4 * k + 1] = v.y; u[4 * k + 2] = v.z; u[4 * k + 3] = v.w;
    }
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < WORDS; ++k) u[k] = 0;
  }
  __device__ __forceinline__ void store(void* p) const {
    u32x4* q = reinterpret_cast<u32x4*>(p);
#pragma unroll
    for (int k = 0; k < WORDS / 4; ++k) {
      u32x4 v = {u[4 * k + 0], u[4 * k + 1], u[4 * k + 2], u[4 * k + 3]};
      __builtin_nontemporal_store(v, q + k);
    }
  }
};

// pack 8 codes (0..255) of consecutive elements; CODES == 4: 4 B (low nibble = even element),
// CODES == 8: 8 B.
template <int CODES>
__device__ __forceinline__ void store_codes8(uint8_t* base, int64_t elem0, const uint32_t (&c)[8]) {
  if constexpr (CODES == 4) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v |= (c[i] & 0xFu) << (4 * i);
    *reinterpret_cast<uint32_t*>(base + elem0 / 2) = v;
  } else if constexpr (CODES == 8) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) lo |= (c[i] & 0xFFu) << (8 * i);
#pragma unroll
    for (int i = 0; i < 4; ++i) hi |= (c[4 + i] & 0xFFu) << (8 * i);
    *reinterpret_cast<uint2*>(base + elem0) = make_uint2(lo, hi);
  }
}

}  // namespace iwq

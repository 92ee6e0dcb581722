// iwq_common.cuh — device-side building blocks for the gfx950 min-max quantizer.
//
// Numerics contract (SURVEY.md §7 "Hard parts", §8a): the reference evaluates
//   quant_funcs.py:16-38  /  quant_linear.py:909-947
// as a chain of ATen ops on 16-bit tensors; each op computes in fp32 and rounds RNE to the
// storage dtype.  The *exact* path below replays that chain literally (one rounding per op).
// The *fast* path (fp16, finite groups) computes the same bits with fewer instructions; each
// shortcut is justified next to it and the two non-obvious ones (reciprocal, corrected
// division) are checked exhaustively over all fp16 operands by iwq_selftest_division.
// Compiled with -ffp-contract=off and IEEE fp32 division (no fast-math).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// IWQ_AB=1 (build.py --ab / IWQ_AB=1 in the environment -> _lib/libiwq_ab.so): also compile the kernel
// variants kept for A/B timing and their bit-identity tests (flags bits 16..23 that no default path
// takes).  The product library (IWQ_AB=0) carries the defaults plus the forms the tests pin, and
// answers any other variant with IWQ_ERR_ARG.
#ifndef IWQ_AB
#define IWQ_AB 0
#endif

namespace iwq {

// last HIP error of this host thread, shared by every translation unit (iwq_last_hip_error)
int& last_hip_error();

// Zeroing without hipMemsetAsync (round 5): a memset captured into a hipGraph comes back right on the
// graph's FIRST replay only -- from the second on it leaves ~60 % of the bytes non-zero (every size
// tried, 16 B to 8 KiB; tools/diag_graph_memset.py, profiles/r05_diag_graph_memset.log; eager memsets
// are fine).  Every zeroing a caller may capture therefore goes through this kernel: 16-B vector
// stores for the aligned body, byte stores for the head and tail.
namespace {
__global__ __launch_bounds__(256) void k_zero_bytes(unsigned char* p, uint64_t n, uint64_t head, uint64_t body16) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * 256;
  if (t < head) p[t] = 0;
  uint4* b = reinterpret_cast<uint4*>(p + head);
  for (uint64_t i = t; i < body16; i += nt) b[i] = make_uint4(0u, 0u, 0u, 0u);
  const uint64_t tail0 = head + body16 * 16;
  if (tail0 + t < n) p[tail0 + t] = 0;  // < 16 tail bytes
}

// in the same unnamed namespace as its kernel: each translation unit launches its own k_zero_bytes
// (an inline function with external linkage would be one definition per TU of a different kernel)
hipError_t zero_async(void* p, uint64_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  unsigned char* c = static_cast<unsigned char*>(p);
  uint64_t head = (16 - (reinterpret_cast<uintptr_t>(c) & 15)) & 15;
  if (head > n) head = n;
  const uint64_t body16 = (n - head) / 16;
  uint64_t blocks = (body16 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_zero_bytes, dim3((unsigned)blocks), dim3(256), 0, st, c, n, head, body16);
  return hipGetLastError();
}
}  // namespace


enum : int { DT_F16 = 0, DT_BF16 = 1, DT_F32 = 2 };

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

constexpr int WAVE = 64;

// Global-address-space views: plain `T*` kernel pointers are generic (flat) to the compiler, and
// flat loads are counted on both vmcnt and lgkmcnt, which forces full drains between them.
#define IWQ_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ IWQ_GLOBAL T* gp(void* p) { return (IWQ_GLOBAL T*)(p); }
template <typename T>
__device__ __forceinline__ const IWQ_GLOBAL T* gp(const void* p) { return (const IWQ_GLOBAL T*)(p); }

// Value barrier: forces x to exist as an fp32 register value.  Stops LLVM from folding
// "fptrunc(fma(..))" into one v_fma_mixlo_f16 (a single rounding straight to fp16, which is NOT
// RN16(RN32(.))) and "fptrunc(fdiv(fpext, fpext))" into an fp16 division.
__device__ __forceinline__ float opaque(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

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
  __device__ __forceinline__ static float R(float x) { return (float)(_Float16)opaque(x); }
};

template <>
struct Fmt<DT_BF16> {
  static constexpr int BYTES = 2;
  static constexpr int NB = 16;
  __device__ __forceinline__ static float to_f(uint32_t b) { return __builtin_bit_cast(float, (uint32_t)(b << 16)); }
  __device__ __forceinline__ static uint32_t from_f(float x) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x);  // v_cvt_pk_bf16_f32, RNE, NaN-preserving
  }
  __device__ __forceinline__ static float R(float x) { return to_f(from_f(opaque(x))); }
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
// fast reciprocal / division for operands that are fp16 values (held in fp32)
// ---------------------------------------------------------------------------------------------
// RN32(1/s) for every positive finite fp16 s: v_rcp_f32 (<= 1 ulp) + one Newton step.
// (exhaustively checked, iwq_selftest_division counter 2)
__device__ __forceinline__ float rcp_f16val(float s) {
  float r = __builtin_amdgcn_rcpf(s);
  float e = __builtin_fmaf(-s, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}
// RN32(w/s) given rs = RN32(1/s) (Markstein: q0 = RN(w*rs), the residual w - q0*s is exact in one
// fma, q1 = RN(q0 + e*rs) is the correctly rounded quotient).  Exhaustive over all finite fp16 w
// and all positive fp16 s: iwq_selftest_division counters 0/1.
__device__ __forceinline__ float div_f16vals(float w, float s, float rs) {
  float q0 = w * rs;
  float e = __builtin_fmaf(-q0, s, w);
  return opaque(__builtin_fmaf(e, rs, q0));
}
// Same, with IEEE's sign for a zero quotient (-0 / s = -0; the corrected form yields +0 there).
// Needed where the sign of a zero is stored (the zero point of min_val = -0 groups); the
// elementwise path does not need it (see quant2_fast).
__device__ __forceinline__ float div_f16vals_signed(float w, float s, float rs) {
  const float q0 = w * rs;
  const float e = __builtin_fmaf(-q0, s, w);
  return opaque(__builtin_copysignf(__builtin_fmaf(e, rs, q0), q0));
}

// ---------------------------------------------------------------------------------------------
// per-group parameters
// ---------------------------------------------------------------------------------------------
struct GroupParams {
  float s;    // scale (storage-rounded)
  float rs;   // RN(1/s) (fp32), for the corrected division
  float z;    // zero point (storage-rounded; +0 for symmetric)
  float lo;   // min_int (storage-rounded)
  float hi;   // max_int (storage-rounded)
  bool fast;  // the fast elementwise path is exact for this group
};

// zero_point=True branch, literal op chain: quant_funcs.py:17-22 == quant_linear.py:917-922
template <int DT>
__device__ __forceinline__ GroupParams params_asym_exact(float mn, float mx, int n_bits) {
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
  p.fast = false;
  return p;
}

// zero_point=False branch, literal op chain: quant_funcs.py:24-29 == quant_linear.py:910-915
template <int DT>
__device__ __forceinline__ GroupParams params_sym_exact(float amax, int n_bits) {
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
  p.fast = false;
  return p;
}

// Same values for fp16 groups with a finite range and a nonzero scale, n_bits <= 10, without
// IEEE divisions: rng/max_int and mn/s are quotients of fp16 values -> div_f16vals.
// rmax = RN32(1/max_int) (per-kernel constant).  Otherwise falls back to the exact chain.
template <int DT>
__device__ __forceinline__ GroupParams params_asym(float mn, float mx, int n_bits, float rmax) {
  if constexpr (DT == DT_F16) {
    if (n_bits <= 10) {
      GroupParams p;
      const float max_int = (float)((1u << n_bits) - 1u);
      const float eps = (float)(_Float16)1e-5f;
      float rng = (float)(_Float16)(mx - mn);  // exact-then-round == ATen's fp16 subtraction
      rng = rng < eps ? eps : rng;
      p.s = (float)(_Float16)div_f16vals(rng, max_int, rmax);
      p.rs = rcp_f16val(p.s);
      p.hi = max_int;                          // exact in fp16 for n_bits <= 10
      p.lo = 0.0f;
      float zq = (float)(_Float16)div_f16vals_signed(mn, p.s, p.rs);
      p.z = clamp_nan(-__builtin_rintf(zq), 0.0f, p.hi);
      // rng finite (so mn, mx finite) and s > 0: every shortcut above is exact; z is finite
      // because the clamp maps +-inf into [0, max_int].
      p.fast = (rng <= 65504.0f) && (p.s > 0.0f);
      if (p.fast) return p;
    }
  }
  return params_asym_exact<DT>(mn, mx, n_bits);
}

template <int DT>
__device__ __forceinline__ GroupParams params_sym(float amax, int n_bits, float rmax) {
  if constexpr (DT == DT_F16) {
    if (n_bits <= 10) {
      GroupParams p;
      const float max_int = (float)((1u << (n_bits - 1)) - 1u);
      const float eps = (float)(_Float16)1e-5f;
      float m = amax < eps ? eps : amax;
      p.s = (float)(_Float16)div_f16vals(m, max_int, rmax);
      p.rs = rcp_f16val(p.s);
      p.z = 0.0f;
      p.hi = max_int;
      p.lo = -(float)(1u << (n_bits - 1));
      p.fast = (m <= 65504.0f) && (p.s > 0.0f);
      if (p.fast) return p;
    }
  }
  return params_sym_exact<DT>(amax, n_bits);
}

// reciprocal of max_int used by the fast parameter path (IEEE division, once per thread)
__device__ __forceinline__ float rmax_for(int n_bits, bool sym) {
  const float max_int = sym ? (float)((1u << (n_bits - 1)) - 1u) : (float)((1u << n_bits) - 1u);
  return 1.0f / max_int;
}

// ---------------------------------------------------------------------------------------------
// elementwise quantize->dequantize, exact path: literally the reference op chain, each op rounded
// to the storage dtype.  Handles NaN/inf/zero scales exactly as ATen does.
// ---------------------------------------------------------------------------------------------
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

// Per-element form of the fast path (used where neighbouring elements belong to different groups,
// e.g. quant_dim = 1).  Same arguments as quant2_fast; r = rint(t) exactly here.
template <int DT, bool SYM>
__device__ __forceinline__ float quant_exact_or_fast(float w, const GroupParams& p, float& c_out) {
  if constexpr (DT == DT_F16) {
    if (p.fast) {
      const float t = (float)(_Float16)div_f16vals(w, p.s, p.rs);
      const float r = __builtin_rintf(t);
      const float a = r + p.z;  // exact below 2^11; larger values clamp to the same bound
      const float c = __builtin_amdgcn_fmed3f(a, p.lo, p.hi);
      c_out = c;
      return SYM ? c * p.s : (c - p.z) * p.s;  // exact fp32 product; rounded once on store
    }
  }
  return quant_exact<DT, SYM>(w, p, c_out);
}

// ---------------------------------------------------------------------------------------------
// elementwise fast path: fp16 pairs in packed math (p.fast groups only)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ uint32_t as_u32(h2 h) { return __builtin_bit_cast(uint32_t, h); }
__device__ __forceinline__ h2 pk_max(h2 a, h2 b) {
  h2 r;
  asm("v_pk_max_f16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ h2 pk_min(h2 a, h2 b) {
  h2 r;
  asm("v_pk_min_f16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

struct FastPk {  // group constants broadcast to both halves
  h2 z, lo, hi, s, codeoff;  // codeoff = code offset + 1024 (see codes below)
};
template <bool SYM>
__device__ __forceinline__ FastPk fast_pk(const GroupParams& p, int n_bits) {
  FastPk k;
  k.z = h2{(_Float16)p.z, (_Float16)p.z};
  k.lo = h2{(_Float16)p.lo, (_Float16)p.lo};
  k.hi = h2{(_Float16)p.hi, (_Float16)p.hi};
  k.s = h2{(_Float16)p.s, (_Float16)p.s};
  const float off = (SYM ? (float)(1u << (n_bits - 1)) : 0.0f) + 1024.0f;
  k.codeoff = h2{(_Float16)off, (_Float16)off};
  return k;
}

// Two fp16 weights -> two dequantized fp16 (bit pattern) + two clamped integer values c (fp16).
//  t = RN16(w/s)           corrected division in fp32 + v_cvt_pk_f16_f32 (RNE)
//  r = rint(t)             (t + m) - m with m = copysign(1024, t): RNE to an integer for |t| < 1024;
//                          for |t| >= 1024 it stays >= 1024 in magnitude with t's sign, and such
//                          values clamp to the same bound as rint(t) (|bounds| <= 1023).  r is never
//                          -0, which matches "round(.) + zeros" (-0 + z) for every z the clamp can
//                          see (outputs and codes identical).
//  a = r + z, c = clamp    v_pk_add_f16, v_pk_max_f16/v_pk_min_f16 (no NaN can occur here)
//  y = (c - z) * s         exact difference, one correctly rounded fp16 product == RN16(RN32(.))
template <bool SYM>
__device__ __forceinline__ uint32_t quant2_fast(uint32_t wpair, const GroupParams& p, const FastPk& k,
                                                uint32_t& cpair) {
  const h2 w = as_h2(wpair);
  const float q0 = div_f16vals((float)w.x, p.s, p.rs);
  const float q1 = div_f16vals((float)w.y, p.s, p.rs);
  const h2 t = __builtin_convertvector((f2){q0, q1}, h2);
  const h2 m = as_h2((as_u32(t) & 0x80008000u) | 0x64006400u);
  const h2 r = (t + m) - m;
  const h2 c = pk_min(pk_max(r + k.z, k.lo), k.hi);
  cpair = as_u32(c);
  if constexpr (SYM) return as_u32(c * k.s);
  else return as_u32((c - k.z) * k.s);
}

// integer codes of two clamped values: c + off + 1024 lies in [1024, 2048) where fp16 spacing is 1,
// so its low 10 mantissa bits ARE the code.
__device__ __forceinline__ uint32_t codes2_fast(uint32_t cpair, const FastPk& k) {
  return as_u32(as_h2(cpair) + k.codeoff) & 0x03FF03FFu;
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
  template <bool NT = true>
  __device__ __forceinline__ void load(const void* p) {
    const IWQ_GLOBAL u32x4* q = gp<u32x4>(p);
#pragma unroll
    for (int k = 0; k < WORDS / 4; ++k) {
      u32x4 v;
      if constexpr (NT) v = __builtin_nontemporal_load(q + k);
      else v = q[k];
      u[4 * k + 0] = v.x; u[4 * k + 1] = v.y; u[4 * k + 2] = v.z; u[4 * k + 3] = v.w;
    }
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < WORDS; ++k) u[k] = 0;
  }
  template <bool NT = true>
  __device__ __forceinline__ void store(void* p) const {
    IWQ_GLOBAL u32x4* q = gp<u32x4>(p);
#pragma unroll
    for (int k = 0; k < WORDS / 4; ++k) {
      u32x4 v = {u[4 * k + 0], u[4 * k + 1], u[4 * k + 2], u[4 * k + 3]};
      if constexpr (NT) __builtin_nontemporal_store(v, q + k);
      else q[k] = v;
    }
  }
};

// min/max order keys of 8 elements (16-bit dtypes in packed int16 math)
template <int DT, bool SYM>
__device__ __forceinline__ void minmax8(const Vec8<DT>& v, int32_t& mn, int32_t& mx) {
  if constexpr (Fmt<DT>::NB == 16) {
    if constexpr (SYM) {
      u16x2 m[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) m[i] = __builtin_bit_cast(u16x2, v.u[i] & 0x7FFF7FFFu);
      u16x2 a = __builtin_elementwise_max(__builtin_elementwise_max(m[0], m[1]), __builtin_elementwise_max(m[2], m[3]));
      mx = (int32_t)max(a.x, a.y);
      mn = 0;
    } else {
      s16x2 k[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s16x2 x = __builtin_bit_cast(s16x2, v.u[i]);
        k[i] = x ^ ((x >> (short)15) & (short)0x7FFF);
      }
      s16x2 a = __builtin_elementwise_min(__builtin_elementwise_min(k[0], k[1]), __builtin_elementwise_min(k[2], k[3]));
      s16x2 b = __builtin_elementwise_max(__builtin_elementwise_max(k[0], k[1]), __builtin_elementwise_max(k[2], k[3]));
      mn = min((int32_t)a.x, (int32_t)a.y);
      mx = max((int32_t)b.x, (int32_t)b.y);
    }
  } else {
    if constexpr (SYM) {
      mn = 0;
      mx = mag_key<DT>(v.get(0));
#pragma unroll
      for (int i = 1; i < 8; ++i) mx = max(mx, mag_key<DT>(v.get(i)));
    } else {
      mn = mx = key_of<DT>(v.get(0));
#pragma unroll
      for (int i = 1; i < 8; ++i) {
        int32_t kk = key_of<DT>(v.get(i));
        mn = min(mn, kk);
        mx = max(mx, kk);
      }
    }
  }
}

// store one storage-dtype value (scales / zeros)
template <int DT>
__device__ __forceinline__ void store_param(void* base, int64_t idx, float v) {
  if constexpr (Fmt<DT>::NB == 16) gp<uint16_t>(base)[idx] = (uint16_t)Fmt<DT>::from_f(v);
  else gp<uint32_t>(base)[idx] = Fmt<DT>::from_f(v);
}

template <int DT, bool SYM>
__device__ __forceinline__ GroupParams params_from_keys(int32_t mn, int32_t mx, int n_bits, float rmax) {
  using F = Fmt<DT>;
  if constexpr (SYM) return params_sym<DT>(F::to_f(bits_of_key<DT>(mx)), n_bits, rmax);
  else return params_asym<DT>(F::to_f(bits_of_key<DT>(mn)), F::to_f(bits_of_key<DT>(mx)), n_bits, rmax);
}

// Quantize 8 elements with one group's parameters.  codes[j] (j < 4) receives the integer codes of
// elements 2j, 2j+1 in its two 16-bit halves.  Returns true if a dequantized value is NaN.
template <int DT, bool SYM>
__device__ __forceinline__ bool quant8(const Vec8<DT>& v, const GroupParams& p, int n_bits, Vec8<DT>& o,
                                       uint32_t (&codes)[4]) {
  if constexpr (DT == DT_F16) {
    if (p.fast) {
      const FastPk k = fast_pk<SYM>(p, n_bits);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t cp;
        o.u[j] = quant2_fast<SYM>(v.u[j], p, k, cp);
        codes[j] = codes2_fast(cp, k);
      }
      return false;
    }
  }
  using F = Fmt<DT>;
  bool any_nan = false;
  const uint32_t off = SYM ? (1u << (n_bits - 1)) : 0u;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float cf;
    const float y = quant_exact<DT, SYM>(F::to_f(v.get(i)), p, cf);
    any_nan |= (y != y);
    o.set(i, F::from_f(y));
    const uint32_t c = (cf == cf) ? ((uint32_t)(int32_t)cf + off) & 0xFFFFu : 0u;
    if (i & 1) codes[i >> 1] |= c << 16;
    else codes[i >> 1] = c;
  }
  return any_nan;
}

// ---------------------------------------------------------------------------------------------
// biased fast path (fp16, n_bits <= 9, p.fast groups): 11 VALU ops per element pair
// ---------------------------------------------------------------------------------------------
// With B = 1536:  u = RN16(t + B) is rint(t) + B exactly for |t| < 512 (u in [1024, 2048), where
// fp16 spacing is 1; B is even, so RNE ties go to the same integer as torch.round's); and
// c - z = clamp(rint(t) + z, lo, hi) - z = clamp(rint(t), lo - z, hi - z)  (integers, exact), so
//   y = (clamp(u, B + lo - z, B + hi - z) - B) * s
// For n_bits <= 9 both bounds lie in [1025, 2047]: a t with |t| >= 512 gives a u outside
// [1024, 2048) that clamps to the same bound as rint(t) would.  The code is
// c + off = u_clamped + (z + off - B) (an integer in [0, 2^b), exact), read from the mantissa of
// u_clamped + (z + off - B + 1024) in [1024, 2048).
// The division w / s is the corrected (Markstein) quotient of div_f16vals, two lanes per
// v_pk_mul_f32 / v_pk_fma_f32 (scalar operands broadcast by op_sel_hi).
constexpr float BIAS = 1536.0f;

__device__ __forceinline__ f2 opaque2(f2 x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ f2 pk_div_f16vals(f2 w, float rs1, float s1) {
  const f2 rs = {rs1, rs1}, s = {s1, s1};
  const f2 q0 = w * rs;
  const f2 e = __builtin_elementwise_fma(-q0, s, w);
  return opaque2(__builtin_elementwise_fma(e, rs, q0));
}
// both halves clamped to [bounds.lo, bounds.hi]
__device__ __forceinline__ h2 pk_clamp_bc(h2 u, uint32_t bounds) {
  h2 r;
  asm("v_pk_max_f16 %0, %1, %2 op_sel_hi:[1,0]\n\t"
      "v_pk_min_f16 %0, %0, %2 op_sel:[0,1]"
      : "=&v"(r) : "v"(u), "v"(bounds));
  return r;
}
// d * (s_lo, s_lo)
__device__ __forceinline__ h2 pk_mul_bc_lo(h2 d, uint32_t s) {
  h2 r;
  asm("v_pk_mul_f16 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(d), "v"(s));
  return r;
}

// Per-group words of the biased path, built once per group by the lane that owns its parameters.
struct BiasedWords {
  uint32_t bounds;  // fp16 (B + lo - z) | (B + hi - z) << 16
  uint32_t sz;      // fp16 s | z << 16 (the stored scale / zero bits)
  uint32_t kc;      // fp16 (z + off - B + 1024) in both halves (codes)
  // RN(1/s) and s in fp32.  Kept as two scalars, never an f2: ROCm 7.2's LLVM merged the DPP
  // broadcasts of the two halves of an f2 into ONE (both lanes got .x) -- a silent miscompile.
  float rs, s;
};
template <bool SYM>
__device__ __forceinline__ BiasedWords biased_words(const GroupParams& p, int n_bits) {
  BiasedWords b;
  const uint32_t lo = Fmt<DT_F16>::from_f(BIAS + p.lo - p.z), hi = Fmt<DT_F16>::from_f(BIAS + p.hi - p.z);
  b.bounds = lo | (hi << 16);
  b.sz = Fmt<DT_F16>::from_f(p.s) | (Fmt<DT_F16>::from_f(p.z) << 16);
  const float off = SYM ? (float)(1u << (n_bits - 1)) : 0.0f;
  const uint32_t k = Fmt<DT_F16>::from_f(p.z + off - BIAS + 1024.0f);
  b.kc = k | (k << 16);
  b.rs = p.rs;
  b.s = p.s;
  return b;
}

// Two fp16 weights -> two dequantized fp16 (bits); cpair receives the codes (CODES only).
template <int CODES>
__device__ __forceinline__ uint32_t quant2_biased(uint32_t wpair, const BiasedWords& b, uint32_t& cpair) {
  const f2 w = __builtin_convertvector(as_h2(wpair), f2);
  const h2 t = __builtin_convertvector(pk_div_f16vals(w, b.rs, b.s), h2);
  const h2 bias = {(_Float16)BIAS, (_Float16)BIAS};
  const h2 u = pk_clamp_bc(t + bias, b.bounds);
  if constexpr (CODES != 0) cpair = as_u32(u + as_h2(b.kc)) & 0x03FF03FFu;
  return as_u32(pk_mul_bc_lo(u - bias, b.sz));
}

// Biased path with DIFFERENT groups in the two halves of a pair (quant_dim = 1: adjacent columns):
// the same 11 operations with per-half operands instead of broadcasts.
struct BiasedPair {
  f2 rs, s;        // per-half RN(1/s), s (fp32)
  uint32_t lo, hi;  // per-half fp16 bounds B + lo - z, B + hi - z
  uint32_t s16;     // per-half fp16 scales
  uint32_t kc;      // per-half fp16 z + off - B + 1024
};
template <bool SYM>
__device__ __forceinline__ BiasedPair biased_pair(const GroupParams& p0, const GroupParams& p1, int n_bits) {
  const BiasedWords a = biased_words<SYM>(p0, n_bits), b = biased_words<SYM>(p1, n_bits);
  BiasedPair r;
  r.rs = f2{a.rs, b.rs};
  r.s = f2{a.s, b.s};
  r.lo = (a.bounds & 0xFFFFu) | (b.bounds << 16);
  r.hi = (a.bounds >> 16) | (b.bounds & 0xFFFF0000u);
  r.s16 = (a.sz & 0xFFFFu) | (b.sz << 16);
  r.kc = (a.kc & 0xFFFFu) | (b.kc << 16);
  return r;
}
template <int CODES>
__device__ __forceinline__ uint32_t quant2_biased_pair(uint32_t wpair, const BiasedPair& b, uint32_t& cpair) {
  const f2 w = __builtin_convertvector(as_h2(wpair), f2);
  const f2 q0 = w * b.rs;
  const f2 e = __builtin_elementwise_fma(-q0, b.s, w);
  const h2 t = __builtin_convertvector(opaque2(__builtin_elementwise_fma(e, b.rs, q0)), h2);
  const h2 bias = {(_Float16)BIAS, (_Float16)BIAS};
  const h2 u = pk_min(pk_max(t + bias, as_h2(b.lo)), as_h2(b.hi));
  if constexpr (CODES != 0) cpair = as_u32(u + as_h2(b.kc)) & 0x03FF03FFu;
  return as_u32((u - bias) * as_h2(b.s16));
}

// Store the codes of 8 consecutive elements (element index elem0, multiple of 8):
// CODES == 4: 4 B (low nibble = even element), CODES == 8: 8 B.
template <int CODES>
__device__ __forceinline__ void store_codes8(uint8_t* base, int64_t elem0, const uint32_t (&c)[4]) {
  if constexpr (CODES == 4) {
    // c[j] holds the codes of elements 2j / 2j + 1 (< 16) in bytes 0 / 2: gather the even elements'
    // bytes and the odd elements' bytes (four byte permutes), then one shift-or interleaves the nibbles
    const uint32_t p01 = __builtin_amdgcn_perm(c[1], c[0], 0x06020400u);  // [e0, e2, e1, e3]
    const uint32_t p23 = __builtin_amdgcn_perm(c[3], c[2], 0x06020400u);  // [e4, e6, e5, e7]
    const uint32_t ev = __builtin_amdgcn_perm(p23, p01, 0x05040100u);     // [e0, e2, e4, e6]
    const uint32_t od = __builtin_amdgcn_perm(p23, p01, 0x07060302u);     // [e1, e3, e5, e7]
    *gp<uint32_t>(base + elem0 / 2) = ev | (od << 4);
  } else if constexpr (CODES == 8) {
    const uint32_t lo = __builtin_amdgcn_perm(c[1], c[0], 0x06040200u);
    const uint32_t hi = __builtin_amdgcn_perm(c[3], c[2], 0x06040200u);
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    *gp<u32x2>(base + elem0) = (u32x2){lo, hi};
  }
}

}  // namespace iwq

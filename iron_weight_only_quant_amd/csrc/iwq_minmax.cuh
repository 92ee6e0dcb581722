// iwq_minmax.cuh -- the min-max quantize kernels (device code + launch helpers shared by the
// host dispatch of iwq_minmax.hip and the batched-table launches of iwq_batched.hip).
// Included by exactly those two translation units; everything lives in an anonymous namespace,
// so each TU instantiates only the templates it launches.
#pragma once
#include "iwq_common.cuh"
#include "iwq_seg.cuh"
#include "../../include/iwq.h"

#include <stdio.h>
#include <string.h>

#include <atomic>

using namespace iwq;
using iwq::seg::SegArgs;
using iwq::seg::SEG_RUN;
using iwq::seg::seg_locate;
using iwq::seg::k_seg_init;
using iwq::seg::k_seg_reduce;

namespace {


#define IWQ_HIP(call)                                   \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) {                             \
      iwq::last_hip_error() = (int)e_;                  \
      return IWQ_ERR_HIP;                               \
    }                                                   \
  } while (0)

constexpr int BLOCK = 256;
constexpr int WAVES_PER_BLOCK = BLOCK / WAVE;
constexpr int UNIT = WAVE * 8;  // elements per wave-instruction span (k_group)

int device_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

// Resident 256-thread blocks per CU for a kernel (occupancy API: VGPRs/LDS; SGPRs are capped at
// 80 on the persistent kernels so the API answer is exact).  Cached per instantiation & device.
template <typename Kern>
int resident_blocks_per_cu(Kern kernel, int* cache) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, BLOCK, 0) != hipSuccess || n <= 0) n = 1;
    cache[dev] = n > 8 ? 8 : n;
  }
  return cache[dev];
}

// wave-uniform 64-bit values / pointers (readfirstlane of both halves)
__device__ __forceinline__ int64_t rfl64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <typename P>
__device__ __forceinline__ P rflp(P p) {
  return (P)(uintptr_t)rfl64((int64_t)(uintptr_t)p);
}

__device__ __forceinline__ void flag_nan(uint32_t* nan_flag, bool any_nan) {
  // one atomic per wave at most
  uint64_t m = __ballot(any_nan);
  if (m != 0 && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(m) && nan_flag) atomicOr(nan_flag, 1u);
}

// =============================================================================================
// k_group: contiguous groups of G in {8..512}
// =============================================================================================
struct GroupTensor {
  const void* w;
  void* out;
  void* codes;
  void* scales;
  void* zeros;
  int64_t numel;
};

struct GroupArgs {
  GroupTensor single;              // used when !BATCHED
  const iwq_batch_entry* entries;  // used when BATCHED
  int32_t n_entries;
  int64_t total_units;
  int n_bits;
  uint32_t* nan_flag;
};

// Resolved target of one 512-element unit.
struct UnitRef {
  GroupTensor t;
  int64_t e0;     // first element of this lane
  bool valid;
};

template <int DT, int G, bool SYM, int CODES, bool NTS = true>
__device__ __forceinline__ bool group_unit_compute(const UnitRef& r, const Vec8<DT>& v, int lane, int n_bits,
                                                   float rmax) {
  using F = Fmt<DT>;
  constexpr int LPG = G / 8;  // lanes per group
  int32_t mn, mx;
  minmax8<DT, SYM>(v, mn, mx);
  if constexpr (SYM) group_max<LPG>(mx);
  else group_minmax<LPG>(mn, mx);
  const GroupParams p = params_from_keys<DT, SYM>(mn, mx, n_bits, rmax);
  Vec8<DT> o;
  uint32_t c[4];
  const bool any_nan = quant8<DT, SYM>(v, p, n_bits, o, c);
  if (r.valid) {
    if (r.t.out) o.template store<NTS>(static_cast<char*>(r.t.out) + r.e0 * F::BYTES);
    if constexpr (CODES != 0) store_codes8<CODES>(static_cast<uint8_t*>(r.t.codes), r.e0, c);
    if ((lane % LPG) == 0) {
      const int64_t gidx = r.e0 / G;
      if (r.t.scales) store_param<DT>(r.t.scales, gidx, p.s);
      if (!SYM && r.t.zeros) store_param<DT>(r.t.zeros, gidx, p.z);
    }
  }
  return r.valid && any_nan;
}

// quad_perm broadcasts read inside the quad, so no source lane is out of range and bound_ctrl changes
// nothing -- but with it set the compiler drops the v_mov 0 it otherwise emits for the `old` operand
// (one VALU per broadcast, 4-5 per unit)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, CTRL, 0xF, 0xF, true);
}
template <int K, int CODES>
__device__ __forceinline__ BiasedWords bcast_words_k(const BiasedWords& w) {
  constexpr int C = K * 0x55;  // quad_perm [K,K,K,K]
  BiasedWords b;
  b.bounds = dpp_u32<C>(w.bounds);
  b.sz = dpp_u32<C>(w.sz);
  b.rs = __builtin_bit_cast(float, dpp_u32<C>(__builtin_bit_cast(uint32_t, w.rs)));
  b.s = __builtin_bit_cast(float, dpp_u32<C>(__builtin_bit_cast(uint32_t, w.s)));
  b.kc = CODES != 0 ? dpp_u32<C>(w.kc) : 0u;
  return b;
}
// the words of unit k of this lane's group (held by lane k of the quad)
template <int CODES>
__device__ __forceinline__ BiasedWords bcast_words(const BiasedWords& w, int k) {
  switch (k) {
    case 0: return bcast_words_k<0, CODES>(w);
    case 1: return bcast_words_k<1, CODES>(w);
    case 2: return bcast_words_k<2, CODES>(w);
    default: return bcast_words_k<3, CODES>(w);
  }
}

// One iteration of NU (<= UNROLL) units of an fp16 tensor with SHARED group parameters: the
// NU x (64 / LPG) groups of the iteration get their parameters from ONE pass of the parameter
// math (lane l computes unit (l % UNROLL) of its own group), instead of one pass per unit in which
// every lane of a group repeats it; each unit then takes its group's words from lane k of the quad
// by DPP broadcast (quads never straddle a group: LPG >= 4).  Elementwise: quant2_biased.
// Returns false (nothing stored) when some group of the iteration is not on the fast path or
// n_bits > 9; the caller then runs the per-unit path.
template <int G, bool SYM, int CODES, int UNROLL, bool NTS>
__device__ __forceinline__ bool iter_shared_f16(const GroupTensor& t, int64_t e0, int32_t nu,
                                                const Vec8<DT_F16> (&v)[UNROLL], int lane, int n_bits,
                                                float rmax) {
  static_assert(G >= 32 && (UNROLL == 1 || UNROLL == 2 || UNROLL == 4), "quad broadcast layout");
  constexpr int LPG = G / 8;
  int32_t mn[UNROLL], mx[UNROLL];
#pragma unroll
  for (int k = 0; k < UNROLL; ++k) {
    minmax8<DT_F16, SYM>(v[k], mn[k], mx[k]);
    if constexpr (SYM) group_max<LPG>(mx[k]);
    else group_minmax<LPG>(mn[k], mx[k]);
  }
  const int kk = lane & (UNROLL - 1);
  int32_t smn = mn[0], smx = mx[0];
#pragma unroll
  for (int k = 1; k < UNROLL; ++k) {
    if (kk == k) { smn = mn[k]; smx = mx[k]; }
  }
  const GroupParams p = params_from_keys<DT_F16, SYM>(smn, smx, n_bits, rmax);
  if (n_bits > 9 || __ballot(kk < nu && !p.fast) != 0) return false;
  const BiasedWords bw = biased_words<SYM>(p, n_bits);
#pragma unroll
  for (int k = 0; k < UNROLL; ++k) {
    if (k < nu) {
      const BiasedWords b = bcast_words<CODES>(bw, k);
      Vec8<DT_F16> o;
      uint32_t c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o.u[j] = quant2_biased<CODES>(v[k].u[j], b, c[j]);
      const int64_t e = e0 + (int64_t)k * UNIT;
      if (e < t.numel) {
        if (t.out) o.template store<NTS>(static_cast<char*>(t.out) + e * 2);
        if constexpr (CODES != 0) store_codes8<CODES>(static_cast<uint8_t*>(t.codes), e, c);
        if ((lane % LPG) == 0) {
          const int64_t gidx = e / G;
          if (t.scales) gp<uint16_t>(t.scales)[gidx] = (uint16_t)b.sz;
          if (!SYM && t.zeros) gp<uint16_t>(t.zeros)[gidx] = (uint16_t)(b.sz >> 16);
        }
      }
    }
  }
  return true;
}

// Persistent launch; wave w owns the contiguous unit range [w*per, (w+1)*per) and walks it in
// iterations of up to UNROLL units that never straddle two tensors, so one iteration has ONE
// (wave-uniform, SGPR-resident) tensor descriptor and the lane offsets of its units differ by
// immediates.  All loads of an iteration are issued before any compute/store (the output may
// alias the input, so the compiler cannot hoist later loads above earlier stores on its own);
// with PF the next iteration's loads are issued before this iteration's compute (register double
// buffering; prefetched units never overlap the ones being stored).
template <bool BATCHED>
struct TensorCursor {
  int32_t cur = 0;
  int64_t begin = 0, next = INT64_MAX;  // unit range [begin, next) of the current tensor
  GroupTensor t;
  __device__ __forceinline__ void init(const GroupArgs& a) {
    t = a.single;
    if constexpr (BATCHED) {
      next = -1;
    }
  }
  // make u (< total) fall inside the current tensor; all values wave-uniform
  __device__ __forceinline__ void seek(const GroupArgs& a, int64_t u) {
    if constexpr (BATCHED) {
      if (u >= next || next < 0) {
        const IWQ_GLOBAL iwq_batch_entry* tab = gp<iwq_batch_entry>(a.entries);
        if (next < 0) {  // first seek: binary search (the last entry whose range starts at or before u)
          int32_t lo = cur, hi = a.n_entries - 1;
          while (lo < hi) {
            const int32_t mid = (lo + hi + 1) >> 1;
            if (tab[mid].unit_begin <= u) lo = mid;
            else hi = mid - 1;
          }
          cur = lo;
        }
        while (cur + 1 < a.n_entries && u >= tab[cur + 1].unit_begin) ++cur;
        cur = __builtin_amdgcn_readfirstlane(cur);
        t.w = rfl_ptr(tab[cur].w);
        t.out = rfl_ptr(tab[cur].out_deq);
        t.codes = rfl_ptr(tab[cur].out_codes);
        t.scales = rfl_ptr(tab[cur].out_scales);
        t.zeros = rfl_ptr(tab[cur].out_zeros);
        t.numel = rfl_i64(tab[cur].rows * tab[cur].cols);
        begin = rfl_i64(tab[cur].unit_begin);
        next = (cur + 1 < a.n_entries) ? rfl_i64(tab[cur + 1].unit_begin) : INT64_MAX;
      }
    }
  }
  __device__ __forceinline__ static int64_t rfl_i64(int64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
  }
  template <typename P>
  __device__ __forceinline__ static P rfl_ptr(P p) {
    return (P)(uintptr_t)rfl_i64((int64_t)(uintptr_t)p);
  }
};

struct Iter {
  GroupTensor t;
  int64_t e0;      // this lane's first element in unit 0 of the iteration
  int32_t n;       // units in this iteration (1..UNROLL), wave-uniform
};

template <int DT, int UNROLL, bool NTL>
__device__ __forceinline__ void load_iter(const Iter& it, Vec8<DT> (&v)[UNROLL]) {
  // unconditional loads (units past it.n and lanes past numel re-read the tensor's first 16 B and
  // are never stored): no exec-masked branches around the loads
  const char* base = static_cast<const char*>(it.t.w);
#pragma unroll
  for (int k = 0; k < UNROLL; ++k) {
    const int64_t e = it.e0 + (int64_t)k * UNIT;
    const bool ok = (k < it.n) && (e < it.t.numel);
    v[k].template load<NTL>(base + (ok ? e : 0) * Fmt<DT>::BYTES);
  }
}

// SGPRs capped at 80: above that the hardware admits 7 (not 8) 256-thread blocks per CU while the
// occupancy API still answers 8 (MI355X_MICROARCH.md "Residency"), and this persistent grid is
// sized for full residency.
// SKEL (roofline probe only, variant 118): the same walk, loads and 16-B stores with the arithmetic
// removed (the input is copied to the output) -- this kernel's own memory stream as a ceiling.
// PHASE (A/B, contiguous walk only): wave w starts its chunk at a wave-dependent iteration (a hash
// of w) and wraps around to the chunk's start, so the waves do not sweep their chunks in lockstep
// (without it every wave's address is congruent to the others' modulo the chunk length at every
// moment).  PFD 2 (A/B): the loads of iteration i + 2 are in flight while iteration i is stored
// (three register images).  RW > 1 (A/B, region walk): the units are cut into nwaves / RW
// contiguous regions, RW consecutive waves share one and take its UNROLL-unit chunks round-robin
// (RW = 1 is the contiguous walk, one region per wave; the grid-stride walk is one region for all) --
// fewer distinct pages in flight at once.
template <int DT, int G, bool SYM, int CODES, bool BATCHED, int UNROLL, bool PF = false, bool NTL = true,
          bool NTS = true, bool SHARED = true, bool GS = false, bool SKEL = false, bool PHASE = false, int PFD = 0,
          int RW = 1>
__device__ __forceinline__ void k_group_body(const GroupArgs& a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * WAVES_PER_BLOCK + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
  const float rmax = rmax_for(a.n_bits, SYM);
  // The walk: contiguous (one chunk [wave*per, +per) per wave) or, with GS, grid-stride chunks of
  // UNROLL units (c*UNROLL for c = wave, wave + nwaves, ...: at any moment the grid works on one
  // contiguous window).  u0 = next unit, cend = end of the current chunk; u0 < cend <=> work left.
  int64_t u0, cend;
  int64_t wrap_lo = 0, wrap_hi = 0;  // PHASE: the chunk's head, walked after its tail
  int64_t rend = 0;                   // RW: end of this wave's region
  // RW: waves per region, at most the grid's (a grid of fewer than RW waves is one region)
  const int64_t rw = RW > 1 && nwaves < RW ? nwaves : RW;
  if constexpr (GS) {
    u0 = wave * UNROLL;
    cend = min(u0 + UNROLL, a.total_units);
  } else if constexpr (RW > 1) {
    const int64_t nreg = nwaves / rw;
    const int64_t r = wave / rw;
    int64_t per = (a.total_units + nreg - 1) / nreg;
    per = (per + UNROLL - 1) / UNROLL * UNROLL;
    const int64_t rbeg = r < nreg ? r * per : a.total_units;
    rend = min(rbeg + per, a.total_units);
    u0 = rbeg + (wave % rw) * UNROLL;
    cend = min(u0 + UNROLL, rend);
  } else {
    int64_t per = (a.total_units + nwaves - 1) / nwaves;
    per = (per + UNROLL - 1) / UNROLL * UNROLL;
    u0 = wave * per;
    cend = min(u0 + per, a.total_units);
    if constexpr (PHASE) {
      if (u0 < cend) {
        const int64_t nit = (cend - u0 + UNROLL - 1) / UNROLL;
        const uint32_t h = (uint32_t)wave * 0x9E3779B1u;
        const int64_t ph = (int64_t)((uint64_t)(h >> 8) % (uint64_t)nit) * UNROLL;
        wrap_lo = u0;
        wrap_hi = u0 + ph;
        u0 += ph;
      }
    }
  }
  bool any_nan = false;
  TensorCursor<BATCHED> cursor;
  cursor.init(a);
  auto advance = [&](int64_t n) {
    u0 += n;
    if constexpr (GS) {
      if (u0 >= cend) {
        u0 += (nwaves - 1) * UNROLL;
        cend = min(u0 + UNROLL, a.total_units);
      }
    }
    if constexpr (RW > 1 && !GS) {
      if (u0 >= cend) {
        u0 += (rw - 1) * UNROLL;
        cend = min(u0 + UNROLL, rend);
      }
    }
    if constexpr (PHASE && !GS) {
      if (u0 >= cend && wrap_hi > wrap_lo) {
        u0 = wrap_lo;
        cend = wrap_hi;
        wrap_hi = wrap_lo;
        cursor.cur = 0;  // the cursor only moves forward: search again from the first entry
        cursor.next = BATCHED ? -1 : INT64_MAX;
      }
    }
  };
  auto plan_iter = [&](int64_t u, Iter& it) {
    cursor.seek(a, u);
    const int64_t lim = min(cend, cursor.next);
    it.t = cursor.t;
    it.n = (int32_t)min((int64_t)UNROLL, lim - u);
    it.e0 = (u - cursor.begin) * UNIT + (int64_t)lane * 8;
  };
  auto compute_iter = [&](const Iter& it, const Vec8<DT> (&v)[UNROLL]) {
    if constexpr (SKEL) {
#pragma unroll
      for (int k = 0; k < UNROLL; ++k) {
        const int64_t e = it.e0 + (int64_t)k * UNIT;
        if (k < it.n && e < it.t.numel && it.t.out)
          v[k].template store<NTS>(static_cast<char*>(it.t.out) + e * Fmt<DT>::BYTES);
      }
      return;
    }
    if constexpr (SHARED && DT == DT_F16 && G >= 32 && (UNROLL == 1 || UNROLL == 2 || UNROLL == 4)) {
      if (iter_shared_f16<G, SYM, CODES, UNROLL, NTS>(it.t, it.e0, it.n, v, lane, a.n_bits, rmax)) return;
    }
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      if (k < it.n) {
        UnitRef r;
        r.t = it.t;
        r.e0 = it.e0 + (int64_t)k * UNIT;
        r.valid = r.e0 < it.t.numel;
        any_nan |= group_unit_compute<DT, G, SYM, CODES, NTS>(r, v[k], lane, a.n_bits, rmax);
      }
    }
  };
  if (!(u0 < cend)) {
    flag_nan(a.nan_flag, false);
    return;
  }
  if constexpr (PFD == 2) {
    // three register images: slot s is computed while slot (s + 2) % 3 loads
    Iter it[3];
    Vec8<DT> v[3][UNROLL];
    bool has[3];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      has[s] = u0 < cend;
      if (has[s]) {
        plan_iter(u0, it[s]);
        load_iter<DT, UNROLL, NTL>(it[s], v[s]);
        advance(it[s].n);
      }
    }
    auto step = [&](auto S) -> bool {
      constexpr int s = decltype(S)::value;
      constexpr int l = (s + 2) % 3;
      has[l] = u0 < cend;
      if (has[l]) {
        plan_iter(u0, it[l]);
        load_iter<DT, UNROLL, NTL>(it[l], v[l]);
        advance(it[l].n);
      }
      if (!has[s]) return false;
      compute_iter(it[s], v[s]);
      return true;
    };
    while (step(std::integral_constant<int, 0>{}) && step(std::integral_constant<int, 1>{}) &&
           step(std::integral_constant<int, 2>{})) {
    }
  } else if constexpr (PF) {
    Iter itn;
    Vec8<DT> vn[UNROLL];
    plan_iter(u0, itn);
    load_iter<DT, UNROLL, NTL>(itn, vn);
    while (true) {
      const Iter it = itn;
      Vec8<DT> v[UNROLL];
#pragma unroll
      for (int k = 0; k < UNROLL; ++k) v[k] = vn[k];
      advance(it.n);
      const bool more = u0 < cend;
      if (more) {
        plan_iter(u0, itn);
        load_iter<DT, UNROLL, NTL>(itn, vn);
      }
      compute_iter(it, v);
      if (!more) break;
    }
  } else {
    while (u0 < cend) {
      Iter it;
      Vec8<DT> v[UNROLL];
      plan_iter(u0, it);
      load_iter<DT, UNROLL, NTL>(it, v);
      compute_iter(it, v);
      advance(it.n);
    }
  }
  flag_nan(a.nan_flag, any_nan);
}

template <int DT, int G, bool SYM, int CODES, bool BATCHED, int UNROLL, bool PF = false, bool NTL = true,
          bool NTS = true, bool SHARED = true, bool GS = false, bool SKEL = false, int RW = 1>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80))) void k_group(GroupArgs a) {
  k_group_body<DT, G, SYM, CODES, BATCHED, UNROLL, PF, NTL, NTS, SHARED, GS, SKEL, false, 0, RW>(a);
}
// walk-order forms (A/B): PHASE / PFD as in k_group_body
template <int DT, int G, bool SYM, int CODES, bool BATCHED, int UNROLL, bool SKEL, bool PHASE, int PFD, int RW = 1>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80))) void k_group_walk(GroupArgs a) {
  k_group_body<DT, G, SYM, CODES, BATCHED, UNROLL, false, true, true, true, false, SKEL, PHASE, PFD, RW>(a);
}
// the same walk held to 64 VGPRs, i.e. 8 waves per SIMD (k_group needs 67-68 at fp16 g128: 7 waves)
template <int DT, int G, bool SYM, int CODES, bool BATCHED, int UNROLL, bool PF = false, bool NTL = true,
          bool NTS = true, bool SHARED = true, bool GS = false, bool SKEL = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8, 8))) void k_group8(
    GroupArgs a) {
  k_group_body<DT, G, SYM, CODES, BATCHED, UNROLL, PF, NTL, NTS, SHARED, GS, SKEL>(a);
}

// =============================================================================================
// k_rowwave: one wavefront per contiguous group of length L (L % 8 == 0, L <= CPL*512)
// =============================================================================================
struct RowArgs {
  const char* w;
  char* out;
  uint8_t* codes;
  void* scales;
  void* zeros;
  int64_t ld_w, ld_out;   // elements
  int64_t cols;           // row length of the weight (codes layout)
  int64_t L;              // group length
  int64_t gpr;            // groups per row = cols / L
  int64_t G;              // number of groups
  int n_bits;
  uint32_t* nan_flag;
};

template <int DT, int CPL>
__device__ __forceinline__ void row_load(const RowArgs& a, int64_t j, int lane, Vec8<DT> (&v)[CPL]) {
  using F = Fmt<DT>;
  const int64_t row = j / a.gpr;
  const int64_t col0 = (j - row * a.gpr) * a.L;
  const char* src = a.w + (row * a.ld_w + col0) * F::BYTES;
  const int64_t nchunks = a.L / 8;
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int64_t ch = (int64_t)k * WAVE + lane;
    if (ch < nchunks) v[k].load(src + ch * 8 * F::BYTES);
  }
}

// reduce + quantize + store one group held in registers; returns whether a NaN was produced
template <int DT, int CPL, bool SYM, int CODES>
__device__ __forceinline__ bool row_compute(const RowArgs& a, int64_t j, int lane, const Vec8<DT> (&v)[CPL],
                                            float rmax) {
  using F = Fmt<DT>;
  const int64_t row = j / a.gpr;
  const int64_t col0 = (j - row * a.gpr) * a.L;
  const int64_t nchunks = a.L / 8;
  int32_t mn = 0x7FFFFFFF, mx = (int32_t)0x80000000;
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int64_t ch = (int64_t)k * WAVE + lane;
    if (ch < nchunks) {
      int32_t a_mn, a_mx;
      minmax8<DT, SYM>(v[k], a_mn, a_mx);
      mn = min(mn, a_mn);
      mx = max(mx, a_mx);
    }
  }
  if constexpr (SYM) group_max<64>(mx);
  else group_minmax<64>(mn, mx);
  const GroupParams p = params_from_keys<DT, SYM>(mn, mx, a.n_bits, rmax);
  bool any_nan = false;
  char* dst = a.out ? a.out + (row * a.ld_out + col0) * F::BYTES : nullptr;
  bool biased = false;
  BiasedWords bw{};
  if constexpr (DT == DT_F16) {
    biased = p.fast && a.n_bits <= 9;  // wave-uniform (one group per wave)
    if (biased) bw = biased_words<SYM>(p, a.n_bits);
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int64_t ch = (int64_t)k * WAVE + lane;
    if (ch < nchunks) {
      Vec8<DT> o;
      uint32_t c[4];
      if (DT == DT_F16 && biased) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) o.u[jj] = quant2_biased<CODES>(v[k].u[jj], bw, c[jj]);
      } else {
        any_nan |= quant8<DT, SYM>(v[k], p, a.n_bits, o, c);
      }
      if (dst) o.store(dst + ch * 8 * F::BYTES);
      if constexpr (CODES != 0) store_codes8<CODES>(a.codes, row * a.cols + col0 + ch * 8, c);
    }
  }
  if (lane == 0) {
    if (a.scales) store_param<DT>(a.scales, j, p.s);
    if (!SYM && a.zeros) store_param<DT>(a.zeros, j, p.z);
  }
  return any_nan;
}

template <int DT, int CPL, bool SYM, int CODES>
__global__ __launch_bounds__(BLOCK) void k_rowwave(RowArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * WAVES_PER_BLOCK + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (j >= a.G) return;  // whole wave exits together
  Vec8<DT> v[CPL];
  row_load<DT, CPL>(a, j, lane, v);
  flag_nan(a.nan_flag, row_compute<DT, CPL, SYM, CODES>(a, j, lane, v, rmax_for(a.n_bits, SYM)));
}

// Persistent form for short groups (CPL <= 8, rows up to 4096 elements): wave w takes groups
// w, w + nwaves, ... and loads group j + nwaves while it quantizes group j (two register images),
// so a 1.3-round grid (11008 rows of 4096) has neither a second-round tail nor exposed load latency.
template <int DT, int CPL, bool SYM, int CODES>
__global__ __launch_bounds__(BLOCK) void k_rowwave_pf(RowArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
  int64_t j = (int64_t)blockIdx.x * WAVES_PER_BLOCK + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  bool any_nan = false;
  if (j < a.G) {
    const float rmax = rmax_for(a.n_bits, SYM);
    Vec8<DT> v[CPL];
    row_load<DT, CPL>(a, j, lane, v);
    while (true) {
      const int64_t jn = j + nwaves;
      Vec8<DT> vn[CPL];
      if (jn < a.G) row_load<DT, CPL>(a, jn, lane, vn);
      any_nan |= row_compute<DT, CPL, SYM, CODES>(a, j, lane, v, rmax);
      if (jn >= a.G) break;
#pragma unroll
      for (int k = 0; k < CPL; ++k) v[k] = vn[k];
      j = jn;
    }
  }
  flag_nan(a.nan_flag, any_nan);
}

// =============================================================================================
// k_column: quant_dim = 1.  Groups of g consecutive ROWS in one column of W [rows, cols].
// Block = TX column-chunks (8 columns each) x TY row slices; grid = (cols/(8*TX), rows/g).
// Group j of column c sits at scales[c * (rows/g) + jr] (reference order of weight.t()).
// =============================================================================================
struct ColArgs {
  const char* w;
  char* out;
  uint8_t* codes;
  void* scales;
  void* zeros;
  int64_t rows, cols, ld_w, ld_out;
  int64_t g;      // rows per group
  int n_bits;
  uint32_t* nan_flag;
};

// bx, by: the block's column-chunk and row-group index (blockIdx.x / .y of the per-tensor grid;
// the batched kernels derive them from a flattened grid)
template <int DT, bool SYM, int CODES, int TX, int TY>
__device__ __forceinline__ void column_body(const ColArgs& a, int64_t bx, int64_t by) {
  using F = Fmt<DT>;
  __shared__ int32_t s_mn[TY][TX * 8];
  __shared__ int32_t s_mx[TY][TX * 8];
  const int tx = threadIdx.x % TX;
  const int ty = threadIdx.x / TX;
  const int64_t c0 = (bx * TX + tx) * 8;                       // first of this lane's 8 columns
  const int64_t jr = by;                                       // group index along rows
  const int64_t r0 = jr * a.g;
  const bool cvalid = c0 < a.cols;
  const float rmax = rmax_for(a.n_bits, SYM);
  int32_t mn[8], mx[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { mn[i] = 0x7FFFFFFF; mx[i] = (int32_t)0x80000000; }
  if (cvalid) {
    for (int64_t r = r0 + ty; r < r0 + a.g; r += TY) {
      Vec8<DT> v;
      v.load(a.w + (r * a.ld_w + c0) * F::BYTES);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (SYM) {
          mx[i] = max(mx[i], mag_key<DT>(v.get(i)));
        } else {
          int32_t k = key_of<DT>(v.get(i));
          mn[i] = min(mn[i], k);
          mx[i] = max(mx[i], k);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { s_mn[ty][tx * 8 + i] = mn[i]; s_mx[ty][tx * 8 + i] = mx[i]; }
  __syncthreads();
  GroupParams p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    int32_t a_mn = 0x7FFFFFFF, a_mx = (int32_t)0x80000000;
    for (int y = 0; y < TY; ++y) { a_mn = min(a_mn, s_mn[y][tx * 8 + i]); a_mx = max(a_mx, s_mx[y][tx * 8 + i]); }
    p[i] = params_from_keys<DT, SYM>(a_mn, a_mx, a.n_bits, rmax);
  }
  bool any_nan = false;
  if (cvalid) {
    if (ty == 0) {
      const int64_t ng = a.rows / a.g;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int64_t gidx = (c0 + i) * ng + jr;
        if (a.scales) store_param<DT>(a.scales, gidx, p[i].s);
        if (!SYM && a.zeros) store_param<DT>(a.zeros, gidx, p[i].z);
      }
    }
    const uint32_t off = SYM ? (1u << (a.n_bits - 1)) : 0u;
    for (int64_t r = r0 + ty; r < r0 + a.g; r += TY) {
      Vec8<DT> v, o;
      v.load(a.w + (r * a.ld_w + c0) * F::BYTES);
      uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float cf, y;
        y = quant_exact_or_fast<DT, SYM>(F::to_f(v.get(i)), p[i], cf);
        any_nan |= (y != y);
        o.set(i, F::from_f(y));
        const uint32_t cc = (cf == cf) ? ((uint32_t)(int32_t)cf + off) & 0xFFFFu : 0u;
        c[i >> 1] |= (i & 1) ? (cc << 16) : cc;
      }
      if (a.out) o.store(a.out + (r * a.ld_out + c0) * F::BYTES);
      if constexpr (CODES != 0) store_codes8<CODES>(a.codes, r * a.cols + c0, c);
    }
  }
  flag_nan(a.nan_flag, any_nan);
}

template <int DT, bool SYM, int CODES, int TX, int TY>
__global__ __launch_bounds__(TX * TY) void k_column(ColArgs a) {
  column_body<DT, SYM, CODES, TX, TY>(a, blockIdx.x, blockIdx.y);
}


// k_column_reg: k_column for g = RPT * TY rows per group (g in {32, 64, 128, 256}): every thread
// issues the loads of its RPT rows once, keeps them in registers across the reduction, and the
// block's per-column (min, max) is folded by 64 threads instead of every thread re-reading all
// TY partials (one pass over HBM, no second read of the tile).
template <int DT, bool SYM, int CODES, int TX, int TY, int RPT>
__device__ __forceinline__ void column_reg_body(const ColArgs& a, int64_t bx, int64_t by) {
  using F = Fmt<DT>;
  constexpr int NC = TX * 8;  // columns per block
  // Round 5 (LDS bank conflicts were 78 % of the kernel's LDS cycles, PMC): the partials live as
  // [ty][i][tx] with a row pitch of NC + TX dwords, so the 8-column stores of a wave's lanes (tx, ty)
  // hit distinct banks, and the fold threads (i, tx) read them in lane order; the fp16 fast path's
  // per-column words go out structure-of-arrays [i][tx] (16 lanes of distinct tx, 64 consecutive
  // dwords), replacing 8 GroupParams reads whose 192-B stride folded onto 4 banks and the 16-fold
  // redundant biased_words math of the TY row slices.
  // (SOA: fp16 up to 32 x 8 blocks; the 64 x 4 form of the short groups keeps the GroupParams
  // reads, whose 12 KiB more LDS would cost it two of its five workgroups per CU)
  // (the 64 x 4 form keeps the column-major partials [ty][8 tx + i]: its 8 consecutive dwords per
  // thread go out as two b128 writes, and the transposed layout measured 3 % slower there, g = 32)
  constexpr bool TL = TX <= 32;
  constexpr int PP = TL ? NC + TX : NC;
  constexpr bool SOA = DT == DT_F16 && TL;
  constexpr int NW = SOA ? NC : 1;
  __shared__ int32_t s_mn[TY * PP];
  __shared__ int32_t s_mx[TY * PP];
  __shared__ GroupParams f_p[NC];
  __shared__ uint32_t w_bounds[NW], w_sz[NW], w_kc[NW], w_fast[NW];
  __shared__ float w_rs[NW], w_s[NW];
  const int tx = threadIdx.x % TX;
  const int ty = threadIdx.x / TX;
  const int64_t c0 = (bx * TX + tx) * 8;
  const int64_t jr = by;
  const int64_t r0 = jr * a.g;
  const bool cvalid = c0 < a.cols;
  const int64_t cl = cvalid ? c0 : 0;  // unconditional loads (clamped column)
  Vec8<DT> v[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) v[k].load(a.w + ((r0 + ty + k * TY) * a.ld_w + cl) * F::BYTES);
  int32_t mn[8], mx[8];
  if constexpr (Fmt<DT>::NB == 16) {
    // per-column keys of the 16-bit dtypes in packed int16 (two columns per op), unpacked once
    s16x2 pmn[4], pmx[4];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        s16x2 kk;
        if constexpr (SYM) {
          kk = __builtin_bit_cast(s16x2, v[k].u[jj] & 0x7FFF7FFFu);
        } else {
          const s16x2 x = __builtin_bit_cast(s16x2, v[k].u[jj]);
          kk = x ^ ((x >> (short)15) & (short)0x7FFF);
        }
        if (k == 0) {
          pmn[jj] = kk;
          pmx[jj] = kk;
        } else {
          if constexpr (!SYM) pmn[jj] = __builtin_elementwise_min(pmn[jj], kk);
          pmx[jj] = __builtin_elementwise_max(pmx[jj], kk);
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      mn[2 * jj] = SYM ? 0 : (int32_t)pmn[jj].x;
      mn[2 * jj + 1] = SYM ? 0 : (int32_t)pmn[jj].y;
      mx[2 * jj] = (int32_t)pmx[jj].x;
      mx[2 * jj + 1] = (int32_t)pmx[jj].y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) { mn[i] = 0x7FFFFFFF; mx[i] = (int32_t)0x80000000; }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (SYM) {
          mx[i] = max(mx[i], mag_key<DT>(v[k].get(i)));
        } else {
          const int32_t kk = key_of<DT>(v[k].get(i));
          mn[i] = min(mn[i], kk);
          mx[i] = max(mx[i], kk);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = ty * PP + (TL ? i * TX + tx : tx * 8 + i);
    s_mn[e] = mn[i];
    s_mx[e] = mx[i];
  }
  __syncthreads();
  // one thread per column folds the TY partials AND derives the group's parameters once (not once
  // per row slice: 8x less parameter math at TY = 8), shared through LDS
  for (int t = threadIdx.x; t < NC; t += TX * TY) {  // NC > threads for the 64 x 4 shape
    const int fi = t / TX, ftx = t - fi * TX;          // TL: column ftx * 8 + fi
    const int cc = TL ? ftx * 8 + fi : t;
    int32_t a_mn = 0x7FFFFFFF, a_mx = (int32_t)0x80000000;
#pragma unroll 8
    for (int y = 0; y < TY; ++y) { a_mn = min(a_mn, s_mn[y * PP + t]); a_mx = max(a_mx, s_mx[y * PP + t]); }
    const GroupParams q = params_from_keys<DT, SYM>(a_mn, a_mx, a.n_bits, rmax_for(a.n_bits, SYM));
    f_p[cc] = q;
    if constexpr (SOA) {
      const BiasedWords bw = biased_words<SYM>(q, a.n_bits);
      w_bounds[t] = bw.bounds;
      w_sz[t] = bw.sz;
      w_kc[t] = bw.kc;
      w_rs[t] = bw.rs;
      w_s[t] = bw.s;
      w_fast[t] = q.fast ? 1u : 0u;
    }
    const int64_t col = bx * NC + cc;
    if (col < a.cols) {
      const int64_t gidx = col * (a.rows / a.g) + jr;
      if (a.scales) store_param<DT>(a.scales, gidx, q.s);
      if (!SYM && a.zeros) store_param<DT>(a.zeros, gidx, q.z);
    }
  }
  __syncthreads();
  bool any_nan = false;
  if (cvalid) {
    const uint32_t off = SYM ? (1u << (a.n_bits - 1)) : 0u;
    if constexpr (DT == DT_F16) {
      // all 8 columns of this thread on the fast path: packed pairs with per-half group operands
      // (the pairs assembled from the fold's per-column words, biased_pair's packing)
      bool fast = a.n_bits <= 9;
      GroupParams pf[8];
      if constexpr (SOA) {
#pragma unroll
        for (int i = 0; i < 8; ++i) fast = fast && w_fast[i * TX + tx] != 0u;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          pf[i] = f_p[tx * 8 + i];
          fast = fast && pf[i].fast;
        }
      }
      if (fast) {
        BiasedPair bp[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          if constexpr (SOA) {
            const int e0 = (2 * jj) * TX + tx, e1 = (2 * jj + 1) * TX + tx;
            bp[jj].rs = f2{w_rs[e0], w_rs[e1]};
            bp[jj].s = f2{w_s[e0], w_s[e1]};
            const uint32_t b0 = w_bounds[e0], b1 = w_bounds[e1];
            bp[jj].lo = (b0 & 0xFFFFu) | (b1 << 16);
            bp[jj].hi = (b0 >> 16) | (b1 & 0xFFFF0000u);
            bp[jj].s16 = (w_sz[e0] & 0xFFFFu) | (w_sz[e1] << 16);
            bp[jj].kc = (w_kc[e0] & 0xFFFFu) | (w_kc[e1] << 16);
          } else {
            bp[jj] = biased_pair<SYM>(pf[2 * jj], pf[2 * jj + 1], a.n_bits);
          }
        }
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
          const int64_t r = r0 + ty + k * TY;
          Vec8<DT> o;
          uint32_t c[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) o.u[jj] = quant2_biased_pair<CODES>(v[k].u[jj], bp[jj], c[jj]);
          if (a.out) o.store(a.out + (r * a.ld_out + c0) * F::BYTES);
          if constexpr (CODES != 0) store_codes8<CODES>(a.codes, r * a.cols + c0, c);
        }
        flag_nan(a.nan_flag, false);
        return;
      }
    }
    GroupParams p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = f_p[tx * 8 + i];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int64_t r = r0 + ty + k * TY;
      Vec8<DT> o;
      uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float cf, y;
        y = quant_exact_or_fast<DT, SYM>(F::to_f(v[k].get(i)), p[i], cf);
        any_nan |= (y != y);
        o.set(i, F::from_f(y));
        const uint32_t cc = (cf == cf) ? ((uint32_t)(int32_t)cf + off) & 0xFFFFu : 0u;
        c[i >> 1] |= (i & 1) ? (cc << 16) : cc;
      }
      if (a.out) o.store(a.out + (r * a.ld_out + c0) * F::BYTES);
      if constexpr (CODES != 0) store_codes8<CODES>(a.codes, r * a.cols + c0, c);
    }
  }
  flag_nan(a.nan_flag, any_nan);
}

template <int DT, bool SYM, int CODES, int TX, int TY, int RPT>
__global__ __launch_bounds__(TX * TY) void k_column_reg(ColArgs a) {
  column_reg_body<DT, SYM, CODES, TX, TY, RPT>(a, blockIdx.x, blockIdx.y);
}


// =============================================================================================
// per-tensor (group -1; one group, so the element-wise apply is the same for quant_dim 0 and 1):
//   k_tensor_reduce  persistent grid, 16-B loads, one (min, max) key pair per workgroup -> workspace
//   k_tensor_apply   every workgroup folds the partials (<= a few thousand x 8 B, L2-resident),
//                    derives the tensor's scale / zero point and quantizes its share
// 6 B per fp16 element of HBM traffic (read, read, write) instead of the segmented path's scalar walk.
// =============================================================================================
template <int DT, bool SYM, bool NTL>
__global__ __launch_bounds__(BLOCK) void k_tensor_reduce(const char* w, int64_t nunits, int32_t* partial) {
  using F = Fmt<DT>;
  constexpr int UN = 4;
  __shared__ int32_t smn[WAVES_PER_BLOCK], smx[WAVES_PER_BLOCK];
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  int32_t mn = 0x7FFFFFFF, mx = (int32_t)0x80000000;
  for (int64_t u0 = (int64_t)blockIdx.x * BLOCK + threadIdx.x; u0 < nunits; u0 += nthreads * UN) {
    Vec8<DT> v[UN];
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int64_t u = u0 + k * nthreads;
      v[k].template load<NTL>(w + (u < nunits ? u : 0) * 8 * F::BYTES);
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      if (u0 + k * nthreads < nunits) {
        int32_t a, b;
        minmax8<DT, SYM>(v[k], a, b);
        mn = min(mn, a);
        mx = max(mx, b);
      }
    }
  }
  group_minmax<64>(mn, mx);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[wv] = mn; smx[wv] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 1; i < WAVES_PER_BLOCK; ++i) { mn = min(mn, smn[i]); mx = max(mx, smx[i]); }
    partial[2 * blockIdx.x] = mn;
    partial[2 * blockIdx.x + 1] = mx;
  }
}

template <int DT, bool SYM, int CODES, bool NTL, bool REV, int UN = 1>
__global__ __launch_bounds__(BLOCK) void k_tensor_apply(const char* w, char* out, uint8_t* codes, void* scales,
                                                        void* zeros, int64_t nunits, const int32_t* partial,
                                                        int nparts, int n_bits, uint32_t* nan_flag) {
  using F = Fmt<DT>;
  __shared__ int32_t smn[WAVES_PER_BLOCK], smx[WAVES_PER_BLOCK];
  int32_t mn = 0x7FFFFFFF, mx = (int32_t)0x80000000;
  for (int i = threadIdx.x; i < nparts; i += BLOCK) {
    mn = min(mn, partial[2 * i]);
    mx = max(mx, partial[2 * i + 1]);
  }
  group_minmax<64>(mn, mx);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[wv] = mn; smx[wv] = mx; }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < WAVES_PER_BLOCK; ++i) { mn = min(mn, smn[i]); mx = max(mx, smx[i]); }
  const GroupParams p = params_from_keys<DT, SYM>(mn, mx, n_bits, rmax_for(n_bits, SYM));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (scales) store_param<DT>(scales, 0, p.s);
    if (!SYM && zeros) store_param<DT>(zeros, 0, p.z);
  }
  bool any_nan = false;
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  // UN units per thread per iteration, all loads issued before the first store (UN > 1)
  for (int64_t t0 = (int64_t)blockIdx.x * BLOCK + threadIdx.x; t0 < nunits; t0 += nthreads * UN) {
    Vec8<DT> v[UN];
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int64_t t = t0 + k * nthreads;
      const int64_t u = REV ? nunits - 1 - t : t;  // REV: the units the reduce read last (MALL) first
      v[k].template load<NTL>(w + (t < nunits ? u : 0) * 8 * F::BYTES);
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int64_t t = t0 + k * nthreads;
      if (t < nunits) {
        const int64_t u = REV ? nunits - 1 - t : t;
        Vec8<DT> o;
        uint32_t c[4];
        any_nan |= quant8<DT, SYM>(v[k], p, n_bits, o, c);
        if (out) o.store(out + u * 8 * F::BYTES);
        if constexpr (CODES != 0) store_codes8<CODES>(codes, u * 8, c);
      }
    }
  }
  flag_nan(nan_flag, any_nan);
}

// ---------------------------------------------------------------------------------------------
// k_tensor_onepass (round 3): per-tensor (-1) in ONE pass over HBM for fp16 weights that fit the
// chip's registers.  One 512-thread workgroup per CU (2 waves per SIMD, up to 256 registers per lane:
// two would not fit, so the grid of CU-count workgroups is co-resident -- up to ~100 MB of fp16
// held, every Llama-2-7B shape); every thread loads its NV 16-B vectors (grid-stride,
// coalesced) and KEEPS them in registers; the workgroup's (min, max) order keys (int16 for 16-bit
// dtypes, packed in one dword) are published as one 8-byte granule {tag = 1, keys} by an agent-scope
// atomic store (cdna_hip_programming.md Guideline 16 R2: the data is the flag, no fence); wave 0 of
// every workgroup sweeps all granules (relaxed agent-scope atomic loads, bounded spin) until every
// tag is 1, folds them, and the workgroup quantizes its registers and stores -- 4 B per element of
// HBM traffic instead of the two-kernel pair's 6.  The granules (8 B x CU count, at the workspace's
// start), the CONSENSUS word and the done counter after them are zero before every launch (a zeroing
// kernel, or IWQ_FLAG_WS_ZEROED: the kernel's last workgroup leaves them zero).
//
// Fail-safe hand-off (round 4): the hand-off needs every workgroup resident at once; when another
// kernel holds CUs a sweep can give up.  Every workgroup stores NOTHING until the launch has agreed
// on one outcome, decided by the first compare-and-swap on the consensus word:
//   * a sweep that saw every granule CASes 0 -> GO; a sweep that gave up CASes 0 -> ABORT;
//   * a workgroup stores (output, codes, parameters) only if the word reads GO;
//   * a workgroup that gave up but finds GO sweeps again: the GO-er saw every granule, so all of
//     them are published and this sweep ends (bounded; a second give-up -- not reachable while
//     stores become visible -- sets nan_flag bit 2: outputs invalid).
// On ABORT no byte of any output is written and nan_flag bit 1 is set, so the host can re-run the
// same call on the two-kernel pair, IN PLACE too: the input is untouched.  Round 6: with outputs that
// cannot alias the input, a completed sweep goes without the CAS (the CAS decides only give-ups); an
// ABORT then may leave some outputs written, which the host's re-run on the pair overwrites.
// ---------------------------------------------------------------------------------------------
constexpr int OP_THR = 512;
constexpr uint32_t OP_SPIN_LIMIT = 1u << 22;
constexpr int OP_NT = 2;  // buffer-instruction cache bits: non-temporal (streamed once)
constexpr unsigned long long OP_GO = 1, OP_ABORT = 2;

// Workgroup b owns the contiguous vectors [b * nvt * 512, (b + 1) * nvt * 512) (vectors of 8
// elements: 16 B for fp16 / bf16, 32 B for fp32; nvt <= NV vectors per thread, chosen so the chunks
// spread over every CU); vector i of thread t is b * nvt * 512 + i * 512 + t: every load / store
// instruction covers 8 KiB contiguous per workgroup (fp32: two instructions over 16 KiB).  The loads
// go through a buffer descriptor over the workgroup's chunk (one 32-bit per-lane offset for all
// vectors; the range check zero-fills loads beyond the chunk -- i >= nvt, or the last chunk's tail --
// without touching memory, and the key fold masks them).  A granule counts once its tag equals 1.
// Keys: 16-bit dtypes publish (min, max) as packed int16 in ONE granule per workgroup; fp32 (round 5)
// publishes two granules, {tag, min key} and {tag, max key} (granules[2b], granules[2b + 1]); the
// consensus word and a done counter follow the last granule.  All are zero on entry (the per-launch
// memset, or IWQ_FLAG_WS_ZEROED) and the last workgroup to finish its hand-off zeroes them again.
// Elementwise: fp16 takes the packed fast path, bf16 / fp32 (round 5) a Markstein-division fast path
// on the register-held vectors; non-finite or extreme ranges re-read the input for the literal chain.
template <int DT, bool SYM, int CODES, int NV>
__global__ __launch_bounds__(OP_THR) void k_tensor_onepass(const char* w, char* out, uint8_t* codes, void* scales,
                                                           void* zeros, int64_t nvec, int nvt,
                                                           unsigned long long* granules, int n_bits,
                                                           uint32_t* nan_flag, uint32_t spin_limit) {
  constexpr uint32_t tag = 1;
  using F = Fmt<DT>;
  constexpr bool K32 = F::NB == 32;       // 32-bit order keys: two granules per workgroup
  constexpr int KG = K32 ? 2 : 1;         // granules per workgroup
  constexpr int VB = F::BYTES * 8;        // bytes per 8-element vector
  constexpr int32_t KMIN = K32 ? (int32_t)0x80000000 : -0x8000, KMAX = K32 ? 0x7FFFFFFF : 0x7FFF;
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  __shared__ int32_t smn[OP_THR / 64], smx[OP_THR / 64];
  __shared__ int32_t fin[3];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t chunk = (int64_t)nvt * OP_THR;                    // vectors per workgroup
  const int64_t v0 = (int64_t)blockIdx.x * chunk;                 // this workgroup's first vector
  const int64_t nv_here = nvec - v0 < chunk ? nvec - v0 : chunk;  // > 0: one workgroup per non-empty chunk
  const int nbytes = (int)(nv_here * VB);
  const char* wb = static_cast<const char*>(rflp(static_cast<const void*>(w + v0 * VB)));
  const auto rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wb), 0, nbytes, 0x00020000);
  // fp32: the two 16-B halves of a thread's vector i are chunks 2i and 2i + 1 of 512 x 16 B each
  // (chunk c of thread t at byte (c * 512 + t) * 16 of the workgroup's range), so every load / store
  // instruction still covers 8 KiB contiguous; elementwise work does not care which 8 elements share
  // a register vector.  16-bit dtypes: one chunk per vector.
  const int voff = threadIdx.x * 16;
  const int64_t nch = nv_here * (VB / 16);  // valid 16-B chunks of this workgroup
  Vec8<DT> v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int h = 0; h < VB / 16; ++h) {
      const u32x4v x = __builtin_amdgcn_raw_buffer_load_b128(rin, voff, (i * (VB / 16) + h) * OP_THR * 16, OP_NT);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[i].u[4 * h + j] = x[j];
    }
  }
  int32_t mn = KMAX, mx = KMIN;  // identities (every order key lies in between)
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (i < nvt) {  // uniform (a branch, not a break: the loop must stay fully unrolled)
      if constexpr (K32) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if ((int64_t)(2 * i + h) * OP_THR + threadIdx.x < nch) {
#pragma unroll
            for (int e = 4 * h; e < 4 * h + 4; ++e) {
              const int32_t kk = SYM ? mag_key<DT>(v[i].get(e)) : key_of<DT>(v[i].get(e));
              mn = min(mn, SYM ? 0 : kk);
              mx = max(mx, kk);
            }
          }
        }
      } else {
        int32_t a, b;
        minmax8<DT, SYM>(v[i], a, b);
        if ((int64_t)i * OP_THR + threadIdx.x < nv_here) {
          mn = min(mn, a);
          mx = max(mx, b);
        }
      }
    }
  }
  group_minmax<64>(mn, mx);
  if (lane == 0) { smn[wv] = mn; smx[wv] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 1; i < OP_THR / 64; ++i) { mn = min(mn, smn[i]); mx = max(mx, smx[i]); }
    if constexpr (K32) {
      __hip_atomic_store(granules + 2 * blockIdx.x, ((unsigned long long)tag << 32) | (uint32_t)mn,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(granules + 2 * blockIdx.x + 1, ((unsigned long long)tag << 32) | (uint32_t)mx,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint32_t keys = (uint32_t)(uint16_t)(int16_t)mn | ((uint32_t)(uint16_t)(int16_t)mx << 16);
      __hip_atomic_store(granules + blockIdx.x, ((unsigned long long)tag << 32) | keys, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    // the publish is acknowledged at agent scope before this thread issues anything else -- in
    // particular before its done-counter increment below (a workgroup that gives up its
    // sweep early must not let its publish land after the last workgroup's clearing stores).  A wait,
    // not a release fence: the granules are agent-scope atomic stores, there is no cached data to
    // write back, and the wait sits where this wave waits for the other publishes anyway.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // Round 6: when the outputs cannot alias the input (out of place -- pseudo_quantize_tensor's
  // default -- or codes / parameters only) a workgroup whose sweep saw every granule goes WITHOUT the
  // consensus compare-and-swap (one agent-scope round trip less on the hand-off's critical path):
  // if another workgroup gives up, it still CASes ABORT and sets nan_flag bit 1, and the host re-runs
  // the call on the pair, which rewrites every output from the untouched input.  In place, the CAS
  // protocol stands (an input overwritten by a GO-er could not be re-read by the retry).
  const int64_t tbytes = nvec * VB;
  const bool alias = out != nullptr && out < w + tbytes && w < out + tbytes;
  if (wv == 0) {
    // sweep every workgroup's granule(s) until all carry the tag (relaxed agent-scope loads bypass L1)
    const int ng = (int)gridDim.x * KG;
    int32_t gmn, gmx;
    auto fold = [&](unsigned long long x, int g) {
      if constexpr (K32) {
        if (g & 1) gmx = max(gmx, (int32_t)(uint32_t)x);
        else gmn = min(gmn, (int32_t)(uint32_t)x);
      } else {
        gmn = min(gmn, (int32_t)(int16_t)(uint16_t)(x & 0xFFFFu));
        gmx = max(gmx, (int32_t)(int16_t)(uint16_t)((x >> 16) & 0xFFFFu));
      }
    };
    // round 5: every granule a lane still waits for is loaded in the same spin iteration (up to 8 x 64
    // granules: one relaxed agent-scope round trip per iteration instead of one per 64 granules in
    // sequence -- four on a 256-CU chip, eight with fp32's two granules per workgroup)
    constexpr int SWK = 8;
    auto sweep = [&](uint32_t limit) -> bool {  // true: gave up before seeing every granule
      gmn = KMAX;
      gmx = KMIN;
      bool gave_up = false;
      if (ng <= 64 * SWK) {
        const int nk = (ng + 63) / 64;
        uint32_t have = 0;  // bit k: granule 64 k + lane seen with the tag (or beyond ng)
#pragma unroll
        for (int k = 0; k < SWK; ++k)
          if (k >= nk || 64 * k + lane >= ng) have |= 1u << k;
        uint32_t spins = 0;
        while (true) {
          unsigned long long xv[SWK];
#pragma unroll
          for (int k = 0; k < SWK; ++k)
            if (!((have >> k) & 1u)) xv[k] = __hip_atomic_load(granules + 64 * k + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int k = 0; k < SWK; ++k) {
            if (!((have >> k) & 1u) && (uint32_t)(xv[k] >> 32) == tag) {
              have |= 1u << k;
              fold(xv[k], 64 * k + lane);
            }
          }
          if (__all(have == (1u << SWK) - 1u)) break;
          if (++spins > limit) {
            gave_up = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        return gave_up;
      }
      for (int g0 = 0; g0 < ng; g0 += 64) {  // (more workgroups than 8 x 64 granules: chunk by chunk)
        const int g = g0 + lane;
        uint32_t spins = 0;
        unsigned long long x = 0;
        while (true) {
          x = g < ng ? __hip_atomic_load(granules + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : ((unsigned long long)tag << 32);
          if (__all((uint32_t)(x >> 32) == tag)) break;
          if (++spins > limit) {
            gave_up = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (g < ng && (uint32_t)(x >> 32) == tag) fold(x, g);
      }
      return gave_up;
    };
    // spin_limit 0 (test-only variant 9): every workgroup gives up, so the launch ABORTs
    bool timed_out = sweep(spin_limit) || spin_limit == 0;
    // one outcome for the whole launch: the first CAS on the consensus word decides (in place, or
    // after a give-up; out of place a completed sweep is its own decision)
    unsigned long long decided = (!alias && !timed_out) ? OP_GO : 0;
    if (lane == 0 && decided == 0) {
      unsigned long long expect = 0;
      const unsigned long long want = timed_out ? OP_ABORT : OP_GO;
      decided = __hip_atomic_compare_exchange_strong(granules + ng, &expect, want, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    ? want
                    : expect;
    }
    decided = (unsigned long long)__shfl((long long)decided, 0);
    bool go = decided == OP_GO;
    if (go && timed_out) {
      // another workgroup saw every granule: they are all published, so this sweep completes
      if (sweep(OP_SPIN_LIMIT * 4)) {
        go = false;
        if (lane == 0 && nan_flag) atomicOr(nan_flag, 4u);
      }
    }
    group_minmax<64>(gmn, gmx);
    if (lane == 0) {
      fin[0] = gmn;
      fin[1] = gmx;
      fin[2] = go ? 1 : 0;
      if (!go && decided == OP_ABORT && nan_flag) atomicOr(nan_flag, 2u);
    }
  }
  __syncthreads();
  // round 5: past the barrier no wave of this workgroup reads a granule any more -- count the
  // workgroup done; the LAST one zeroes the granules, the consensus word and the counter, so the next
  // launch on the same workspace needs no memset (IWQ_FLAG_WS_ZEROED).  The increment is made by the
  // thread that published this workgroup's granule(s), after its explicit wait for that publish's
  // acknowledgement (above), so every publish is performed before its workgroup's count; the last
  // workgroup issues its clearing stores only once its increment has returned the final count (a
  // data dependency on an agent-scope atomic).  Issued here, its value used only at the end
  // (clear_if_last), so its round trip overlaps this workgroup's output stores.
  unsigned long long done = 0;
  if (threadIdx.x == 0)
    done = __hip_atomic_fetch_add(granules + (int)gridDim.x * KG + 1, 1ull, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  auto clear_if_last = [&]() {
    if (threadIdx.x < 64) {
      done = (unsigned long long)__shfl((long long)done, 0);
      if (done == (unsigned long long)gridDim.x - 1) {
        const int ng = (int)gridDim.x * KG;
        for (int g = threadIdx.x; g < ng + 2; g += 64)
          __hip_atomic_store(granules + g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };
  if (fin[2] == 0) {  // ABORT: no output byte is written (the input is untouched)
    clear_if_last();
    return;
  }
  const GroupParams p = params_from_keys<DT, SYM>(fin[0], fin[1], n_bits, rmax_for(n_bits, SYM));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (scales) store_param<DT>(scales, 0, p.s);
    if (!SYM && zeros) store_param<DT>(zeros, 0, p.z);
  }
  // the stores are global stores: ROCm 7.2's LLVM omits the wait state a buffer_store_dwordx4 with an
  // SGPR soffset needs before a VALU overwrites its data registers (the first dword of the stored
  // vector was clobbered -- caught by the bit-exact tests), so the output leaves through 64-bit
  // addresses with the range check done by hand
  char* ob = out ? out + v0 * VB + threadIdx.x * 16 : nullptr;
  bool any_nan = false;
  if constexpr (DT == DT_F16) {
    if (p.fast) {  // the packed fp16 path on the register-held vectors (uniform: one group)
      const FastPk k = fast_pk<SYM>(p, n_bits);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        if (i < nvt) {  // uniform
          u32x4v o;
          uint32_t c[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t cp;
            o[j] = quant2_fast<SYM>(v[i].u[j], p, k, cp);
            c[j] = codes2_fast(cp, k);
          }
          if ((int64_t)i * OP_THR + threadIdx.x < nv_here) {
            if (ob) __builtin_nontemporal_store(o, gp<u32x4v>(static_cast<void*>(ob + (int64_t)i * OP_THR * 16)));
            if constexpr (CODES != 0) store_codes8<CODES>(codes, (v0 + (int64_t)i * OP_THR + threadIdx.x) * 8, c);
          }
        }
      }
    } else {
      // non-finite range / zero scale (never on real weights): the exact chain, each thread re-reading
      // its own vectors (nothing else writes them, so this is right in place too)
      for (int i = 0; i < nvt; ++i) {
        const int64_t u = v0 + (int64_t)i * OP_THR + threadIdx.x;
        if (u < v0 + nv_here) {
          Vec8<DT> x, o;
          x.template load<true>(w + u * 8 * F::BYTES);
          uint32_t c[4];
          any_nan |= quant8<DT, SYM>(x, p, n_bits, o, c);
          if (out) o.template store<true>(out + u * 8 * F::BYTES);
          if constexpr (CODES != 0) store_codes8<CODES>(codes, u * 8, c);
        }
      }
    }
  } else {
    // bf16 / fp32 (round 5).  Fast path (one group, so a uniform branch): the quotient as Markstein's
    // corrected product, q = RN32(w / s) from rs = RN32(1 / s) (exact IEEE reciprocal, once); then one
    // rounding to the storage dtype, rint, the bound clamp and RN((c - z) * s) -- bit-identical to the
    // literal chain quant_exact (iwq_common.cuh) whenever tensor_fast_dt holds: s normal and
    // >= 2^-40 (the reference clamps the range at 1e-5 first, so s >= 1.5e-10 for <= 16 bits), and
    // max |w| * rs < 2^100 (no overflow in q0 or the residual).  A quotient that matters (|w / s| >=
    // 0.5) then has |w| >= s / 2, a normal number whose residual w - q0 s cannot underflow, so the
    // correction is exact (the fp16 selftest checks the same construction exhaustively); smaller
    // quotients round to 0 whatever their last bits.  r + z needs no rounding: exact below 2^8 (bf16)
    // / 2^24 (fp32), and beyond that the clamp to [lo, hi] gives the same bound; (c - z) * s is the
    // reference's product: fp32-rounded, then (bf16) rounded to the storage dtype.
    const float mxa = fmaxf(fabsf(F::to_f(bits_of_key<DT>(fin[0]))), fabsf(F::to_f(bits_of_key<DT>(fin[1]))));
    // (bf16 represents every integer only up to 2^8: above 8 bits the reference's R(r + z) can move
    // an in-range integer, so wider bf16 codes take the literal chain)
    const bool fastdt = p.s >= 0x1p-40f && p.s <= 0x1p100f && mxa * p.rs < 0x1p100f &&
                        n_bits <= (F::NB == 16 ? 8 : 16);
    if (fastdt) {
      const float rs = p.rs, sc = p.s, zz = p.z, lo = p.lo, hi = p.hi;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        if (i < nvt) {  // uniform
          Vec8<DT> o;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = F::to_f(v[i].get(e));
            const float q0 = x * rs;
            const float q = opaque(__builtin_fmaf(__builtin_fmaf(-q0, sc, x), rs, q0));  // RN32(x / s)
            const float t = F::R(q);
            const float c = __builtin_amdgcn_fmed3f(__builtin_rintf(t) + zz, lo, hi);
            o.set(e, F::from_f(SYM ? c * sc : (c - zz) * sc));
          }
          if (ob) {
            if constexpr (K32) {
#pragma unroll
              for (int h = 0; h < 2; ++h)
                if ((int64_t)(2 * i + h) * OP_THR + threadIdx.x < nch)
                  __builtin_nontemporal_store((u32x4v){o.u[4 * h], o.u[4 * h + 1], o.u[4 * h + 2], o.u[4 * h + 3]},
                                              gp<u32x4v>(static_cast<void*>(ob + (int64_t)(2 * i + h) * OP_THR * 16)));
            } else if ((int64_t)i * OP_THR + threadIdx.x < nv_here) {
              o.template store<true>(ob + (int64_t)i * OP_THR * VB);
            }
          }
        }
      }
    } else {
      // non-finite / extreme ranges: the literal op chain, each thread re-reading its own vectors
      // (nothing else writes them, so this is right in place too)
      for (int i = 0; i < nvt; ++i) {
        const int64_t u = v0 + (int64_t)i * OP_THR + threadIdx.x;
        if (u < v0 + nv_here) {
          Vec8<DT> x, o;
          x.template load<true>(w + u * 8 * F::BYTES);
          uint32_t c[4];
          any_nan |= quant8<DT, SYM>(x, p, n_bits, o, c);
          if (out) o.template store<true>(out + u * 8 * F::BYTES);
          if constexpr (CODES != 0) store_codes8<CODES>(codes, u * 8, c);
        }
      }
    }
  }
  flag_nan(nan_flag, any_nan);
  clear_if_last();
}

template <int DT, bool SYM>
__global__ __launch_bounds__(BLOCK) void k_seg_apply(SegArgs a) {
  using F = Fmt<DT>;
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  const int64_t tid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  int64_t curj = -1;
  GroupParams p{};
  bool any_nan = false;
  for (int64_t f0 = tid * SEG_RUN; f0 < a.total; f0 += nthreads * SEG_RUN) {
    const int64_t fend = min(f0 + SEG_RUN, a.total);
    for (int64_t f = f0; f < fend; ++f) {
      const int64_t j = f / a.L;
      if (j != curj) {
        curj = j;
        if constexpr (SYM) p = params_sym_exact<DT>(F::to_f(bits_of_key<DT>(a.keys[2 * j + 1])), a.n_bits);
        else p = params_asym_exact<DT>(F::to_f(bits_of_key<DT>(a.keys[2 * j])), F::to_f(bits_of_key<DT>(a.keys[2 * j + 1])), a.n_bits);
        if (f == j * a.L) {
          if (a.scales) store_param<DT>(a.scales, j, p.s);
          if (!SYM && a.zeros) store_param<DT>(a.zeros, j, p.z);
        }
      }
      int64_t ow, oo, r, c;
      seg_locate(a, f, ow, oo, r, c);
      uint32_t b;
      if constexpr (F::NB == 16) b = gp<uint16_t>(a.w)[ow];
      else b = gp<uint32_t>(a.w)[ow];
      float cf;
      float y = quant_exact<DT, SYM>(F::to_f(b), p, cf);
      any_nan |= (y != y);
      const uint32_t yb = F::from_f(y);
      if (a.out) {
        if constexpr (F::NB == 16) gp<uint16_t>(a.out)[oo] = (uint16_t)yb;
        else gp<uint32_t>(a.out)[oo] = yb;
      }
      if (a.codes_bits) {
        const uint32_t code = (cf == cf) ? (uint32_t)(int32_t)cf + (SYM ? (1u << (a.n_bits - 1)) : 0u) : 0u;
        const int64_t e = r * a.cols + c;
        if (a.codes_bits == 8) {
          gp<uint8_t>(a.codes)[e] = (uint8_t)code;
        } else {
          // nibbles: OR into the (pre-zeroed) 32-bit word; neighbours may belong to other threads
          const int64_t byte = e >> 1;
          const int shift = (int)((byte & 3) * 8 + (e & 1) * 4);
          atomicOr(reinterpret_cast<uint32_t*>(a.codes + (byte & ~(int64_t)3)), (code & 0xFu) << shift);
        }
      }
    }
  }
  flag_nan(a.nan_flag, any_nan);
}

// =============================================================================================
// Batched forms of the row / column / per-tensor kernels: whole-model launches for the group modes
// the k_group walk does not cover (per-channel and long or non-power-of-two groups, quant_dim 1,
// per-tensor), quant_wrapper.py:52-82's loop for those configurations.  The table is
// iwq_batch_entry[] in device memory; entry e's work items -- groups (rows), blocks of its own 2-D
// column grid, or 512-element units (per-tensor) -- start at unit_begin (iwq_batch_plan_ex).  A
// work item finds its entry by a wave-uniform binary search over unit_begin (a few KiB of table,
// scalar-cache resident), then runs the per-tensor kernel's body on that entry: every tensor gets
// exactly the bits of its single-tensor launch.
// =============================================================================================
struct BatchExArgs {
  const iwq_batch_entry* entries;
  int32_t n_entries;
  int64_t total_units;
  int64_t group;     // > 0, or IWQ_GROUP_PER_CHANNEL (the row / column length of each entry)
  int n_bits;
  uint32_t* nan_flag;
};


// largest e with entries[e].unit_begin <= u (u wave-uniform)
__device__ __forceinline__ int32_t find_entry(const iwq_batch_entry* entries, int32_t n, int64_t u) {
  const IWQ_GLOBAL iwq_batch_entry* tab = gp<iwq_batch_entry>(entries);
  int32_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const int32_t mid = (lo + hi + 1) >> 1;
    if (rfl64(tab[mid].unit_begin) <= u) lo = mid;
    else hi = mid - 1;
  }
  return __builtin_amdgcn_readfirstlane(lo);
}

struct RowRef {
  RowArgs a;
  int64_t jl;  // group index within the entry
};

__device__ __forceinline__ RowRef row_ref(const BatchExArgs& b, int64_t j) {
  const int32_t e = find_entry(b.entries, b.n_entries, j);
  const IWQ_GLOBAL iwq_batch_entry* t = gp<iwq_batch_entry>(b.entries) + e;
  RowRef r;
  const int64_t cols = rfl64(t->cols);
  r.a.w = static_cast<const char*>(rflp(t->w));
  r.a.out = static_cast<char*>(rflp(t->out_deq));
  r.a.codes = static_cast<uint8_t*>(rflp(t->out_codes));
  r.a.scales = rflp(t->out_scales);
  r.a.zeros = rflp(t->out_zeros);
  r.a.ld_w = cols;
  r.a.ld_out = cols;
  r.a.cols = cols;
  r.a.L = b.group > 0 ? b.group : cols;
  r.a.gpr = cols / r.a.L;
  r.a.G = rfl64(t->rows) * r.a.gpr;
  r.a.n_bits = b.n_bits;
  r.a.nan_flag = nullptr;
  r.jl = j - rfl64(t->unit_begin);
  return r;
}

// one wave per group (row or row segment), persistent over the whole table; PF: the next group's
// loads are issued before this one's arithmetic (k_rowwave_pf's two register images)
template <int DT, int CPL, bool SYM, int CODES, bool PF>
__global__ __launch_bounds__(BLOCK) void k_rowwave_b(BatchExArgs b) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
  int64_t j = (int64_t)blockIdx.x * WAVES_PER_BLOCK + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  bool any_nan = false;
  if (j < b.total_units) {
    const float rmax = rmax_for(b.n_bits, SYM);
    RowRef cur = row_ref(b, j);
    Vec8<DT> v[CPL];
    row_load<DT, CPL>(cur.a, cur.jl, lane, v);
    while (true) {
      const int64_t jn = j + nwaves;
      const bool more = jn < b.total_units;
      if constexpr (PF) {
        RowRef nxt = cur;
        Vec8<DT> vn[CPL];
        if (more) {
          nxt = row_ref(b, jn);
          row_load<DT, CPL>(nxt.a, nxt.jl, lane, vn);
        }
        any_nan |= row_compute<DT, CPL, SYM, CODES>(cur.a, cur.jl, lane, v, rmax);
        if (!more) break;
        cur = nxt;
#pragma unroll
        for (int k = 0; k < CPL; ++k) v[k] = vn[k];
      } else {
        any_nan |= row_compute<DT, CPL, SYM, CODES>(cur.a, cur.jl, lane, v, rmax);
        if (!more) break;
        cur = row_ref(b, jn);
        row_load<DT, CPL>(cur.a, cur.jl, lane, v);
      }
      j = jn;
    }
  }
  flag_nan(b.nan_flag, any_nan);
}

// quant_dim 1: one block of the entry's (column chunk, row group) grid per flattened block index;
// RPT 0 = the generic two-pass body (any g, e.g. per-channel g = rows), else column_reg_body
template <int DT, bool SYM, int CODES, int TX, int TY, int RPT>
__global__ __launch_bounds__(TX * TY) void k_column_b(BatchExArgs b) {
  const int64_t u = blockIdx.x;
  const int32_t e = find_entry(b.entries, b.n_entries, u);
  const IWQ_GLOBAL iwq_batch_entry* t = gp<iwq_batch_entry>(b.entries) + e;
  ColArgs a{};
  a.w = static_cast<const char*>(rflp(t->w));
  a.out = static_cast<char*>(rflp(t->out_deq));
  a.codes = static_cast<uint8_t*>(rflp(t->out_codes));
  a.scales = rflp(t->out_scales);
  a.zeros = rflp(t->out_zeros);
  a.rows = rfl64(t->rows);
  a.cols = rfl64(t->cols);
  a.ld_w = a.cols;
  a.ld_out = a.cols;
  a.g = b.group > 0 ? b.group : a.rows;
  a.n_bits = b.n_bits;
  a.nan_flag = b.nan_flag;
  const int64_t gx = (a.cols + 8 * TX - 1) / (8 * TX);
  const int64_t lb = u - rfl64(t->unit_begin);
  if constexpr (RPT == 0) column_body<DT, SYM, CODES, TX, TY>(a, lb % gx, lb / gx);
  else column_reg_body<DT, SYM, CODES, TX, TY, RPT>(a, lb % gx, lb / gx);
}

// per-tensor (-1): keys[2e], keys[2e + 1] = the (min, max) order keys of entry e
__global__ __launch_bounds__(BLOCK) void k_keys_init(int32_t* keys, int32_t n) {
  const int32_t i = (int32_t)(blockIdx.x * BLOCK + threadIdx.x);
  if (i < n) {
    keys[2 * i] = 0x7FFFFFFF;
    keys[2 * i + 1] = (int32_t)0x80000000;
  }
}

// the k_group walk (contiguous chunk of 512-element units per wave, TensorCursor over the table);
// per-lane keys folded per wave and merged into the entry's keys by one atomic pair per wave and
// entry touched (min / max of integer order keys: exact and order-independent)
template <int DT, bool SYM>
__global__ __launch_bounds__(BLOCK) void k_tensor_reduce_b(GroupArgs a, int32_t* keys) {
  constexpr int UN = 4;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * WAVES_PER_BLOCK + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
  const int64_t per = (a.total_units + nwaves - 1) / nwaves;
  int64_t u = wave * per;
  const int64_t uend = min(u + per, a.total_units);
  TensorCursor<true> cur;
  cur.init(a);
  int32_t owner = -1, mn = 0x7FFFFFFF, mx = (int32_t)0x80000000;
  auto flush = [&]() {
    group_minmax<64>(mn, mx);
    if (lane == 0) {
      if (!SYM) atomicMin(keys + 2 * owner, mn);
      atomicMax(keys + 2 * owner + 1, mx);
    }
  };
  while (u < uend) {
    cur.seek(a, u);
    if (cur.cur != owner) {
      if (owner >= 0) flush();
      owner = cur.cur;
      mn = 0x7FFFFFFF;
      mx = (int32_t)0x80000000;
    }
    const int64_t lim = min(uend, cur.next);
    for (; u < lim; u += UN) {
      Vec8<DT> v[UN];
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int64_t e = (u + k - cur.begin) * UNIT + (int64_t)lane * 8;
        const bool ok = u + k < lim && e < cur.t.numel;
        v[k].template load<true>(static_cast<const char*>(cur.t.w) + (ok ? e : 0) * Fmt<DT>::BYTES);
      }
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int64_t e = (u + k - cur.begin) * UNIT + (int64_t)lane * 8;
        if (u + k < lim && e < cur.t.numel) {
          int32_t a_mn, a_mx;
          minmax8<DT, SYM>(v[k], a_mn, a_mx);
          mn = min(mn, a_mn);
          mx = max(mx, a_mx);
        }
      }
    }
    u = lim;
  }
  if (owner >= 0) flush();
}

template <int DT, bool SYM, int CODES>
__global__ __launch_bounds__(BLOCK) void k_tensor_apply_b(GroupArgs a, const int32_t* keys) {
  using F = Fmt<DT>;
  constexpr int UN = 4;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * WAVES_PER_BLOCK + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
  const int64_t per = (a.total_units + nwaves - 1) / nwaves;
  int64_t u = wave * per;
  const int64_t uend = min(u + per, a.total_units);
  const float rmax = rmax_for(a.n_bits, SYM);
  TensorCursor<true> cur;
  cur.init(a);
  int32_t owner = -1;
  GroupParams p{};
  bool any_nan = false;
  while (u < uend) {
    cur.seek(a, u);
    if (cur.cur != owner) {
      owner = cur.cur;
      const int32_t kmn = __builtin_amdgcn_readfirstlane(keys[2 * owner]);
      const int32_t kmx = __builtin_amdgcn_readfirstlane(keys[2 * owner + 1]);
      p = params_from_keys<DT, SYM>(kmn, kmx, a.n_bits, rmax);
      if (u == cur.begin && lane == 0) {
        if (cur.t.scales) store_param<DT>(cur.t.scales, 0, p.s);
        if (!SYM && cur.t.zeros) store_param<DT>(cur.t.zeros, 0, p.z);
      }
    }
    const int64_t lim = min(uend, cur.next);
    for (; u < lim; u += UN) {
      Vec8<DT> v[UN];
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int64_t e = (u + k - cur.begin) * UNIT + (int64_t)lane * 8;
        const bool ok = u + k < lim && e < cur.t.numel;
        v[k].template load<true>(static_cast<const char*>(cur.t.w) + (ok ? e : 0) * F::BYTES);
      }
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int64_t e = (u + k - cur.begin) * UNIT + (int64_t)lane * 8;
        if (u + k < lim && e < cur.t.numel) {
          Vec8<DT> o;
          uint32_t c[4];
          any_nan |= quant8<DT, SYM>(v[k], p, a.n_bits, o, c);
          if (cur.t.out) o.template store<true>(static_cast<char*>(cur.t.out) + e * F::BYTES);
          if constexpr (CODES != 0) store_codes8<CODES>(static_cast<uint8_t*>(cur.t.codes), e, c);
        }
      }
    }
    u = lim;
  }
  flag_nan(a.nan_flag, any_nan);
}


// ---- host helpers shared by both translation units ----
bool is_pow2(int64_t x) { return x > 0 && (x & (x - 1)) == 0; }
bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
int elem_bytes(int dt) { return dt == IWQ_F32 ? 4 : 2; }
constexpr int64_t ROW_MAX_L = 32 * 64 * 8;  // 16384 elements held in registers

}  // namespace

// iwq_minmax.hip — gfx950 kernels + C-ABI for min-max weight quantization.
//
// Replaces (reference, /root/reference):
//   quant_funcs.pseudo_quantize_tensor                quant_funcs.py:4-46
//   QuantLinear.quantize_weight INT branch            quant_linear.py:885-956 (quant_dim: :640-647)
//   the per-layer RTN loop of quantize_model          quant_wrapper.py:52-82   (batched entry)
//
// Kernels:
//   k_group    contiguous groups, 8 <= g <= 512 (power of two): 8 elements per lane, a group spans
//              g/8 lanes, min/max by DPP; persistent grid-stride over 512-element units; optional
//              multi-tensor table (whole model in one launch).  HBM-bound, 4 B/elem (fp16 in/out).
//   k_rowwave  one wavefront per long contiguous group (per-channel rows, g > 512), the group
//              held in registers between the reduction and the quantize pass.
//   k_column   quant_dim = 1: groups run down a column; each lane owns 8 adjacent columns and
//              (TY row slices per block) reduces through LDS.
//   k_seg_*    universal path (any layout / length / n_bits): init keys, atomic segmented
//              min/max, apply.  Per-tensor (-1) always uses it.
#include "iwq_common.cuh"
#include "iwq_seg.cuh"
#include "../../include/iwq.h"

#include <stdio.h>
#include <string.h>

using namespace iwq;
using iwq::seg::SegArgs;
using iwq::seg::SEG_RUN;
using iwq::seg::seg_locate;
using iwq::seg::k_seg_init;
using iwq::seg::k_seg_reduce;

int& iwq::last_hip_error() {
  static thread_local int e = 0;
  return e;
}

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

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, CTRL, 0xF, 0xF, false);
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
template <int DT, int G, bool SYM, int CODES, bool BATCHED, int UNROLL, bool PF = false, bool NTL = true,
          bool NTS = true, bool SHARED = true, bool GS = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80))) void k_group(GroupArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * WAVES_PER_BLOCK + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
  const float rmax = rmax_for(a.n_bits, SYM);
  // The walk: contiguous (one chunk [wave*per, +per) per wave) or, with GS, grid-stride chunks of
  // UNROLL units (c*UNROLL for c = wave, wave + nwaves, ...: at any moment the grid works on one
  // contiguous window).  u0 = next unit, cend = end of the current chunk; u0 < cend <=> work left.
  int64_t u0, cend;
  if constexpr (GS) {
    u0 = wave * UNROLL;
    cend = min(u0 + UNROLL, a.total_units);
  } else {
    int64_t per = (a.total_units + nwaves - 1) / nwaves;
    per = (per + UNROLL - 1) / UNROLL * UNROLL;
    u0 = wave * per;
    cend = min(u0 + per, a.total_units);
  }
  auto advance = [&](int64_t n) {
    u0 += n;
    if constexpr (GS) {
      if (u0 >= cend) {
        u0 += (nwaves - 1) * UNROLL;
        cend = min(u0 + UNROLL, a.total_units);
      }
    }
  };
  bool any_nan = false;
  TensorCursor<BATCHED> cursor;
  cursor.init(a);
  auto plan_iter = [&](int64_t u, Iter& it) {
    cursor.seek(a, u);
    const int64_t lim = min(cend, cursor.next);
    it.t = cursor.t;
    it.n = (int32_t)min((int64_t)UNROLL, lim - u);
    it.e0 = (u - cursor.begin) * UNIT + (int64_t)lane * 8;
  };
  auto compute_iter = [&](const Iter& it, const Vec8<DT> (&v)[UNROLL]) {
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
  if constexpr (PF) {
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

template <int DT, bool SYM, int CODES, int TX, int TY>
__global__ __launch_bounds__(TX * TY) void k_column(ColArgs a) {
  using F = Fmt<DT>;
  __shared__ int32_t s_mn[TY][TX * 8];
  __shared__ int32_t s_mx[TY][TX * 8];
  const int tx = threadIdx.x % TX;
  const int ty = threadIdx.x / TX;
  const int64_t c0 = ((int64_t)blockIdx.x * TX + tx) * 8;     // first of this lane's 8 columns
  const int64_t jr = blockIdx.y;                               // group index along rows
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


// k_column_reg: k_column for g = RPT * TY rows per group (g in {32, 64, 128, 256}): every thread
// issues the loads of its RPT rows once, keeps them in registers across the reduction, and the
// block's per-column (min, max) is folded by 64 threads instead of every thread re-reading all
// TY partials (one pass over HBM, no second read of the tile).
template <int DT, bool SYM, int CODES, int TX, int TY, int RPT>
__global__ __launch_bounds__(TX * TY) void k_column_reg(ColArgs a) {
  using F = Fmt<DT>;
  constexpr int NC = TX * 8;  // columns per block
  __shared__ int32_t s_mn[TY][NC];
  __shared__ int32_t s_mx[TY][NC];
  __shared__ GroupParams f_p[NC];
  const int tx = threadIdx.x % TX;
  const int ty = threadIdx.x / TX;
  const int64_t c0 = ((int64_t)blockIdx.x * TX + tx) * 8;
  const int64_t jr = blockIdx.y;
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
  for (int i = 0; i < 8; ++i) { s_mn[ty][tx * 8 + i] = mn[i]; s_mx[ty][tx * 8 + i] = mx[i]; }
  __syncthreads();
  // one thread per column folds the TY partials AND derives the group's parameters once (not once
  // per row slice: 8x less parameter math at TY = 8), shared through LDS
  for (int cc = threadIdx.x; cc < NC; cc += TX * TY) {  // NC > threads for the 64 x 4 shape
    int32_t a_mn = 0x7FFFFFFF, a_mx = (int32_t)0x80000000;
#pragma unroll 8
    for (int y = 0; y < TY; ++y) { a_mn = min(a_mn, s_mn[y][cc]); a_mx = max(a_mx, s_mx[y][cc]); }
    const GroupParams q = params_from_keys<DT, SYM>(a_mn, a_mx, a.n_bits, rmax_for(a.n_bits, SYM));
    f_p[cc] = q;
    const int64_t col = (int64_t)blockIdx.x * NC + cc;
    if (col < a.cols) {
      const int64_t gidx = col * (a.rows / a.g) + jr;
      if (a.scales) store_param<DT>(a.scales, gidx, q.s);
      if (!SYM && a.zeros) store_param<DT>(a.zeros, gidx, q.z);
    }
  }
  __syncthreads();
  GroupParams p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] = f_p[tx * 8 + i];
  bool any_nan = false;
  if (cvalid) {
    const uint32_t off = SYM ? (1u << (a.n_bits - 1)) : 0u;
    if constexpr (DT == DT_F16) {
      // all 8 columns of this thread on the fast path: packed pairs with per-half group operands
      bool fast = a.n_bits <= 9;
#pragma unroll
      for (int i = 0; i < 8; ++i) fast = fast && p[i].fast;
      if (fast) {
        BiasedPair bp[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) bp[jj] = biased_pair<SYM>(p[2 * jj], p[2 * jj + 1], a.n_bits);
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
// host-side dispatch
// =============================================================================================
bool is_pow2(int64_t x) { return x > 0 && (x & (x - 1)) == 0; }
bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
int elem_bytes(int dt) { return dt == IWQ_F32 ? 4 : 2; }

// Walk policy, picked by cold in-run A/B (tools/ab_single.py rotating over >= 1 GB of distinct
// tensors, bench.py --variants; profiles/r01_ab_*):
//  * whole-model batched walk (hundreds of iterations per wave): contiguous chunk per wave, no
//    prefetch (grid-stride: 4.68 vs 4.40 ms per 7B);
//  * single fp16 tensors of >= 2 grid-rounds (11008x4096: 34.3 vs 36.8 us): grid-stride chunks;
//  * smaller single tensors (4096x4096, ~1 round): contiguous chunk with the next iteration's
//    loads prefetched (14.2 vs 15.1 us).
// All with non-temporal loads.
template <typename Kern>
hipError_t launch_persistent(Kern kern, int* cache, int unroll, const GroupArgs& a, hipStream_t st) {
  const int64_t waves_needed = (a.total_units + unroll - 1) / unroll;
  int64_t blocks = (waves_needed + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  const int64_t cap = (int64_t)device_cu_count() * resident_blocks_per_cu(kern, cache);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}

template <int DT, int G, bool SYM, int CODES, bool BATCHED>
hipError_t launch_group_t(const GroupArgs& a, hipStream_t st) {
  constexpr int UNROLL = 4;
  static int cache[64] = {0};
  auto kern = k_group<DT, G, SYM, CODES, BATCHED, UNROLL, /*PF*/ !BATCHED, /*NTL*/ true>;
  if constexpr (!BATCHED && DT == DT_F16) {
    static int cache_gs[64] = {0};
    auto kern_gs = k_group<DT, G, SYM, CODES, false, UNROLL, /*PF*/ false, /*NTL*/ true, /*NTS*/ true,
                           /*SHARED*/ true, /*GS*/ true>;
    const int64_t round_units =
        (int64_t)device_cu_count() * resident_blocks_per_cu(kern_gs, cache_gs) * WAVES_PER_BLOCK * UNROLL;
    if (a.total_units >= 2 * round_units) return launch_persistent(kern_gs, cache_gs, UNROLL, a, st);
  }
  return launch_persistent(kern, cache, UNROLL, a, st);
}

// Tuning variants of the headline configuration (fp16, g=128, asymmetric, no codes, batched),
// selected by flags bits 16..23 for in-process A/B timing (bench.py --variants).
template <int UNROLL, bool PF, bool NTL, bool NTS, bool SHARED = true, bool GS = false>
hipError_t launch_variant_t(const GroupArgs& a, hipStream_t st, int max_blocks_per_cu = 8) {
  static int cache[64] = {0};
  auto kern = k_group<DT_F16, 128, false, 0, true, UNROLL, PF, NTL, NTS, SHARED, GS>;
  const int64_t waves_needed = (a.total_units + UNROLL - 1) / UNROLL;
  int64_t blocks = (waves_needed + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  const int per_cu = resident_blocks_per_cu(kern, cache);
  const int64_t cap = (int64_t)device_cu_count() * (per_cu < max_blocks_per_cu ? per_cu : max_blocks_per_cu);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}
// Roofline probes (variants >= 100): the same bytes moved without arithmetic, to measure the
// achievable HBM rate of a given access style on the box at hand.  Timing reference only.
//   MODE 0: copy, nt load + nt store     MODE 1: copy, plain       MODE 2: copy, 4 x 16 B in flight/lane (nt)
//   MODE 3: read only (xor-reduce)       MODE 4: write only (nt)
//   k_probe_pol<POL, COPY>: write-only (COPY false) or nt-load copy (COPY true) with the store's
//   cache policy POL: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 nt sc1, 5 sc0 sc1 nt (vector stores only).
template <int POL>
__device__ __forceinline__ void store_pol(IWQ_GLOBAL u32x4* p, u32x4 v) {
  if constexpr (POL == 0) *p = v;
  else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
  else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}
template <int POL, bool COPY>
__global__ __launch_bounds__(BLOCK) void k_probe_pol(const iwq_batch_entry* entries, int32_t n) {
  for (int32_t i = 0; i < n; ++i) {
    const IWQ_GLOBAL iwq_batch_entry* tab = gp<iwq_batch_entry>(entries);
    const int64_t nvec = tab[i].rows * tab[i].cols / 8;
    const IWQ_GLOBAL u32x4* src = gp<u32x4>(tab[i].w);
    IWQ_GLOBAL u32x4* dst = gp<u32x4>(tab[i].out_deq);
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < nvec; j += stride) {
      if constexpr (COPY) store_pol<POL>(dst + j, __builtin_nontemporal_load(src + j));
      else store_pol<POL>(dst + j, (u32x4){(uint32_t)j, 0u, 0u, 0u});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_probe(const iwq_batch_entry* entries, int32_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (int32_t i = 0; i < n; ++i) {
    const IWQ_GLOBAL iwq_batch_entry* tab = gp<iwq_batch_entry>(entries);
    const int64_t nvec = tab[i].rows * tab[i].cols / 8;
    const IWQ_GLOBAL u32x4* src = gp<u32x4>(tab[i].w);
    IWQ_GLOBAL u32x4* dst = gp<u32x4>(tab[i].out_deq);
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    const int64_t t0 = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if constexpr (MODE == 2) {
      int64_t j = t0;
      for (; j + 3 * stride < nvec; j += 4 * stride) {
        u32x4 a0 = __builtin_nontemporal_load(src + j), a1 = __builtin_nontemporal_load(src + j + stride);
        u32x4 a2 = __builtin_nontemporal_load(src + j + 2 * stride), a3 = __builtin_nontemporal_load(src + j + 3 * stride);
        __builtin_nontemporal_store(a0, dst + j);
        __builtin_nontemporal_store(a1, dst + j + stride);
        __builtin_nontemporal_store(a2, dst + j + 2 * stride);
        __builtin_nontemporal_store(a3, dst + j + 3 * stride);
      }
      for (; j < nvec; j += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + j), dst + j);
    } else {
      for (int64_t j = t0; j < nvec; j += stride) {
        if constexpr (MODE == 0) __builtin_nontemporal_store(__builtin_nontemporal_load(src + j), dst + j);
        if constexpr (MODE == 1) dst[j] = src[j];
        if constexpr (MODE == 3) { u32x4 x = __builtin_nontemporal_load(src + j); acc ^= x.x ^ x.y ^ x.z ^ x.w; }
        if constexpr (MODE == 4) __builtin_nontemporal_store((u32x4){(uint32_t)j, 0u, 0u, 0u}, dst + j);
      }
    }
  }
  if (MODE == 3 && acc == 0x12345678u) sink[0] = acc;
}

hipError_t launch_variant(int v, const GroupArgs& a, hipStream_t st) {
  switch (v) {
    case 1: return launch_variant_t<4, true, true, true>(a, st);
    case 2: return launch_variant_t<4, true, false, true>(a, st);
    case 3: return launch_variant_t<4, false, true, true, false>(a, st);   // per-unit parameters (r1 default)
    case 4: return launch_variant_t<2, true, true, true>(a, st);
    case 5: return launch_variant_t<4, false, true, true, true, true>(a, st);   // grid-stride walk
    case 6: return launch_variant_t<4, true, true, true, true, true>(a, st);    // grid-stride + prefetch
    case 7: return launch_variant_t<2, true, true, true, true, true>(a, st);    // grid-stride, UNROLL 2, prefetch
    case 8: return launch_variant_t<1, true, true, true, true, true>(a, st);    // grid-stride, UNROLL 1, prefetch
    case 9: return launch_variant_t<4, false, true, true>(a, st, 7);            // default kernel, 7 waves/SIMD
    case 10: return launch_variant_t<4, false, true, true>(a, st, 6);           // default kernel, 6 waves/SIMD
    case 11: return launch_variant_t<4, false, true, true>(a, st, 4);           // default kernel, 4 waves/SIMD
    case 12: return launch_variant_t<4, false, true, true>(a, st, 8);           // default kernel (same as 0)
    case 13: return launch_variant_t<4, false, true, false>(a, st);             // default walk, plain stores
    case 14: return launch_variant_t<4, false, false, false>(a, st);            // plain loads + plain stores
    case 100: hipLaunchKernelGGL(k_probe<0>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 101: hipLaunchKernelGGL(k_probe<1>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 102: hipLaunchKernelGGL(k_probe<2>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 103: hipLaunchKernelGGL(k_probe<3>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 104: hipLaunchKernelGGL(k_probe<4>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 105: hipLaunchKernelGGL(k_probe<0>, dim3((unsigned)(device_cu_count() * 32)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
#define IWQ_PROBE_POL(V, POL, COPY)                                                                  \
  case V: hipLaunchKernelGGL((k_probe_pol<POL, COPY>), dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, \
                             a.entries, a.n_entries); return hipGetLastError();
    IWQ_PROBE_POL(106, 0, false) IWQ_PROBE_POL(107, 1, false) IWQ_PROBE_POL(108, 2, false)
    IWQ_PROBE_POL(109, 3, false) IWQ_PROBE_POL(110, 4, false) IWQ_PROBE_POL(111, 5, false)
    IWQ_PROBE_POL(112, 0, true) IWQ_PROBE_POL(113, 1, true) IWQ_PROBE_POL(114, 2, true)
    IWQ_PROBE_POL(115, 3, true) IWQ_PROBE_POL(116, 4, true) IWQ_PROBE_POL(117, 5, true)
#undef IWQ_PROBE_POL
  }
  return hipErrorInvalidValue;
}

template <int DT, bool SYM, int CODES, bool BATCHED>
hipError_t launch_group_g(int64_t g, const GroupArgs& a, hipStream_t st) {
  switch (g) {
    case 8: return launch_group_t<DT, 8, SYM, CODES, BATCHED>(a, st);
    case 16: return launch_group_t<DT, 16, SYM, CODES, BATCHED>(a, st);
    case 32: return launch_group_t<DT, 32, SYM, CODES, BATCHED>(a, st);
    case 64: return launch_group_t<DT, 64, SYM, CODES, BATCHED>(a, st);
    case 128: return launch_group_t<DT, 128, SYM, CODES, BATCHED>(a, st);
    case 256: return launch_group_t<DT, 256, SYM, CODES, BATCHED>(a, st);
    case 512: return launch_group_t<DT, 512, SYM, CODES, BATCHED>(a, st);
  }
  return hipErrorInvalidValue;
}

template <bool BATCHED>
hipError_t launch_group(int dt, int64_t g, bool sym, int codes, const GroupArgs& a, hipStream_t st) {
#define IWQ_G_CODES(DT, SYM)                                                          \
  switch (codes) {                                                                    \
    case 0: return launch_group_g<DT, SYM, 0, BATCHED>(g, a, st);                     \
    case 4: return launch_group_g<DT, SYM, 4, BATCHED>(g, a, st);                     \
    default: return launch_group_g<DT, SYM, 8, BATCHED>(g, a, st);                    \
  }
  if (dt == IWQ_F16) { if (sym) { IWQ_G_CODES(DT_F16, true) } else { IWQ_G_CODES(DT_F16, false) } }
  if (dt == IWQ_BF16) { if (sym) { IWQ_G_CODES(DT_BF16, true) } else { IWQ_G_CODES(DT_BF16, false) } }
  if (sym) { IWQ_G_CODES(DT_F32, true) } else { IWQ_G_CODES(DT_F32, false) }
#undef IWQ_G_CODES
}

template <int DT, int CPL, bool SYM, int CODES>
hipError_t launch_row_pf(const RowArgs& a, hipStream_t st) {
  static int cache[64] = {0};
  auto kern = k_rowwave_pf<DT, CPL, SYM, CODES>;
  int64_t blocks = (a.G + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  const int64_t cap = (int64_t)device_cu_count() * resident_blocks_per_cu(kern, cache);
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}

template <int DT, int CPL, bool SYM>
hipError_t launch_row_t(int codes, const RowArgs& a, hipStream_t st) {
  if constexpr (CPL <= 8 && DT != DT_F32) {
    // persistent + prefetch once the groups overflow one resident grid (~8k waves)
    if (a.G > (int64_t)device_cu_count() * 8 * WAVES_PER_BLOCK) {
      if (codes == 0) return launch_row_pf<DT, CPL, SYM, 0>(a, st);
      if (codes == 4) return launch_row_pf<DT, CPL, SYM, 4>(a, st);
      return launch_row_pf<DT, CPL, SYM, 8>(a, st);
    }
  }
  const int64_t blocks = (a.G + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  if (codes == 0) hipLaunchKernelGGL((k_rowwave<DT, CPL, SYM, 0>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  else if (codes == 4) hipLaunchKernelGGL((k_rowwave<DT, CPL, SYM, 4>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  else hipLaunchKernelGGL((k_rowwave<DT, CPL, SYM, 8>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}

template <int DT, bool SYM>
hipError_t launch_row_c(int codes, const RowArgs& a, hipStream_t st) {
  const int64_t chunks = a.L / 8;
  if (chunks <= 64 * 1) return launch_row_t<DT, 1, SYM>(codes, a, st);
  if (chunks <= 64 * 2) return launch_row_t<DT, 2, SYM>(codes, a, st);
  if (chunks <= 64 * 4) return launch_row_t<DT, 4, SYM>(codes, a, st);
  if (chunks <= 64 * 8) return launch_row_t<DT, 8, SYM>(codes, a, st);
  if (chunks <= 64 * 12) return launch_row_t<DT, 12, SYM>(codes, a, st);
  if (chunks <= 64 * 16) return launch_row_t<DT, 16, SYM>(codes, a, st);
  if (chunks <= 64 * 24) return launch_row_t<DT, 24, SYM>(codes, a, st);
  return launch_row_t<DT, 32, SYM>(codes, a, st);
}
constexpr int64_t ROW_MAX_L = 32 * 64 * 8;  // 16384 elements held in registers

hipError_t launch_row(int dt, bool sym, int codes, const RowArgs& a, hipStream_t st) {
  if (dt == IWQ_F16) return sym ? launch_row_c<DT_F16, true>(codes, a, st) : launch_row_c<DT_F16, false>(codes, a, st);
  if (dt == IWQ_BF16) return sym ? launch_row_c<DT_BF16, true>(codes, a, st) : launch_row_c<DT_BF16, false>(codes, a, st);
  return sym ? launch_row_c<DT_F32, true>(codes, a, st) : launch_row_c<DT_F32, false>(codes, a, st);
}

// Block = TX column chunks (8 columns, 16 B each) x TY row slices.  Default 32 x 8 (512-B row
// segments; 16 x 16 at g = 256 to bound registers), picked by tools/ab_col.py (profiles/r01_ab_col.jsonl:
// 11008x4096 g=128 39.1 us vs 41.2 for the r1 8 x 32 shape, g=32 45.3 vs 67.7).  flags variant
// 1 = 8 x 32, 2 = 32 x 8, 3 = 16 x 16.
template <int DT, bool SYM, int CODES, int TX, int TY>
hipError_t launch_col_t(const ColArgs& a, hipStream_t st) {
  dim3 grid((unsigned)((a.cols + 8 * TX - 1) / (8 * TX)), (unsigned)(a.rows / a.g));
  static_assert(32 % TY == 0, "k_column_reg needs g % TY == 0 for g >= 32");
  const dim3 blk(TX * TY);
  if (a.g == 32) hipLaunchKernelGGL((k_column_reg<DT, SYM, CODES, TX, TY, 32 / TY>), grid, blk, 0, st, a);
  else if (a.g == 64) hipLaunchKernelGGL((k_column_reg<DT, SYM, CODES, TX, TY, 64 / TY>), grid, blk, 0, st, a);
  else if (a.g == 128) hipLaunchKernelGGL((k_column_reg<DT, SYM, CODES, TX, TY, 128 / TY>), grid, blk, 0, st, a);
  else if (a.g == 256) hipLaunchKernelGGL((k_column_reg<DT, SYM, CODES, TX, TY, 256 / TY>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((k_column<DT, SYM, CODES, TX, TY>), grid, blk, 0, st, a);
  return hipGetLastError();
}
// 64 column chunks x 4 row slices (1 KiB row segments; g / 4 rows per thread): short groups only
template <int DT, bool SYM, int CODES>
hipError_t launch_col_wide(const ColArgs& a, hipStream_t st) {
  constexpr int TX = 64, TY = 4;
  dim3 grid((unsigned)((a.cols + 8 * TX - 1) / (8 * TX)), (unsigned)(a.rows / a.g));
  if (a.g == 32) hipLaunchKernelGGL((k_column_reg<DT, SYM, CODES, TX, TY, 8>), grid, dim3(TX * TY), 0, st, a);
  else hipLaunchKernelGGL((k_column_reg<DT, SYM, CODES, TX, TY, 16>), grid, dim3(TX * TY), 0, st, a);
  return hipGetLastError();
}
template <int DT, bool SYM, int CODES>
hipError_t launch_col_v(int variant, const ColArgs& a, hipStream_t st) {
  if constexpr (DT == DT_F16) {  // g = 32: 1 KiB row segments win (cold 11008x4096 44.7 -> 41.0 us);
                                 // g = 64: 37.7 -> 39.4 us, so only as variant 4 (r01_ab_col_wide.jsonl)
    if ((variant == 4 && a.g == 64) || ((variant == 0 || variant == 4) && a.g == 32))
      return launch_col_wide<DT, SYM, CODES>(a, st);
  }
  if (variant == 1) return launch_col_t<DT, SYM, CODES, 8, 32>(a, st);
  if (variant == 2) return launch_col_t<DT, SYM, CODES, 32, 8>(a, st);
  if (variant == 3 || a.g == 256) return launch_col_t<DT, SYM, CODES, 16, 16>(a, st);  // 16 rows/thread at g=256
  return launch_col_t<DT, SYM, CODES, 32, 8>(a, st);
}
template <int DT, bool SYM>
hipError_t launch_col_c(int codes, int variant, const ColArgs& a, hipStream_t st) {
  if (codes == 0) return launch_col_v<DT, SYM, 0>(variant, a, st);
  if (codes == 4) return launch_col_v<DT, SYM, 4>(variant, a, st);
  return launch_col_v<DT, SYM, 8>(variant, a, st);
}
hipError_t launch_col(int dt, bool sym, int codes, int variant, const ColArgs& a, hipStream_t st) {
  if (dt == IWQ_F16)
    return sym ? launch_col_c<DT_F16, true>(codes, variant, a, st) : launch_col_c<DT_F16, false>(codes, variant, a, st);
  if (dt == IWQ_BF16)
    return sym ? launch_col_c<DT_BF16, true>(codes, variant, a, st) : launch_col_c<DT_BF16, false>(codes, variant, a, st);
  return sym ? launch_col_c<DT_F32, true>(codes, variant, a, st) : launch_col_c<DT_F32, false>(codes, variant, a, st);
}

template <int DT, bool SYM>
hipError_t launch_seg_t(const SegArgs& a, hipStream_t st) {
  const int64_t cap = (int64_t)device_cu_count() * 8;
  int64_t ib = (a.G + BLOCK - 1) / BLOCK;
  if (ib > cap) ib = cap;
  hipLaunchKernelGGL(k_seg_init, dim3((unsigned)ib), dim3(BLOCK), 0, st, a.keys, a.G);
  int64_t blocks = (a.total + (int64_t)BLOCK * SEG_RUN - 1) / ((int64_t)BLOCK * SEG_RUN);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((k_seg_reduce<DT, SYM>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  hipLaunchKernelGGL((k_seg_apply<DT, SYM>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_seg(int dt, bool sym, const SegArgs& a, hipStream_t st) {
  if (dt == IWQ_F16) return sym ? launch_seg_t<DT_F16, true>(a, st) : launch_seg_t<DT_F16, false>(a, st);
  if (dt == IWQ_BF16) return sym ? launch_seg_t<DT_BF16, true>(a, st) : launch_seg_t<DT_BF16, false>(a, st);
  return sym ? launch_seg_t<DT_F32, true>(a, st) : launch_seg_t<DT_F32, false>(a, st);
}


constexpr int TENSOR_PARTS_MAX = 4096;

// Per-tensor variants (flags bits 16..23; profiles/r01_ab_tensor.jsonl):
//   0/2: temporal loads in both passes (default: cold 11008x4096 51.1 -> 49.0 us, 4096^2 22.6 -> 20.0 us)
//   1: non-temporal loads in both passes (the previous default)
//   3: temporal loads, apply walks the tensor backwards (the most recently read units first): no gain
//   4 / 5: apply with 4 / 2 units in flight per thread: within +-2.5 % (profiles/r01_ab_tensor_unroll.jsonl)
template <int DT, bool SYM, int CODES, bool NTL, bool REV, int UN = 1>
void launch_tensor_pair(const void* w, void* out, void* codes, void* scales, void* zeros, int64_t nunits,
                        int64_t blocks, int32_t* ws, int n_bits, uint32_t* nan_flag, hipStream_t st) {
  hipLaunchKernelGGL((k_tensor_reduce<DT, SYM, NTL>), dim3((unsigned)blocks), dim3(BLOCK), 0, st,
                     static_cast<const char*>(w), nunits, ws);
  hipLaunchKernelGGL((k_tensor_apply<DT, SYM, CODES, NTL, REV, UN>), dim3((unsigned)blocks), dim3(BLOCK), 0, st,
                     static_cast<const char*>(w), static_cast<char*>(out), static_cast<uint8_t*>(codes), scales,
                     zeros, nunits, ws, (int)blocks, n_bits, nan_flag);
}

template <int DT, bool SYM, int CODES>
hipError_t launch_tensor_t(const void* w, void* out, void* codes, void* scales, void* zeros, int64_t numel,
                           int32_t* ws, int n_bits, uint32_t* nan_flag, hipStream_t st, int variant) {
  const int64_t nunits = numel / 8;
  int64_t blocks = (int64_t)device_cu_count() * 8;
  const int64_t need = (nunits + BLOCK - 1) / BLOCK;
  if (blocks > need) blocks = need;
  if (blocks > TENSOR_PARTS_MAX) blocks = TENSOR_PARTS_MAX;
  if (blocks < 1) blocks = 1;
  if (variant == 1)
    launch_tensor_pair<DT, SYM, CODES, true, false>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else if (variant == 3)
    launch_tensor_pair<DT, SYM, CODES, false, true>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else if (variant == 4)
    launch_tensor_pair<DT, SYM, CODES, false, false, 4>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else if (variant == 5)
    launch_tensor_pair<DT, SYM, CODES, false, false, 2>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else
    launch_tensor_pair<DT, SYM, CODES, false, false>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  return hipGetLastError();
}

template <int DT, bool SYM>
hipError_t launch_tensor_c(int codes, const void* w, void* out, void* cd, void* sc, void* zr, int64_t numel,
                           int32_t* ws, int n_bits, uint32_t* nan_flag, hipStream_t st, int v) {
  if (codes == 0) return launch_tensor_t<DT, SYM, 0>(w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v);
  if (codes == 4) return launch_tensor_t<DT, SYM, 4>(w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v);
  return launch_tensor_t<DT, SYM, 8>(w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v);
}

hipError_t launch_tensor(int dt, bool sym, int codes, const void* w, void* out, void* cd, void* sc, void* zr,
                         int64_t numel, int32_t* ws, int n_bits, uint32_t* nan_flag, hipStream_t st, int v) {
  if (dt == IWQ_F16)
    return sym ? launch_tensor_c<DT_F16, true>(codes, w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v)
               : launch_tensor_c<DT_F16, false>(codes, w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v);
  if (dt == IWQ_BF16)
    return sym ? launch_tensor_c<DT_BF16, true>(codes, w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v)
               : launch_tensor_c<DT_BF16, false>(codes, w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v);
  return sym ? launch_tensor_c<DT_F32, true>(codes, w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v)
             : launch_tensor_c<DT_F32, false>(codes, w, out, cd, sc, zr, numel, ws, n_bits, nan_flag, st, v);
}

int group_geometry(int64_t rows, int64_t cols, int64_t group, int quant_dim, int64_t& L, int64_t& G) {
  const int64_t vr = quant_dim == 1 ? cols : rows;
  const int64_t vc = quant_dim == 1 ? rows : cols;
  if (group > 0) {
    if (vc % group != 0) return IWQ_ERR_GROUP;
    L = group;
    G = vr * vc / group;
  } else if (group == IWQ_GROUP_PER_TENSOR) {
    L = vr * vc;
    G = 1;
  } else if (group == IWQ_GROUP_PER_CHANNEL) {
    L = vc;
    G = vr;
  } else {
    return IWQ_ERR_GROUP_MODE;
  }
  return IWQ_OK;
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

int64_t iwq_workspace_bytes(int64_t rows, int64_t cols, int64_t group, int quant_dim) {
  int64_t L = 0, G = 0;
  if (rows <= 0 || cols <= 0) return 0;
  if (group_geometry(rows, cols, group, quant_dim, L, G) != IWQ_OK) return 0;
  if (group == IWQ_GROUP_PER_TENSOR) return (int64_t)TENSOR_PARTS_MAX * 8;  // per-workgroup partial keys
  return ((8 * G + 255) / 256) * 256;
}

int iwq_quantize_minmax(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int n_bits,
                        int64_t group, int symmetric, int quant_dim, void* out_deq, int64_t ld_out,
                        void* out_codes, void* out_scales, void* out_zeros, void* workspace,
                        int64_t workspace_bytes, uint32_t* nan_flag, unsigned flags, void* stream) {
  if (dtype != IWQ_F16 && dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (!w) return IWQ_ERR_ARG;
  if (rows <= 0 || cols <= 0 || ld_w < cols || (out_deq && ld_out < cols)) return IWQ_ERR_SHAPE;
  if (quant_dim != 0 && quant_dim != 1) return IWQ_ERR_ARG;
  if (n_bits < 1 || n_bits > 24) return IWQ_ERR_BITS;
  if (symmetric && n_bits < 2) return IWQ_ERR_BITS;
  int64_t L = 0, G = 0;
  int st = group_geometry(rows, cols, group, quant_dim, L, G);
  if (st != IWQ_OK) return st;
  int codes = 0;
  if (out_codes) {
    if (n_bits > 8) return IWQ_ERR_CODES;
    codes = n_bits <= 4 ? 4 : 8;
    if (codes == 4 && (cols & 1)) return IWQ_ERR_CODES;
  }
  const bool sym = symmetric != 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int eb = elem_bytes(dtype);
  const bool generic = (flags & IWQ_FLAG_FORCE_GENERIC) != 0;
  const bool al = aligned16(w) && (!out_deq || aligned16(out_deq)) && (ld_w * eb) % 16 == 0 &&
                  (!out_deq || (ld_out * eb) % 16 == 0) && (!out_codes || aligned16(out_codes));
  const bool fastbits = n_bits <= 8;

  if (!generic && quant_dim == 0 && group > 0 && group >= 8 && group <= 512 && is_pow2(group) && al &&
      fastbits && ld_w == cols && (!out_deq || ld_out == cols)) {
    GroupArgs a{};
    a.single = GroupTensor{w, out_deq, out_codes, out_scales, sym ? nullptr : out_zeros, rows * cols};
    a.total_units = (rows * cols + UNIT - 1) / UNIT;
    a.n_entries = 1;
    a.n_bits = n_bits;
    a.nan_flag = nan_flag;
    IWQ_HIP(launch_group<false>(dtype, group, sym, codes, a, s));
    return IWQ_OK;
  }
  if (!generic && group == IWQ_GROUP_PER_TENSOR && al && fastbits && ld_w == cols &&
      (!out_deq || ld_out == cols) && (rows * cols) % 8 == 0) {
    const int64_t need = iwq_workspace_bytes(rows, cols, group, quant_dim);
    if (!workspace || workspace_bytes < need || !aligned16(workspace)) return IWQ_ERR_WORKSPACE;
    IWQ_HIP(launch_tensor(dtype, sym, codes, w, out_deq, out_codes, out_scales, sym ? nullptr : out_zeros,
                          rows * cols, static_cast<int32_t*>(workspace), n_bits, nan_flag, s,
                          (int)((flags >> 16) & 0xFFu)));
    return IWQ_OK;
  }
  if (!generic && quant_dim == 0 && group != IWQ_GROUP_PER_TENSOR && L % 8 == 0 && L <= ROW_MAX_L && al && fastbits) {
    RowArgs a{};
    a.w = static_cast<const char*>(w);
    a.out = static_cast<char*>(out_deq);
    a.codes = static_cast<uint8_t*>(out_codes);
    a.scales = out_scales;
    a.zeros = sym ? nullptr : out_zeros;
    a.ld_w = ld_w;
    a.ld_out = ld_out;
    a.cols = cols;
    a.L = L;
    a.gpr = cols / L;
    a.G = G;
    a.n_bits = n_bits;
    a.nan_flag = nan_flag;
    IWQ_HIP(launch_row(dtype, sym, codes, a, s));
    return IWQ_OK;
  }
  if (!generic && quant_dim == 1 && group != IWQ_GROUP_PER_TENSOR && cols % 8 == 0 && al && fastbits) {
    ColArgs a{};
    a.w = static_cast<const char*>(w);
    a.out = static_cast<char*>(out_deq);
    a.codes = static_cast<uint8_t*>(out_codes);
    a.scales = out_scales;
    a.zeros = sym ? nullptr : out_zeros;
    a.rows = rows;
    a.cols = cols;
    a.ld_w = ld_w;
    a.ld_out = ld_out;
    a.g = L;  // rows per group (L = group, or rows for per-channel)
    a.n_bits = n_bits;
    a.nan_flag = nan_flag;
    IWQ_HIP(launch_col(dtype, sym, codes, (int)((flags >> 16) & 0xFFu), a, s));
    return IWQ_OK;
  }
  // universal path
  const int64_t need = iwq_workspace_bytes(rows, cols, group, quant_dim);
  if (!workspace || workspace_bytes < need || !aligned16(workspace)) return IWQ_ERR_WORKSPACE;
  if (codes == 4) {
    const int64_t nbytes = rows * (cols / 2);
    if ((reinterpret_cast<uintptr_t>(out_codes) & 3u) != 0) return IWQ_ERR_ARG;
    IWQ_HIP(hipMemsetAsync(out_codes, 0, (size_t)nbytes, s));
  }
  SegArgs a{};
  a.w = static_cast<const char*>(w);
  a.out = static_cast<char*>(out_deq);
  a.codes = static_cast<uint8_t*>(out_codes);
  a.scales = out_scales;
  a.zeros = sym ? nullptr : out_zeros;
  a.keys = static_cast<int32_t*>(workspace);
  a.rows = rows;
  a.cols = cols;
  a.ld_w = ld_w;
  a.ld_out = ld_out;
  a.vc = quant_dim == 1 ? rows : cols;
  a.L = L;
  a.G = G;
  a.total = rows * cols;
  a.quant_dim = quant_dim;
  a.n_bits = n_bits;
  a.codes_bits = codes;
  a.nan_flag = nan_flag;
  IWQ_HIP(launch_seg(dtype, sym, a, s));
  return IWQ_OK;
}

int iwq_batch_plan(iwq_batch_entry* h_entries, int32_t n_entries, int dtype, int n_bits, int64_t group,
                   int64_t* h_total_units) {
  if (!h_entries || n_entries <= 0 || !h_total_units) return IWQ_ERR_ARG;
  if (dtype != IWQ_F16 && dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (n_bits < 2 || n_bits > 8) return IWQ_ERR_BITS;
  if (!(group >= 8 && group <= 512 && is_pow2(group))) return IWQ_ERR_GROUP_MODE;
  int64_t u = 0;
  for (int32_t i = 0; i < n_entries; ++i) {
    iwq_batch_entry& e = h_entries[i];
    if (!e.w || e.rows <= 0 || e.cols <= 0) return IWQ_ERR_SHAPE;
    if (e.cols % group != 0) return IWQ_ERR_GROUP;
    if (!aligned16(e.w) || (e.out_deq && !aligned16(e.out_deq)) || (e.out_codes && !aligned16(e.out_codes)))
      return IWQ_ERR_ARG;
    if (e.out_codes && n_bits <= 4 && (e.cols & 1)) return IWQ_ERR_CODES;
    e.unit_begin = u;
    u += (e.rows * e.cols + UNIT - 1) / UNIT;
  }
  *h_total_units = u;
  return IWQ_OK;
}

int iwq_quantize_minmax_batched(const iwq_batch_entry* d_entries, int32_t n_entries, int64_t total_units,
                                int dtype, int n_bits, int64_t group, int symmetric, uint32_t* nan_flag,
                                unsigned flags, void* stream) {
  if (!d_entries || n_entries <= 0 || total_units <= 0) return IWQ_ERR_ARG;
  if (dtype != IWQ_F16 && dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (n_bits < 2 || n_bits > 8) return IWQ_ERR_BITS;
  if (!(group >= 8 && group <= 512 && is_pow2(group))) return IWQ_ERR_GROUP_MODE;
  (void)flags;
  GroupArgs a{};
  a.entries = d_entries;
  a.n_entries = n_entries;
  a.total_units = total_units;
  a.n_bits = n_bits;
  a.nan_flag = nan_flag;
  // the codes width is a template parameter and the entries are device-resident, so the caller
  // states with IWQ_FLAG_BATCH_CODES that every entry carries out_codes.
  const int codes = (flags & IWQ_FLAG_BATCH_CODES) ? (n_bits <= 4 ? 4 : 8) : 0;
  const int variant = (int)((flags >> 16) & 0xFFu);
  if (variant != 0 && dtype == IWQ_F16 && group == 128 && !symmetric && codes == 0) {
    IWQ_HIP(launch_variant(variant, a, static_cast<hipStream_t>(stream)));
    return IWQ_OK;
  }
  IWQ_HIP(launch_group<true>(dtype, group, symmetric != 0, codes, a, static_cast<hipStream_t>(stream)));
  return IWQ_OK;
}

const char* iwq_status_string(int status) {
  switch (status) {
    case IWQ_OK: return "ok";
    case IWQ_ERR_SHAPE: return "bad shape";
    case IWQ_ERR_GROUP: return "last dimension not divisible by group size";
    case IWQ_ERR_GROUP_MODE: return "Invalid w_group_size";
    case IWQ_ERR_BITS: return "unsupported n_bits";
    case IWQ_ERR_DTYPE: return "unsupported dtype";
    case IWQ_ERR_WORKSPACE: return "workspace missing or too small";
    case IWQ_ERR_CODES: return "codes output unsupported for this n_bits / shape";
    case IWQ_ERR_HIP: return "HIP runtime error";
    case IWQ_ERR_ARG: return "bad argument";
    case IWQ_ERR_FORMAT: return "value cannot be converted to type c10::Half without overflow";
  }
  return "unknown status";
}

int iwq_last_hip_error(void) { return iwq::last_hip_error(); }

}  // extern "C"

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
//              min/max, apply.
// The kernels themselves live in iwq_minmax.cuh (shared with iwq_batched.hip, the batched-table
// launches for the other group modes); this file holds their host dispatch and the C-ABI.
#include "iwq_minmax.cuh"

int& iwq::last_hip_error() {
  static thread_local int e = 0;
  return e;
}


namespace {

// =============================================================================================
// host-side dispatch
// =============================================================================================

// Walk policy, picked by cold in-run A/B (tools/ab_single.py rotating over >= 1 GB of distinct
// tensors, bench.py --variants; profiles/r01_ab_*):
//  * whole-model batched walk (hundreds of iterations per wave): no prefetch (grid-stride: 4.68 vs
//    4.40 ms per 7B); round 6: the REGION walk, 256 consecutive waves share one contiguous region and
//    take its 4-unit chunks round-robin (RW = 256: 32 regions at 8192 waves), instead of one contiguous
//    chunk per wave -- +1...+3.5 % on every output placement measured, most where the placement is
//    slow (tools/ab_outplace.py, profiles/r06_ab_outplace_regions.jsonl / r06_ab_outplace_rw.jsonl:
//    per-tensor outputs 0.759 -> 0.764 / 0.735 -> 0.749, in place 0.735 -> 0.748 / 0.741 -> 0.750,
//    one packed arena 0.629 -> 0.647 / 0.631 -> 0.649; same bits, checked on every weight);
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

constexpr int BATCH_RW = 256;  // the batched walk's waves per region (k_group_body RW)
template <int DT, int G, bool SYM, int CODES, bool BATCHED>
hipError_t launch_group_t(const GroupArgs& a, hipStream_t st) {
  constexpr int UNROLL = 4;
  static int cache[64] = {0};
  auto kern = k_group<DT, G, SYM, CODES, BATCHED, UNROLL, /*PF*/ !BATCHED, /*NTL*/ true, /*NTS*/ true,
                      /*SHARED*/ true, /*GS*/ false, /*SKEL*/ false, /*RW*/ BATCHED ? BATCH_RW : 1>;
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
template <int UNROLL, bool PF, bool NTL, bool NTS, bool SHARED = true, bool GS = false, bool SKEL = false,
          bool BATCHED = true, int RW = 1>
hipError_t launch_variant_t(const GroupArgs& a, hipStream_t st, int max_blocks_per_cu = 8) {
  static int cache[64] = {0};
  auto kern = k_group<DT_F16, 128, false, 0, BATCHED, UNROLL, PF, NTL, NTS, SHARED, GS, SKEL, RW>;
  const int64_t waves_needed = (a.total_units + UNROLL - 1) / UNROLL;
  int64_t blocks = (waves_needed + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  const int per_cu = resident_blocks_per_cu(kern, cache);
  const int64_t cap = (int64_t)device_cu_count() * (per_cu < max_blocks_per_cu ? per_cu : max_blocks_per_cu);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}
template <int UNROLL, bool SKEL, bool PHASE, int PFD, int RW = 1>
hipError_t launch_walk_t(const GroupArgs& a, hipStream_t st) {
  static int cache[64] = {0};
  auto kern = k_group_walk<DT_F16, 128, false, 0, true, UNROLL, SKEL, PHASE, PFD, RW>;
  return launch_persistent(kern, cache, UNROLL, a, st);
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

// the roofline probes bench.py measures its ceiling with (CEILING_PROBES): in every library
bool is_ceiling_probe(int v) { return v == 100 || v == 101 || v == 102 || v == 118; }

hipError_t launch_variant(int v, const GroupArgs& a, hipStream_t st) {
  switch (v) {
    case 100: hipLaunchKernelGGL(k_probe<0>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 101: hipLaunchKernelGGL(k_probe<1>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 102: hipLaunchKernelGGL(k_probe<2>, dim3((unsigned)(device_cu_count() * 8)), dim3(BLOCK), 0, st, a.entries, a.n_entries, a.nan_flag); return hipGetLastError();
    case 118:  // the default (region) walk, no arithmetic
      return launch_variant_t<4, false, true, true, true, false, true, true, BATCH_RW>(a, st);
  }
#if IWQ_AB
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
    case 12: return launch_variant_t<4, false, true, true>(a, st, 8);           // the contiguous walk (r1-r5 default)
    case 163: return launch_variant_t<4, false, true, true, true, false, true>(a, st);  // skeleton of 12
    case 13: return launch_variant_t<4, false, true, false>(a, st);             // default walk, plain stores
    case 14: return launch_variant_t<4, false, false, false>(a, st);            // plain loads + plain stores
    // memory-stream probes on the same skeleton (no arithmetic): which walk moves the bytes fastest
    case 119: return launch_variant_t<8, false, true, true, true, false, true>(a, st);     // 8 units in flight
    case 120: return launch_variant_t<2, false, true, true, true, false, true>(a, st);     // 2 units in flight
    case 121: return launch_variant_t<4, true, true, true, true, false, true>(a, st);      // + next loads prefetched
    case 122: return launch_variant_t<4, false, true, true, true, true, true>(a, st);      // grid-stride walk
    case 123: return launch_variant_t<4, false, true, true, true, false, true>(a, st, 4);  // 4 waves / SIMD
    case 124: return launch_variant_t<8, false, true, true, true, false, true>(a, st, 4);  // 8 units, 4 waves / SIMD
    case 125: return launch_variant_t<4, false, true, false, true, false, true>(a, st);    // plain stores
    case 126: return launch_variant_t<4, false, false, true, true, false, true>(a, st);    // plain loads
    case 127: return launch_variant_t<8, true, true, true, true, false, true>(a, st, 4);   // 8 units + prefetch, 4 waves
    // the real kernel at lower residency (fewer concurrent streams), and more skeleton residencies
    case 128: return launch_variant_t<4, false, true, true>(a, st, 3);                     // 3 waves / SIMD
    case 129: return launch_variant_t<4, false, true, true>(a, st, 2);                     // 2 waves / SIMD
    case 130: return launch_variant_t<4, false, true, true>(a, st, 5);                     // 5 waves / SIMD
    case 131: return launch_variant_t<4, true, true, true>(a, st, 4);                      // prefetch, 4 waves / SIMD
    case 132: return launch_variant_t<2, false, true, true>(a, st, 4);                     // 2 units, 4 waves / SIMD
    case 133: return launch_variant_t<4, false, true, true, true, false, true>(a, st, 3);  // skeleton, 3 waves / SIMD
    case 134: return launch_variant_t<4, false, true, true, true, false, true>(a, st, 2);  // skeleton, 2 waves / SIMD
    case 135: return launch_variant_t<8, false, true, true, true, false, true>(a, st, 2);  // skeleton, 8 units, 2 waves
    // grid-stride walks at copy-like granularity (single-tensor calls: the plain copy 100 beats the
    // contiguous walk by ~12 % on one 11008 x 4096 weight)
    case 136: return launch_variant_t<1, false, true, true, true, true>(a, st);            // grid-stride, 1 unit
    case 137: return launch_variant_t<2, false, true, true, true, true>(a, st);            // grid-stride, 2 units
    case 138: return launch_variant_t<4, false, true, false, true, true>(a, st);           // grid-stride, plain stores
    case 139: return launch_variant_t<1, false, true, true, true, true, true>(a, st);      // skeleton, grid-stride, 1 unit
    case 140: return launch_variant_t<2, false, true, true, true, true, true>(a, st);      // skeleton, grid-stride, 2 units
    case 141: return launch_variant_t<1, false, true, true, true, true>(a, st, 4);         // grid-stride, 1 unit, 4 waves
    // walk order vs output placement (round 6, tools/ab_outplace.py): per-wave phase rotation,
    // stores lagging the loads by two iterations, and their skeletons
    case 142: return launch_walk_t<4, false, true, 0>(a, st);   // phase rotation
    case 143: return launch_walk_t<4, false, false, 2>(a, st);  // loads of i + 2 in flight at the stores of i
    case 144: return launch_walk_t<2, false, false, 2>(a, st);  // the same with 2-unit iterations
    case 145: return launch_walk_t<2, false, true, 2>(a, st);   // both, 2-unit iterations
    case 146: return launch_walk_t<4, true, true, 0>(a, st);    // skeleton of 142
    case 147: return launch_walk_t<4, true, false, 2>(a, st);   // skeleton of 143
    // region walks: RW consecutive waves share a contiguous region, chunks round-robin
    case 148: return launch_walk_t<4, false, false, 0, 2>(a, st);
    case 149: return launch_walk_t<4, false, false, 0, 4>(a, st);
    case 150: return launch_walk_t<4, false, false, 0, 8>(a, st);
    case 151: return launch_walk_t<4, false, false, 0, 16>(a, st);
    case 152: return launch_walk_t<4, false, false, 0, 64>(a, st);
    case 153: return launch_walk_t<4, true, false, 0, 8>(a, st);    // skeleton of 150
    case 154: return launch_walk_t<4, true, false, 0, 64>(a, st);   // skeleton of 152
    case 155: return launch_walk_t<4, false, false, 0, 256>(a, st);
    case 156: return launch_walk_t<4, false, false, 0, 128>(a, st);
    case 157: return launch_walk_t<4, false, false, 0, 512>(a, st);
    case 158: return launch_walk_t<4, false, false, 0, 1024>(a, st);
    case 159: return launch_walk_t<4, false, false, 0, 2048>(a, st);
    case 160: return launch_walk_t<4, true, false, 0, 256>(a, st);   // skeleton of 155
    case 161: return launch_walk_t<2, false, false, 0, 256>(a, st);  // 2-unit chunks
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
#else
  (void)v;
  (void)a;
  (void)st;
#endif
  return hipErrorInvalidValue;
}

#if IWQ_AB
// A/B forms of the single-tensor walk (fp16, g = 128, asymmetric, no codes; one launch per weight,
// pseudo_quantize_tensor's drop-in call; tools/single_trace.py): 1 / 2 the two defaults forced
// (contiguous UNROLL 4 + prefetch / grid-stride UNROLL 4), 3 / 4 contiguous UNROLL 2 / 1 + prefetch,
// 5 / 6 grid-stride UNROLL 2 / 1, 7 / 8 contiguous UNROLL 4 / 2 + prefetch on half the resident waves,
// 9 grid-stride + prefetch, 10 / 11 UNROLL 8 grid-stride / contiguous, 12 / 13 the walks of 1 / 2
// without the arithmetic (roofline probes: wrong results), 14 / 15 the walks of 1 / 2 at 64 VGPRs
// (8 waves per SIMD instead of 7)
hipError_t launch_single_variant(int v, const GroupArgs& a, hipStream_t st) {
  static int c14[64] = {0}, c15[64] = {0};
  switch (v) {
    case 1: return launch_variant_t<4, true, true, true, true, false, false, false>(a, st);
    case 2: return launch_variant_t<4, false, true, true, true, true, false, false>(a, st);
    case 3: return launch_variant_t<2, true, true, true, true, false, false, false>(a, st);
    case 4: return launch_variant_t<1, true, true, true, true, false, false, false>(a, st);
    case 5: return launch_variant_t<2, false, true, true, true, true, false, false>(a, st);
    case 6: return launch_variant_t<1, false, true, true, true, true, false, false>(a, st);
    case 7: return launch_variant_t<4, true, true, true, true, false, false, false>(a, st, 4);
    case 8: return launch_variant_t<2, true, true, true, true, false, false, false>(a, st, 4);
    case 9: return launch_variant_t<4, true, true, true, true, true, false, false>(a, st);      // grid-stride + prefetch
    case 10: return launch_variant_t<8, false, true, true, true, true, false, false>(a, st);    // grid-stride UNROLL 8
    case 11: return launch_variant_t<8, true, true, true, true, false, false, false>(a, st);    // contiguous UNROLL 8
    case 12: return launch_variant_t<4, true, true, true, true, false, true, false>(a, st);     // 1's walk, no arithmetic
    case 13: return launch_variant_t<4, false, true, true, true, true, true, false>(a, st);     // 2's walk, no arithmetic
    case 14: return launch_persistent(k_group8<DT_F16, 128, false, 0, false, 4, true, true>, c14, 4, a, st);
    case 15: return launch_persistent(k_group8<DT_F16, 128, false, 0, false, 4, false, true, true, true, true>, c15, 4,
                                      a, st);
  }
  return hipErrorInvalidValue;
}
#endif

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

hipError_t launch_row(int dt, bool sym, int codes, const RowArgs& a, hipStream_t st) {
  if (dt == IWQ_F16) return sym ? launch_row_c<DT_F16, true>(codes, a, st) : launch_row_c<DT_F16, false>(codes, a, st);
  if (dt == IWQ_BF16) return sym ? launch_row_c<DT_BF16, true>(codes, a, st) : launch_row_c<DT_BF16, false>(codes, a, st);
  return sym ? launch_row_c<DT_F32, true>(codes, a, st) : launch_row_c<DT_F32, false>(codes, a, st);
}

// Block = TX column chunks (8 columns, 16 B each) x TY row slices.  Default 32 x 8 (512-B row
// segments) for g = 64, 16 x 16 at g = 128 (round 5, below) and g = 256 (to bound registers), picked
// by tools/ab_col.py (profiles/r01_ab_col.jsonl:
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
#if IWQ_AB
  if (variant == 1) return launch_col_t<DT, SYM, CODES, 8, 32>(a, st);
  if (variant == 2) return launch_col_t<DT, SYM, CODES, 32, 8>(a, st);
#endif
  // 16 x 16 at g = 128 (round 5: 37.8-37.9 vs 38.2-39.5 us for 32 x 8 on 11008 x 4096, two rounds of
  // the same box, profiles/r05_ab_col.jsonl; 512-thread 32 x 16 / 64 x 8 / 16 x 32 blocks 38.8-40.4)
  // and at g = 256 (16 rows per thread)
  if (variant == 3 || a.g == 256 || (variant == 0 && a.g == 128)) return launch_col_t<DT, SYM, CODES, 16, 16>(a, st);
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
// A per-tensor workspace holds two regions of TENSOR_PARTS_MAX 8-byte words: the one-pass kernel's
// granules, consensus word and done counter in the first (zeroed before its launch, or kept zero by
// the caller and the kernel -- IWQ_FLAG_WS_ZEROED), the pair's / universal path's partial keys in the
// second (fully written before they are read: never needs zeroing), so the pair leaves the first
// region zero without a clearing launch.
constexpr int TENSOR_SCRATCH_WORDS32 = TENSOR_PARTS_MAX * 2;  // the second region, in int32 units

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

// One-pass form (k_tensor_onepass, fp16): the tensor held in registers across the
// in-launch exchange of the per-workgroup keys; NV 16-B vectors per thread, one 512-thread
// workgroup per CU.  Returns false (nothing launched) when the tensor does not fit (> 48 vectors per
// thread: ~100 MB on 256 CUs) or there is no nan_flag to report a hand-off timeout through.
template <int DT, bool SYM, int CODES, int NV>
hipError_t launch_tensor_onepass_nv(const void* w, void* out, void* codes, void* scales, void* zeros, int64_t nvec,
                                    int nvt, int32_t* ws, int n_bits, uint32_t* nan_flag, hipStream_t st, int cus,
                                    uint32_t spin_limit, bool wsz) {
  // one workgroup per nvt * 512 vectors (<= the CU count: every chunk is non-empty and all are resident)
  const int64_t chunk = (int64_t)nvt * OP_THR;
  const int64_t nblk = (nvec + chunk - 1) / chunk;
  if (nvt < 1 || nvt > NV || nblk < 1 || nblk > cus) return hipErrorInvalidValue;
  // the granules (two per workgroup for fp32's 32-bit keys), the consensus word and the done counter
  // after them: zeroed before the launch unless the caller states they are (IWQ_FLAG_WS_ZEROED: the
  // kernel's last workgroup leaves them zero, so a workspace kept per stream needs no memset launch)
  if (!wsz) {
    const size_t gbytes = ((size_t)(nblk * (DT == DT_F32 ? 2 : 1) + 2) * 8 + 15) / 16 * 16;
    hipError_t e = zero_async(ws, gbytes, st);  // (not hipMemsetAsync: iwq_common.cuh)
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((k_tensor_onepass<DT, SYM, CODES, NV>), dim3((unsigned)nblk), dim3(OP_THR), 0, st,
                     static_cast<const char*>(w), static_cast<char*>(out), static_cast<uint8_t*>(codes), scales, zeros,
                     nvec, nvt, reinterpret_cast<unsigned long long*>(ws), n_bits, nan_flag, spin_limit);
  return hipGetLastError();
}
// fp16: every codes width; bf16 / fp32 (round 5): the fake-quant output only (CODES 0) -- with packed
// codes they take the pair.  Register budget: NV vectors of 8 elements per thread, up to 48 x 16 B
// (16-bit dtypes) or 24 x 32 B (fp32) = 192 VGPRs of data: ~100 MB of weights on 256 CUs either way.
template <int DT, bool SYM, int CODES>
bool launch_tensor_onepass(const void* w, void* out, void* codes, void* scales, void* zeros, int64_t numel,
                           int32_t* ws, int n_bits, uint32_t* nan_flag, hipStream_t st, hipError_t* err,
                           bool fixed_nv, uint32_t spin_limit, bool wsz) {
  if constexpr (DT != DT_F16 && CODES != 0) {
    return false;
  } else {
    if (nan_flag == nullptr) return false;  // an aborted hand-off must be reportable (bit 1)
    const int cus = device_cu_count();
    // granules (two per workgroup for fp32) + the consensus word + the done counter must fit the workspace
    if ((int64_t)cus * (DT == DT_F32 ? 2 : 1) + 2 > (int64_t)TENSOR_PARTS_MAX) return false;
    const int64_t nvec = numel / 8;
    const int64_t per = (nvec + (int64_t)cus * OP_THR - 1) / ((int64_t)cus * OP_THR);
    // nvt = per spreads the chunks over every CU; fixed_nv (A/B) uses the template's NV instead
    if constexpr (DT == DT_F32) {
      if (per <= 16) *err = launch_tensor_onepass_nv<DT, SYM, CODES, 16>(w, out, codes, scales, zeros, nvec, fixed_nv ? 16 : (int)per, ws, n_bits, nan_flag, st, cus, spin_limit, wsz);
      else if (per <= 24) *err = launch_tensor_onepass_nv<DT, SYM, CODES, 24>(w, out, codes, scales, zeros, nvec, fixed_nv ? 24 : (int)per, ws, n_bits, nan_flag, st, cus, spin_limit, wsz);
      else return false;
    } else {
      if (per <= 16) *err = launch_tensor_onepass_nv<DT, SYM, CODES, 16>(w, out, codes, scales, zeros, nvec, fixed_nv ? 16 : (int)per, ws, n_bits, nan_flag, st, cus, spin_limit, wsz);
      else if (per <= 32) *err = launch_tensor_onepass_nv<DT, SYM, CODES, 32>(w, out, codes, scales, zeros, nvec, fixed_nv ? 32 : (int)per, ws, n_bits, nan_flag, st, cus, spin_limit, wsz);
      else if (per <= 48) *err = launch_tensor_onepass_nv<DT, SYM, CODES, 48>(w, out, codes, scales, zeros, nvec, fixed_nv ? 48 : (int)per, ws, n_bits, nan_flag, st, cus, spin_limit, wsz);
      else return false;
    }
    return true;
  }
}

// variants: 0 = one pass where it pays (tensor_onepass_pays) and the tensor fits the registers, else
// the pair below; 6 = the pair (round-2 default) forced; 7 = one pass with NV vectors per thread (the
// first form: fewer, fuller chunks, some CUs idle); 8 = one pass wherever it fits (any size);
// 9 = TEST ONLY: one pass whose every sweep gives up at once (spin limit 0), so the launch ABORTs:
// nothing is written, nan_flag bit 1 is set, and the host's retry on the pair can be exercised
// variant bit 8 (set by iwq_quantize_minmax from IWQ_FLAG_WS_ZEROED): the first workspace region is
// zero on entry and must be zero on exit -- the one-pass kernel cleans up after itself, the pair never
// touches it
// Round 5 (profiles/r05_tensor_dt_sizes.jsonl, cold calls, zeroed workspace): the one pass pays from
// 32 MiB of fp16 / fp32 and 16 MiB of bf16 (ties there); below, the hand-off's fixed cost (publish,
// sweep and consensus round trips, ~4-5 us) exceeds the pair's second read, which mostly hits the
// MALL at these sizes (8 MiB fp16: 14.7 us one pass vs 10.1 us pair; 48 MiB: 27.5 vs 30.5).
template <int DT>
bool tensor_onepass_pays(int64_t numel) {
  const int64_t bytes = numel * (DT == DT_F32 ? 4 : 2);
  return bytes >= (DT == DT_BF16 ? (16ll << 20) : (32ll << 20));
}

template <int DT, bool SYM, int CODES>
hipError_t launch_tensor_t(const void* w, void* out, void* codes, void* scales, void* zeros, int64_t numel,
                           int32_t* ws, int n_bits, uint32_t* nan_flag, hipStream_t st, int variant) {
  const bool wsz = (variant & 0x100) != 0;
  variant &= 0xFF;
  if ((variant == 0 && tensor_onepass_pays<DT>(numel)) || variant == 7 || variant == 8 || variant == 9) {
    hipError_t e = hipSuccess;
    if (launch_tensor_onepass<DT, SYM, CODES>(w, out, codes, scales, zeros, numel, ws, n_bits, nan_flag, st, &e,
                                              IWQ_AB && variant == 7, variant == 9 ? 0u : OP_SPIN_LIMIT, wsz))
      return e;
  }
  ws += TENSOR_SCRATCH_WORDS32;  // the pair's partial keys: the second region
  const int64_t nunits = numel / 8;
  int64_t blocks = (int64_t)device_cu_count() * 8;
  const int64_t need = (nunits + BLOCK - 1) / BLOCK;
  if (blocks > need) blocks = need;
  if (blocks > TENSOR_PARTS_MAX) blocks = TENSOR_PARTS_MAX;
  if (blocks < 1) blocks = 1;
#if IWQ_AB
  if (variant == 1)
    launch_tensor_pair<DT, SYM, CODES, true, false>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else if (variant == 3)
    launch_tensor_pair<DT, SYM, CODES, false, true>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else if (variant == 4)
    launch_tensor_pair<DT, SYM, CODES, false, false, 4>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else if (variant == 5)
    launch_tensor_pair<DT, SYM, CODES, false, false, 2>(w, out, codes, scales, zeros, nunits, blocks, ws, n_bits, nan_flag, st);
  else
#endif
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
  if (group == IWQ_GROUP_PER_TENSOR) return (int64_t)TENSOR_PARTS_MAX * 16;  // the two regions above
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
  // product library: the default, and per tensor the pair forced (6: the host's retry), the one pass
  // forced (8) and the test-only abort (9); every other variant is an A/B form (IWQ_AB builds)
  const int variant = (int)((flags >> 16) & 0xFFu);
  if (!IWQ_AB && variant != 0 &&
      !(group == IWQ_GROUP_PER_TENSOR && (variant == 6 || variant == 8 || variant == 9)))
    return IWQ_ERR_ARG;

  if (!generic && quant_dim == 0 && group > 0 && group >= 8 && group <= 512 && is_pow2(group) && al &&
      fastbits && ld_w == cols && (!out_deq || ld_out == cols)) {
    GroupArgs a{};
    a.single = GroupTensor{w, out_deq, out_codes, out_scales, sym ? nullptr : out_zeros, rows * cols};
    a.total_units = (rows * cols + UNIT - 1) / UNIT;
    a.n_entries = 1;
    a.n_bits = n_bits;
    a.nan_flag = nan_flag;
#if IWQ_AB
    if (variant != 0 && dtype == IWQ_F16 && group == 128 && !sym && codes == 0) {
      IWQ_HIP(launch_single_variant(variant, a, s));
      return IWQ_OK;
    }
#endif
    IWQ_HIP(launch_group<false>(dtype, group, sym, codes, a, s));
    return IWQ_OK;
  }
  if (!generic && group == IWQ_GROUP_PER_TENSOR && al && fastbits && ld_w == cols &&
      (!out_deq || ld_out == cols) && (rows * cols) % 8 == 0) {
    const int64_t need = iwq_workspace_bytes(rows, cols, group, quant_dim);
    if (!workspace || workspace_bytes < need || !aligned16(workspace)) return IWQ_ERR_WORKSPACE;
    IWQ_HIP(launch_tensor(dtype, sym, codes, w, out_deq, out_codes, out_scales, sym ? nullptr : out_zeros,
                          rows * cols, static_cast<int32_t*>(workspace), n_bits, nan_flag, s,
                          variant | ((flags & IWQ_FLAG_WS_ZEROED) ? 0x100 : 0)));
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
    IWQ_HIP(launch_col(dtype, sym, codes, variant, a, s));
    return IWQ_OK;
  }
  // universal path
  const int64_t need = iwq_workspace_bytes(rows, cols, group, quant_dim);
  if (!workspace || workspace_bytes < need || !aligned16(workspace)) return IWQ_ERR_WORKSPACE;
  if (codes == 4) {
    const int64_t nbytes = rows * (cols / 2);
    if ((reinterpret_cast<uintptr_t>(out_codes) & 3u) != 0) return IWQ_ERR_ARG;
    IWQ_HIP(zero_async(out_codes, (uint64_t)nbytes, s));
  }
  SegArgs a{};
  a.w = static_cast<const char*>(w);
  a.out = static_cast<char*>(out_deq);
  a.codes = static_cast<uint8_t*>(out_codes);
  a.scales = out_scales;
  a.zeros = sym ? nullptr : out_zeros;
  // per tensor: the second region (the first stays zero for IWQ_FLAG_WS_ZEROED callers)
  a.keys = static_cast<int32_t*>(workspace) + (group == IWQ_GROUP_PER_TENSOR ? TENSOR_SCRATCH_WORDS32 : 0);
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
  if (!IWQ_AB && variant != 0 && !is_ceiling_probe(variant)) return IWQ_ERR_ARG;  // A/B forms: IWQ_AB builds
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

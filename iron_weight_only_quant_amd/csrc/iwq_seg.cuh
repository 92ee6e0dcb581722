// iwq_seg.cuh — the universal segmented min/max reduction shared by the INT and FP paths.
// Groups are runs of L consecutive elements of the grouped view V (V = W or W^T, quant_dim),
// any L, any row stride: k_seg_init + k_seg_reduce leave per-group order keys in a workspace
// (atomic min/max), then a path-specific apply kernel quantizes.
#pragma once
#include "iwq_common.cuh"

namespace iwq {
namespace seg {
namespace {  // internal linkage: included by several translation units

constexpr int BLOCK = 256;

struct SegArgs {
  const char* w;
  char* out;
  uint8_t* codes;
  void* scales;
  void* zeros;
  int32_t* keys;      // [2*G]: (min key, max key) — symmetric uses the max slot only
  int64_t rows, cols, ld_w, ld_out;
  int64_t vc;         // columns of V
  int64_t L, G, total;
  int quant_dim;
  int n_bits;
  int codes_bits;     // 0, 4, 8
  uint32_t* nan_flag;
};

constexpr int SEG_RUN = 16;

__device__ __forceinline__ void seg_locate(const SegArgs& a, int64_t f, int64_t& off_w, int64_t& off_o,
                                           int64_t& r, int64_t& c) {
  const int64_t vr_i = f / a.vc;
  const int64_t vc_i = f - vr_i * a.vc;
  if (a.quant_dim == 0) { r = vr_i; c = vc_i; }
  else { r = vc_i; c = vr_i; }
  off_w = r * a.ld_w + c;
  off_o = r * a.ld_out + c;
}

__global__ __launch_bounds__(BLOCK) void k_seg_init(int32_t* keys, int64_t G) {
  for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < G; j += (int64_t)gridDim.x * BLOCK) {
    keys[2 * j] = 0x7FFFFFFF;
    keys[2 * j + 1] = (int32_t)0x80000000;
  }
}

template <int DT, bool SYM>
__global__ __launch_bounds__(BLOCK) void k_seg_reduce(SegArgs a) {
  using F = Fmt<DT>;
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  const int64_t tid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  int64_t curj = -1;
  int32_t mn = 0x7FFFFFFF, mx = (int32_t)0x80000000;
  for (int64_t f0 = tid * SEG_RUN; f0 < a.total; f0 += nthreads * SEG_RUN) {
    const int64_t fend = min(f0 + SEG_RUN, a.total);
    for (int64_t f = f0; f < fend; ++f) {
      const int64_t j = f / a.L;
      if (j != curj) {
        if (curj >= 0) {
          if (!SYM) atomicMin(&a.keys[2 * curj], mn);
          atomicMax(&a.keys[2 * curj + 1], mx);
        }
        curj = j;
        mn = 0x7FFFFFFF;
        mx = (int32_t)0x80000000;
      }
      int64_t ow, oo, r, c;
      seg_locate(a, f, ow, oo, r, c);
      uint32_t b;
      if constexpr (F::NB == 16) b = gp<uint16_t>(a.w)[ow];
      else b = gp<uint32_t>(a.w)[ow];
      if constexpr (SYM) {
        mx = max(mx, mag_key<DT>(b));
      } else {
        int32_t k = key_of<DT>(b);
        mn = min(mn, k);
        mx = max(mx, k);
      }
    }
  }
  // flush: combine across the wave first when every lane holds the same group (per-tensor case)
  const int64_t j0 = __shfl(curj, 0);
  const bool same = __all(curj == j0);
  if (same) {
    if (j0 >= 0) {
      int32_t m1 = mn, m2 = mx;
      group_minmax<64>(m1, m2);
      if ((threadIdx.x & 63) == 0) {
        if (!SYM) atomicMin(&a.keys[2 * j0], m1);
        atomicMax(&a.keys[2 * j0 + 1], m2);
      }
    }
  } else if (curj >= 0) {
    if (!SYM) atomicMin(&a.keys[2 * curj], mn);
    atomicMax(&a.keys[2 * curj + 1], mx);
  }
}


}  // namespace
}  // namespace seg
}  // namespace iwq

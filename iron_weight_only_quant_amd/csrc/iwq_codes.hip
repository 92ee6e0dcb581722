// iwq_codes.hip — packed codes (include/iwq.h layout) -> the dequantized weight, every INT mode.
//
// The reference keeps no integer codes; this is the inverse of the packed format
// the quantize kernels write, used where only (codes, scales, zeros) exist: the packed checkpoint
// (checkpoint.py) restores QuantLinear.weight from it, and the packed-only layer (PackedLinear)
// dequantizes a weight for the library GEMM.  Element (r, c) of W:
//   code  = nibble c & 1 of byte r * cols/2 + c/2 (n_bits <= 4) or byte r * cols + c (5..8 bits)
//   group = flat index of (r, c) in the grouped view V (W, or W^T for quant_dim 1), divided by the
//           group length L (group, the row length of V for per-channel, rows * cols for per-tensor)
//   out   = RN_dtype((code - z) * s), z = zeros[group] (asymmetric) or 2^(b-1) (symmetric)
// (code - z) is an exact small integer and the fp32 product of two 16-bit values is exact, so for
// fp16 / bf16 the one rounding is the reference's RN16((q - z) * s) (quant_funcs.py:38,
// quant_linear.py:947); for fp32 it is the fp32 multiply ATen does.
// HBM-bound (0.5-1 B read + the output written per element; load-time work, not the hot path):
// a thread takes 8 consecutive columns of one row, one code load and one output store per 8 where
// the row allows it.
#include "iwq_common.cuh"
#include "../../include/iwq.h"

using namespace iwq;

namespace {

struct CodesArgs {
  const uint8_t* codes;
  const void* scales;
  const void* zeros;
  void* out;
  int64_t rows, cols, ld_out, L;
  float zsym;
};

template <int DT>
__device__ __forceinline__ float param_at(const void* p, int64_t i) {
  if constexpr (Fmt<DT>::NB == 16) return Fmt<DT>::to_f(gp<uint16_t>(p)[i]);
  else return Fmt<DT>::to_f(gp<uint32_t>(p)[i]);
}

template <int DT>
__device__ __forceinline__ uint32_t deq(uint32_t code, float s, float z) {
  return Fmt<DT>::from_f(opaque(((float)code - z) * s));
}

// NIB: 4-bit codes (two per byte); QD: quant_dim; FULL8: cols % 8 == 0 (every chunk is 8 in-row
// columns, its codes one aligned 4- / 8-byte word); SAME: additionally quant_dim 0 and L % 8 == 0 (the
// 8 share one group)
template <int DT, bool NIB, int QD, bool FULL8, bool SAME>
__global__ __launch_bounds__(256) void k_dequant_codes(CodesArgs a) {
  const int64_t cpr = (a.cols + 7) / 8;
  const int64_t total = a.rows * cpr;
  const bool sym = a.zeros == nullptr;
  for (int64_t ci = (int64_t)blockIdx.x * 256 + threadIdx.x; ci < total; ci += (int64_t)gridDim.x * 256) {
    const int64_t r = ci / cpr;
    const int64_t c0 = (ci - r * cpr) * 8;
    const int n = FULL8 ? 8 : (int)(a.cols - c0 < 8 ? a.cols - c0 : 8);
    uint32_t code[8];
    if constexpr (FULL8) {
      if constexpr (NIB) {
        const uint32_t w = gp<uint32_t>(a.codes)[(r * a.cols + c0) / 8];
#pragma unroll
        for (int j = 0; j < 8; ++j) code[j] = (w >> (4 * j)) & 15u;
      } else {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 w = gp<u32x2>(a.codes)[(r * a.cols + c0) / 8];
#pragma unroll
        for (int j = 0; j < 8; ++j) code[j] = ((j < 4 ? w.x : w.y) >> (8 * (j & 3))) & 255u;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        code[j] = 0;
        if (j < n) {
          const int64_t c = c0 + j;
          if constexpr (NIB) code[j] = (gp<uint8_t>(a.codes)[r * (a.cols / 2) + c / 2] >> (4 * (c & 1))) & 15u;
          else code[j] = gp<uint8_t>(a.codes)[r * a.cols + c];
        }
      }
    }
    uint32_t y[8];
    if constexpr (SAME) {
      const int64_t gi = (r * a.cols + c0) / a.L;
      const float s = param_at<DT>(a.scales, gi);
      const float z = sym ? a.zsym : param_at<DT>(a.zeros, gi);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = deq<DT>(code[j], s, z);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        y[j] = 0;
        if (j < n) {
          const int64_t c = c0 + j;
          const int64_t gi = (QD == 0 ? r * a.cols + c : c * a.rows + r) / a.L;
          const float s = param_at<DT>(a.scales, gi);
          const float z = sym ? a.zsym : param_at<DT>(a.zeros, gi);
          y[j] = deq<DT>(code[j], s, z);
        }
      }
    }
    const int64_t o = r * a.ld_out + c0;  // element offset of this chunk's first output
    if constexpr (FULL8 && Fmt<DT>::NB == 16) {
      if ((o & 7) == 0) {  // 16-B aligned (the base is checked on the host)
        gp<u32x4>(a.out)[o / 8] = u32x4{y[0] | (y[1] << 16), y[2] | (y[3] << 16), y[4] | (y[5] << 16), y[6] | (y[7] << 16)};
        continue;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < n) {
        if constexpr (Fmt<DT>::NB == 16) gp<uint16_t>(a.out)[o + j] = (uint16_t)y[j];
        else gp<uint32_t>(a.out)[o + j] = y[j];
      }
    }
  }
}

template <int DT, bool NIB, int QD>
void launch_codes(const CodesArgs& a, bool full8, bool same, unsigned blocks, hipStream_t st) {
  if (full8 && same && QD == 0)
    hipLaunchKernelGGL((k_dequant_codes<DT, NIB, QD, true, true>), dim3(blocks), dim3(256), 0, st, a);
  else if (full8)
    hipLaunchKernelGGL((k_dequant_codes<DT, NIB, QD, true, false>), dim3(blocks), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((k_dequant_codes<DT, NIB, QD, false, false>), dim3(blocks), dim3(256), 0, st, a);
}

template <int DT>
void launch_codes_dt(const CodesArgs& a, bool nib, int qd, bool full8, bool same, unsigned blocks, hipStream_t st) {
  if (nib) {
    if (qd == 0) launch_codes<DT, true, 0>(a, full8, same, blocks, st);
    else launch_codes<DT, true, 1>(a, full8, same, blocks, st);
  } else {
    if (qd == 0) launch_codes<DT, false, 0>(a, full8, same, blocks, st);
    else launch_codes<DT, false, 1>(a, full8, same, blocks, st);
  }
}

}  // namespace

extern "C" int iwq_dequant_codes(const void* codes, const void* scales, const void* zeros, int dtype, int n_bits,
                                 int64_t group, int symmetric, int quant_dim, int64_t rows, int64_t cols, void* out,
                                 int64_t ld_out, void* stream) {
  if (!codes || !scales || !out || (!symmetric && !zeros)) return IWQ_ERR_ARG;
  if (dtype != IWQ_F16 && dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (n_bits < 1 || n_bits > 8 || (symmetric && n_bits < 2)) return IWQ_ERR_BITS;
  if (quant_dim != 0 && quant_dim != 1) return IWQ_ERR_ARG;
  if (rows <= 0 || cols <= 0 || ld_out < cols) return IWQ_ERR_SHAPE;
  const bool nib = n_bits <= 4;
  if (nib && (cols & 1)) return IWQ_ERR_CODES;
  const int64_t vc = quant_dim == 0 ? cols : rows;  // row length of the grouped view
  int64_t L;
  if (group == IWQ_GROUP_PER_TENSOR) L = rows * cols;
  else if (group == IWQ_GROUP_PER_CHANNEL) L = vc;
  else if (group > 0) {
    if (vc % group != 0) return IWQ_ERR_GROUP;
    L = group;
  } else {
    return IWQ_ERR_GROUP_MODE;
  }
  const int esz = dtype == IWQ_F32 ? 4 : 2;
  const bool full8 = cols % 8 == 0 && (reinterpret_cast<uintptr_t>(codes) & 7u) == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 15u) == 0;
  if ((reinterpret_cast<uintptr_t>(out) % esz) || (reinterpret_cast<uintptr_t>(scales) % esz) ||
      (zeros && (reinterpret_cast<uintptr_t>(zeros) % esz)))
    return IWQ_ERR_ARG;
  const bool same = quant_dim == 0 && L % 8 == 0;
  CodesArgs a{static_cast<const uint8_t*>(codes), scales, symmetric ? nullptr : zeros, out, rows, cols, ld_out, L,
              (float)(1 << (n_bits - 1))};
  const int64_t chunks = rows * ((cols + 7) / 8);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  int64_t blocks = (chunks + 255) / 256;
  if (blocks > (int64_t)cus * 16) blocks = (int64_t)cus * 16;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == IWQ_F16) launch_codes_dt<DT_F16>(a, nib, quant_dim, full8, same, (unsigned)blocks, st);
  else if (dtype == IWQ_BF16) launch_codes_dt<DT_BF16>(a, nib, quant_dim, full8, same, (unsigned)blocks, st);
  else launch_codes_dt<DT_F32>(a, nib, quant_dim, full8, same, (unsigned)blocks, st);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    iwq::last_hip_error() = (int)e;
    return IWQ_ERR_HIP;
  }
  return IWQ_OK;
}

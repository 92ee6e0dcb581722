// iwq_bfp.hip — block floating point (BFP) fake quantization on gfx950.
//
// Replaces (reference, /root/reference): QuantLinear.quantize_weight, weight_format "bfp"
// (quant_linear.py:648-723).  Per group of w_group_size consecutive elements of the (transposed when
// quant_dim == 1) weight, taken to fp16:
//   shared exponent  e_max = max 5-bit fp16 exponent field of the group
//   mantissa         (leading 1 for normals | 10-bit field) >> (e_max - e)   (a subnormal's e is 0)
//   rounding         round-half-up right shift by 11 - b, b = min(w_bit - 1, 11); saturate 2^b - 1
//   dequant          mant * 2^(e_max - 15 - (b - 1)) * sign   (exact in fp32, one rounding to dtype)
// Integer work only (exponent max + shifts): HBM-bound, 2 bytes read + 2 written per fp16 element.
//
// Kernels:
//   k_bfp_group    quant_dim 0, contiguous, group 8..512 (power of two): 8 elements per lane, the
//                  group's exponent max by DPP across its G/8 lanes, one pass.
//   k_bfp_generic  any group / quant_dim / strides: one thread per group, two passes over it
//                  (quant_dim 1: consecutive threads take consecutive columns -> coalesced).
#include "iwq_common.cuh"
#include "../../include/iwq.h"

using namespace iwq;

namespace {

constexpr int BLOCK = 256;

struct BfpArgs {
  const char* w;
  char* out;
  int64_t rows, cols, ld_w, ld_out;
  int64_t numel;
  int64_t g, gpr, ngroups;   // group length, groups per grouped row, group count
  int quant_dim;
  int tmb, sd, mant_max;     // kept mantissa bits, rounding shift, saturation
};

// fp16 bits of an element of the weight dtype (.to(torch.float16): RNE)
template <int DT>
__device__ __forceinline__ uint32_t to_h(uint32_t b) {
  if constexpr (DT == DT_F16) return b;
  else return Fmt<DT_F16>::from_f(Fmt<DT>::to_f(b));
}

__device__ __forceinline__ int rrshift(int v, int s) {  // quant_linear.py:112-123 (s in 1..11)
  return (v + (1 << (s - 1))) >> s;
}

// BFP value of one fp16 element given the group's max exponent field: exact in fp32
__device__ __forceinline__ float bfp_value(uint32_t h, int eb, const BfpArgs& a) {
  const int e = (int)((h >> 10) & 0x1Fu);
  const int mwl = (e ? 1024 : 0) | (int)(h & 0x3FFu);
  int m = mwl >> (eb - e);                                 // eb >= e; shift <= 31
  if (a.sd > 0) m = rrshift(m, a.sd);
  m = m < a.mant_max ? m : a.mant_max;
  const float v = __builtin_ldexpf((float)m, eb - 15 - (a.tmb - 1));
  return (h >> 15) ? -v : v;
}

template <int DT, int G>
__global__ __launch_bounds__(BLOCK) void k_bfp_group(BfpArgs a) {
  using F = Fmt<DT>;
  constexpr int LPG = G / 8;
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  // wave-uniform trip count: a wave covers 512 consecutive elements = whole groups (G | 512)
  const int64_t nunits = (a.numel + 511) / 512 * 64;
  for (int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x; t < nunits; t += nthreads) {
    const int64_t e0 = t * 8;
    const bool ok = e0 < a.numel;
    Vec8<DT> v;
    v.load(a.w + (ok ? e0 : 0) * F::BYTES);
    uint32_t h[8];
    int32_t mx = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      h[i] = to_h<DT>(v.get(i));
      const int32_t e = (int32_t)((h[i] >> 10) & 0x1Fu);
      mx = e > mx ? e : mx;
    }
    group_max<LPG>(mx);
    Vec8<DT> o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.set(i, F::from_f(bfp_value(h[i], mx, a)));
    if (ok) o.store(a.out + e0 * F::BYTES);
  }
}

template <int DT>
__global__ __launch_bounds__(BLOCK) void k_bfp_generic(BfpArgs a) {
  using F = Fmt<DT>;
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  for (int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x; t < a.ngroups; t += nthreads) {
    // first element (r0, c0) and element stride of this group in the weight / output
    int64_t r0, c0, sw, so;
    if (a.quant_dim == 0) {
      r0 = t / a.gpr;
      c0 = (t - r0 * a.gpr) * a.g;
      sw = 1;
      so = 1;
    } else {  // transposed groups run down a column; consecutive threads = consecutive columns
      const int64_t rb = t / a.cols;
      c0 = t - rb * a.cols;
      r0 = rb * a.g;
      sw = a.ld_w;
      so = a.ld_out;
    }
    const char* wp = a.w + (r0 * a.ld_w + c0) * F::BYTES;
    char* op = a.out + (r0 * a.ld_out + c0) * F::BYTES;
    int eb = 0;
    for (int64_t k = 0; k < a.g; ++k) {
      const uint32_t b = F::NB == 16 ? (uint32_t)gp<uint16_t>(wp)[k * sw] : gp<uint32_t>(wp)[k * sw];
      const int e = (int)((to_h<DT>(b) >> 10) & 0x1Fu);
      eb = e > eb ? e : eb;
    }
    for (int64_t k = 0; k < a.g; ++k) {
      const uint32_t b = F::NB == 16 ? (uint32_t)gp<uint16_t>(wp)[k * sw] : gp<uint32_t>(wp)[k * sw];
      const uint32_t y = F::from_f(bfp_value(to_h<DT>(b), eb, a));
      if constexpr (F::NB == 16) gp<uint16_t>(op)[k * so] = (uint16_t)y;
      else gp<uint32_t>(op)[k * so] = y;
    }
  }
}

int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
  return n;
}

template <int DT>
hipError_t launch_bfp(const BfpArgs& a, bool fast, hipStream_t st) {
  const int64_t cap = (int64_t)cu_count() * 16;
  if (fast) {
    int64_t blocks = ((a.numel + 511) / 512 * 64 + BLOCK - 1) / BLOCK;
    blocks = blocks > cap ? cap : (blocks < 1 ? 1 : blocks);
    switch (a.g) {
      case 8: hipLaunchKernelGGL((k_bfp_group<DT, 8>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a); break;
      case 16: hipLaunchKernelGGL((k_bfp_group<DT, 16>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a); break;
      case 32: hipLaunchKernelGGL((k_bfp_group<DT, 32>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a); break;
      case 64: hipLaunchKernelGGL((k_bfp_group<DT, 64>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a); break;
      case 128: hipLaunchKernelGGL((k_bfp_group<DT, 128>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a); break;
      case 256: hipLaunchKernelGGL((k_bfp_group<DT, 256>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a); break;
      default: hipLaunchKernelGGL((k_bfp_group<DT, 512>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a); break;
    }
  } else {
    int64_t blocks = (a.ngroups + BLOCK - 1) / BLOCK;
    blocks = blocks > cap ? cap : (blocks < 1 ? 1 : blocks);
    hipLaunchKernelGGL(k_bfp_generic<DT>, dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace

extern "C" {

int iwq_quantize_bfp(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int w_bit, int64_t group,
                     int quant_dim, void* out, int64_t ld_out, unsigned flags, void* stream) {
  if (!w || !out) return IWQ_ERR_ARG;
  if (dtype != IWQ_F16 && dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (rows <= 0 || cols <= 0 || ld_w < cols || ld_out < cols) return IWQ_ERR_SHAPE;
  if (quant_dim != 0 && quant_dim != 1) return IWQ_ERR_ARG;
  if (group <= 0) return IWQ_ERR_GROUP_MODE;           // BFP needs a positive group (ValueError)
  if (w_bit < 1) return IWQ_ERR_BITS;                  // (1 << (w_bit-1)) - 1 with w_bit < 1: ValueError
  const int64_t vr = quant_dim == 1 ? cols : rows, vc = quant_dim == 1 ? rows : cols;
  if (vc % group != 0) return IWQ_ERR_GROUP;           // AssertionError in the reference
  BfpArgs a{};
  a.w = static_cast<const char*>(w);
  a.out = static_cast<char*>(out);
  a.rows = rows;
  a.cols = cols;
  a.ld_w = ld_w;
  a.ld_out = ld_out;
  a.numel = rows * cols;
  a.g = group;
  a.gpr = vc / group;
  a.ngroups = vr * vc / group;
  a.quant_dim = quant_dim;
  a.tmb = w_bit - 1 < 11 ? w_bit - 1 : 11;
  a.sd = 11 - a.tmb;
  a.mant_max = (1 << a.tmb) - 1;
  const bool al = ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  const bool fast = !(flags & IWQ_FLAG_FORCE_GENERIC) && quant_dim == 0 && ld_w == cols && ld_out == cols && al &&
                    group >= 8 && group <= 512 && (group & (group - 1)) == 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = hipSuccess;
  if (dtype == IWQ_F16) e = launch_bfp<DT_F16>(a, fast, st);
  else if (dtype == IWQ_BF16) e = launch_bfp<DT_BF16>(a, fast, st);
  else e = launch_bfp<DT_F32>(a, fast, st);
  if (e != hipSuccess) {
    iwq::last_hip_error() = (int)e;
    return IWQ_ERR_HIP;
  }
  return IWQ_OK;
}

}  // extern "C"

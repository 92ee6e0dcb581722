// iwq_synth.hip — synthetic weight generator (bit-identical to oracle/synth.py), the exhaustive
// division self-test, and build info.  Test/bench utilities of the C-ABI; not on the hot path.
#include "iwq_common.cuh"
#include "../../include/iwq.h"

using namespace iwq;

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <int DT>
__global__ __launch_bounds__(256) void k_synth(void* out, int64_t n, uint64_t seed, int64_t off) {
  const float scale = (float)(0.02 / 37837.23);  // == np.float32(0.02 / 37837.23)
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t h = splitmix64(seed * 0xD2B74407B1CE6E93ull + (uint64_t)(i + off));
    const int64_t u0 = (int64_t)(h & 0xFFFF), u1 = (int64_t)((h >> 16) & 0xFFFF);
    const int64_t u2 = (int64_t)((h >> 32) & 0xFFFF), u3 = (int64_t)((h >> 48) & 0xFFFF);
    float x = (float)(u0 + u1 + u2 + u3 - 131070) * scale;
    if (((u0 ^ u3) & 0x3FF) == 0) x = x * 8.0f;
    if constexpr (Fmt<DT>::NB == 16) static_cast<uint16_t*>(out)[i] = (uint16_t)Fmt<DT>::from_f(x);
    else static_cast<float*>(out)[i] = x;
  }
}

// Every finite fp16 numerator (63488 incl. +-0) against fp16 divisors s in [2^-24, 65504]:
// the hot loop's reciprocal (rcp_f16val) and corrected quotient (div_f16vals) vs IEEE fp32 division.
__global__ __launch_bounds__(256) void k_selftest_div(unsigned long long* counts) {
  const uint32_t dbits = blockIdx.y + 1;  // 0x0001 .. 0x7BFF
  const float s = (float)__builtin_bit_cast(_Float16, (uint16_t)dbits);
  const float rs_ref = opaque(1.0f / s);
  const float rs = rcp_f16val(s);
  unsigned long long bad32 = 0, bad16 = 0;
  for (uint32_t wb = blockIdx.x * 256 + threadIdx.x; wb < 65536u; wb += gridDim.x * 256) {
    if ((wb & 0x7C00u) == 0x7C00u) continue;  // inf / NaN numerators never take the fast path
    const float w = (float)__builtin_bit_cast(_Float16, (uint16_t)wb);
    const float q1 = div_f16vals(w, s, rs);
    const float ref = opaque(w / s);
    const bool z1 = (q1 == 0.0f && ref == 0.0f);  // sign of a zero quotient is irrelevant downstream
    bad32 += (!z1 && __builtin_bit_cast(uint32_t, q1) != __builtin_bit_cast(uint32_t, ref)) ? 1 : 0;
    const uint16_t h1 = __builtin_bit_cast(uint16_t, (_Float16)q1), h2v = __builtin_bit_cast(uint16_t, (_Float16)ref);
    bad16 += (!z1 && h1 != h2v) ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) {
    bad32 += __shfl_down(bad32, o);
    bad16 += __shfl_down(bad16, o);
  }
  if ((threadIdx.x & 63) == 0 && (bad32 | bad16)) {
    atomicAdd(&counts[0], bad32);
    atomicAdd(&counts[1], bad16);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && __builtin_bit_cast(uint32_t, rs) != __builtin_bit_cast(uint32_t, rs_ref))
    atomicAdd(&counts[2], 1ull);
}

}  // namespace

extern "C" {

int iwq_fill_synthetic(void* out, int64_t n, int dtype, uint64_t seed, int64_t index_offset, void* stream) {
  if (!out || n < 0) return IWQ_ERR_ARG;
  if (n == 0) return IWQ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (dtype == IWQ_F16) hipLaunchKernelGGL(k_synth<DT_F16>, dim3((unsigned)blocks), dim3(256), 0, st, out, n, seed, index_offset);
  else if (dtype == IWQ_BF16) hipLaunchKernelGGL(k_synth<DT_BF16>, dim3((unsigned)blocks), dim3(256), 0, st, out, n, seed, index_offset);
  else if (dtype == IWQ_F32) hipLaunchKernelGGL(k_synth<DT_F32>, dim3((unsigned)blocks), dim3(256), 0, st, out, n, seed, index_offset);
  else return IWQ_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? IWQ_OK : IWQ_ERR_HIP;
}

int iwq_selftest_division(uint64_t* d_counts, void* stream) {
  if (!d_counts) return IWQ_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hipMemsetAsync(d_counts, 0, 3 * sizeof(uint64_t), st) != hipSuccess) return IWQ_ERR_HIP;
  hipLaunchKernelGGL(k_selftest_div, dim3(64, 0x7BFF), dim3(256), 0, st,
                     reinterpret_cast<unsigned long long*>(d_counts));
  return hipGetLastError() == hipSuccess ? IWQ_OK : IWQ_ERR_HIP;
}

const char* iwq_build_info(void) {
#if IWQ_AB
  return "iwq 0.1 gfx950 (-O3 -ffp-contract=off, IEEE fp32 div, denormals preserved) ab=1";
#else
  return "iwq 0.1 gfx950 (-O3 -ffp-contract=off, IEEE fp32 div, denormals preserved) ab=0";
#endif
}

}  // extern "C"

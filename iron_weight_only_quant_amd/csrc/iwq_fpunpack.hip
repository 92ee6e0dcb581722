// iwq_fpunpack.hip — FP4/FP6/FP8 packed codes -> fp16 weights (the "unpack" half of config 5).
//
// Replaces the dequant step of the QuantLinear FP branches (quant_linear.py:724-883):
//   dequantized = _fp_to_float(codes).to(fp16) * scales (+ zeros)          (:773-777, :825-829, :876-880)
// and of fp4_quantize_cpu.quantize_fp16_to_fp4_e1m2 (fp4_quantize_cpu.py:66-72: q * S) for codes
// produced by iwq_quantize_fp / iwq_fp4_grid_packed.  Output bit-identical to those kernels' out_deq.
//
// Decode: _fp_to_float's values are exact in fp16 for every format whose fp_max fits fp16, so
// out = RN16(RN16(decode(c)) * s) = one fp16 multiply of the exact decoded value (+ one fp16 add of
// the zero point).  The decode itself:
//   E2M1 (nibbles)  v_cvt_scalef32_pk_f16_fp4 (scale 1.0): the reference's E2M1 (bias 1, no inf /
//                   NaN codes) is the OCP e2m1 value set bit for bit, sign of zero included;
//   E4M3 (bytes)    v_cvt_scalef32_pk_f16_fp8: the reference's E4M3 (bias 7) differs from OCP e4m3fn
//                   only in codes 0x7F / 0xFF (OCP: NaN; reference: +-480 = (1 + 7/8) 2^8), which a
//                   SWAR test finds per dword and a wave-uniform slow path rewrites;
//   any other E/M   a 256-entry fp16 table built in LDS by each workgroup from the reference formula.
// Walk: as k_dequant_packed (iwq_gemm.hip): a wave takes 2048 consecutive elements per step, lane l
// of piece j owns elements 512 j + 8 l .. +8 (one code dword / dword pair, one 16-B store); a piece
// never straddles a scale group (group % 8 == 0, K % 8 == 0).  HBM-bound: 2 + 0.5 (or 1) + 2/g B
// per weight (+ 2/g for zeros).
#include "iwq_common.cuh"
#include "../../include/iwq.h"

namespace iwq {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

enum : int { FMT_HW4 = 0, FMT_HW8 = 1, FMT_TAB4 = 2, FMT_TAB8 = 3 };

struct UnpackArgs {
  const uint8_t* codes;
  const _Float16* scales;
  const _Float16* zeros;  // null: symmetric
  _Float16* out;
  int64_t total;          // N * K
  int64_t group;          // elements per scale group (flat order)
  int gshift;             // log2(group) or -1
  int E, M, bias;
};

__device__ __forceinline__ h2 as_h2u(uint32_t u) { return __builtin_bit_cast(h2, u); }

// exact decode of one code (quant_linear.py:213-235) as fp16 bits
__device__ __forceinline__ uint16_t decode_bits(uint32_t c, int E, int M, int bias) {
  const uint32_t sign = (c >> (E + M)) & 1u;
  const int e = (int)((c >> M) & ((1u << E) - 1u));
  const int m = (int)(c & ((1u << M) - 1u));
  const float mag = e == 0 ? __builtin_ldexpf((float)m, 1 - bias - M) : __builtin_ldexpf((float)((1 << M) + m), e - bias - M);
  float v = sign ? -mag : mag;
  if (c == 0) v = 0.0f;  // code 0 -> +0; the sign-only code keeps its -0
  return __builtin_bit_cast(uint16_t, (_Float16)v);
}

template <int FMT, bool ASYM>
__global__ __launch_bounds__(256) void k_dequant_fp_packed(UnpackArgs a) {
  __shared__ uint16_t tab[256];
  if constexpr (FMT == FMT_TAB4 || FMT == FMT_TAB8) {
    tab[threadIdx.x] = decode_bits(threadIdx.x, a.E, a.M, a.bias);
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  IWQ_GLOBAL h8* out = gp<h8>(a.out);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  constexpr bool NIB = FMT == FMT_HW4 || FMT == FMT_TAB4;
  // one step = 2048 elements per wave: the codes AND the group parameters of the step are loaded
  // together (no second dependent round trip for the scales), and the next step's loads are issued
  // before this step's decode and stores (register double buffer)
  struct Step {
    u32x2 w[4];
    _Float16 sc[4], zv[4];
  };
  auto load_step = [&](int64_t base, Step& st) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = base + 512 * j + 8 * lane;
      const int64_t ee = e < a.total ? e : 0;
      if constexpr (NIB) st.w[j] = u32x2{__builtin_nontemporal_load(gp<uint32_t>(a.codes) + ee / 8), 0u};
      else st.w[j] = __builtin_nontemporal_load(gp<u32x2>(a.codes) + ee / 8);
      const int64_t gi = a.gshift >= 0 ? (ee >> a.gshift) : ee / a.group;
      st.sc[j] = gp<_Float16>(a.scales)[gi];
      if constexpr (ASYM) st.zv[j] = gp<_Float16>(a.zeros)[gi];
    }
  };
  int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2048;
  if (base >= a.total) return;
  Step nxt;
  load_step(base, nxt);
  while (true) {
    const Step cur = nxt;
    const int64_t b0 = base;
    base += nwaves * 2048;
    const bool more = base < a.total;
    if (more) load_step(base, nxt);
    const u32x2* w = cur.w;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = b0 + 512 * j + 8 * lane;
      if (e >= a.total) continue;
      const h2 s2 = {cur.sc[j], cur.sc[j]};
      h2 z2 = {(_Float16)0.0f, (_Float16)0.0f};
      if constexpr (ASYM) z2 = h2{cur.zv[j], cur.zv[j]};
      h2 d[4];
      if constexpr (FMT == FMT_HW4) {
        d[0] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(w[j].x, 1.0f, 0);
        d[1] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(w[j].x, 1.0f, 1);
        d[2] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(w[j].x, 1.0f, 2);
        d[3] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(w[j].x, 1.0f, 3);
      } else if constexpr (FMT == FMT_HW8) {
        d[0] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w[j].x, 1.0f, false);
        d[1] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w[j].x, 1.0f, true);
        d[2] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w[j].y, 1.0f, false);
        d[3] = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w[j].y, 1.0f, true);
        // codes 0x7F / 0xFF: OCP NaN, the reference's +-480 (a byte of (c & 0x7F) ^ 0x7F is zero)
        const uint32_t t0 = (w[j].x & 0x7F7F7F7Fu) ^ 0x7F7F7F7Fu, t1 = (w[j].y & 0x7F7F7F7Fu) ^ 0x7F7F7F7Fu;
        const bool hit = (((t0 - 0x01010101u) & ~t0) | ((t1 - 0x01010101u) & ~t1)) & 0x80808080u;
        if (__builtin_expect(__ballot(hit) != 0, 0)) {
          if (hit) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const uint32_t c = ((i < 4 ? w[j].x : w[j].y) >> (8 * (i & 3))) & 0xFFu;
              if ((c & 0x7Fu) == 0x7Fu) {
                const _Float16 v = (c & 0x80u) ? (_Float16)-480.0f : (_Float16)480.0f;
                if (i & 1) d[i >> 1].y = v;
                else d[i >> 1].x = v;
              }
            }
          }
        }
      } else {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          uint32_t c0, c1;
          if constexpr (FMT == FMT_TAB4) {
            c0 = (w[j].x >> (8 * p)) & 0xFu;
            c1 = (w[j].x >> (8 * p + 4)) & 0xFu;
          } else {
            const uint32_t ww = p < 2 ? w[j].x : w[j].y;
            c0 = (ww >> (16 * (p & 1))) & 0xFFu;
            c1 = (ww >> (16 * (p & 1) + 8)) & 0xFFu;
          }
          d[p] = as_h2u((uint32_t)tab[c0] | ((uint32_t)tab[c1] << 16));
        }
      }
      h8 o;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        h2 y = d[p] * s2;      // RN16 of the exact product (decode(c) is exact in fp16)
        if constexpr (ASYM) y = y + z2;
        o[2 * p] = y.x;
        o[2 * p + 1] = y.y;
      }
      __builtin_nontemporal_store(o, out + e / 8);
    }
    if (!more) break;
  }
}

template <int FMT>
hipError_t launch_unpack(const UnpackArgs& a, bool asym, hipStream_t st) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  int64_t blocks = (a.total + 4 * 2048 - 1) / (4 * 2048);
  if (blocks > (int64_t)cus * 8) blocks = (int64_t)cus * 8;
  if (asym) hipLaunchKernelGGL((k_dequant_fp_packed<FMT, true>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((k_dequant_fp_packed<FMT, false>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace
}  // namespace iwq

using namespace iwq;

extern "C" {

int iwq_dequant_fp_packed(const void* codes, const void* scales, const void* zeros, int exp_bits, int mant_bits,
                          int64_t group, int64_t N, int64_t K, void* out, int64_t ld_out, void* stream) {
  if (!codes || !scales || !out) return IWQ_ERR_ARG;
  if (N <= 0 || K <= 0 || K % 8 != 0 || ld_out != K) return IWQ_ERR_SHAPE;
  if (exp_bits < 1 || mant_bits < 0 || 1 + exp_bits + mant_bits > 8) return IWQ_ERR_BITS;
  const int bias = (1 << (exp_bits - 1)) - 1;
  // fp_max = (1 + (2^M - 1) / 2^M) 2^(2^E - 1 - bias) must fit fp16 (as in iwq_quantize_fp)
  const double fp_max = (1.0 + ((1 << mant_bits) - 1) / (double)(1 << mant_bits)) *
                        __builtin_ldexp(1.0, (1 << exp_bits) - 1 - bias);
  if (fp_max > 65504.0) return IWQ_ERR_FORMAT;
  int64_t g;
  if (group == IWQ_GROUP_PER_CHANNEL) g = K;
  else if (group == IWQ_GROUP_PER_TENSOR) g = N * K;
  else if (group > 0) g = group;
  else return IWQ_ERR_GROUP_MODE;
  if (g % 8 != 0 || (group > 0 && K % g != 0)) return IWQ_ERR_GROUP;
  const bool nib = 1 + exp_bits + mant_bits <= 4;
  if ((reinterpret_cast<uintptr_t>(codes) & (nib ? 3u : 7u)) || (reinterpret_cast<uintptr_t>(out) & 15u))
    return IWQ_ERR_ARG;
  UnpackArgs a{};
  a.codes = static_cast<const uint8_t*>(codes);
  a.scales = static_cast<const _Float16*>(scales);
  a.zeros = static_cast<const _Float16*>(zeros);
  a.out = static_cast<_Float16*>(out);
  a.total = N * K;
  a.group = g;
  a.gshift = (g & (g - 1)) == 0 ? __builtin_ctzll((unsigned long long)g) : -1;
  a.E = exp_bits;
  a.M = mant_bits;
  a.bias = bias;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool asym = zeros != nullptr;
  hipError_t e;
  if (exp_bits == 2 && mant_bits == 1) e = launch_unpack<FMT_HW4>(a, asym, st);
  else if (exp_bits == 4 && mant_bits == 3) e = launch_unpack<FMT_HW8>(a, asym, st);
  else if (nib) e = launch_unpack<FMT_TAB4>(a, asym, st);
  else e = launch_unpack<FMT_TAB8>(a, asym, st);
  if (e != hipSuccess) {
    iwq::last_hip_error() = (int)e;
    return IWQ_ERR_HIP;
  }
  return IWQ_OK;
}

}  // extern "C"

// iwq_fpdt.hip — the reference's FP weight formats on bf16 and fp32 weights (round 4).
//
// Replaces (reference, /root/reference), for a weight stored in bf16 or fp32 (T):
//   QuantLinear.quantize_weight FP4/FP6/FP8 branches   quant_linear.py:724-883
//   QuantLinear.quantize_weight_approximate             quant_linear.py:470-632 (single / double)
// The fp16 forms live in iwq_fp.hip (LDS decode tables, DPP group reductions).  Here every op runs
// in T exactly as ATen evaluates it on a T tensor -- fp32 arithmetic, one rounding to T per op:
//   scales = RN_T(max(|w|max, eps_T) / fp_max) clamped at eps_T (sym), or from mid = RN_T(RN_T(max +
//   min) * 0.5), span = RN_T(RN_T(max - min) * 0.5) (asym); t = clamp(RN_T((w [- mid]) / scales),
//   +-RN_T(fp_max)); the exponent floor(torch.log2(|t|)) with torch's own rounding in T (per-binade
//   thresholds, iwq_fp_tables_dt.h) and the .to(int8) wrap of :139; decoded value * scales
//   rounded to T; asym: + the zero point AS STORED, i.e. RN_T(RN16(mid)) (self.zeros is .half()).
//   The stored scales / zeros buffers are fp16 (.half()), as the reference's.
// E5M2 (fp_max 114688) is representable in bf16 / fp32, so it runs here (fp16 raises).
// Structure: iwq::seg's atomic group-key reduction (any group mode, quant_dim 0/1, any stride), then
// one apply kernel per element; the double-approximate decode adds a pass over quads of codes.
// HBM traffic is not the point of this path (fp16 is what the reference's models load); exactness is.
#include "iwq_common.cuh"
#include "iwq_fp.cuh"
#include "iwq_fp_tables_dt.h"
#include "iwq_seg.cuh"
#include "../../include/iwq.h"

using namespace iwq;
using iwq::seg::SegArgs;
using iwq::seg::SEG_RUN;
using iwq::seg::seg_locate;

namespace {

constexpr int BLOCK = 256;
constexpr int NTHR = 277;  // threshold entries: true exponents -149 .. 127
enum { DT_CODEC_FP = 0, DT_CODEC_APX = 1, DT_CODEC_APXD = 2 };

#define IWQ_HIP_DT(call)              \
  do {                                \
    hipError_t e_ = (call);           \
    if (e_ != hipSuccess) {           \
      iwq::last_hip_error() = (int)e_; \
      return IWQ_ERR_HIP;             \
    }                                 \
  } while (0)

// floor(torch.log2(x)) computed in T for a positive finite magnitude (fp32 bits), then .to(int8)
__device__ __forceinline__ int floor_log2_t(uint32_t mb, const uint32_t* thr) {
  const int ef = (int)(mb >> 23);
  const int e_true = ef > 0 ? ef - 127 : (31 - __builtin_clz(mb)) - 149;
  const int e = e_true + (mb >= thr[e_true + 149] ? 1 : 0);
  return (int)(int8_t)(uint8_t)(e & 0xFF);  // |x| < 2^-128 wraps to a large positive exponent
}

// _float_to_fp (quant_linear.py:126-163) on a T value t (finite, clamped), exact fp32 steps
__device__ __forceinline__ uint32_t fp_encode_t(float t, const FpSpec& f, const uint32_t* thr) {
  const uint32_t tb = __builtin_bit_cast(uint32_t, t);
  const uint32_t mb = tb & 0x7FFFFFFFu;
  if (mb == 0 || mb > 0x7F800000u) return 0;  // zero_mask; NaN (its group's output is NaN anyway)
  const uint32_t sign = tb >> 31;
  const int e = floor_log2_t(mb, thr);
  const float xa = __builtin_bit_cast(float, mb);
  const float ms = (float)(1u << f.M);
  uint32_t exp_field, mant;
  if (e >= f.emin) {  // normal path: T / fp32 tensor -> fp32 (exact)
    const int ec = e < f.emax ? e : f.emax;
    float m = __builtin_rintf((__builtin_ldexpf(xa, -ec) - 1.0f) * ms);
    m = m < 0.0f ? 0.0f : (m > ms - 1.0f ? ms - 1.0f : m);
    exp_field = (uint32_t)(ec + f.bias);
    mant = (uint32_t)m;
  } else {            // subnormal path: RN_T(x / 2^emin) * 2^M, exact in T
    float m = __builtin_rintf(__builtin_ldexpf(xa, -f.emin) * ms);
    m = m > ms - 1.0f ? ms - 1.0f : m;
    exp_field = 0;
    mant = (uint32_t)m;
  }
  return ((sign << (f.E + f.M)) | (exp_field << f.M) | mant) & 0xFFu;
}

// fp_decode_aligned_double_approx (quant_linear.py:288-363) on one quad, decode_dtype = T: the
// int8 steps of iwq_fp.cuh's fp_decode_double4, the value mant / 2^(M+tail) * 2^(tgt-bias) exact in
// fp32 (and in T: at most 8 significant bits; T's range holds every format's values)
__device__ __forceinline__ void fp_decode_double4_exact(const uint32_t (&code)[4], const FpSpec& f, float (&out)[4]) {
  int ae[4], mpad[4], sg[4];
  bool zero[4];
  int cnt = 0, gmax = -128;
  bool has_max = false;
  const int maxv = (1 << f.E) - 1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t c = code[k] & 0xFFu;
    zero[k] = c == 0;
    sg[k] = w8((int)((c >> (f.E + f.M)) & 1u));
    const int ef = w8((int)((c >> f.M) & ((1u << f.E) - 1u)));
    const int mf = w8((int)(c & ((1u << f.M) - 1u)));
    ae[k] = ef == 0 ? 1 : ef;
    const int mfull = w8(lsh8(ef == 0 ? 0 : 1, f.M) | mf);
    mpad[k] = f.tp >= 0 ? lsh8(mfull, f.tp) : rrsh8(mfull, -f.tp);
    const bool outl = ae[k] < f.hs || ae[k] > f.hf;
    cnt += outl ? 1 : 0;
    gmax = ae[k] > gmax ? ae[k] : gmax;
    has_max |= outl && ae[k] == maxv;
  }
  int tgt = cnt <= 1 ? w8(f.hf) : gmax;
  if (has_max) tgt = w8(maxv);
  const int capr = ((1 << (f.M + 1)) - 1);
  const int cap = w8(f.tp >= 0 ? (capr << f.tp) : (capr >> (-f.tp)));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int sh = w8(tgt - ae[k]);
    const int shr = sh > 0 ? sh : 0;
    const int nsh = w8(-sh);
    const int shl = nsh > 0 ? nsh : 0;
    const int mr = rrsh8(mpad[k], shr);
    int ml = lsh8(mpad[k], shl);
    ml = ml > cap ? cap : ml;
    const int mal = sh >= 0 ? mr : ml;
    float v = __builtin_ldexpf((float)mal, w8(tgt - f.bias) - (f.M + f.tp));
    v = sg[k] == 1 ? -v : v;
    out[k] = zero[k] ? 0.0f : v;
  }
}

struct ParamsT {
  float s;    // scales in T
  float z;    // zero point as added back: RN_T(RN16(mid)); 0 symmetric
  float mid;  // zero point in T (the normalization's)
};

template <int DT, bool SYM>
__device__ __forceinline__ ParamsT params_t(int32_t mnk, int32_t mxk, const FpSpec& f) {
  using F = Fmt<DT>;
  const float eps = F::R(1e-5f);
  ParamsT p{};
  if constexpr (SYM) {
    const float am = F::to_f(bits_of_key<DT>(mxk));
    const float m = am < eps ? eps : am;  // NaN stays NaN
    float s = F::R(m / f.fp_max);
    p.s = s < eps ? eps : s;
  } else {
    const float mx = F::to_f(bits_of_key<DT>(mxk)), mn = F::to_f(bits_of_key<DT>(mnk));
    const float mid = F::R(F::R(mx + mn) * 0.5f);
    float span = F::R(F::R(mx - mn) * 0.5f);
    span = span < eps ? eps : span;
    float s = F::R(span / f.fp_max);
    p.s = s < eps ? eps : s;
    p.mid = mid;
    p.z = F::R((float)(_Float16)mid);
  }
  return p;
}

__device__ __forceinline__ void store_h(void* base, int64_t i, float v) {
  gp<_Float16>(base)[i] = (_Float16)v;
}

struct DtArgs {
  SegArgs s;
  FpSpec f;
  float fpm;        // RN_T(fp_max): the clamp bounds
  float* scales_t;  // double approximate: the T scales per group (workspace), else null
};

// one element per step (iwq::seg layout); CODEC: FP (optionally codes), APX (single aligned), APXD
// (codes into the workspace + T scales for the quad pass)
template <int DT, int CODEC, bool SYM>
__global__ __launch_bounds__(BLOCK) void k_fpdt_apply(DtArgs d) {
  using F = Fmt<DT>;
  const SegArgs& a = d.s;
  __shared__ uint32_t thr[NTHR];
  for (int i = threadIdx.x; i < NTHR; i += BLOCK) thr[i] = DT == DT_BF16 ? kLog2UpBf16[i] : kLog2UpF32[i];
  __syncthreads();
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  const int64_t tid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  int64_t curj = -1;
  ParamsT p{};
  bool any_nan = false;
  for (int64_t f0 = tid * SEG_RUN; f0 < a.total; f0 += nthreads * SEG_RUN) {
    const int64_t fend = min(f0 + SEG_RUN, a.total);
    for (int64_t fi = f0; fi < fend; ++fi) {
      const int64_t j = fi / a.L;
      if (j != curj) {
        curj = j;
        p = params_t<DT, SYM>(a.keys[2 * j], a.keys[2 * j + 1], d.f);
        if (fi == j * a.L) {
          if (a.scales) store_h(a.scales, j, p.s);
          if (!SYM && a.zeros) store_h(a.zeros, j, p.mid);
          if (CODEC == DT_CODEC_APXD) d.scales_t[j] = p.s;
        }
      }
      int64_t ow, oo, r, c;
      seg_locate(a, fi, ow, oo, r, c);
      float w;
      if constexpr (F::NB == 16) w = F::to_f(gp<uint16_t>(a.w)[ow]);
      else w = F::to_f(gp<uint32_t>(a.w)[ow]);
      float t = SYM ? F::R(w / p.s) : F::R(F::R(w - p.mid) / p.s);
      t = clamp_nan(t, -d.fpm, d.fpm);
      const uint32_t code = fp_encode_t(t, d.f, thr);
      if constexpr (CODEC == DT_CODEC_APXD) {
        gp<uint8_t>(a.codes)[r * a.cols + c] = (uint8_t)code;
        continue;
      }
      float y;
      if constexpr (CODEC == DT_CODEC_APX) {
        y = F::R(F::R(fp_decode_aligned(code, d.f)) * p.s);
      } else {
        y = F::R(F::R(fp_decode(code, d.f)) * p.s);
        if constexpr (!SYM) y = F::R(y + p.z);
      }
      if (t != t) y = t;  // NaN scale: NaN out
      any_nan |= (y != y);
      if constexpr (F::NB == 16) gp<uint16_t>(a.out)[oo] = (uint16_t)F::from_f(y);
      else gp<uint32_t>(a.out)[oo] = F::from_f(y);
      if (CODEC == DT_CODEC_FP && a.codes_bits) {
        const int64_t e = r * a.cols + c;
        if (a.codes_bits == 8) {
          gp<uint8_t>(a.codes)[e] = (uint8_t)code;
        } else {
          const int64_t byte = e >> 1;
          const int shift = (int)((byte & 3) * 8 + (e & 1) * 4);
          atomicOr(reinterpret_cast<uint32_t*>(a.codes + (byte & ~(int64_t)3)), (code & 0xFu) << shift);
        }
      }
    }
  }
  const uint64_t m = __ballot(any_nan);
  if (m != 0 && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(m) && a.nan_flag) atomicOr(a.nan_flag, 1u);
}

struct QuadArgs {
  const uint8_t* codes;   // weight layout [rows, cols], one byte per element
  const float* scales_t;  // [G] T scales
  char* out;
  int64_t rows, cols, ld_out;
  int64_t g, G, gpr, nquads;
  int quant_dim;
  FpSpec f;
};

__device__ __forceinline__ void quad_locate(const QuadArgs& a, int64_t j, int64_t i, int64_t& r, int64_t& c) {
  const int64_t jr = j / a.gpr, jg = j - jr * a.gpr;
  if (a.quant_dim == 0) { r = jr; c = jg * a.g + i; }
  else { c = jr; r = jg * a.g + i; }
}

// quads = 4 consecutive elements of the grouped code matrix's transpose, flattened ([g, G] order)
template <int DT>
__global__ __launch_bounds__(BLOCK) void k_fpdt_double(QuadArgs a) {
  using F = Fmt<DT>;
  const int64_t nthreads = (int64_t)gridDim.x * BLOCK;
  for (int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x; t < a.nquads; t += nthreads) {
    int64_t rr[4], cc[4], jj[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t fi = 4 * t + k, i = fi / a.G;
      jj[k] = fi - i * a.G;
      quad_locate(a, jj[k], i, rr[k], cc[k]);
    }
    uint32_t code[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) code[k] = a.codes[rr[k] * a.cols + cc[k]];
    float v[4];
    fp_decode_double4_exact(code, a.f, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float y = F::R(F::R(v[k]) * a.scales_t[jj[k]]);
      if constexpr (F::NB == 16) gp<uint16_t>(a.out)[rr[k] * a.ld_out + cc[k]] = (uint16_t)F::from_f(y);
      else gp<uint32_t>(a.out)[rr[k] * a.ld_out + cc[k]] = F::from_f(y);
    }
  }
}

int cu_count_dt() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
  return n;
}

template <int DT>
hipError_t launch_dt(int codec, bool sym, const DtArgs& d, hipStream_t st) {
  const SegArgs& a = d.s;
  const int64_t cap = (int64_t)cu_count_dt() * 8;
  int64_t ib = (a.G + BLOCK - 1) / BLOCK;
  if (ib > cap) ib = cap;
  hipLaunchKernelGGL(iwq::seg::k_seg_init, dim3((unsigned)ib), dim3(BLOCK), 0, st, a.keys, a.G);
  int64_t blocks = (a.total + (int64_t)BLOCK * SEG_RUN - 1) / ((int64_t)BLOCK * SEG_RUN);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  if (sym) hipLaunchKernelGGL((iwq::seg::k_seg_reduce<DT, true>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  else hipLaunchKernelGGL((iwq::seg::k_seg_reduce<DT, false>), dim3((unsigned)blocks), dim3(BLOCK), 0, st, a);
  const dim3 grid((unsigned)blocks), blk(BLOCK);
  if (codec == DT_CODEC_APX) hipLaunchKernelGGL((k_fpdt_apply<DT, DT_CODEC_APX, true>), grid, blk, 0, st, d);
  else if (codec == DT_CODEC_APXD) hipLaunchKernelGGL((k_fpdt_apply<DT, DT_CODEC_APXD, true>), grid, blk, 0, st, d);
  else if (sym) hipLaunchKernelGGL((k_fpdt_apply<DT, DT_CODEC_FP, true>), grid, blk, 0, st, d);
  else hipLaunchKernelGGL((k_fpdt_apply<DT, DT_CODEC_FP, false>), grid, blk, 0, st, d);
  return hipGetLastError();
}

float rn_bf16_host(float x) {  // finite x: round to nearest even at bf16 precision
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
  float r;
  __builtin_memcpy(&r, &u, 4);
  return r;
}

bool spec_dt(int exp_bits, int mant_bits, FpSpec& f) {
  if (exp_bits < 1 || mant_bits < 0 || exp_bits + mant_bits > 7) return false;
  f.E = exp_bits;
  f.M = mant_bits;
  f.bias = (1 << (exp_bits - 1)) - 1;
  f.emin = 1 - f.bias;
  f.emax = ((1 << exp_bits) - 1) - f.bias;
  f.fp_max = (float)((1.0 + (double)((1 << mant_bits) - 1) / (double)(1 << mant_bits)) * __builtin_ldexp(1.0, f.emax));
  return true;
}

}  // namespace

namespace iwq {

int64_t fp_dt_workspace_bytes(int64_t rows, int64_t cols, int64_t G, bool double_approx) {
  auto r256 = [](int64_t b) { return (b + 255) / 256 * 256; };
  return r256(8 * G) + (double_approx ? r256(rows * cols) + r256(4 * G) : 0);
}

// bf16 / fp32 weights (dtype IWQ_BF16 / IWQ_F32): codec 0 FP (sym / asym, optional codes), 1 APX,
// 2 APX double.  scales / zeros: fp16 [G] (the reference's .half() buffers).  Workspace:
// fp_dt_workspace_bytes.  Status codes as iwq_quantize_fp.
int run_fp_dt(int codec, const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int exp_bits,
              int mant_bits, int64_t group, int symmetric, int quant_dim, void* out, int64_t ld_out, void* codes_out,
              void* scales, void* zeros, void* ws, int64_t ws_bytes, uint32_t* nan_flag, void* stream, int hs,
              int hf, int tp) {
  if (dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (!w || !out) return IWQ_ERR_ARG;
  if (rows <= 0 || cols <= 0 || ld_w < cols || ld_out < cols) return IWQ_ERR_SHAPE;
  if (quant_dim != 0 && quant_dim != 1) return IWQ_ERR_ARG;
  FpSpec f{};
  if (!spec_dt(exp_bits, mant_bits, f)) return IWQ_ERR_BITS;
  f.hs = hs;
  f.hf = hf;
  f.tp = tp;
  const int64_t vr = quant_dim == 1 ? cols : rows, vc = quant_dim == 1 ? rows : cols;
  int64_t L, G;
  if (group > 0) {
    if (vc % group != 0) return IWQ_ERR_GROUP;
    L = group;
    G = vr * vc / group;
  } else if (group == IWQ_GROUP_PER_TENSOR && codec == DT_CODEC_FP) {
    L = vr * vc;
    G = 1;
  } else if (group == IWQ_GROUP_PER_CHANNEL && codec == DT_CODEC_FP) {
    L = vc;
    G = vr;
  } else {
    return IWQ_ERR_GROUP_MODE;
  }
  const bool dbl = codec == DT_CODEC_APXD;
  if (dbl && (G * L) % 4 != 0) return IWQ_ERR_SHAPE;
  int codes = 0;
  if (codes_out) {
    if (codec != DT_CODEC_FP) return IWQ_ERR_CODES;
    codes = (exp_bits + mant_bits + 1) <= 4 ? 4 : 8;
    if (codes == 4 && (cols & 1)) return IWQ_ERR_CODES;
  }
  if (!ws || ws_bytes < fp_dt_workspace_bytes(rows, cols, G, dbl) || (reinterpret_cast<uintptr_t>(ws) & 15))
    return IWQ_ERR_WORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (codes == 4) IWQ_HIP_DT(zero_async(codes_out, (uint64_t)(rows * (cols / 2)), s));
  auto r256 = [](int64_t b) { return (b + 255) / 256 * 256; };
  uint8_t* wsb = static_cast<uint8_t*>(ws);
  DtArgs d{};
  SegArgs& a = d.s;
  a.w = static_cast<const char*>(w);
  a.out = static_cast<char*>(out);
  a.codes = dbl ? wsb + r256(8 * G) : static_cast<uint8_t*>(codes_out);
  a.scales = scales;
  a.zeros = (symmetric || codec != DT_CODEC_FP) ? nullptr : zeros;
  a.keys = reinterpret_cast<int32_t*>(wsb);
  a.rows = rows;
  a.cols = cols;
  a.ld_w = ld_w;
  a.ld_out = ld_out;
  a.vc = vc;
  a.L = L;
  a.G = G;
  a.total = rows * cols;
  a.quant_dim = quant_dim;
  a.n_bits = 8;
  a.codes_bits = codes;
  a.nan_flag = nan_flag;
  d.f = f;
  d.scales_t = dbl ? reinterpret_cast<float*>(wsb + r256(8 * G) + r256(rows * cols)) : nullptr;
  const bool sym = codec != DT_CODEC_FP || symmetric;
  if (dtype == IWQ_BF16) {
    d.fpm = rn_bf16_host(f.fp_max);  // torch.clamp converts its bounds to bf16
    IWQ_HIP_DT(launch_dt<DT_BF16>(codec, sym, d, s));
  } else {
    d.fpm = f.fp_max;
    IWQ_HIP_DT(launch_dt<DT_F32>(codec, sym, d, s));
  }
  if (!dbl) return IWQ_OK;
  QuadArgs q{};
  q.codes = a.codes;
  q.scales_t = d.scales_t;
  q.out = static_cast<char*>(out);
  q.rows = rows;
  q.cols = cols;
  q.ld_out = ld_out;
  q.g = L;
  q.G = G;
  q.gpr = vc / L;
  q.nquads = G * L / 4;
  q.quant_dim = quant_dim;
  q.f = f;
  int64_t blocks = (q.nquads + BLOCK - 1) / BLOCK;
  const int64_t cap = (int64_t)cu_count_dt() * 16;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  if (dtype == IWQ_BF16) hipLaunchKernelGGL((k_fpdt_double<DT_BF16>), dim3((unsigned)blocks), dim3(BLOCK), 0, s, q);
  else hipLaunchKernelGGL((k_fpdt_double<DT_F32>), dim3((unsigned)blocks), dim3(BLOCK), 0, s, q);
  IWQ_HIP_DT(hipGetLastError());
  return IWQ_OK;
}

}  // namespace iwq

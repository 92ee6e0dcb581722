// iwq_gemm.hip — fused dequant -> GEMM forward for packed INT4 weights on gfx950 MFMA.
//
// Replaces the fake-quant forward of the reference, QuantLinear.forward = F.linear(x, W_deq, b)
// (quant_linear.py:960-972), where W_deq is the fp16 dequantized weight written by
// quantize_weight (:935-949).  Here the weight stays packed (4 bits + per-channel / per-group fp16
// scale and zero point, include/iwq.h layout, 4x fewer weight bytes than fp16) and is dequantized
// in registers inside the GEMM: each fp16 weight element is exactly the reference's
// RN16((q - z) * s), so the result differs from F.linear on the dequantized weight only in fp32
// accumulation order.
//
// Structure (k_w4a16): 128x128 output tile per 256-thread workgroup, 4 waves as 2 (M) x 2 (N),
// each wave 64x64 = 4x4 v_mfma_f32_16x16x32_f16 tiles; K in steps of 128.
//   X tile [128 x 128] fp16: global -> registers -> LDS (double-buffered, XOR-swizzled 16-B slots,
//     halves permuted (0,4,1,5,2,6,3,7) inside each 8-element chunk), read with ds_read_b128.
//   W: each lane streams 16 B of packed codes = 32 consecutive k of one output column per 128-k
//     step straight into registers (no LDS), and per MFMA step dequantizes one dword: 8 nibbles ->
//     (1024+q) fp16 pairs by one and-or each -> minus (1024+z) (exact) -> times s (RN16).  The
//     nibble pairs come out as (k, k+4), which is why X is permuted the same way when staged: the
//     MFMA's 32-wide k slice of lane group q is the logical k range [32q+8s, 32q+8s+8) of the tile.
//   XCD-aware tile order: consecutive tiles of one X row panel are dealt to one XCD (L2 reuse).
#include "iwq_common.cuh"
#include "iwq_prefill.h"
#include "../../include/iwq.h"

using namespace iwq;

namespace {

constexpr int BM = 128, BN = 128, BK = 128, NTHR = 256;
constexpr int LDS_TILE = BM * BK * 2;  // bytes of one X tile

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const _Float16* x;    // [M, K], row stride lda
  int64_t lda;
  const uint8_t* codes; // [N, K/2] (two 4-bit codes per byte, low nibble = even k)
  const _Float16* scales;
  const _Float16* zeros;  // nullable: symmetric (z = 2^(b-1) offset folded in zoff)
  const _Float16* bias;   // nullable
  _Float16* y;          // [M, N], row stride ldy
  int64_t ldy;
  int M, N, K;
  int gpr;              // scale groups per row = K / group
  int group;            // group length along K (K for per-channel)
  int gshift;           // log2(group) when group is a power of two, else -1
  float zsym;           // symmetric code offset 2^(b-1)
  // the cross-workgroup K-split of the batched decode (k_w4a16_gemv_ct<.., KSX>, round 6): ks K ranges
  // per column group, fp32 slabs ksws[ks][M][N], one arrival counter per column group (zero on entry,
  // left zero by the last arrival)
  float* ksws;
  int* kscnt;
  int ks;
  int ksxcd;  // A/B: the ks workgroups of a column group on one XCD (block b on XCD b % 8)
};

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// 8 packed 4-bit codes (nibble p of w = k offset p) -> 8 dequantized fp16 RN16((q - z) * s) in the
// MFMA k order (0,4,1,5,2,6,3,7).  Nibbles 0/4 and 2/6 become (1024 + q) by one and-or with 0x6400
// (fp16 mantissa ulp 1 at 1024); nibbles 1/5 and 3/7 sit at mantissa bits 4..7, so or-ing 0x5400
// (64, ulp 1/16) gives (64 + q) with no shift.  (q - z) is then one exact subtraction and the only
// rounding is the multiply by s — the reference's fp16 dequant, element for element.
// Each mask-and-magic is ONE v_and_or_b32 (gfx9 VOP3 takes no literal: masks live in SGPRs, the
// magics in VGPRs, see DqConst); left to itself the compiler splits it into a VOP2 and + or.
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t mask_s, uint32_t magic_v) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(mask_s), "v"(magic_v));
  return r;
}
struct DqConst {
  uint32_t m0, m1;  // SGPR masks 0x000F000F, 0x00F000F0
  uint32_t k0, k1;  // VGPR magics 0x64006400, 0x54005400
  __device__ __forceinline__ DqConst() {
    m0 = __builtin_amdgcn_readfirstlane(0x000F000Fu);
    m1 = __builtin_amdgcn_readfirstlane(0x00F000F0u);
    asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(k0));
    asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(k1));
  }
};
__device__ __forceinline__ h8 dequant8(uint32_t w, h2 z1024, h2 z64, h2 s, const DqConst& c) {
  const uint32_t w8 = w >> 8;
  const h2 d0 = (as_h2(and_or(w, c.m0, c.k0)) - z1024) * s;
  const h2 d1 = (as_h2(and_or(w, c.m1, c.k1)) - z64) * s;
  const h2 d2 = (as_h2(and_or(w8, c.m0, c.k0)) - z1024) * s;
  const h2 d3 = (as_h2(and_or(w8, c.m1, c.k1)) - z64) * s;
  return h8{d0.x, d0.y, d1.x, d1.y, d2.x, d2.y, d3.x, d3.y};
}

// (q - z) exactly, the per-channel scale factored out into the epilogue (decode kernels, PC)
__device__ __forceinline__ h8 dequant8_ns(uint32_t w, h2 z1024, h2 z64, const DqConst& c) {
  const uint32_t w8 = w >> 8;
  const h2 d0 = as_h2(and_or(w, c.m0, c.k0)) - z1024;
  const h2 d1 = as_h2(and_or(w, c.m1, c.k1)) - z64;
  const h2 d2 = as_h2(and_or(w8, c.m0, c.k0)) - z1024;
  const h2 d3 = as_h2(and_or(w8, c.m1, c.k1)) - z64;
  return h8{d0.x, d0.y, d1.x, d1.y, d2.x, d2.y, d3.x, d3.y};
}

__device__ __forceinline__ int64_t swizzled_block(int64_t bid, int64_t nblocks) {
  const int64_t xcd = bid % 8, i = bid / 8;
  const int64_t q = nblocks / 8, r = nblocks % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
}

__global__ __launch_bounds__(NTHR) void k_w4a16(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * LDS_TILE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int q = lane >> 4, r16 = lane & 15;
  const int tiles_n = a.N / BN;
  const int64_t nblocks = (int64_t)gridDim.x;
  const int64_t t = swizzled_block(blockIdx.x, nblocks);
  const int tm = (int)(t / tiles_n), tn = (int)(t % tiles_n);
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = a.K / BK;

  // ---- X staging: 2048 16-B chunks per tile, 8 per thread (row = c >> 4, slot = c & 15)
  u32x4 xr[8];
  auto load_x = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + NTHR * i;
      const int row = c >> 4, slot = c & 15;
      const int gm = m0 + row;
      const int64_t off = (int64_t)(gm < a.M ? gm : a.M - 1) * a.lda + (int64_t)kt * BK + slot * 8;
      xr[i] = *gp<u32x4>(a.x + off);
      if (gm >= a.M) xr[i] = (u32x4){0u, 0u, 0u, 0u};
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + NTHR * i;
      const int row = c >> 4, slot = c & 15;
      const u32x4 d = xr[i];
      const u32x4 pd = {perm(d.z, d.x, 0x05040100u), perm(d.z, d.x, 0x07060302u),
                        perm(d.w, d.y, 0x05040100u), perm(d.w, d.y, 0x07060302u)};
      *reinterpret_cast<u32x4*>(smem + buf * LDS_TILE + row * 256 + ((slot ^ (row & 15)) << 4)) = pd;
    }
  };

  // ---- per-lane weight columns (one per 16-wide n subtile)
  int ncol[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) ncol[nt] = n0 + wn * 64 + nt * 16 + r16;

  const DqConst dq;
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f4){0.f, 0.f, 0.f, 0.f};

  load_x(0);
  store_x(0);
  __syncthreads();

  const int64_t crow = a.K / 2;  // bytes per packed row
  // packed codes of this lane for one 128-k step: k in [k0 + 32q, k0 + 32q + 32) of 4 columns, and
  // the scale / zero point of the group holding k0 + 32q (groups are >= 32 wide and aligned)
  auto load_b = [&](int kt, u32x4 (&bc)[4], h2 (&sv)[4], h2 (&zv)[4]) {
    const int k0 = kt * BK;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      bc[nt] = __builtin_nontemporal_load(gp<u32x4>(a.codes + (int64_t)ncol[nt] * crow + (k0 >> 1) + q * 16));
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int64_t gi = (int64_t)ncol[nt] * a.gpr + (k0 + 32 * q) / a.group;
      const _Float16 sc = gp<_Float16>(a.scales)[gi];
      const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[gi] : a.zsym;
      const _Float16 zz = (_Float16)zf;  // exact: z is a small integer
      sv[nt] = h2{sc, sc};
      zv[nt] = h2{zz, zz};
    }
  };
  const h2 k1024 = h2{(_Float16)1024.0f, (_Float16)1024.0f}, k64 = h2{(_Float16)64.0f, (_Float16)64.0f};
  u32x4 bc[4];
  h2 sv[4], zv[4];
  load_b(0, bc, sv, zv);
  for (int kt = 0; kt < nk; ++kt) {
    // next step's weights and X tile are in flight during this step's MFMAs
    u32x4 bcn[4];
    h2 svn[4], zvn[4];
    if (kt + 1 < nk) {
      load_b(kt + 1, bcn, svn, zvn);
      load_x(kt + 1);
    }
    const uint8_t* xb = smem + (kt & 1) * LDS_TILE;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      h8 af[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int row = wm * 64 + mt * 16 + r16;
        const int slot = 4 * q + s;
        af[mt] = *reinterpret_cast<const h8*>(xb + row * 256 + ((slot ^ (row & 15)) << 4));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const h8 bf = dequant8(bc[nt][s], zv[nt] + k1024, zv[nt] + k64, sv[nt], dq);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mt], bf, acc[mt][nt], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) {
      store_x((kt + 1) & 1);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        bc[nt] = bcn[nt];
        sv[nt] = svn[nt];
        zv[nt] = zvn[nt];
      }
    }
    __syncthreads();
  }

  // ---- epilogue: C layout col = lane & 15, row = 4 * (lane >> 4) + reg
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = ncol[nt];
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + mt * 16 + 4 * q + r;
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(acc[mt][nt][r] + b);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_decode: M <= 16 (token decode).  HBM-bound on the packed weight bytes (0.5 B/weight +
// scales), so the work is laid out for streaming, not for MFMA throughput: one workgroup per 16
// output columns, its WAVES waves split K and each issues ALL its 16-B code loads (one per 128-k
// step) before computing; the 16x16x32 MFMA (rows >= M zero) does the dot products, the waves'
// partial tiles are summed through LDS.  X rows are read from L2 (16 B per lane per MFMA step,
// permuted like the prefill kernel's LDS image).
// ---------------------------------------------------------------------------------------------
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_w4a16_decode(GemmArgs a) {
  constexpr int CH = 4;  // 128-k steps per chunk: all their code, scale and X loads are in flight together
  __shared__ __attribute__((aligned(16))) float red[WAVES][64 * 4];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int n = blockIdx.x * 16 + r16;
  const int nk = a.K / BK;
  const int per = (nk + WAVES - 1) / WAVES;
  const int kb = wid * per, ke = min(kb + per, nk);
  const int64_t crow = a.K / 2;
  const bool mvalid = r16 < a.M;  // A row of this lane = r16
  const _Float16* xrow = a.x + (int64_t)(mvalid ? r16 : 0) * a.lda;
  const DqConst dq;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = kb; c0 < ke; c0 += CH) {
    const int ns = min(CH, ke - c0);
    u32x4 bc[CH];
    u32x4 xa[CH][4];
    _Float16 sc[CH];
    float zf[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int kt = c0 + (i < ns ? i : 0);
      const int k0 = kt * BK;
      bc[i] = __builtin_nontemporal_load(gp<u32x4>(a.codes + (int64_t)n * crow + kt * (BK / 2) + q * 16));
      const int64_t gi = (int64_t)n * a.gpr + (k0 + 32 * q) / a.group;
      sc[i] = gp<_Float16>(a.scales)[gi];
      zf[i] = a.zeros ? (float)gp<_Float16>(a.zeros)[gi] : a.zsym;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        xa[i][s] = *gp<u32x4>(xrow + k0 + 32 * q + 8 * s);  // unconditional (row 0 for padding lanes)
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (i >= ns) break;
      const h2 sv = h2{sc[i], sc[i]};
      const _Float16 zz = (_Float16)(1024.0f + zf[i]), z6 = (_Float16)(64.0f + zf[i]);
      const h2 zv = h2{zz, zz}, zv64 = h2{z6, z6};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const u32x4 x4 = mvalid ? xa[i][s] : (u32x4){0u, 0u, 0u, 0u};
        const u32x4 pa = {perm(x4.z, x4.x, 0x05040100u), perm(x4.z, x4.x, 0x07060302u),
                          perm(x4.w, x4.y, 0x05040100u), perm(x4.w, x4.y, 0x07060302u)};
        const h8 af = __builtin_bit_cast(h8, pa);
        const h8 bf = dequant8(bc[i][s], zv, zv64, sv, dq);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, acc, 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wid][lane * 4 + r] = acc[r];
  __syncthreads();
  if (wid == 0) {
    f4 t = acc;
#pragma unroll
    for (int w = 1; w < WAVES; ++w)
#pragma unroll
      for (int r = 0; r < 4; ++r) t[r] += red[w][lane * 4 + r];
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[n] : 0.0f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * q + r;  // C layout: col = lane & 15, row = 4 * (lane >> 4) + reg
      if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + n] = (_Float16)(t[r] + b);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_gemv: M <= 16 (token decode), the weight-streaming kernel.  HBM-bound on the packed
// weight bytes, so it is organised around bytes in flight:
//   - a workgroup of T*S waves owns T tiles of 16 output columns; wave (tile, ks) takes the 128-k
//     steps ks, ks+S, ks+2S, ... of its tile (consecutive steps of one column row are loaded by
//     neighbouring waves at the same time);
//   - each wave keeps a ring of PF steps of packed-code loads (1 KiB each) in flight: step j is
//     dequantized + MFMA'd, then its slot is refilled with step j+PF;
//   - X (M x K fp16, L2-resident, shared by all workgroups) is staged once per workgroup into LDS,
//     pre-permuted to the nibble-pair order, when it fits (XLDS); then the A operand is an LDS read
//     (lgkmcnt) that never makes a wave wait behind its own code prefetches on the in-order
//     vmcnt.  Otherwise the X fragments of a step ride in the same ring slot as its codes.
//   - lanes whose A row is >= M read row M-1 (their C rows are discarded); the S partial tiles of a
//     column tile are summed through LDS in k-split order (deterministic).
// ---------------------------------------------------------------------------------------------
constexpr int XLDS_MAX = 64 * 1024;  // dynamic LDS per workgroup for the X image (2+ workgroups per CU)
// Round 6, batched decode (M = 8..16): where the grid is at most one workgroup per CU (q / o / down
// shapes, N / 16 <= 256 column tiles; the fused q/k/v at CT 4) the X image may take most of the CU's
// LDS -- 16 rows of K = 4096 are 128 KiB -- instead of being re-read from L2 at every k-step (the
// ring form below 64 KiB); staged with XB rows of loads in flight per thread.
constexpr int XLDS_BIG = 150 * 1024;
inline int gemm_cu_count() {
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
// the X image of M rows into LDS, pre-permuted to the nibble-pair order (chunk c of row m at
// dsm + m * xpitch + 16 c); XB > 1: XB rows' loads issued before their stores
template <int XB>
__device__ __forceinline__ void stage_x(const GemmArgs& a, uint8_t* dsm, int xpitch, int nthr) {
  const int cpr = a.K / 8;
  if constexpr (XB <= 1) {
    // load and store chunk by chunk: preloading the chunks first measured 3-4 % slower at M = 1 and
    // 15 % at gate M = 4, per channel (profiles/r05_ab_gemv_xpre.jsonl)
    for (int m = 0; m < a.M; ++m) {
      const _Float16* xr = a.x + (int64_t)m * a.lda;
      for (int c = threadIdx.x; c < cpr; c += nthr) {
        const u32x4 d = *gp<u32x4>(xr + 8 * c);
        const u32x4 pd = {perm(d.z, d.x, 0x05040100u), perm(d.z, d.x, 0x07060302u),
                          perm(d.w, d.y, 0x05040100u), perm(d.w, d.y, 0x07060302u)};
        *reinterpret_cast<u32x4*>(dsm + m * xpitch + 16 * c) = pd;
      }
    }
  } else {
    for (int m0 = 0; m0 < a.M; m0 += XB) {
      for (int c = threadIdx.x; c < cpr; c += nthr) {
        u32x4 d[XB];
#pragma unroll
        for (int r = 0; r < XB; ++r) {
          const int m = m0 + r < a.M ? m0 + r : a.M - 1;
          d[r] = *gp<u32x4>(a.x + (int64_t)m * a.lda + 8 * c);
        }
#pragma unroll
        for (int r = 0; r < XB; ++r) {
          if (m0 + r < a.M) {
            const u32x4 pd = {perm(d[r].z, d[r].x, 0x05040100u), perm(d[r].z, d[r].x, 0x07060302u),
                              perm(d[r].w, d[r].y, 0x05040100u), perm(d[r].w, d[r].y, 0x07060302u)};
            *reinterpret_cast<u32x4*>(dsm + (m0 + r) * xpitch + 16 * c) = pd;
          }
        }
      }
    }
  }
}
// grouped decode (round 5): the (s, z) rows of np / gpr consecutive columns starting at parameter
// index pbase, staged as one dword per group (s | z << 16), rows padded to gpr + 1 dwords.  The first
// PRE chunks per thread are loaded by pst_preload (issued together with the X image's loads) and
// written by pst_store, which also walks any longer rows.
constexpr int PST_LDS_MAX = 80 * 1024;  // X image + staged parameters per workgroup (2 per CU)
template <int PRE>
__device__ __forceinline__ void pst_preload(const GemmArgs& a, int64_t pbase, int np, int nthr, uint32_t (&ps)[PRE],
                                            uint32_t (&pz)[PRE]) {
  const uint32_t zs = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a.zsym);
#pragma unroll
  for (int r = 0; r < PRE; ++r) {
    const int i = (int)threadIdx.x + r * nthr;
    ps[r] = i < np ? (uint32_t)gp<uint16_t>(a.scales)[pbase + i] : 0u;
    pz[r] = i < np && a.zeros ? (uint32_t)gp<uint16_t>(a.zeros)[pbase + i] : zs;
  }
}
template <int PRE>
__device__ __forceinline__ void pst_store(const GemmArgs& a, uint32_t* pst, int64_t pbase, int np, int nthr,
                                          const uint32_t (&ps)[PRE], const uint32_t (&pz)[PRE]) {
#pragma unroll
  for (int r = 0; r < PRE; ++r) {
    const int i = (int)threadIdx.x + r * nthr;
    if (i < np) {
      const int c = i / a.gpr, g = i - c * a.gpr;
      pst[c * (a.gpr + 1) + g] = ps[r] | (pz[r] << 16);
    }
  }
  const uint32_t zs = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a.zsym);
  for (int i = (int)threadIdx.x + PRE * nthr; i < np; i += nthr) {  // rows longer than PRE chunks
    const int c = i / a.gpr, g = i - c * a.gpr;
    const uint32_t sv16 = gp<uint16_t>(a.scales)[pbase + i];
    const uint32_t zv16 = a.zeros ? (uint32_t)gp<uint16_t>(a.zeros)[pbase + i] : zs;
    pst[c * (a.gpr + 1) + g] = sv16 | (zv16 << 16);
  }
}

// TILED: codes in the decode tile layout (iwq_tile_codes): the 1 KiB a wave loads for one 128-k
// step of its 16 columns is contiguous (lane l = 16 q + r at byte 16 l), instead of 16 column rows x
// 64 B at a K/2 stride -- one DRAM-friendly 1 KiB burst per load instruction.
// PC (per channel, a.gpr == 1): B = (q - z) exactly and the fp32 result is scaled once in the
// epilogue, y = RN16(s * sum x (q - z) + b), as the prefill kernels' FACTOR path (4 fewer VALU per
// 8 weights; A = I still gives W_deq exactly: s (q - z) is exact in fp32)
// PST (grouped, round 5): the workgroup's parameter rows -- its 16 T columns of the reference's
// [N, K/g] scales and zero points, one contiguous run each -- are staged into LDS beside the X image
// by coalesced loads, (s, z) interleaved in one dword and the rows padded to gpr + 1 dwords (the 16
// columns a step reads land in distinct banks); a step then takes its (s, z) with one ds_read_b32
// instead of two 2-byte global gathers over 16 rows on the in-order vmcnt behind its code loads.
// GF (grouped, round 5): the scale FACTORED per k-step (group % 128 == 0: a step lies in one group):
// B = (q - z) exactly as PC, the step's four MFMAs into a fresh accumulator, then
// acc += s_g * step -- the PC numerics per group, y = RN16(sum_g s_g sum_{k in g} x (q - z) + b)
// (A = I still gives W_deq exactly), 16 fewer VALU per k-step than RN16((q - z) s) per weight.
template <int PF, int S, int T, bool XLDS, int PROBE = 0, bool TILED = false, bool PC = false, bool PST = false,
          bool GF = false, int XB = 1>
__global__ __launch_bounds__(S * T * 64) void k_w4a16_gemv(GemmArgs a) {
  static_assert(!PST || !PC, "staged parameters: grouped weights only");
  constexpr int WPB = S * T;
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = wid % T, ks = wid / T;
  const int q = lane >> 4, r16 = lane & 15;
  const int n = (blockIdx.x * T + tile) * 16 + r16;
  const int nks = a.K / BK;
  const int nj = nks > ks ? (nks - ks + S - 1) / S : 0;  // steps of this wave: kt = ks + j*S
  const int64_t crow = a.K / 2;
  const int arow = r16 < a.M ? r16 : a.M - 1;
  const int xpitch = a.K * 2 + 16;                       // LDS row pitch (bytes), +16 vs bank conflicts
  // PROBE 2 (A/B only, wrong results): k-major tile order, (kt * tiles + tile) KiB -- at any moment
  // the chip reads one contiguous window instead of one stream per tile
  const uint8_t* cbase = PROBE == 2 ? a.codes + (int64_t)(blockIdx.x * T + tile) * 1024 + lane * 16
                         : TILED ? a.codes + (int64_t)(blockIdx.x * T + tile) * nks * 1024 + lane * 16
                                 : a.codes + (int64_t)n * crow + q * 16;
  const int64_t kstride = PROBE == 2 ? (int64_t)(a.N / 16) * 1024 : (TILED ? 1024 : BK / 2);
  const _Float16* xrow = a.x + (int64_t)arow * a.lda + 32 * q;
  constexpr bool perch = PC;                              // one scale/zero per column: hoisted

  _Float16 sc0 = (_Float16)0.f, zz0 = (_Float16)0.f;
  if (perch) {
    sc0 = gp<_Float16>(a.scales)[n];
    zz0 = a.zeros ? gp<_Float16>(a.zeros)[n] : (_Float16)a.zsym;
  }
  const h2 k1024 = h2{(_Float16)1024.0f, (_Float16)1024.0f}, k64 = h2{(_Float16)64.0f, (_Float16)64.0f};
  u32x4 bc[PF];
  _Float16 sv[PF], zv[PF];
  u32x4 xa[XLDS ? 1 : PF][4];
  auto load = [&](int j, int u) {
    const int kt = ks + j * S;
    bc[u] = __builtin_nontemporal_load(gp<u32x4>(cbase + kt * kstride));
    if (!perch && !PST) {
      const int kk = kt * BK + 32 * q;
      const int64_t gi = (int64_t)n * a.gpr + (a.gshift >= 0 ? (kk >> a.gshift) : kk / a.group);
      sv[u] = gp<_Float16>(a.scales)[gi];
      zv[u] = a.zeros ? gp<_Float16>(a.zeros)[gi] : (_Float16)a.zsym;
    }
    if constexpr (!XLDS) {
      if constexpr (PROBE == 5) {  // A/B probe (wrong results): the same X bytes, lanes q of a row on
        // one contiguous 64 B per instruction (piece 4 s + q instead of 4 q + s)
#pragma unroll
        for (int s = 0; s < 4; ++s) xa[u][s] = *gp<u32x4>(xrow - 32 * q + kt * BK + 32 * s + 8 * q);
      } else if constexpr (PROBE == 6) {  // A/B probe (wrong results): no X loads at all
#pragma unroll
        for (int s = 0; s < 4; ++s) xa[u][s] = (u32x4){(uint32_t)kt, (uint32_t)s, 0x3C003C00u, 0u};
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) xa[u][s] = *gp<u32x4>(xrow + kt * BK + 8 * s);
      }
    }
  };
  // the code prefetch first (DRAM: the longest latency); then the staged parameters' first PRE
  // chunks (PST) and the X image (XLDS).  (Issuing X before the codes, so that its wait does not
  // include them in vmcnt order, measured 4-7 % SLOWER on every shape: the codes' DRAM latency is
  // the critical path.)
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nj) load(u, u);
  constexpr int PRE = 4;
  // PST: after the X image (or at the start without one)
  uint32_t* pst = reinterpret_cast<uint32_t*>(dsm + (XLDS ? (a.M * xpitch + 15) / 16 * 16 : 0));
  const int np = PST ? T * 16 * a.gpr : 0;
  const int64_t pbase = (int64_t)blockIdx.x * np;
  uint32_t pre_s[PRE], pre_z[PRE];
  if constexpr (PST) pst_preload<PRE>(a, pbase, np, WPB * 64, pre_s, pre_z);  // before X's waits
  if constexpr (XLDS || PST) {
    // 16-B chunk c of X row m -> permuted (0,4,1,5,2,6,3,7) at dsm + m*xpitch + 16c
    if constexpr (XLDS) stage_x<XB>(a, dsm, xpitch, WPB * 64);
    if constexpr (PST) pst_store<PRE>(a, pst, pbase, np, WPB * 64, pre_s, pre_z);
    __syncthreads();
  }
  const uint8_t* xsrow = dsm + arow * xpitch + 64 * q;
  // PST: this lane's column row of the staged parameters (tile, r16)
  const uint32_t* prow = pst + (tile * 16 + r16) * (a.gpr + 1);
  const DqConst dq;

  f4 acc = {0.f, 0.f, 0.f, 0.f};
  // GF: the running k-step's partial tile, and the previous step's (folded into acc only after this
  // step's MFMAs are issued, so the VALU never waits on the MFMA chain it just fed)
  f4 accs = {0.f, 0.f, 0.f, 0.f}, accp = {0.f, 0.f, 0.f, 0.f};
  float sfp = 0.f;
  for (int j0 = 0; j0 < nj; j0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int j = j0 + u;
      if (j >= nj) break;
      const int kt = ks + j * S;
      h2 s2, z2;
      float sf = 0.f;  // GF: the step's group scale
      if constexpr (PST) {
        const int kk = kt * BK + 32 * q;
        const uint32_t sz = prow[a.gshift >= 0 ? (kk >> a.gshift) : kk / a.group];
        if constexpr (GF) sf = (float)__builtin_bit_cast(_Float16, (uint16_t)(sz & 0xFFFFu));
        else s2 = as_h2(__builtin_amdgcn_perm(sz, sz, 0x01000100u));
        z2 = as_h2(__builtin_amdgcn_perm(sz, sz, 0x03020302u));
      } else {
        s2 = perch ? h2{sc0, sc0} : h2{sv[u], sv[u]};
        z2 = perch ? h2{zz0, zz0} : h2{zv[u], zv[u]};
        if constexpr (GF) sf = (float)sv[u];
      }
      const h2 z1024 = z2 + k1024, z64 = z2 + k64;  // exact: z is a small integer
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        h8 af;
        if constexpr (XLDS) {
          af = *reinterpret_cast<const h8*>(xsrow + kt * (BK * 2) + 16 * s);
        } else {
          const u32x4 x4 = xa[u][s];
          const u32x4 pa = {perm(x4.z, x4.x, 0x05040100u), perm(x4.z, x4.x, 0x07060302u),
                            perm(x4.w, x4.y, 0x05040100u), perm(x4.w, x4.y, 0x07060302u)};
          af = __builtin_bit_cast(h8, pa);
        }
        h8 bf;
        if constexpr (PROBE == 1 || PROBE == 2) {  // A/B probe only: no dequantization (wrong results)
          const uint32_t w = bc[u][s];
          bf = __builtin_bit_cast(h8, (u32x4){w, w ^ 1u, w ^ 2u, w ^ 3u});
        } else if constexpr (PC || GF) {
          bf = dequant8_ns(bc[u][s], z1024, z64, dq);
        } else {
          bf = dequant8(bc[u][s], z1024, z64, s2, dq);
        }
        if constexpr (GF) accs = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, s == 0 ? f4{0.f, 0.f, 0.f, 0.f} : accs, 0, 0, 0);
        else acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, acc, 0, 0, 0);
      }
      if constexpr (GF) {  // this lane's 4 accumulators all belong to its column r16: one scale
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(sfp, accp[e], acc[e]);  // step j - 1 (0 at j = 0)
        accp = accs;
        sfp = sf;
      }
      if (j + PF < nj) load(j + PF, u);
    }
  }
  if constexpr (GF) {
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(sfp, accp[e], acc[e]);  // the last step
  }
  if constexpr (XLDS || PST) __syncthreads();  // X image / parameters dead: the LDS now holds the partial tiles
  float* red = reinterpret_cast<float*>(dsm);  // [WPB][256], wave (tile, ks) at index ks*T + tile
  *reinterpret_cast<f4*>(red + wid * 256 + lane * 4) = acc;
  __syncthreads();
  for (int o = threadIdx.x; o < T * 256; o += WPB * 64) {
    const int t = o >> 8, e = o & 255;                    // e = lane' * 4 + reg of the C layout
    const int ln = e >> 2, reg = e & 3;
    const int row = 4 * (ln >> 4) + reg, col = (blockIdx.x * T + t) * 16 + (ln & 15);
    if (row < a.M) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) v += red[(k * T + t) * 256 + e];
      if constexpr (PC) v = opaque(v * (float)gp<_Float16>(a.scales)[col]);  // no fma_mix fold
      if (a.bias) v += (float)gp<_Float16>(a.bias)[col];
      gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)v;
    }
  }
}

// k_w4a16_gemv_ct: the same weight stream for 4 <= M <= 16, where X, not the codes, dominates the
// on-chip traffic: k_w4a16_gemv reads (or stages) X once per 16-column tile, M * 256 B per 1 KiB of
// codes (M = 16: 4x the code bytes from L2).  Here each wave applies one A fragment to CT column
// tiles (CT code loads per k-step, CT accumulators), so X traffic per code byte drops CT-fold.
// Same k-split S and the same per-tile accumulation order as k_w4a16_gemv<.., S, ..>: identical bits
// (GF: the grouped scale factored per k-step, as k_w4a16_gemv's PM 2).
template <int PF, int S, int CT, bool XLDS, bool TILED, bool PC = false, bool GF = false, bool PST = false,
          int XB = 1, bool KSX = false>
__global__ __launch_bounds__(S * 64) void k_w4a16_gemv_ct(GemmArgs a) {
  static_assert(!PST || !PC, "staged parameters: grouped weights only");
  static_assert(!KSX || !XLDS, "the K-split form reads X per k-step (no whole-row image)");
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int lane = threadIdx.x & 63;
  const int ks = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  // KSX: workgroup b = column group b / a.ks, K range b % a.ks (k-steps [kb, ke) of the nks)
  int cgrp = KSX ? (int)blockIdx.x / a.ks : (int)blockIdx.x;
  int ksi = KSX ? (int)blockIdx.x - cgrp * a.ks : 0;
  if (KSX && a.ksxcd) {  // block b = x + 8 j: XCD x's j-th workgroup -> group x + 8 (j / ks), range j % ks
    const int xj = (int)blockIdx.x >> 3;
    cgrp = ((int)blockIdx.x & 7) + 8 * (xj / a.ks);
    ksi = xj - (xj / a.ks) * a.ks;
  }
  const int tile0 = cgrp * CT;
  const int nks = a.K / BK;
  const int kb = KSX ? (int)((int64_t)nks * ksi / a.ks) : 0;
  const int nkr = KSX ? (int)((int64_t)nks * (ksi + 1) / a.ks) - kb : nks;
  const int nj = nkr > ks ? (nkr - ks + S - 1) / S : 0;
  const int64_t crow = a.K / 2;
  const int arow = r16 < a.M ? r16 : a.M - 1;
  const int xpitch = a.K * 2 + 16;
  const int64_t tstride = TILED ? (int64_t)nks * 1024 : 16 * crow;  // code bytes between column tiles
  const uint8_t* cbase = TILED ? a.codes + (int64_t)tile0 * tstride + lane * 16
                               : a.codes + (int64_t)(tile0 * 16 + r16) * crow + q * 16;
  const _Float16* xrow = a.x + (int64_t)arow * a.lda + 32 * q;
  constexpr bool perch = PC;

  _Float16 sc0[CT], zz0[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int n = (tile0 + c) * 16 + r16;
    sc0[c] = perch ? gp<_Float16>(a.scales)[n] : (_Float16)0.f;
    zz0[c] = perch ? (a.zeros ? gp<_Float16>(a.zeros)[n] : (_Float16)a.zsym) : (_Float16)0.f;
  }
  const h2 k1024 = h2{(_Float16)1024.0f, (_Float16)1024.0f}, k64 = h2{(_Float16)64.0f, (_Float16)64.0f};
  u32x4 bc[PF][CT];
  _Float16 sv[PF][CT], zv[PF][CT];
  u32x4 xa[XLDS ? 1 : PF][4];
  auto load = [&](int j, int u) {
    const int kt = kb + ks + j * S;
#pragma unroll
    for (int c = 0; c < CT; ++c)
      bc[u][c] = __builtin_nontemporal_load(gp<u32x4>(cbase + c * tstride + kt * (TILED ? 1024 : BK / 2)));
    if (!perch && !PST) {
      const int kk = kt * BK + 32 * q;
      const int gk = a.gshift >= 0 ? (kk >> a.gshift) : kk / a.group;
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int64_t gi = (int64_t)((tile0 + c) * 16 + r16) * a.gpr + gk;
        sv[u][c] = gp<_Float16>(a.scales)[gi];
        zv[u][c] = a.zeros ? gp<_Float16>(a.zeros)[gi] : (_Float16)a.zsym;
      }
    }
    if constexpr (!XLDS) {
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[u][s] = *gp<u32x4>(xrow + kt * BK + 8 * s);
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nj) load(u, u);

  // PST (round 5, as k_w4a16_gemv): the CT tiles' parameter rows, after the X image
  constexpr int PRE = 4;
  uint32_t* pst = reinterpret_cast<uint32_t*>(dsm + (XLDS ? (a.M * xpitch + 15) / 16 * 16 : 0));
  const int np = PST ? CT * 16 * a.gpr : 0;
  const int64_t pbase = (int64_t)tile0 * 16 * a.gpr;
  uint32_t pre_s[PRE], pre_z[PRE];
  if constexpr (PST) pst_preload<PRE>(a, pbase, np, S * 64, pre_s, pre_z);
  if constexpr (XLDS || PST) {
    if constexpr (XLDS) stage_x<XB>(a, dsm, xpitch, S * 64);
    if constexpr (PST) pst_store<PRE>(a, pst, pbase, np, S * 64, pre_s, pre_z);
    __syncthreads();
  }
  const uint8_t* xsrow = dsm + arow * xpitch + 64 * q;
  const DqConst dq;

  f4 acc[CT], accs[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) acc[c] = accs[c] = f4{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nj; j0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int j = j0 + u;
      if (j >= nj) break;
      const int kt = kb + ks + j * S;
      h2 s2[CT], z1024[CT], z64[CT];
      float sf[CT];  // GF: the step's group scale per tile
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        h2 z2;
        if constexpr (PST) {
          const int kk = kt * BK + 32 * q;
          const uint32_t sz = pst[(c * 16 + r16) * (a.gpr + 1) + (a.gshift >= 0 ? (kk >> a.gshift) : kk / a.group)];
          s2[c] = as_h2(__builtin_amdgcn_perm(sz, sz, 0x01000100u));
          z2 = as_h2(__builtin_amdgcn_perm(sz, sz, 0x03020302u));
          sf[c] = (float)__builtin_bit_cast(_Float16, (uint16_t)(sz & 0xFFFFu));
        } else {
          s2[c] = perch ? h2{sc0[c], sc0[c]} : h2{sv[u][c], sv[u][c]};
          z2 = perch ? h2{zz0[c], zz0[c]} : h2{zv[u][c], zv[u][c]};
          sf[c] = perch ? 0.f : (float)sv[u][c];
        }
        z1024[c] = z2 + k1024;
        z64[c] = z2 + k64;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        h8 af;
        if constexpr (XLDS) {
          af = *reinterpret_cast<const h8*>(xsrow + kt * (BK * 2) + 16 * s);
        } else {
          const u32x4 x4 = xa[u][s];
          const u32x4 pa = {perm(x4.z, x4.x, 0x05040100u), perm(x4.z, x4.x, 0x07060302u),
                            perm(x4.w, x4.y, 0x05040100u), perm(x4.w, x4.y, 0x07060302u)};
          af = __builtin_bit_cast(h8, pa);
        }
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          if constexpr (GF)
            accs[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dequant8_ns(bc[u][c][s], z1024[c], z64[c], dq),
                                                             s == 0 ? f4{0.f, 0.f, 0.f, 0.f} : accs[c], 0, 0, 0);
          else
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, PC ? dequant8_ns(bc[u][c][s], z1024[c], z64[c], dq) : dequant8(bc[u][c][s], z1024[c], z64[c], s2[c], dq),
                acc[c], 0, 0, 0);
        }
      }
      if constexpr (GF) {
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[c][e] = __builtin_fmaf(sf[c], accs[c][e], acc[c][e]);
      }
      if (j + PF < nj) load(j + PF, u);
    }
  }
  if constexpr (XLDS || PST) __syncthreads();
  float* red = reinterpret_cast<float*>(dsm);  // [S][CT][256]
#pragma unroll
  for (int c = 0; c < CT; ++c) *reinterpret_cast<f4*>(red + (ks * CT + c) * 256 + lane * 4) = acc[c];
  __syncthreads();
  auto finish = [&](float v, int row, int col) {
    if constexpr (PC) v = opaque(v * (float)gp<_Float16>(a.scales)[col]);  // no fma_mix fold
    if (a.bias) v += (float)gp<_Float16>(a.bias)[col];
    gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)v;
  };
  const bool split = KSX && a.ks > 1;
  for (int o = threadIdx.x; o < CT * 256; o += S * 64) {
    const int c = o >> 8, e = o & 255;
    const int ln = e >> 2, reg = e & 3;
    const int row = 4 * (ln >> 4) + reg, col = (tile0 + c) * 16 + (ln & 15);
    if (row < a.M) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) v += red[(k * CT + c) * 256 + e];
      if (split)  // this K range's partial, device-coherent (the last arrival may sit on another XCD)
        __hip_atomic_store(a.ksws + ((int64_t)ksi * a.M + row) * a.N + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        finish(v, row, col);
    }
  }
  if constexpr (KSX) {
    if (split) {
      // every wave's slab stores complete before the arrival (the stores are device-coherent: a wait
      // for them, not an agent-scope release fence -- on gfx950 that fence writes back the whole L2,
      // and one per workgroup serialised the grid: 20-550 us per call, profiles/r06_gemv_ksx_ab.jsonl);
      // the last of the a.ks workgroups of the column group sums the slabs in K-range order
      // (deterministic) with device-coherent loads, finishes the tile and clears the counter
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      __shared__ int last;
      if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(a.kscnt + cgrp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = old == a.ks - 1;
        if (last) __hip_atomic_store(a.kscnt + cgrp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (last) {
        for (int o = threadIdx.x; o < CT * 256; o += S * 64) {
          const int c = o >> 8, e = o & 255;
          const int ln = e >> 2, reg = e & 3;
          const int row = 4 * (ln >> 4) + reg, col = (tile0 + c) * 16 + (ln & 15);
          if (row < a.M) {
            float v = 0.f;
            for (int k = 0; k < a.ks; ++k)
              v += __hip_atomic_load(a.ksws + ((int64_t)k * a.M + row) * a.N + col, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            finish(v, row, col);
          }
        }
      }
    }
  }
}

// k_w4a16_gemv_ks (round 6): batched decode, 8 <= M <= 16, where X (M x K fp16) outgrows the LDS
// image and every workgroup would otherwise re-read all of it from L2 -- at M = 16 the X bytes a CU
// reads per call are 4x its code bytes (7B down_proj: 352 KiB of X per 16-column tile; the whole
// call 90 MB of L2 traffic against 22.5 MB of codes).  The K range is split over KS workgroups per CT
// column tiles: each stages its X SLICE (M x K / KS) in LDS once, streams its k-steps with
// k_w4a16_gemv_ct's inner loop (wave w: the slice's k-steps w, w + S, ...), sums its S waves' partial
// tiles in LDS in wave order and writes one fp32 slab ws[ks][m][n]; k_gemv_ks_reduce then sums the
// KS slabs in ks order, applies the per-channel scale and the bias and rounds to fp16 once --
// deterministic, X traffic / KS, one extra launch.  Per-channel numerics as PC (y = RN16(s sum x (q - z)
// + b)), grouped as GF (acc += s_g step); X = rows of the identity still gives W_deq bit for bit.
template <int PF, int S, int CT, bool TILED, bool PC = false, bool GF = false, bool PST = false>
__global__ __launch_bounds__(S * 64) void k_w4a16_gemv_ks(GemmArgs a, float* ws, int KS) {
  static_assert(!PST || !PC, "staged parameters: grouped weights only");
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int cg = blockIdx.x / KS, ksi = blockIdx.x - (blockIdx.x / KS) * KS;
  const int tile0 = cg * CT;
  const int nks = a.K / BK;
  const int k0 = (int)((int64_t)nks * ksi / KS), k1 = (int)((int64_t)nks * (ksi + 1) / KS);
  const int nkr = k1 - k0;
  const int nj = nkr > wv ? (nkr - wv + S - 1) / S : 0;  // steps of this wave: kt = k0 + wv + j S
  const int64_t crow = a.K / 2;
  const int arow = r16 < a.M ? r16 : a.M - 1;
  const int xpitch = nkr * BK * 2 + 16;
  const int64_t tstride = TILED ? (int64_t)nks * 1024 : 16 * crow;
  const uint8_t* cbase = TILED ? a.codes + (int64_t)tile0 * tstride + lane * 16
                               : a.codes + (int64_t)(tile0 * 16 + r16) * crow + q * 16;
  constexpr bool perch = PC;
  _Float16 zz0[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int n = (tile0 + c) * 16 + r16;
    zz0[c] = perch ? (a.zeros ? gp<_Float16>(a.zeros)[n] : (_Float16)a.zsym) : (_Float16)0.f;
  }
  const h2 k1024 = h2{(_Float16)1024.0f, (_Float16)1024.0f}, k64 = h2{(_Float16)64.0f, (_Float16)64.0f};
  u32x4 bc[PF][CT];
  _Float16 sv[PF][CT], zv[PF][CT];
  auto load = [&](int j, int u) {
    const int kt = k0 + wv + j * S;
#pragma unroll
    for (int c = 0; c < CT; ++c)
      bc[u][c] = __builtin_nontemporal_load(gp<u32x4>(cbase + c * tstride + kt * (TILED ? 1024 : BK / 2)));
    if (!perch && !PST) {
      const int kk = kt * BK + 32 * q;
      const int gk = a.gshift >= 0 ? (kk >> a.gshift) : kk / a.group;
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int64_t gi = (int64_t)((tile0 + c) * 16 + r16) * a.gpr + gk;
        sv[u][c] = gp<_Float16>(a.scales)[gi];
        zv[u][c] = a.zeros ? gp<_Float16>(a.zeros)[gi] : (_Float16)a.zsym;
      }
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nj) load(u, u);
  // the X slice (permuted as the image of k_w4a16_gemv), then the staged parameters (PST)
  constexpr int PRE = 4;
  uint32_t* pst = reinterpret_cast<uint32_t*>(dsm + (a.M * xpitch + 15) / 16 * 16);
  const int np = PST ? CT * 16 * a.gpr : 0;
  const int64_t pbase = (int64_t)tile0 * 16 * a.gpr;
  uint32_t pre_s[PRE], pre_z[PRE];
  if constexpr (PST) pst_preload<PRE>(a, pbase, np, S * 64, pre_s, pre_z);
  {
    const int cpr = nkr * (BK / 8);  // 16-B chunks per row of the slice
    for (int m0 = 0; m0 < a.M; m0 += 8) {
      for (int c = threadIdx.x; c < cpr; c += S * 64) {
        u32x4 d[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int m = m0 + r < a.M ? m0 + r : a.M - 1;
          d[r] = *gp<u32x4>(a.x + (int64_t)m * a.lda + (int64_t)k0 * BK + 8 * c);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if (m0 + r < a.M) {
            const u32x4 pd = {perm(d[r].z, d[r].x, 0x05040100u), perm(d[r].z, d[r].x, 0x07060302u),
                              perm(d[r].w, d[r].y, 0x05040100u), perm(d[r].w, d[r].y, 0x07060302u)};
            *reinterpret_cast<u32x4*>(dsm + (m0 + r) * xpitch + 16 * c) = pd;
          }
        }
      }
    }
  }
  if constexpr (PST) pst_store<PRE>(a, pst, pbase, np, S * 64, pre_s, pre_z);
  __syncthreads();
  const uint8_t* xsrow = dsm + arow * xpitch + 64 * q;
  const DqConst dq;
  f4 acc[CT], accs[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) acc[c] = accs[c] = f4{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nj; j0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int j = j0 + u;
      if (j >= nj) break;
      const int kt = k0 + wv + j * S;
      h2 s2[CT], z1024[CT], z64[CT];
      float sf[CT];
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        h2 z2;
        if constexpr (PST) {
          const int kk = kt * BK + 32 * q;
          const uint32_t sz = pst[(c * 16 + r16) * (a.gpr + 1) + (a.gshift >= 0 ? (kk >> a.gshift) : kk / a.group)];
          s2[c] = as_h2(__builtin_amdgcn_perm(sz, sz, 0x01000100u));
          z2 = as_h2(__builtin_amdgcn_perm(sz, sz, 0x03020302u));
          sf[c] = (float)__builtin_bit_cast(_Float16, (uint16_t)(sz & 0xFFFFu));
        } else {
          s2[c] = perch ? h2{(_Float16)0.f, (_Float16)0.f} : h2{sv[u][c], sv[u][c]};
          z2 = perch ? h2{zz0[c], zz0[c]} : h2{zv[u][c], zv[u][c]};
          sf[c] = perch ? 0.f : (float)sv[u][c];
        }
        z1024[c] = z2 + k1024;
        z64[c] = z2 + k64;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const h8 af = *reinterpret_cast<const h8*>(xsrow + (kt - k0) * (BK * 2) + 16 * s);
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          if constexpr (GF)
            accs[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dequant8_ns(bc[u][c][s], z1024[c], z64[c], dq),
                                                             s == 0 ? f4{0.f, 0.f, 0.f, 0.f} : accs[c], 0, 0, 0);
          else
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, PC ? dequant8_ns(bc[u][c][s], z1024[c], z64[c], dq) : dequant8(bc[u][c][s], z1024[c], z64[c], s2[c], dq),
                acc[c], 0, 0, 0);
        }
      }
      if constexpr (GF) {
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[c][e] = __builtin_fmaf(sf[c], accs[c][e], acc[c][e]);
      }
      if (j + PF < nj) load(j + PF, u);
    }
  }
  __syncthreads();  // the X slice and parameters are dead: the LDS now holds the waves' partial tiles
  float* red = reinterpret_cast<float*>(dsm);  // [S][CT][256]
#pragma unroll
  for (int c = 0; c < CT; ++c) *reinterpret_cast<f4*>(red + (wv * CT + c) * 256 + lane * 4) = acc[c];
  __syncthreads();
  float* slab = ws + (int64_t)ksi * a.M * a.N;
  for (int o = threadIdx.x; o < CT * 256; o += S * 64) {
    const int c = o >> 8, e = o & 255;
    const int ln = e >> 2, reg = e & 3;
    const int row = 4 * (ln >> 4) + reg, col = (tile0 + c) * 16 + (ln & 15);
    if (row < a.M) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) v += red[(k * CT + c) * 256 + e];
      slab[(int64_t)row * a.N + col] = v;
    }
  }
}

// the KS fp32 slabs of k_w4a16_gemv_ks summed in ks order, per-channel scale (PC) and bias, one
// rounding to fp16; 4 consecutive columns per thread (N % 16 == 0)
template <bool PC>
__global__ __launch_bounds__(256) void k_gemv_ks_reduce(GemmArgs a, const float* ws, int KS) {
  const int64_t total = (int64_t)a.M * a.N, n4 = total / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f4 v = *gp<f4>(ws + 4 * i);
    for (int k = 1; k < KS; ++k) {
      const f4 t = *gp<f4>(ws + (int64_t)k * total + 4 * i);
      v = v + t;
    }
    const int64_t e0 = 4 * i;
    const int row = (int)(e0 / a.N), col = (int)(e0 - (int64_t)row * a.N);
    _Float16* yr = a.y + (int64_t)row * a.ldy + col;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float r = v[j];
      if constexpr (PC) r = opaque(r * (float)gp<_Float16>(a.scales)[col + j]);  // no fma_mix fold
      if (a.bias) r += (float)gp<_Float16>(a.bias)[col + j];
      gp<_Float16>(yr)[j] = (_Float16)r;
    }
  }
}

// The K-split decode plan: 8 <= M <= 16, X over the 64 KiB image budget; CT 4 column tiles per
// workgroup, KS the smallest power of two whose X slice fits 80 KiB (two workgroups per CU) and whose
// grid covers the CUs.  Returns false where the one-launch kernels keep X resident.
inline bool gemv_ks_plan(int64_t M, int64_t N, int64_t K, int* ct_out, int* ks_out) {
  if (M < 8 || M > 16 || N % 64 != 0 || K % BK != 0) return false;
  if (M * (2 * K + 16) <= XLDS_MAX) return false;
  const int64_t nks = K / BK, groups = N / 64;
  for (int ks = 2; ks <= 16; ks *= 2) {
    const int64_t steps = (nks + ks - 1) / ks;
    if (steps < 8) return false;  // at least one k-step per wave
    if (M * (steps * BK * 2 + 16) > 80 * 1024) continue;
    if (groups * ks < gemm_cu_count() && ks < 16) continue;
    if (ct_out) *ct_out = 4;
    if (ks_out) *ks_out = ks;
    return true;
  }
  return false;
}
constexpr bool GEMV_KS_DEFAULT = false;
inline int64_t gemv_ks_bytes(int64_t M, int64_t N, int64_t K) {
  int ks = 0;
  return gemv_ks_plan(M, N, K, nullptr, &ks) ? (int64_t)ks * M * N * 4 : 0;
}

template <int PF, int S, bool TILED>
void launch_gemv_ks(const GemmArgs& a, hipStream_t st, float* ws, int KS) {
  constexpr int CT = 4;
  const int nks = a.K / BK;
  const int smax = (nks + KS - 1) / KS;
  const int64_t xbytes = ((int64_t)a.M * (smax * BK * 2 + 16) + 15) / 16 * 16;
  const unsigned blocks = (unsigned)(a.N / (16 * CT) * KS);
  const size_t red = (size_t)S * CT * 256 * 4;
  const bool pc = a.gpr == 1;
  const bool gf = !pc && a.group % BK == 0;
  const int64_t pend = xbytes + (int64_t)16 * CT * (a.gpr + 1) * 4;
  const bool pst = gf && pend <= 96 * 1024;
  const size_t lds = red > (size_t)(pst ? pend : xbytes) ? red : (size_t)(pst ? pend : xbytes);
  if (pc) hipLaunchKernelGGL((k_w4a16_gemv_ks<PF, S, CT, TILED, true>), dim3(blocks), dim3(S * 64), lds, st, a, ws, KS);
  else if (pst) hipLaunchKernelGGL((k_w4a16_gemv_ks<PF, S, CT, TILED, false, true, true>), dim3(blocks), dim3(S * 64), lds, st, a, ws, KS);
  else if (gf) hipLaunchKernelGGL((k_w4a16_gemv_ks<PF, S, CT, TILED, false, true>), dim3(blocks), dim3(S * 64), lds, st, a, ws, KS);
  else hipLaunchKernelGGL((k_w4a16_gemv_ks<PF, S, CT, TILED>), dim3(blocks), dim3(S * 64), lds, st, a, ws, KS);
  const int64_t n4 = (int64_t)a.M * a.N / 4;
  int64_t rb = (n4 + 255) / 256;
  if (rb > 1024) rb = 1024;
  if (pc) hipLaunchKernelGGL(k_gemv_ks_reduce<true>, dim3((unsigned)rb), dim3(256), 0, st, a, ws, KS);
  else hipLaunchKernelGGL(k_gemv_ks_reduce<false>, dim3((unsigned)rb), dim3(256), 0, st, a, ws, KS);
}

// The cross-workgroup K-split of the batched decode (round 6, k_w4a16_gemv_ct<.., KSX>).  At M = 16
// the X rows, not the codes, are what a workgroup waits for: every workgroup of the unsplit kernels reads
// all of X (M x K fp16) from L2 -- 128 KiB per CU on K = 4096, 344 KiB on K = 11008 -- at the ~70 GB/s
// per CU an L2-served stream gets (MI355X_MICROARCH.md §Indexed rows), 2.3 / 5.7 us of the 6.7 / 13.6
// us q / down calls (an A/B probe without X loads runs M = 16 at the M = 1 time: profiles/
// r06_gemv_xstream.jsonl).  X bytes per workgroup are M * 2 * (its K range) against 8 * CT * (its K
// range) of codes, so CT = 4 tiles per workgroup make X 1 : 1 with the codes at M = 16, and KS K ranges
// per column group bring the grid back to the CU count: KS times less X per CU.  The KS partial tiles
// meet in fp32 slabs; the last workgroup of a column group to arrive (one agent-scope counter per group,
// zero on entry and cleared again by that workgroup: IWQ_FLAG_WS_ZEROED) sums them in K-range order and
// finishes the tile in the same launch.  Workspace: the counters (GEMV_KSX_CNT_BYTES, G <= 4096 of them
// used), then KS * M * N fp32.
constexpr int GEMV_KSX_CT = 4;
// the counter region has one fixed size, whatever the call's N: a per-stream workspace serves calls of
// every shape, and one call's slabs must never lie where another call expects zero counters
constexpr int64_t GEMV_KSX_CNT_BYTES = 16384;
inline bool gemv_ksx_plan(int64_t M, int64_t N, int64_t K, int* ct_out, int* ks_out) {
  if (M < 8 || M > 16 || N % (16 * GEMV_KSX_CT) != 0 || K % BK != 0) return false;
  const int64_t g = N / (16 * GEMV_KSX_CT), nks = K / BK, cus = gemm_cu_count();
  if (g >= cus || g * 4 > GEMV_KSX_CNT_BYTES) return false;
  const int64_t ks = (cus + g - 1) / g;
  if (nks / ks < 4) return false;
  if (ct_out) *ct_out = GEMV_KSX_CT;
  if (ks_out) *ks_out = (int)ks;
  return true;
}
inline int64_t gemv_ksx_cnt_bytes(int64_t N, int ct) { return (void)N, (void)ct, GEMV_KSX_CNT_BYTES; }
inline int64_t gemv_ksx_bytes_for(int64_t M, int64_t N, int ct, int ks) {
  return gemv_ksx_cnt_bytes(N, ct) + (int64_t)ks * M * N * 4;
}
inline int64_t gemv_ksx_bytes(int64_t M, int64_t N, int64_t K) {
  int ct = 0, ks = 0;
  return gemv_ksx_plan(M, N, K, &ct, &ks) ? gemv_ksx_bytes_for(M, N, ct, ks) : 0;
}
constexpr bool GEMV_KSX_DEFAULT = false;

template <int PF, int S, int CT, bool TILED>
void launch_gemv_ksx(GemmArgs a, hipStream_t st, void* ws, int KS, bool xcd = false) {
  a.ksxcd = xcd ? 1 : 0;
  a.kscnt = static_cast<int*>(ws);
  a.ksws = reinterpret_cast<float*>(static_cast<uint8_t*>(ws) + gemv_ksx_cnt_bytes(a.N, CT));
  a.ks = KS;
  const unsigned blocks = (unsigned)(a.N / (16 * CT) * KS);
  const size_t red = (size_t)S * CT * 256 * 4;
  const bool pc = a.gpr == 1;
  const bool gf = !pc && a.group % BK == 0;
  const int64_t pend = (int64_t)16 * CT * (a.gpr + 1) * 4;
  const bool pst = gf && pend <= PST_LDS_MAX;
  const size_t ldsp = red > (size_t)pend ? red : (size_t)pend;
  if (pc) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED, true, false, false, 1, true>), dim3(blocks), dim3(S * 64), red, st, a);
  else if (pst) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED, false, true, true, 1, true>), dim3(blocks), dim3(S * 64), ldsp, st, a);
  else if (gf) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED, false, true, false, 1, true>), dim3(blocks), dim3(S * 64), red, st, a);
  else hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED, false, false, false, 1, true>), dim3(blocks), dim3(S * 64), red, st, a);
}

// Column tiles per wave for the decode default (cold sweep, profiles/r01_gemv_ct.jsonl): X traffic
// only matters from M = 4 on, and a CT-fold smaller grid must still cover the chip: CT = 4 when that
// leaves >= 256 workgroups (or >= 160 at M >= 8: 7B gate/up), CT = 2 for >= 256 workgroups once M*K
// is large (70B down, K = 28672); else the one-tile kernel.  70B gate M = 16: 58.5 -> 30.7 us.
// Long reductions at M < 4 (7B down K = 11008, 70B down K = 28672): a 16-way k-split (S = 16) keeps
// twice the waves streaming (cold: 9.4 -> 7.5 us, 26.6 -> 24.2 us); at K <= 8192 the extra partial
// sums cost more than they hide (q/gate/70B gate 4-8 % slower).  Different k-split = different fp32
// summation order than S = 8 (deterministic either way).
inline bool gemv_long_k(int64_t M, int64_t K) { return M < 4 && K >= 10240; }

// M = 3 counts as well (70B gate: staging 49 KB of X per 16-column workgroup, 29.1 us vs 26.8 at
// M = 4 with 4 tiles), and M = 2 once X no longer fits the LDS image (70B down, K = 28672: 34.8 ->
// 28.3 us).
inline int gemv_auto_ct(int64_t M, int64_t N, int64_t K) {
  const bool xlds = M * (2 * K + 16) <= XLDS_MAX;
  if (M < 3 && xlds) return 1;
  if (N / 64 >= 256 || (M >= 8 && N / 64 >= 160)) return 4;
  if (N / 32 >= 256 && (M * K >= 65536 || !xlds)) return 2;
  return 1;
}

template <int PF, int S, int CT, bool TILED, bool BIGX = false>
void launch_gemv_ct(const GemmArgs& a, hipStream_t st, bool allow_pc = true, bool allow_gf = true) {
  const int64_t xbytes = (int64_t)a.M * (a.K * 2 + 16);
  const unsigned blocks = (unsigned)(a.N / (16 * CT));
  const size_t red = (size_t)S * CT * 256 * 4;
  const bool pc = a.gpr == 1 && allow_pc;
  const bool gf = !pc && allow_gf && a.group % BK == 0;  // the grouped scale factored per k-step
  // BIGX: the large image where the grid is at most one workgroup per CU (XLDS_BIG)
  const int64_t xmax = (BIGX && (int64_t)blocks <= gemm_cu_count()) ? XLDS_BIG : XLDS_MAX;
  // grouped + gf: the CT tiles' parameter rows staged after the X image (PST)
  const bool xl = xbytes <= xmax;
  const int64_t pend = (xl ? (xbytes + 15) / 16 * 16 : 0) + (int64_t)16 * CT * (a.gpr + 1) * 4;
  const bool pst = gf && pend <= (BIGX ? xmax + 16 * 1024 : PST_LDS_MAX);
  const size_t ldsp0 = red > (size_t)pend ? red : (size_t)pend;
  if (xl && BIGX && xbytes > XLDS_MAX) {
    const size_t lds = red > (size_t)xbytes ? red : (size_t)xbytes;
    const size_t ldsp = lds > (size_t)pend ? lds : (size_t)pend;
    if (pc) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED, true, false, false, 8>), dim3(blocks), dim3(S * 64), lds, st, a);
    else if (pst) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED, false, true, true, 8>), dim3(blocks), dim3(S * 64), ldsp, st, a);
    else if (gf) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED, false, true, false, 8>), dim3(blocks), dim3(S * 64), lds, st, a);
    else hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED, false, false, false, 8>), dim3(blocks), dim3(S * 64), lds, st, a);
  } else if (xl) {
    const size_t lds = red > (size_t)xbytes ? red : (size_t)xbytes;
    const size_t ldsp = lds > (size_t)pend ? lds : (size_t)pend;
    if (pc) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED, true>), dim3(blocks), dim3(S * 64), lds, st, a);
    else if (pst) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED, false, true, true>), dim3(blocks), dim3(S * 64), ldsp, st, a);
    else if (gf) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED, false, true>), dim3(blocks), dim3(S * 64), lds, st, a);
    else hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, true, TILED>), dim3(blocks), dim3(S * 64), lds, st, a);
  } else {
    if (pc) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED, true>), dim3(blocks), dim3(S * 64), red, st, a);
    else if (pst) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED, false, true, true>), dim3(blocks), dim3(S * 64), ldsp0, st, a);
    else if (gf) hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED, false, true>), dim3(blocks), dim3(S * 64), red, st, a);
    else hipLaunchKernelGGL((k_w4a16_gemv_ct<PF, S, CT, false, TILED>), dim3(blocks), dim3(S * 64), red, st, a);
  }
}

template <int PF, int S, int T, int PROBE = 0, bool TILED = false, bool BIGX = false>
// pm (grouped weights): 0 = parameters per k-step from global memory, scale per weight (the form
// before round 5), 1 = staged in LDS (PST) when they fit beside X, 2 = PST + the scale factored per
// k-step (GF, where every k-step lies in one group; also without PST when X is not staged)
void launch_gemv(const GemmArgs& a, hipStream_t st, bool allow_lds, bool allow_pc = true, int pm = 2) {
  const int64_t xbytes = (int64_t)a.M * (a.K * 2 + 16);
  const unsigned blocks = (unsigned)(a.N / (16 * T));
  const size_t red = (size_t)S * T * 256 * 4;
  const bool pc = a.gpr == 1 && (PROBE == 0 || PROBE >= 5) && allow_pc;  // 5, 6: X-stream probes
  // BIGX: the large image where the grid is at most one workgroup per CU (XLDS_BIG)
  const int64_t xmax = (BIGX && (int64_t)blocks <= gemm_cu_count()) ? XLDS_BIG : XLDS_MAX;
  // grouped: the staged parameters (PST) after the X image, 16 T rows of gpr + 1 dwords
  const bool xl = allow_lds && xbytes <= xmax;
  const int64_t pend = (xl ? (xbytes + 15) / 16 * 16 : 0) + (int64_t)16 * T * (a.gpr + 1) * 4;
  const bool pst = !pc && (PROBE == 0 || PROBE >= 5) && pm > 0 && pend <= (BIGX ? xmax + 16 * 1024 : PST_LDS_MAX);
  const bool gf = !pc && (PROBE == 0 || PROBE >= 5) && pm == 2 && a.group % BK == 0;  // every k-step inside one group
  const size_t ldsp0 = red > (size_t)pend ? red : (size_t)pend;
  if (xl && BIGX && xbytes > XLDS_MAX) {
    const size_t lds = red > (size_t)xbytes ? red : (size_t)xbytes;
    const size_t ldsp = lds > (size_t)pend ? lds : (size_t)pend;
    if (pc) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, true, false, false, 8>), dim3(blocks), dim3(S * T * 64), lds, st, a);
    else if (pst && gf) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, false, true, true, 8>), dim3(blocks), dim3(S * T * 64), ldsp, st, a);
    else if (pst) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, false, true, false, 8>), dim3(blocks), dim3(S * T * 64), ldsp, st, a);
    else if (gf) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, false, false, true, 8>), dim3(blocks), dim3(S * T * 64), lds, st, a);
    else hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, false, false, false, 8>), dim3(blocks), dim3(S * T * 64), lds, st, a);
  } else if (xl) {
    const size_t lds = red > (size_t)xbytes ? red : (size_t)xbytes;
    const size_t ldsp = lds > (size_t)pend ? lds : (size_t)pend;
    if (pc) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, true>), dim3(blocks), dim3(S * T * 64), lds, st, a);
    else if (pst && gf) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, false, true, true>), dim3(blocks), dim3(S * T * 64), ldsp, st, a);
    else if (pst) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, false, true>), dim3(blocks), dim3(S * T * 64), ldsp, st, a);
    else if (gf) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED, false, false, true>), dim3(blocks), dim3(S * T * 64), lds, st, a);
    else hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, true, PROBE, TILED>), dim3(blocks), dim3(S * T * 64), lds, st, a);
  } else {
    if (pc) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, false, PROBE, TILED, true>), dim3(blocks), dim3(S * T * 64), red, st, a);
    else if (pst && gf) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, false, PROBE, TILED, false, true, true>), dim3(blocks), dim3(S * T * 64), ldsp0, st, a);
    else if (pst) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, false, PROBE, TILED, false, true>), dim3(blocks), dim3(S * T * 64), ldsp0, st, a);
    else if (gf) hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, false, PROBE, TILED, false, false, true>), dim3(blocks), dim3(S * T * 64), red, st, a);
    else hipLaunchKernelGGL((k_w4a16_gemv<PF, S, T, false, PROBE, TILED>), dim3(blocks), dim3(S * T * 64), red, st, a);
  }
}

// row-major packed codes [N, K/2] -> decode tile layout: block (t, kt) of 1 KiB at (t * K/128 + kt) KiB,
// byte 16 l + i = row 16 t + (l & 15), code byte 64 kt + 16 (l >> 4) + i.  One thread per 16 B.
__global__ __launch_bounds__(256) void k_tile_codes(const uint8_t* codes, uint8_t* out, int64_t K, int64_t nchunks) {
  const int64_t nks = K / BK;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nchunks; i += (int64_t)gridDim.x * 256) {
    const int64_t blk = i >> 6, l = i & 63;
    const int64_t t = blk / nks, kt = blk - t * nks;
    const int64_t row = 16 * t + (l & 15);
    const u32x4 v = *gp<u32x4>(codes + row * (K / 2) + 64 * kt + 16 * (l >> 4));
    *gp<u32x4>(out + i * 16) = v;
  }
}

// row-major packed codes -> the NIB layout of the prefill kernels (iwq_prefill.hip, variant 75): in
// every code dword (8 consecutive k) byte j = low nibbles of k = 4j', 4j'+2 ... i.e. nibble p holds
// k = (0,2,4,6,1,3,5,7)[p].  Per dword: the 4 low nibbles L (k even) and the 4 high nibbles H (k odd)
// are each compressed from one-per-byte to two-per-byte (x | x >> 4, bytes 0 and 2), L into the low
// half-dword, H into the high one.  One thread per 16 B; safe in place (each thread reads its own 16 B
// before writing them).
__device__ __forceinline__ uint32_t nib_dword(uint32_t w) {
  const uint32_t l = w & 0x0F0F0F0Fu, h = (w >> 4) & 0x0F0F0F0Fu;
  const uint32_t pl = l | (l >> 4), ph = h | (h >> 4);
  return (pl & 0xFFu) | ((pl >> 8) & 0xFF00u) | ((ph & 0xFFu) << 16) | ((ph << 8) & 0xFF000000u);
}

__global__ __launch_bounds__(256) void k_nib_codes(const uint8_t* codes, uint8_t* out, int64_t nchunks) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nchunks; i += (int64_t)gridDim.x * 256) {
    u32x4 v = *gp<u32x4>(codes + i * 16);
    v[0] = nib_dword(v[0]);
    v[1] = nib_dword(v[1]);
    v[2] = nib_dword(v[2]);
    v[3] = nib_dword(v[3]);
    *gp<u32x4>(out + i * 16) = v;
  }
}

// Persistent form of k_w4a16_gemv: the grid is the resident set of workgroups and each one walks
// column groups c = blockIdx.x, blockIdx.x + gridDim.x, ...  X is staged into LDS ONCE per
// workgroup, and each wave's code ring runs across column-group boundaries (the first PF steps of
// group i+1 are in flight while group i's partial tiles are summed), so there is neither a
// second-round tail (70B gate: 1792 groups over 1024 slots) nor a per-workgroup restart.
template <int PF, int S, int T, bool XLDS>
__global__ __launch_bounds__(S * T * 64) void k_w4a16_gemv_p(GemmArgs a, int ngroups) {
  constexpr int WPB = S * T;
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = wid % T, ks = wid / T;
  const int q = lane >> 4, r16 = lane & 15;
  const int nks = a.K / BK;
  const int nj = nks > ks ? (nks - ks + S - 1) / S : 0;  // steps of this wave per column group
  const int ngi = ngroups > (int)blockIdx.x ? (ngroups - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int total = ngi * nj;                            // ring length of this wave
  const int64_t crow = a.K / 2;
  const int arow = r16 < a.M ? r16 : a.M - 1;
  const int xpitch = a.K * 2 + 16;
  const int xbytes = XLDS ? (a.M * xpitch + 15) / 16 * 16 : 0;
  float* red = reinterpret_cast<float*>(dsm + xbytes);   // [WPB][256] partial tiles
  const _Float16* xrow = a.x + (int64_t)arow * a.lda + 32 * q;
  const h2 k1024 = h2{(_Float16)1024.0f, (_Float16)1024.0f}, k64 = h2{(_Float16)64.0f, (_Float16)64.0f};
  u32x4 bc[PF];
  _Float16 sv[PF], zv[PF];
  u32x4 xa[XLDS ? 1 : PF][4];
  auto col_of = [&](int g) { return ((int)blockIdx.x + (g / nj) * (int)gridDim.x) * T * 16 + tile * 16 + r16; };
  auto load = [&](int g, int u) {
    const int kt = ks + (g % nj) * S;
    const int n = col_of(g);
    bc[u] = __builtin_nontemporal_load(gp<u32x4>(a.codes + (int64_t)n * crow + q * 16 + kt * (BK / 2)));
    const int kk = kt * BK + 32 * q;
    const int64_t gi = (int64_t)n * a.gpr + (a.gshift >= 0 ? (kk >> a.gshift) : kk / a.group);
    sv[u] = gp<_Float16>(a.scales)[gi];
    zv[u] = a.zeros ? gp<_Float16>(a.zeros)[gi] : (_Float16)a.zsym;
    if constexpr (!XLDS) {
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[u][s] = *gp<u32x4>(xrow + kt * BK + 8 * s);
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < total) load(u, u);

  if constexpr (XLDS) {
    const int cpr = a.K / 8;
    for (int m = 0; m < a.M; ++m) {
      const _Float16* xr = a.x + (int64_t)m * a.lda;
      for (int c = threadIdx.x; c < cpr; c += WPB * 64) {
        const u32x4 d = *gp<u32x4>(xr + 8 * c);
        const u32x4 pd = {perm(d.z, d.x, 0x05040100u), perm(d.z, d.x, 0x07060302u),
                          perm(d.w, d.y, 0x05040100u), perm(d.w, d.y, 0x07060302u)};
        *reinterpret_cast<u32x4*>(dsm + m * xpitch + 16 * c) = pd;
      }
    }
    __syncthreads();
  }
  const uint8_t* xsrow = dsm + arow * xpitch + 64 * q;
  const DqConst dq;
  // sum the WPB partial tiles of column group cg and store; every wave of the workgroup calls this
  // exactly once per column group (2 barriers), waves without k-steps (nj == 0) included
  auto flush = [&](const f4& acc, int cg) {
    *reinterpret_cast<f4*>(red + wid * 256 + lane * 4) = acc;
    __syncthreads();
    for (int o = threadIdx.x; o < T * 256; o += WPB * 64) {
      const int t = o >> 8, e = o & 255;  // e = lane' * 4 + reg of the C layout
      const int ln = e >> 2, reg = e & 3;
      const int row = 4 * (ln >> 4) + reg, col = (cg * T + t) * 16 + (ln & 15);
      if (row < a.M) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < S; ++k) v += red[(k * T + t) * 256 + e];
        if (a.bias) v += (float)gp<_Float16>(a.bias)[col];
        gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)v;
      }
    }
    __syncthreads();
  };
  if (nj == 0) {
    for (int gi = 0; gi < ngi; ++gi) flush((f4){0.f, 0.f, 0.f, 0.f}, (int)blockIdx.x + gi * (int)gridDim.x);
    return;
  }
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int g0 = 0; g0 < total; g0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int g = g0 + u;
      if (g >= total) break;
      const int kt = ks + (g % nj) * S;
      const h2 s2 = h2{sv[u], sv[u]};
      const h2 z2 = h2{zv[u], zv[u]};
      const h2 z1024 = z2 + k1024, z64 = z2 + k64;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        h8 af;
        if constexpr (XLDS) {
          af = *reinterpret_cast<const h8*>(xsrow + kt * (BK * 2) + 16 * s);
        } else {
          const u32x4 x4 = xa[u][s];
          const u32x4 pa = {perm(x4.z, x4.x, 0x05040100u), perm(x4.z, x4.x, 0x07060302u),
                            perm(x4.w, x4.y, 0x05040100u), perm(x4.w, x4.y, 0x07060302u)};
          af = __builtin_bit_cast(h8, pa);
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, dequant8(bc[u][s], z1024, z64, s2, dq), acc, 0, 0, 0);
      }
      if (g + PF < total) load(g + PF, u);
      if ((g % nj) == nj - 1) {  // this wave's last step of the column group
        flush(acc, (int)blockIdx.x + (g / nj) * (int)gridDim.x);
        acc = (f4){0.f, 0.f, 0.f, 0.f};
      }
    }
  }
}

template <int PF, int S, int T>
void launch_gemv_p(const GemmArgs& a, hipStream_t st) {
  const int64_t xbytes = ((int64_t)a.M * (a.K * 2 + 16) + 15) / 16 * 16;
  const bool xlds = xbytes <= XLDS_MAX;
  const size_t lds = (xlds ? (size_t)xbytes : 0) + (size_t)S * T * 256 * 4;
  const int ngroups = a.N / (16 * T);
  int dev = 0, cus = 256, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  if (xlds) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_w4a16_gemv_p<PF, S, T, true>, S * T * 64, lds) !=
            hipSuccess || occ <= 0)
      occ = 1;
  } else {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_w4a16_gemv_p<PF, S, T, false>, S * T * 64, lds) !=
            hipSuccess || occ <= 0)
      occ = 1;
  }
  int blocks = cus * occ;
  if (blocks > ngroups) blocks = ngroups;
  if (xlds) hipLaunchKernelGGL((k_w4a16_gemv_p<PF, S, T, true>), dim3(blocks), dim3(S * T * 64), lds, st, a, ngroups);
  else hipLaunchKernelGGL((k_w4a16_gemv_p<PF, S, T, false>), dim3(blocks), dim3(S * T * 64), lds, st, a, ngroups);
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_big: prefill (large M), per-channel scales.  256x256 output tile per 512-thread
// workgroup (8 waves as 2 (M) x 4 (N), 128x64 per wave = 8x4 MFMA tiles), K in steps of 64.
// Both operands are staged by LDS-DMA (global_load_lds_dwordx4) into a 3-stage ring
// (X 32 KiB + codes 8 KiB per stage): tile t+2 is in flight while tile t is computed, with ONE
// raw s_barrier per K-step and a counted `s_waitcnt vmcnt(5)` (5 DMA instructions per thread per
// stage), never a full drain inside the loop.  The DMA writes lane-linearly, so the X image is
// XOR-swizzled through the SOURCE addresses (16-B chunk c of row r lands at chunk c ^ ((r>>1)&7):
// conflict-free ds_read_b128 of A fragments).  k runs in natural order on both operands: lane
// group q of k-slice s holds k = 16q + 8s + [0, 8), i.e. one 8-byte codes read per 16-column
// subtile per K-step, dequantized in registers by v_perm + and-or (1024+q / 64+q magic), one exact
// subtraction of the zero point and one rounding multiply by the scale (= the fake-quant weight).
// ---------------------------------------------------------------------------------------------
constexpr int BG_M = 256, BG_N = 256, BG_THR = 512;

template <int BK>
struct BigCfg {
  static constexpr int XS = BG_M * BK * 2;                 // X bytes per stage
  static constexpr int CS = BG_N * BK / 2;                 // codes bytes per stage
  static constexpr int STAGE = XS + CS;
  static constexpr int NSTAGE = BK == 64 ? 3 : 2;          // 120 KiB / 160 KiB of LDS
  static constexpr int XI = BK / 16;                       // X DMA instructions per thread per stage
  static constexpr int CI = BK / 64;                       // codes DMA instructions per thread per stage
  static constexpr int XROWS = 512 / BK;                   // rows per 1-KiB DMA instruction
  static constexpr int XCH = BK / 8;                       // 16-B chunks per X row
  static constexpr int CCOLS = 2048 / BK;                  // columns per 1-KiB codes DMA instruction
  static constexpr int CCH = BK / 32;                      // 16-B chunks per codes column
  static constexpr int KS = BK / 32;                       // MFMA k-slices per stage
  // X: chunk c of row r sits at chunk c ^ xswz(r); 16 lanes reading 16 consecutive rows at one
  // logical chunk hit 16 distinct 16-B slots of the 256-B bank row
  __device__ static int xswz(int r) { return BK == 64 ? ((r >> 1) & 7) : (r & 15); }
  // codes: chunk c of column n sits at c ^ cswz(n) (BK=128: 16 columns x 4 chunks -> distinct slots)
  __device__ static int cswz(int n) { return BK == 64 ? 0 : ((n >> 2) & 3); }
};

typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

// 8 codes (nibble p of w = k offset p) -> 8 fp16 RN16((q - z) * s) in natural k order.
// zz = (1024 + z, 64 + z): even k come out as 1024 + q (low nibble, 0x6400), odd k as 64 + q
// (high nibble at mantissa bits 4..7, 0x5400).
__device__ __forceinline__ h8 dequant8_nat(uint32_t w, h2 zz, h2 s, uint32_t mask_s, uint32_t magic_v) {
  const h2 d0 = (as_h2(and_or(perm(w, w, 0x0C000C00u), mask_s, magic_v)) - zz) * s;
  const h2 d1 = (as_h2(and_or(perm(w, w, 0x0C010C01u), mask_s, magic_v)) - zz) * s;
  const h2 d2 = (as_h2(and_or(perm(w, w, 0x0C020C02u), mask_s, magic_v)) - zz) * s;
  const h2 d3 = (as_h2(and_or(perm(w, w, 0x0C030C03u), mask_s, magic_v)) - zz) * s;
  return h8{d0.x, d0.y, d1.x, d1.y, d2.x, d2.y, d3.x, d3.y};
}

__device__ __forceinline__ void glds16(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void glds2(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 2, 0, 0);
}

// GROUPED: scales / zero points of groups of g (multiple of BK) k: the K-step's 256 scales and 256
// zero points ride in the same ring stage (waves 0-3 DMA the scales, 4-7 the zeros).  A 2-byte
// LDS-DMA writes one zero-extended DWORD per lane (measured: tools/probes/glds_ushort.hip), so each
// parameter occupies 4 bytes of LDS.
template <int BK, bool SOUTER = false, bool GROUPED = false>
__global__ __launch_bounds__(BG_THR) void k_w4a16_big(GemmArgs a) {
  using C = BigCfg<BK>;
  constexpr int STAGE = C::STAGE + (GROUPED ? 2048 : 0);
  constexpr int PER_STAGE = C::XI + C::CI + (GROUPED ? 1 : 0);  // DMA instructions per thread per stage
  static_assert(!GROUPED || C::NSTAGE == 3, "grouped scales: 3-stage ring only");
  __shared__ __attribute__((aligned(16))) uint8_t smem[C::NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int q = lane >> 4, r16 = lane & 15;
  const int tiles_n = a.N / BG_N;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * BG_M, n0 = (int)(t % tiles_n) * BG_N;
  const int nk = a.K / BK;
  const int64_t crow = a.K / 2;

  // DMA sources (per lane); destinations are wave-uniform 1-KiB slots, filled lane-linearly
  const _Float16* xsrc[C::XI];
#pragma unroll
  for (int i = 0; i < C::XI; ++i) {
    const int row = (wid * C::XI + i) * C::XROWS + lane / C::XCH;
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;   // rows past M: any valid row (discarded)
    const int c = (lane % C::XCH) ^ C::xswz(row);
    xsrc[i] = a.x + (int64_t)gm * a.lda + c * 8;
  }
  const uint8_t* csrc[C::CI];
#pragma unroll
  for (int j = 0; j < C::CI; ++j) {
    const int col = (wid * C::CI + j) * C::CCOLS + lane / C::CCH;
    const int c = (lane % C::CCH) ^ C::cswz(col);
    csrc[j] = a.codes + (int64_t)(n0 + col) * crow + c * 16;
  }
  // grouped: wave w < 4 fills the scale of column 64w + lane, wave w >= 4 the zero point
  const _Float16* psrc = nullptr;
  if constexpr (GROUPED) {
    const _Float16* arr = (wid < 4 || !a.zeros) ? a.scales : a.zeros;
    psrc = arr + (int64_t)(n0 + (wid & 3) * 64 + lane) * a.gpr;
  }
  auto issue = [&](int kt, int stg) {
    uint8_t* base = smem + stg * STAGE;
#pragma unroll
    for (int i = 0; i < C::XI; ++i) glds16(xsrc[i] + kt * BK, base + (wid * C::XI + i) * 1024);
#pragma unroll
    for (int j = 0; j < C::CI; ++j) glds16(csrc[j] + kt * (BK / 2), base + C::XS + (wid * C::CI + j) * 1024);
    if constexpr (GROUPED) {
      const int gk = (kt * BK) / a.group;  // a K-step never straddles a group (g % BK == 0)
      glds2(psrc + gk, base + C::XS + C::CS + wid * 256);
    }
  };

  // per-channel scale / zero point of this lane's column in each 16-wide subtile
  h2 sv[4], zz[4];
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = n0 + wn * 64 + nt * 16 + r16;
      const _Float16 sc = gp<_Float16>(a.scales)[col];
      const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
      sv[nt] = h2{sc, sc};
      zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};  // exact: z is a small integer
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  uint32_t magic_v;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));

  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f4){0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  if constexpr (C::NSTAGE == 3) {
    if (nk > 1) issue(1, 1);
  }
  for (int kt = 0; kt < nk; ++kt) {
    // own DMA of tile kt retired (with 3 stages tile kt+1's may stay in flight); the barrier makes
    // every wave's part visible and proves every wave is done reading the stage about to be refilled
    if constexpr (C::NSTAGE == 3) {
      if (kt + 1 < nk) {
        if constexpr (PER_STAGE == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + C::NSTAGE - 1 < nk) issue(kt + C::NSTAGE - 1, (kt + C::NSTAGE - 1) % C::NSTAGE);
    const uint8_t* xs = smem + (kt % C::NSTAGE) * STAGE;
    const uint8_t* cs = xs + C::XS;
    if constexpr (GROUPED) {
      const uint32_t* ps = reinterpret_cast<const uint32_t*>(cs + C::CS);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int col = wn * 64 + nt * 16 + r16;
        const _Float16 sc = __builtin_bit_cast(_Float16, (uint16_t)ps[col]);
        const float zf = a.zeros ? (float)__builtin_bit_cast(_Float16, (uint16_t)ps[256 + col]) : a.zsym;
        sv[nt] = h2{sc, sc};
        zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
      }
    }
    if constexpr (SOUTER && BK == 64) {
      // k-slice-outer order: slice 0's dequant, then its 32 MFMAs with slice 1's dequant VALU
      // interleaved (sched_group_barrier: 1 MFMA : 2 VALU), then slice 1's 32 MFMAs
      u32x2v w2[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        w2[nt] = *reinterpret_cast<const u32x2v*>(cs + (wn * 64 + nt * 16 + r16) * 32 + 8 * q);
      h8 b0[4], b1[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) b0[nt] = dequant8_nat(w2[nt].x, zz[nt], sv[nt], mask_s, magic_v);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) b1[nt] = dequant8_nat(w2[nt].y, zz[nt], sv[nt], mask_s, magic_v);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int row = wm * 128 + mt * 16 + r16;
        const h8 af = *reinterpret_cast<const h8*>(xs + row * 128 + (((2 * q) ^ C::xswz(row)) << 4));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, b0[nt], acc[mt][nt], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // 2 VALU
      }
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int row = wm * 128 + mt * 16 + r16;
        const h8 af = *reinterpret_cast<const h8*>(xs + row * 128 + (((2 * q + 1) ^ C::xswz(row)) << 4));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, b1[nt], acc[mt][nt], 0, 0, 0);
      }
      continue;
    }
    // B fragments: lane group q holds k = (BK/4) q + 8 s + [0, 8) for k-slice s
    h8 bf[4][C::KS];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = wn * 64 + nt * 16 + r16;
      if constexpr (BK == 64) {
        const u32x2v w2 = *reinterpret_cast<const u32x2v*>(cs + col * 32 + 8 * q);
        bf[nt][0] = dequant8_nat(w2.x, zz[nt], sv[nt], mask_s, magic_v);
        bf[nt][1] = dequant8_nat(w2.y, zz[nt], sv[nt], mask_s, magic_v);
      } else {
        const u32x4 w4 = *reinterpret_cast<const u32x4*>(cs + col * 64 + ((q ^ C::cswz(col)) << 4));
        bf[nt][0] = dequant8_nat(w4.x, zz[nt], sv[nt], mask_s, magic_v);
        bf[nt][1] = dequant8_nat(w4.y, zz[nt], sv[nt], mask_s, magic_v);
        bf[nt][2] = dequant8_nat(w4.z, zz[nt], sv[nt], mask_s, magic_v);
        bf[nt][3] = dequant8_nat(w4.w, zz[nt], sv[nt], mask_s, magic_v);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const int row = wm * 128 + mt * 16 + r16;
      const int sw = C::xswz(row);
#pragma unroll
      for (int s2 = 0; s2 < C::KS; ++s2) {
        const h8 af = *reinterpret_cast<const h8*>(xs + row * (BK * 2) + (((C::KS * q + s2) ^ sw) << 4));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[nt][s2], acc[mt][nt], 0, 0, 0);
      }
    }
  }

  // epilogue: C layout col = lane & 15, row = 4 * (lane >> 4) + reg
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = n0 + wn * 64 + nt * 16 + r16;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 128 + mt * 16 + 4 * q + r;
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(acc[mt][nt][r] + b);
      }
    }
  }
}

// Packed codes -> the fp16 dequantized weight W_deq [N, K] (contiguous), element for element the
// reference's RN16((q - z) * s) (quant_linear.py:935-949): the prefill path for packed-only weights
// (dequantize once into a scratch buffer, then one library GEMM), HBM-bound at 2 + 0.5 + 4/g B per
// weight.  The weight is walked flat: a wave takes 2048 consecutive elements per step; lane l's
// piece j (j < 4) is elements 512 j + 8 l .. +8, i.e. code dword 64 j + l, so every load
// instruction reads 256 contiguous bytes and every 16-B store instruction writes 1 KiB contiguous
// (a piece never straddles a row or a scale group: K % 32 == 0, g % 32 == 0).
__global__ __launch_bounds__(256) void k_dequant_packed(GemmArgs a, int64_t total) {
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  uint32_t magic_v;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const IWQ_GLOBAL uint32_t* c32 = gp<uint32_t>(a.codes);
  IWQ_GLOBAL h8* out = gp<h8>(a.y);
  for (int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2048; base < total; base += nwaves * 2048) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = base + 512 * j + 8 * lane;
      w[j] = __builtin_nontemporal_load(c32 + (e < total ? e / 8 : 0));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = base + 512 * j + 8 * lane;
      if (e < total) {
        const int64_t gi = a.gshift >= 0 ? (e >> a.gshift) : e / a.group;  // flat group index
        const _Float16 sc = gp<_Float16>(a.scales)[gi];
        const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[gi] : a.zsym;
        const h2 sv = {sc, sc};
        const h2 zz = {(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};  // exact: z is a small integer
        __builtin_nontemporal_store(dequant8_nat(w[j], zz, sv, mask_s, magic_v), out + e / 8);
      }
    }
  }
}

}  // namespace

extern "C" {

int iwq_tile_codes(const void* codes, int64_t N, int64_t K, void* out, void* stream) {
  if (!codes || !out) return IWQ_ERR_ARG;
  if (N <= 0 || K <= 0 || N % 16 != 0 || K % BK != 0) return IWQ_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(codes) & 15u) || (reinterpret_cast<uintptr_t>(out) & 15u)) return IWQ_ERR_ARG;
  const int64_t nchunks = N * (K / 2) / 16;
  int64_t blocks = (nchunks + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_tile_codes, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(codes), static_cast<uint8_t*>(out), K, nchunks);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    iwq::last_hip_error() = (int)e;
    return IWQ_ERR_HIP;
  }
  return IWQ_OK;
}

int iwq_nib_codes(const void* codes, int64_t N, int64_t K, void* out, void* stream) {
  if (!codes || !out) return IWQ_ERR_ARG;
  if (N <= 0 || K <= 0 || K % 32 != 0) return IWQ_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(codes) & 15u) || (reinterpret_cast<uintptr_t>(out) & 15u)) return IWQ_ERR_ARG;
  const int64_t nchunks = N * (K / 2) / 16;
  int64_t blocks = (nchunks + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_nib_codes, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(codes), static_cast<uint8_t*>(out), nchunks);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    iwq::last_hip_error() = (int)e;
    return IWQ_ERR_HIP;
  }
  return IWQ_OK;
}

int iwq_dequant_packed(const void* codes, const void* scales, const void* zeros, int n_bits, int64_t group,
                       int64_t N, int64_t K, void* out, int64_t ld_out, void* stream) {
  if (!codes || !scales || !out) return IWQ_ERR_ARG;
  if (N <= 0 || K <= 0 || K % 32 != 0 || ld_out != K) return IWQ_ERR_SHAPE;
  if (n_bits < 2 || n_bits > 4) return IWQ_ERR_BITS;
  const int64_t g = group == IWQ_GROUP_PER_CHANNEL ? K : group;
  if (g <= 0 || g % 32 != 0 || K % g != 0) return IWQ_ERR_GROUP;
  if ((reinterpret_cast<uintptr_t>(codes) & 15u) || (reinterpret_cast<uintptr_t>(out) & 15u)) return IWQ_ERR_ARG;
  GemmArgs a{};
  a.codes = static_cast<const uint8_t*>(codes);
  a.scales = static_cast<const _Float16*>(scales);
  a.zeros = static_cast<const _Float16*>(zeros);
  a.y = static_cast<_Float16*>(out);
  a.K = (int)K;
  a.N = (int)N;
  a.group = (int)g;
  a.gpr = (int)(K / g);
  a.zsym = (float)(1 << (n_bits - 1));
  a.gshift = (g & (g - 1)) == 0 ? __builtin_ctzll((unsigned long long)g) : -1;
  const int64_t total = N * K;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  int64_t blocks = (total + 4 * 2048 - 1) / (4 * 2048);
  if (blocks > (int64_t)cus * 8) blocks = (int64_t)cus * 8;
  hipLaunchKernelGGL(k_dequant_packed, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), a,
                     total);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    iwq::last_hip_error() = (int)e;
    return IWQ_ERR_HIP;
  }
  return IWQ_OK;
}

int64_t iwq_w4a16_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K, int64_t group) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (M <= 16) {  // the K-split decodes' slabs (round 6), where the default takes one (A/B forms: the
    // caller sizes its own)
    const int64_t a = GEMV_KS_DEFAULT ? gemv_ks_bytes(M, N, K) : 0, b = GEMV_KSX_DEFAULT ? gemv_ksx_bytes(M, N, K) : 0;
    return a > b ? a : b;
  }
  const int64_t g = group == IWQ_GROUP_PER_CHANNEL ? K : group;
  if (g <= 0 || K % g != 0) return 0;
  int ns = 0, mtw = 2;
  if (prefill_short_split(M, N, K, (int)(K / g), (int)g, &ns, &mtw)) return prefill_splitk_bytes_s(M, N, mtw, ns);
  if (!prefill_split_preferred(M, N, K, (int)(K / g), (int)g)) return 0;
  return prefill_splitk_bytes(M, N, prefill_splitk_count(M, N, K, 0));
}

static int w4a16_gemm_impl(const void* x, int64_t M, int64_t K, int64_t lda, const void* codes, const void* scales,
                           const void* zeros, int n_bits, int64_t group, int64_t N, const void* bias, void* y,
                           int64_t ldy, void* workspace, int64_t workspace_bytes, unsigned flags, void* stream);

int iwq_w4a16_gemm(const void* x, int64_t M, int64_t K, int64_t lda, const void* codes, const void* scales,
                   const void* zeros, int n_bits, int64_t group, int64_t N, const void* bias, void* y, int64_t ldy,
                   unsigned flags, void* stream) {
  return w4a16_gemm_impl(x, M, K, lda, codes, scales, zeros, n_bits, group, N, bias, y, ldy, nullptr, 0, flags,
                         stream);
}

int iwq_w4a16_gemm_ws(const void* x, int64_t M, int64_t K, int64_t lda, const void* codes, const void* scales,
                      const void* zeros, int n_bits, int64_t group, int64_t N, const void* bias, void* y, int64_t ldy,
                      void* workspace, int64_t workspace_bytes, unsigned flags, void* stream) {
  if (workspace_bytes < 0 || (workspace_bytes > 0 && !workspace)) return IWQ_ERR_ARG;
  return w4a16_gemm_impl(x, M, K, lda, codes, scales, zeros, n_bits, group, N, bias, y, ldy, workspace,
                         workspace_bytes, flags, stream);
}

static int w4a16_gemm_impl(const void* x, int64_t M, int64_t K, int64_t lda, const void* codes, const void* scales,
                           const void* zeros, int n_bits, int64_t group, int64_t N, const void* bias, void* y,
                           int64_t ldy, void* workspace, int64_t workspace_bytes, unsigned flags, void* stream) {
  if (!x || !codes || !scales || !y) return IWQ_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldy < N) return IWQ_ERR_SHAPE;
  if (N % BN != 0 || K % BK != 0 || (lda % 8) != 0) return IWQ_ERR_SHAPE;
  if (n_bits < 2 || n_bits > 4) return IWQ_ERR_BITS;
  const int64_t g = group == IWQ_GROUP_PER_CHANNEL ? K : group;
  if (g <= 0 || g % 32 != 0 || K % g != 0) return IWQ_ERR_GROUP;
  if ((reinterpret_cast<uintptr_t>(x) & 15u) || (reinterpret_cast<uintptr_t>(codes) & 15u)) return IWQ_ERR_ARG;
  // the split-K reduces store y in 8-B pieces (4 outputs) and read the fp32 partials with 16-B loads:
  // a caller whose y / ldy cannot take that, or whose workspace is not 16-B aligned, gets the unsplit
  // kernels (a workspace is only ever an optimisation)
  if ((reinterpret_cast<uintptr_t>(y) & 7u) || (ldy % 4) != 0 || (reinterpret_cast<uintptr_t>(workspace) & 15u)) {
    workspace = nullptr;
    workspace_bytes = 0;
  }
  if (M > 0x7FFFFFFF || N > 0x7FFFFFFF || K > 0x7FFFFFFF) return IWQ_ERR_SHAPE;
  GemmArgs a{};
  a.x = static_cast<const _Float16*>(x);
  a.lda = lda;
  a.codes = static_cast<const uint8_t*>(codes);
  a.scales = static_cast<const _Float16*>(scales);
  a.zeros = static_cast<const _Float16*>(zeros);
  a.bias = static_cast<const _Float16*>(bias);
  a.y = static_cast<_Float16*>(y);
  a.ldy = ldy;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.group = (int)g;
  a.gpr = (int)(K / g);
  a.zsym = (float)(1 << (n_bits - 1));
  a.gshift = (g & (g - 1)) == 0 ? __builtin_ctzll((unsigned long long)g) : -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned variant = (flags >> 16) & 0xFFu;
  // the product library takes the default (0) and, at M > 16 on row-major codes, the two fallback
  // kernels for shapes the prefill kernels refuse: k_w4a16 (1) and k_w4a16_big (2); every other
  // variant is an A/B form (IWQ_AB builds)
  if (!IWQ_AB && variant != 0 &&
      !((variant == 1 || variant == 2) && M > 16 && !(flags & (IWQ_FLAG_TILED_CODES | IWQ_FLAG_NIB_CODES))))
    return IWQ_ERR_ARG;
  // default at M > 16: the split-K prefill where it is modelled faster (M >= 256: whenever a split
  // helps; 16 < M < 256: against the mid-M kernel) and the caller gave the workspace it needs
  int short_ns = 0, short_mtw = 2;
  const bool short_pref = variant == 0 && workspace && !(flags & IWQ_FLAG_FORCE_GENERIC) &&
                          prefill_short_split(M, N, K, a.gpr, a.group, &short_ns, &short_mtw) &&
                          workspace_bytes >= prefill_splitk_bytes_s(M, N, short_mtw, short_ns);
  const bool split_pref = !short_pref && variant == 0 && M > 16 && workspace && !(flags & IWQ_FLAG_FORCE_GENERIC) &&
                          prefill_split_preferred(M, N, K, a.gpr, a.group) &&
                          workspace_bytes >= prefill_splitk_bytes(M, N, prefill_splitk_count(M, N, K, 0));
  if (flags & IWQ_FLAG_GROUP_MAJOR) {
    // group-major parameters ([K/group, N]: a transposed copy held next to the codes): the grouped
    // 16x16x32 prefill kernel only (150 / 152 stage a K-step's 256 scales and zero points as contiguous
    // 512-B pieces instead of 256 halves 2 K/group bytes apart), unsplit, M >= 256; row-major or
    // (IWQ_FLAG_NIB_CODES) NIB codes, the same bits as with the reference's parameter order
    // (A/B builds: also the grouped 16x16x32 variants 150-172, codes in the variant's own layout)
    const bool abv = IWQ_AB && variant >= 150 && variant <= 172 && !(flags & IWQ_FLAG_NIB_CODES);
    if ((flags & (IWQ_FLAG_TILED_CODES | IWQ_FLAG_FORCE_GENERIC)) || (variant != 0 && !abv) || M < 256 ||
        a.gpr == 1 || !prefill16_supported(M, N, K, a.gpr, a.group))
      return IWQ_ERR_ARG;
    PrefillArgs p{a.x, a.lda, a.codes, a.scales, a.zeros, a.bias, a.y, a.ldy, a.M, a.N, a.K, a.gpr, a.group, a.zsym};
    p.pgm = 1;
    const hipError_t e = prefill_b32_launch(p, (int)variant, st, (flags & IWQ_FLAG_NIB_CODES) != 0);
    if (e != hipSuccess) {
      iwq::last_hip_error() = (int)e;
      return IWQ_ERR_HIP;
    }
    return IWQ_OK;
  }
  if (flags & IWQ_FLAG_NIB_CODES) {
    // NIB-layout codes (iwq_nib_codes): the prefill kernel only (the row-major default's NIB twin:
    // 172 per channel, 152 grouped, and the split-K form), M >= 256; every other path reads the
    // row-major layout
    if ((flags & (IWQ_FLAG_TILED_CODES | IWQ_FLAG_FORCE_GENERIC)) || variant != 0 || M < 256 ||
        !prefill_b32_supported(M, N, K, a.gpr, a.group))
      return IWQ_ERR_ARG;
    PrefillArgs p{a.x, a.lda, a.codes, a.scales, a.zeros, a.bias, a.y, a.ldy, a.M, a.N, a.K, a.gpr, a.group, a.zsym};
    const int nsplit = prefill_splitk_count(M, N, K, 0);
    hipError_t e;
    if (nsplit > 1 && workspace && workspace_bytes >= prefill_splitk_bytes(M, N, nsplit)) {
      p.ws = static_cast<float*>(workspace);
      p.nsplit = nsplit;
      e = prefill_splitk_launch(p, st, false, true);
    } else {
      e = prefill_b32_launch(p, 0, st, true);  // the default's NIB twin (same bits)
    }
    if (e != hipSuccess) {
      iwq::last_hip_error() = (int)e;
      return IWQ_ERR_HIP;
    }
    return IWQ_OK;
  }
  // the cross-workgroup K-split decode (round 6, KSX) where planned, given a workspace whose counters
  // are zero (IWQ_FLAG_WS_ZEROED); A/B variants 200-239 force (CT, KS) = (4 | 8, 1 + (v - 200) % 20)
  if (M <= 16 && !(flags & IWQ_FLAG_FORCE_GENERIC) && workspace && (flags & IWQ_FLAG_WS_ZEROED) &&
      ((variant == 0 && GEMV_KSX_DEFAULT) || (IWQ_AB && variant >= 200 && variant < 260))) {
    int ct = 0, ksn = 0;
    bool ok = false;
    if (variant == 0) {
      ok = gemv_ksx_plan(M, N, K, &ct, &ksn);
    } else {
      ct = (variant < 220 || variant >= 240) ? 4 : 8;
      ksn = 1 + (int)(variant - 200) % 20;
      ok = N % (16 * ct) == 0 && K / BK >= ksn && N / (16 * ct) * 4 <= GEMV_KSX_CNT_BYTES;
      if (variant >= 240) ok = ok && (N / (16 * ct)) % 8 == 0;  // the XCD-local map
    }
    const bool xcd = variant >= 240;
    if (ok && workspace_bytes >= gemv_ksx_bytes_for(M, N, ct, ksn)) {
      const bool tl = (flags & IWQ_FLAG_TILED_CODES) != 0;
      if (ct == 8) {
        if (tl) launch_gemv_ksx<2, 8, 8, true>(a, st, workspace, ksn, xcd);
        else launch_gemv_ksx<2, 8, 8, false>(a, st, workspace, ksn, xcd);
      } else {
        if (tl) launch_gemv_ksx<2, 8, 4, true>(a, st, workspace, ksn, xcd);
        else launch_gemv_ksx<2, 8, 4, false>(a, st, workspace, ksn, xcd);
      }
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        iwq::last_hip_error() = (int)e;
        return IWQ_ERR_HIP;
      }
      return IWQ_OK;
    }
    if (variant != 0) return IWQ_ERR_ARG;
  }
  // the K-split decode (round 6, k_w4a16_gemv_ks) where planned and the caller gave its workspace;
  // GEMV_KS_DEFAULT decides whether the default takes it (A/B variant 31 forces it, 32 refuses it)
  int ks_ct = 0, ks_n = 0;
  const bool ks_ok = M <= 16 && !(flags & IWQ_FLAG_FORCE_GENERIC) && (variant == 0 || variant == 31 || variant == 32) &&
                     gemv_ks_plan(M, N, K, &ks_ct, &ks_n) && workspace &&
                     workspace_bytes >= gemv_ks_bytes(M, N, K) && (variant == 31 || (variant == 0 && GEMV_KS_DEFAULT));
  if (ks_ok) {
    if (flags & IWQ_FLAG_TILED_CODES) launch_gemv_ks<2, 8, true>(a, st, static_cast<float*>(workspace), ks_n);
    else launch_gemv_ks<2, 8, false>(a, st, static_cast<float*>(workspace), ks_n);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      iwq::last_hip_error() = (int)e;
      return IWQ_ERR_HIP;
    }
    return IWQ_OK;
  }
  if (flags & IWQ_FLAG_TILED_CODES) {  // decode tile layout: the weight-streaming kernel only
    if (M > 16) return IWQ_ERR_ARG;
    switch (variant) {  // same shapes as the row-major variants of the same number (A/B)
#if IWQ_AB
      case 1:
      case 2: launch_gemv<4, 8, 1, 0, true>(a, st, true); break;
      case 4: launch_gemv<4, 4, 2, 0, true>(a, st, true); break;
      case 5: launch_gemv<4, 4, 4, 0, true>(a, st, true); break;
      case 7: launch_gemv<6, 4, 2, 0, true>(a, st, true); break;
      case 8: launch_gemv<4, 16, 1, 0, true>(a, st, true); break;
      case 9: launch_gemv<8, 4, 1, 0, true>(a, st, true); break;
      case 10: launch_gemv<4, 2, 4, 0, true>(a, st, true); break;
      case 12: launch_gemv<2, 4, 1, 0, true>(a, st, true); break;
      case 13: launch_gemv<2, 16, 1, 0, true>(a, st, true); break;
      case 18: launch_gemv<3, 8, 1, 0, true>(a, st, true); break;
      case 19: launch_gemv<8, 8, 1, 0, true>(a, st, true); break;
      case 20: launch_gemv<2, 8, 2, 0, true>(a, st, true); break;
      case 21: launch_gemv_ct<2, 8, 2, true>(a, st); break;
      case 22: launch_gemv_ct<2, 8, 4, true>(a, st); break;
      case 23: launch_gemv_ct<3, 8, 2, true>(a, st); break;
      case 24: launch_gemv_ct<1, 8, 4, true>(a, st); break;
      case 100: launch_gemv<2, 8, 1, 1, true>(a, st, true); break;  // probe: no dequant
      case 102: launch_gemv<2, 8, 1, 2, true>(a, st, true); break;  // probe: k-major order
      case 103: launch_gemv<2, 16, 1, 2, true>(a, st, true); break;
      case 104: launch_gemv<2, 16, 1, 1, true>(a, st, true); break;
      // round 6, the X stream of the ring form (no LDS image) at batched decode: 107 the ring itself,
      // 105 its X loads made line-contiguous (same bytes, wrong results), 106 no X loads (wrong results)
      case 105: launch_gemv<2, 8, 1, 5, true>(a, st, false); break;
      case 106: launch_gemv<2, 8, 1, 6, true>(a, st, false); break;
      case 107: launch_gemv<2, 8, 1, 0, true>(a, st, false); break;
      case 25: launch_gemv<2, 8, 1, 0, true>(a, st, true, false, 0); break;  // per-element scale (A/B)
      case 26: launch_gemv_ct<1, 8, 4, true>(a, st, false, false); break;
      case 27: launch_gemv<2, 8, 1, 0, true>(a, st, true, true, 0); break;  // grouped: params per step, global
      case 28: launch_gemv<2, 8, 1, 0, true>(a, st, true, true, 1); break;  // grouped: staged, scale per weight
      case 29:  // round 6: the default's kernels with the large X image (XLDS_BIG) where it applies
        if (const int ct = gemv_auto_ct(M, N, K); ct == 4) launch_gemv_ct<1, 8, 4, true, true>(a, st);
        else if (ct == 2) launch_gemv_ct<3, 8, 2, true, true>(a, st);
        else if (gemv_long_k(M, K)) launch_gemv<2, 16, 1, 0, true, true>(a, st, true);
        else launch_gemv<2, 8, 1, 0, true, true>(a, st, true);
        break;
      case 30:  // the same with the 16-way k-split (more waves per CU to stage and stream)
        if (const int ct = gemv_auto_ct(M, N, K); ct == 4) launch_gemv_ct<1, 16, 4, true, true>(a, st);
        else launch_gemv<2, 16, 1, 0, true, true>(a, st, true);
        break;
#endif
      default:
        if (const int ct = gemv_auto_ct(M, N, K); ct == 4) launch_gemv_ct<1, 8, 4, true>(a, st);
        else if (ct == 2) launch_gemv_ct<3, 8, 2, true>(a, st);
        else if (gemv_long_k(M, K)) launch_gemv<2, 16, 1, 0, true>(a, st, true);
        // round 6: the large X image where the one-tile grid is at most one workgroup per CU (M >= 8
        // on K = 4096: q / o; variant 29 vs the ring, cold, profiles/r06_gemv_bigx.jsonl: M = 16 per
        // channel 6.84 -> 6.49 us, g128 7.60 -> 6.91; M = 8 g128 6.28 -> 5.84, per channel +2 %)
        else launch_gemv<2, 8, 1, 0, true, true>(a, st, true);
        break;
    }
  } else if (M <= 16 && !(flags & IWQ_FLAG_FORCE_GENERIC)) {
    switch (variant) {
#if IWQ_AB
      case 1:  // previous decode kernel (A/B reference)
        if (K >= 4096) hipLaunchKernelGGL(k_w4a16_decode<8>, dim3((unsigned)(N / 16)), dim3(512), 0, st, a);
        else hipLaunchKernelGGL(k_w4a16_decode<4>, dim3((unsigned)(N / 16)), dim3(256), 0, st, a);
        break;
      case 2: launch_gemv<4, 8, 1>(a, st, true); break;
      case 3: launch_gemv<4, 8, 1>(a, st, false); break;
      case 4: launch_gemv<4, 4, 2>(a, st, true); break;
      case 5: launch_gemv<4, 4, 4>(a, st, true); break;
      case 6: launch_gemv<2, 8, 1>(a, st, true); break;
      case 7: launch_gemv<6, 4, 2>(a, st, true); break;
      case 8: launch_gemv<4, 16, 1>(a, st, true); break;
      case 9: launch_gemv<8, 4, 1>(a, st, true); break;
      case 10: launch_gemv<4, 2, 4>(a, st, true); break;
      case 11: launch_gemv<2, 4, 2>(a, st, false); break;
      case 100: launch_gemv<2, 8, 1, 1>(a, st, true); break;  // probes: no dequant
      case 101: launch_gemv<4, 8, 1, 1>(a, st, true); break;
      case 12: launch_gemv<2, 4, 1>(a, st, true); break;
      case 13: launch_gemv<2, 16, 1>(a, st, true); break;
      // persistent variants (k_w4a16_gemv_p): measured 0-20 % SLOWER than the default on every Llama
      // decode shape (profiles/r01_gemv_persistent.jsonl) -- the per-group flush barriers stall the
      // code ring more than the second-round tail costs; kept for A/B
      case 21: launch_gemv_ct<2, 8, 2, false>(a, st); break;
      case 22: launch_gemv_ct<2, 8, 4, false>(a, st); break;
      case 23: launch_gemv_ct<3, 8, 2, false>(a, st); break;
      case 24: launch_gemv_ct<1, 8, 4, false>(a, st); break;
      case 14: launch_gemv_p<2, 8, 1>(a, st); break;
      case 15: launch_gemv_p<4, 8, 1>(a, st); break;
      case 16: launch_gemv_p<2, 4, 1>(a, st); break;
      case 17: launch_gemv_p<4, 4, 1>(a, st); break;
#endif
      default:  // best or within 5 % of best, M in {1,4,16} (r01 sweep); column tiles for M >= 4
        if (const int ct = gemv_auto_ct(M, N, K); ct == 4) launch_gemv_ct<1, 8, 4, false>(a, st);
        else if (ct == 2) launch_gemv_ct<3, 8, 2, false>(a, st);
        else if (gemv_long_k(M, K)) launch_gemv<2, 16, 1>(a, st, true);
        else launch_gemv<2, 8, 1, 0, false, true>(a, st, true);  // (the large X image, as tiled)
        break;
    }
  } else if (((variant == 0 && !split_pref && !short_pref &&
               (M < 256 || !prefill_b32_supported(M, N, K, a.gpr, a.group) ||
                (M < 512 && prefill_splitk_count(M, N, K, 0) > 1))) ||
              (variant >= 50 && variant < 60)) &&
             !(flags & IWQ_FLAG_FORCE_GENERIC) && mid_supported(M, N, K, a.gpr, a.group)) {
    // 16 < M < 256, or 256 <= M < 512 where a K split would pay but the caller gave no workspace
    // for it: the weight-streaming mid-M kernel.  From M = 256 the prefill kernel runs whenever the
    // split model picks ONE range (wide weights: 70B gate/up, lm_head -- workspace or not), exactly
    // like the NIB path, so both code layouts give the same bits.
    PrefillArgs p{a.x, a.lda, a.codes, a.scales, a.zeros, a.bias, a.y, a.ldy, a.M, a.N, a.K, a.gpr, a.group, a.zsym};
    const hipError_t e = mid_launch(p, (int)variant, false, st);
    if (e != hipSuccess) {
      iwq::last_hip_error() = (int)e;
      return IWQ_ERR_HIP;
    }
    return IWQ_OK;
  } else if ((short_pref || (variant >= 110 && variant < 150)) && !(flags & IWQ_FLAG_FORCE_GENERIC) &&
             prefill_b32_supported(M, N, K, a.gpr, a.group)) {
    // short-tile split prefill: the default's plan, or forced for A/B (110-125: 128-row tiles,
    // 130-145: 64-row tiles, S = v - 108 / v - 128)
    PrefillArgs p{a.x, a.lda, a.codes, a.scales, a.zeros, a.bias, a.y, a.ldy, a.M, a.N, a.K, a.gpr, a.group, a.zsym};
    const int mtw = short_pref ? short_mtw : (variant < 130 ? 4 : 2);
    int ns = short_pref ? short_ns : (int)variant - (variant < 130 ? 108 : 128);
    if (ns > K / 64) ns = (int)(K / 64);
    if (!workspace || workspace_bytes < prefill_splitk_bytes_s(M, N, mtw, ns)) return IWQ_ERR_WORKSPACE;
    p.ws = static_cast<float*>(workspace);
    p.nsplit = ns;
    const hipError_t e = prefill_splitk_launch_s(p, mtw, st);
    if (e != hipSuccess) {
      iwq::last_hip_error() = (int)e;
      return IWQ_ERR_HIP;
    }
    return IWQ_OK;
  } else if (IWQ_AB && variant >= 180 && variant <= 183 && !(flags & IWQ_FLAG_FORCE_GENERIC)) {
    // round 6 A/B: the warp-specialised prefill (iwq_prefill_ws.hip; per channel, row-major codes)
    if (!prefill_ws_supported(M, N, K, a.gpr, a.group)) return IWQ_ERR_ARG;
    PrefillArgs p{a.x, a.lda, a.codes, a.scales, a.zeros, a.bias, a.y, a.ldy, a.M, a.N, a.K, a.gpr, a.group, a.zsym};
    const hipError_t e = prefill_ws_launch(p, (int)variant, st);
    if (e != hipSuccess) {
      iwq::last_hip_error() = (int)e;
      return IWQ_ERR_HIP;
    }
    return IWQ_OK;
  } else if (((variant == 0 && (M >= 256 || split_pref)) || (variant >= 40 && variant < 50) || (variant >= 60 && variant < 82) || variant == 97 || variant == 98 || variant == 99 || (variant >= 150 && variant <= 172) ||
              (variant > 81 && variant < 97)) && !(flags & IWQ_FLAG_FORCE_GENERIC) &&
             prefill_b32_supported(M, N, K, a.gpr, a.group)) {
    // prefill default since round 2 (iwq_prefill.hip: 32x32x16 MFMA, early barrier, per-channel
    // scale factored into the epilogue); the round-1 k_w4a16_big below stays reachable as variant 2.
    // With a workspace and fewer 256 x 256 tiles than CUs it splits K (variant 80 + S forces S ranges).
    PrefillArgs p{a.x, a.lda, a.codes, a.scales, a.zeros, a.bias, a.y, a.ldy, a.M, a.N, a.K, a.gpr, a.group, a.zsym};
    hipError_t e;
    // variant 96: the automatic split on the round-2 first split kernel (A/B)
    const int force = (variant > 81 && variant < 96) ? (int)variant - 80 : 0;
    const int nsplit = (variant == 0 || (variant > 81 && variant < 97)) ? prefill_splitk_count(M, N, K, force) : 1;
    if (nsplit > 1 && workspace && workspace_bytes >= prefill_splitk_bytes(M, N, nsplit)) {
      p.ws = static_cast<float*>(workspace);
      p.nsplit = nsplit;
      e = prefill_splitk_launch(p, st, variant == 96);
    } else {
      if (variant > 81 && variant < 96) return IWQ_ERR_WORKSPACE;
      e = prefill_b32_launch(p, (int)variant, st);
    }
    if (e != hipSuccess) {
      iwq::last_hip_error() = (int)e;
      return IWQ_ERR_HIP;
    }
    return IWQ_OK;
  } else if (N % BG_N == 0 && K % 64 == 0 && M >= 512 && variant != 1 && !(flags & IWQ_FLAG_FORCE_GENERIC) &&
             (a.gpr == 1 || a.group % 64 == 0)) {
    const int64_t blocks = ((M + BG_M - 1) / BG_M) * (N / BG_N);
    if (a.gpr != 1)
      hipLaunchKernelGGL((k_w4a16_big<64, false, true>), dim3((unsigned)blocks), dim3(BG_THR), 0, st, a);
#if IWQ_AB
    else if (variant == 23 && K % 128 == 0)
      hipLaunchKernelGGL((k_w4a16_big<128>), dim3((unsigned)blocks), dim3(BG_THR), 0, st, a);
    else if (variant == 24)
      hipLaunchKernelGGL((k_w4a16_big<64, true>), dim3((unsigned)blocks), dim3(BG_THR), 0, st, a);
#endif
    else
      hipLaunchKernelGGL((k_w4a16_big<64>), dim3((unsigned)blocks), dim3(BG_THR), 0, st, a);
  } else {
    const int64_t blocks = ((M + BM - 1) / BM) * (N / BN);
    hipLaunchKernelGGL(k_w4a16, dim3((unsigned)blocks), dim3(NTHR), 0, st, a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    iwq::last_hip_error() = (int)e;
    return IWQ_ERR_HIP;
  }
  return IWQ_OK;
}

}  // extern "C"

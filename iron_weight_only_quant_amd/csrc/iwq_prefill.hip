// iwq_prefill.hip — prefill (large M) fused dequant -> GEMM for packed INT4 weights, on the
// 32x32x16 f16 MFMA.
//
// Replaces QuantLinear.forward = F.linear(x, W_deq, b) (quant_linear.py:960-972) for weights held
// packed (include/iwq.h layout): y = x @ W_deq^T + b with W_deq = RN16((q - z) * s) rebuilt in
// registers from 4-bit codes inside the K loop.
//
// Why 32x32x16 and not 16x16x32 (k_w4a16_big, iwq_gemm.hip): the dequant is VALU work that has to
// hide in the gaps of the MFMA stream.  A 16x16x32 f16 MFMA occupies its SIMD for 16 cycles and
// holds vector issue for 8 of them, leaving room for 2 four-cycle VALU instructions; a 32x32x16
// occupies 32 cycles for the same 8 of hold, leaving room for 6 (MI355X_MICROARCH.md, cycle
// constants: 'vector-instruction ISSUE cost').  Both do the same FLOP per cycle and each B element
// is dequantized by exactly one lane of its wave either way, so the dequant costs 4 (exact) or 3
// (scale factored out) VALU per 32x32x16 MFMA: inside the 6 free slots, where with 16x16x32 the
// same work needs every free slot and anything else (LDS reads, DMA issue, waits) lands on the
// MFMA critical path.
//
// Structure (k_w4a16_b32): 256 x 256 output tile per 512-thread workgroup, 8 waves as 2 (M) x 4
// (N), 128 x 64 per wave = 4 x 2 MFMA tiles of 32 x 32; K in steps of 64; X and codes staged by
// LDS-DMA (global_load_lds_dwordx4) into a 3-stage ring, ONE raw s_barrier per K-step with a
// counted vmcnt (one stage stays in flight across it).
//   k order: MFMA slice s of a K-step gives lane half h the logical k = 32 h + 8 s + [0, 8): the
//   lane's B codes for all four slices are then ONE contiguous 16-B piece of its column (one
//   ds_read_b128 per 32-column tile per K-step), and its A fragment of slice s one 16-B piece of
//   its X row (ds_read_b128).
//   LDS images: X rows of 128 B, 16-B chunk c of row r at c ^ ((r >> 1) & 7); codes columns of
//   32 B, chunk c of column n at c ^ ((n >> 3) & 1): both read conflict-free (16 lanes hit 16
//   distinct 16-B slots of the 256-B bank row).  The DMA writes lane-linearly, so the swizzle is
//   applied to the per-lane SOURCE address.
//   dequant (natural k order): v_perm_b32 replicates a code byte into both halves, one
//   v_and_or_b32 makes (1024 + q_even, 64 + q_odd), one v_pk_add_f16 subtracts (1024 + z, 64 + z)
//   exactly; grouped / exact mode: one v_pk_mul_f16 by s = RN16((q - z) s), the reference's fp16
//   weight.  FACTOR (per-channel): B = (q - z) exactly and the fp32 accumulator is scaled by s in
//   the epilogue (y = RN16(s * sum x (q - z) + b): no per-element fp16 rounding of the weight, so
//   y differs from F.linear(x, W_deq) by that rounding only -- within the fp16 output tolerance;
//   with x = I the result is still W_deq bit for bit, since s (q - z) is exact in fp32).
#include "iwq_common.cuh"
#include "iwq_prefill.h"

namespace iwq {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int TM = 256, TN = 256, TK = 64, THR = 512, NSTAGE = 3;
constexpr int XS = TM * TK * 2;  // X bytes per stage (32 KiB)
constexpr int CS = TN * TK / 2;  // code bytes per stage (8 KiB)
constexpr int PS = 2 * TN * 4;   // grouped: 256 scales + 256 zero points, one dword each

__device__ __forceinline__ int xswz(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int cswz(int n) { return (n >> 3) & 1; }

__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t mask_s, uint32_t magic_v) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(mask_s), "v"(magic_v));
  return r;
}

__device__ __forceinline__ int64_t swizzled_block(int64_t bid, int64_t nblocks) {
  // consecutive tiles of one X row panel on one XCD (bijective for any block count)
  const int64_t xcd = bid % 8, i = bid / 8;
  const int64_t q = nblocks / 8, r = nblocks % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
}

__device__ __forceinline__ void glds16(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void glds2(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 2, 0, 0);
}

// one code dword (k offsets 0..7, nibble p = offset p) -> 8 fp16 weights in natural k order:
// (q - z) exactly, times s unless the scale is factored out (SCALE = false)
template <bool SCALE>
__device__ __forceinline__ h8 dq8(uint32_t w, h2 zz, h2 s, uint32_t mask_s, uint32_t magic_v) {
  h2 d0 = as_h2(and_or(__builtin_amdgcn_perm(w, w, 0x0C000C00u), mask_s, magic_v)) - zz;
  h2 d1 = as_h2(and_or(__builtin_amdgcn_perm(w, w, 0x0C010C01u), mask_s, magic_v)) - zz;
  h2 d2 = as_h2(and_or(__builtin_amdgcn_perm(w, w, 0x0C020C02u), mask_s, magic_v)) - zz;
  h2 d3 = as_h2(and_or(__builtin_amdgcn_perm(w, w, 0x0C030C03u), mask_s, magic_v)) - zz;
  if constexpr (SCALE) {
    d0 = d0 * s;
    d1 = d1 * s;
    d2 = d2 * s;
    d3 = d3 * s;
  }
  return h8{d0.x, d0.y, d1.x, d1.y, d2.x, d2.y, d3.x, d3.y};
}

// NIB layout (iwq_prefill.hip variant 66; codes repacked so that nibble p of a code dword holds
// k = (0, 2, 4, 6, 1, 3, 5, 7)[p]): two and-or per dword half give (1024 + k0, 1024 + k1) and
// (64 + k2, 64 + k3) (nibble at mantissa bits 4-7 under exponent 64: unit 1/16 x 16), one shift
// for the upper half -- 9 VALU per 8 weights in natural k order instead of 12.
template <bool SCALE>
__device__ __forceinline__ h8 dq8n(uint32_t w, h2 zl, h2 zh, h2 s, uint32_t m0_s, uint32_t m1_s, uint32_t mg64,
                                   uint32_t mg54) {
  const uint32_t t = w >> 8;
  h2 d0 = as_h2(and_or(w, m0_s, mg64)) - zl;
  h2 d1 = as_h2(and_or(w, m1_s, mg54)) - zh;
  h2 d2 = as_h2(and_or(t, m0_s, mg64)) - zl;
  h2 d3 = as_h2(and_or(t, m1_s, mg54)) - zh;
  if constexpr (SCALE) {
    d0 = d0 * s;
    d1 = d1 * s;
    d2 = d2 * s;
    d3 = d3 * s;
  }
  return h8{d0.x, d0.y, d1.x, d1.y, d2.x, d2.y, d3.x, d3.y};
}

// SCHED 0: compiler schedule; 1: slice s+1's dequant interleaved with slice s's MFMAs
// (sched_group_barrier, 1 MFMA : 3 VALU); PRIO: s_setprio(1) over each slice's MFMAs.
template <bool GROUPED, bool FACTOR, int SCHED, bool PRIO>
__global__ __launch_bounds__(THR) void k_w4a16_b32(PrefillArgs a) {
  static_assert(!(GROUPED && FACTOR), "grouped scales change along k: no factoring");
  constexpr int STAGE = XS + CS + (GROUPED ? PS : 0);
  constexpr int PER_STAGE = 4 + 1 + (GROUPED ? 1 : 0);  // DMA instructions per thread per stage
  constexpr bool SCALE = !FACTOR;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int nk = a.K / TK;
  const int64_t crow = a.K / 2;

  // DMA sources (per lane); destinations are wave-uniform 1-KiB slots filled lane-linearly:
  // X: slot 4 wid + i = rows 8 (4 wid + i) + [0, 8), lane = 8 (row % 8) + physical chunk
  const _Float16* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;  // rows past M: any valid row (discarded)
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xswz(row)) << 3);
  }
  // codes: slot wid = columns 32 wid + [0, 32), lane = 2 (col % 32) + physical chunk
  const int ccol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + ccol) * crow + (((lane & 1) ^ cswz(ccol)) << 4);
  const _Float16* psrc = nullptr;
  if constexpr (GROUPED) {  // wave w < 4: scale of column 64 w + lane; w >= 4: its zero point
    const _Float16* arr = (wid < 4 || !a.zeros) ? a.scales : a.zeros;
    psrc = arr + (int64_t)(n0 + (wid & 3) * 64 + lane) * a.gpr;
  }
  auto issue = [&](int kt, int stg) {
    uint8_t* base = smem + stg * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
    if constexpr (GROUPED) glds2(psrc + (kt * TK) / a.group, base + XS + CS + wid * 256);
  };

  h2 sv[2], zz[2];
  float sf[2] = {1.0f, 1.0f};
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int col = n0 + wn * 64 + nt * 32 + r32;
      const _Float16 sc = gp<_Float16>(a.scales)[col];
      const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
      sv[nt] = h2{sc, sc};
      sf[nt] = (float)sc;
      zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};  // exact: z is a small integer
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  uint32_t magic_v;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));

  f16x acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    // own DMA of stage kt retired (stage kt+1's stays in flight); the barrier makes every wave's
    // part visible and proves every wave is done reading the stage about to be refilled
    if (kt + 1 < nk) {
      if constexpr (PER_STAGE == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(kt + 2, (kt + 2) % NSTAGE);
    const uint8_t* xs = smem + (kt % NSTAGE) * STAGE;
    const uint8_t* cs = xs + XS;
    if constexpr (GROUPED) {
      const uint32_t* ps = reinterpret_cast<const uint32_t*>(cs + CS);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int col = wn * 64 + nt * 32 + r32;
        const _Float16 sc = __builtin_bit_cast(_Float16, (uint16_t)ps[col]);
        const float zf = a.zeros ? (float)__builtin_bit_cast(_Float16, (uint16_t)ps[TN + col]) : a.zsym;
        sv[nt] = h2{sc, sc};
        zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
      }
    }
    u32x4 wc[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int col = wn * 64 + nt * 32 + r32;
      wc[nt] = *reinterpret_cast<const u32x4*>(cs + col * 32 + ((h ^ cswz(col)) << 4));
    }
    h8 bf[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) bf[nt][0] = dq8<SCALE>(wc[nt][0], zz[nt], sv[nt], mask_s, magic_v);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      h8 af[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int row = wm * 128 + mt * 32 + r32;
        af[mt] = *reinterpret_cast<const h8*>(xs + row * 128 + (((4 * h + s) ^ xswz(row)) << 4));
      }
      if (s + 1 < 4) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) bf[nt][s + 1] = dq8<SCALE>(wc[nt][s + 1], zz[nt], sv[nt], mask_s, magic_v);
      }
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[mt], bf[nt][s], acc[mt][nt], 0, 0, 0);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      if constexpr (SCHED == 1) {
        // per slice: the A reads, then each MFMA followed by ~3 of the next slice's dequant VALU
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // 4 DS reads
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // 3 VALU
        }
      }
    }
  }

  // epilogue, 32x32 C layout: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int col = n0 + wn * 64 + nt * 32 + r32;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = FACTOR ? opaque(acc[mt][nt][r] * sf[nt]) : acc[mt][nt][r];  // no fma_mix fold
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + b);
      }
    }
  }
}

// Early-barrier form (k_w4a16_b32e): the barrier that publishes stage kt+1 sits BEFORE the last
// MFMA slice of stage kt, whose operands are already in registers.  After the barrier a wave
// issues the next DMA, the LDS reads of stage kt+1's codes and first A slice and that slice's
// dequant, and only then slice 3's 8 MFMAs (256 cycles of MFMA work) -- which cover the LDS read
// latency and the dequant chain of the next K-step instead of leaving the MFMA pipe idle at every
// K-step start.  Same k order, same accumulation order: bit-identical to k_w4a16_b32.
// WAR: a wave's last reads of stage kt (slice 3's A fragments) are retired (lgkmcnt(0)) before the
// barrier after which stage kt is refilled.
// SWAP: the weight fragment is the MFMA's A operand and X's the B operand, so the accumulator holds
// C^T: a lane owns one output row m and, per register quad, 4 consecutive columns n -- the epilogue
// stores 8 B per instruction (4 per 32 x 32 tile) instead of 2 B (16 per tile).  The two operand
// layouts of the 32x32x16 MFMA are the same, so the swap costs nothing in the loop.
// SPLIT: the workgroup's tile and K range come from blockIdx = split * tiles + tile (adjacent tiles of
// one K range share an XCD: the same X rows and K range); the raw fp32 accumulators go to
// a.ws[(tile * nsplit + split)][wave][mt, nt][reg][lane] (256-B coalesced stores) for
// k_splitk_reduce, which applies the epilogue.
template <bool GROUPED, bool FACTOR, int WM, bool PHI = false, bool NIB = false, bool SWAP = false,
          bool SPLIT = false>
__global__ __launch_bounds__(THR) void k_w4a16_b32e(PrefillArgs a) {
  // WM waves along M x WN along N; a wave owns (TM / WM) x (TN / WN) = MTL x NTL tiles of 32 x 32
  constexpr int WN = 8 / WM, MTL = TM / WM / 32, NTL = TN / WN / 32;
  static_assert(WM * WN == 8 && MTL * NTL == 8, "8 waves, 8 MFMA tiles per wave");
  static_assert(!(GROUPED && FACTOR), "grouped scales change along k: no factoring");
  constexpr int STAGE = XS + CS + (GROUPED ? PS : 0);
  constexpr int PER_STAGE = 4 + 1 + (GROUPED ? 1 : 0);
  constexpr bool SCALE = !FACTOR;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  int64_t t;
  int kbase = 0, nk = a.K / TK, split = 0;
  if constexpr (SPLIT) {
    const int64_t tiles = (int64_t)gridDim.x / a.nsplit;
    const int64_t b = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
    split = (int)(b / tiles);
    t = b - (int64_t)split * tiles;
    kbase = split * a.kps;
    nk = min(a.kps, nk - kbase);  // >= 1 by construction (prefill_splitk_count)
  } else {
    t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  }
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int64_t crow = a.K / 2;

  const _Float16* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + kbase * TK + (((lane & 7) ^ xswz(row)) << 3);
  }
  const int ccol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + ccol) * crow + kbase * (TK / 2) + (((lane & 1) ^ cswz(ccol)) << 4);
  const _Float16* psrc = nullptr;
  if constexpr (GROUPED) {
    const _Float16* arr = (wid < 4 || !a.zeros) ? a.scales : a.zeros;
    psrc = arr + (int64_t)(n0 + (wid & 3) * 64 + lane) * a.gpr;
  }
  auto issue = [&](int kt, int stg) {
    uint8_t* base = smem + stg * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
    if constexpr (GROUPED) glds2(psrc + ((kbase + kt) * TK) / a.group, base + XS + CS + wid * 256);
  };

  h2 sv[NTL], zz[NTL], zl[NTL], zh[NTL];
  float sf[NTL];
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) sf[nt] = 1.0f;
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      const int col = n0 + wn * (32 * NTL) + nt * 32 + r32;
      const _Float16 sc = gp<_Float16>(a.scales)[col];
      const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
      sv[nt] = h2{sc, sc};
      sf[nt] = (float)sc;
      zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
      zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
      zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));
#define IWQ_DQ(W, NT)                                                                             \
  (NIB ? dq8n<SCALE>((W), zl[NT], zh[NT], sv[NT], m0_s, m1_s, mg64, mg54)                         \
       : dq8<SCALE>((W), zz[NT], sv[NT], mask_s, magic_v))

  // stage-local reads: grouped parameters, the codes of both 32-column tiles, one A slice
  auto read_params = [&](const uint8_t* xs) {
    if constexpr (GROUPED) {
      const uint32_t* ps = reinterpret_cast<const uint32_t*>(xs + XS + CS);
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt) {
        const int col = wn * (32 * NTL) + nt * 32 + r32;
        const _Float16 sc = __builtin_bit_cast(_Float16, (uint16_t)ps[col]);
        const float zf = a.zeros ? (float)__builtin_bit_cast(_Float16, (uint16_t)ps[TN + col]) : a.zsym;
        sv[nt] = h2{sc, sc};
        zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
        zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
        zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
      }
    }
  };
  auto read_codes = [&](const uint8_t* xs, u32x4 (&wc)[NTL]) {
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      const int col = wn * (32 * NTL) + nt * 32 + r32;
      wc[nt] = *reinterpret_cast<const u32x4*>(xs + XS + col * 32 + ((h ^ cswz(col)) << 4));
    }
  };
  auto read_a = [&](const uint8_t* xs, int s, h8 (&af)[MTL]) {
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt) {
      const int row = wm * (32 * MTL) + mt * 32 + r32;
      af[mt] = *reinterpret_cast<const h8*>(xs + row * 128 + (((4 * h + s) ^ xswz(row)) << 4));
    }
  };

  f16x acc[MTL][NTL];
#pragma unroll
  for (int i = 0; i < MTL; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
#define IWQ_MFMA_SLICE(AF, B0)                                                                   \
  _Pragma("unroll") for (int mt = 0; mt < MTL; ++mt)                                              \
  _Pragma("unroll") for (int nt = 0; nt < NTL; ++nt)                                              \
    acc[mt][nt] = SWAP ? __builtin_amdgcn_mfma_f32_32x32x16_f16(B0[nt], AF[mt], acc[mt][nt], 0, 0, 0) \
                       : __builtin_amdgcn_mfma_f32_32x32x16_f16(AF[mt], B0[nt], acc[mt][nt], 0, 0, 0);

  // PHI: static priority 1 for the second-dispatched half (waves 4-7, the VALU-arbitration loser;
  // cdna_hip_programming.md T5 static form)
  if constexpr (PHI) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    if constexpr (PER_STAGE == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (nk > 2) issue(2, 2);
  u32x4 wc[NTL];
  h8 af[MTL], bcur[NTL];
  read_params(smem);
  read_codes(smem, wc);
  read_a(smem, 0, af);
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) bcur[nt] = IWQ_DQ(wc[nt][0], nt);

  // slices 0..2 of the stage at xs: each slice's MFMAs behind the next slice's reads + dequant
#define IWQ_SLICES_012(XS)                                                                        \
  _Pragma("unroll") for (int s = 0; s < 3; ++s) {                                                 \
    h8 an[MTL], bn[NTL];                                                                          \
    read_a(XS, s + 1, an);                                                                        \
    _Pragma("unroll") for (int nt = 0; nt < NTL; ++nt)                                            \
      bn[nt] = IWQ_DQ(wc[nt][s + 1], nt);                        \
    IWQ_MFMA_SLICE(af, bcur)                                                                      \
    _Pragma("unroll") for (int mt = 0; mt < MTL; ++mt) af[mt] = an[mt];                          \
    _Pragma("unroll") for (int nt = 0; nt < NTL; ++nt) bcur[nt] = bn[nt];                        \
  }
  // the last K-step is peeled: no branch between the barrier and slice 3 inside the loop
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint8_t* xs = smem + (kt % NSTAGE) * STAGE;
    IWQ_SLICES_012(xs)
    // slice 3's operands are in registers; publish stage kt+1, retire this wave's reads of stage kt
    if (kt + 2 < nk) {
      if constexpr (PER_STAGE == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + 3 < nk) issue(kt + 3, kt % NSTAGE);
    const uint8_t* xn = smem + ((kt + 1) % NSTAGE) * STAGE;
    h8 an[MTL], bn[NTL];
    u32x4 wn2[NTL];
    read_params(xn);
    read_codes(xn, wn2);
    read_a(xn, 0, an);
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) bn[nt] = IWQ_DQ(wn2[nt][0], nt);
    IWQ_MFMA_SLICE(af, bcur)
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt) af[mt] = an[mt];
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      bcur[nt] = bn[nt];
      wc[nt] = wn2[nt];
    }
  }
  {
    const uint8_t* xs = smem + ((nk - 1) % NSTAGE) * STAGE;
    IWQ_SLICES_012(xs)
    IWQ_MFMA_SLICE(af, bcur)
  }
#undef IWQ_SLICES_012

  if constexpr (SPLIT) {
    float* dst = a.ws + ((t * a.nsplit + split) * 8 + wid) * 8192 + lane;
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) gp<float>(dst)[((mt * NTL + nt) * 16 + r) * 64] = acc[mt][nt][r];
  } else if constexpr (SWAP) {
    // C^T layout: row m = lane & 31 of the tile, columns n = (r & 3) + 8 (r >> 2) + 4 h
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = n0 + wn * (32 * NTL) + nt * 32 + 8 * g + 4 * h;
        float sc[4], bb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sc[j] = FACTOR ? (float)gp<_Float16>(a.scales)[col + j] : 1.0f;
          bb[j] = a.bias ? (float)gp<_Float16>(a.bias)[col + j] : 0.0f;
        }
#pragma unroll
        for (int mt = 0; mt < MTL; ++mt) {
          const int row = m0 + wm * (32 * MTL) + mt * 32 + r32;
          h2 lo = h2{(_Float16)(opaque(acc[mt][nt][4 * g + 0] * sc[0]) + bb[0]), (_Float16)(opaque(acc[mt][nt][4 * g + 1] * sc[1]) + bb[1])};
          h2 hi = h2{(_Float16)(opaque(acc[mt][nt][4 * g + 2] * sc[2]) + bb[2]), (_Float16)(opaque(acc[mt][nt][4 * g + 3] * sc[3]) + bb[3])};
          typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
          if (row < a.M)
            *reinterpret_cast<IWQ_GLOBAL u32x2v*>(gp<_Float16>(a.y) + (int64_t)row * a.ldy + col) =
                u32x2v{as_u32(lo), as_u32(hi)};
        }
      }
    }
  } else {
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    const int col = n0 + wn * (32 * NTL) + nt * 32 + r32;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (32 * MTL) + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = FACTOR ? opaque(acc[mt][nt][r] * sf[nt]) : acc[mt][nt][r];  // no fma_mix fold
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + b);
      }
    }
  }
  }
}

#undef IWQ_DQ
#undef IWQ_MFMA_SLICE


// ---------------------------------------------------------------------------------------------
// k_w4a16_w4e: the same 256 x 256 tile on FOUR waves (one per SIMD), 128 x 128 per wave = 4 x 4
// MFMA tiles of 32 x 32, the 256 fp32 accumulators in AGPRs (amdgpu_waves_per_eu(1, 1): 512
// registers per lane).  Against the 8-wave form: every dequantized B fragment and every A
// fragment feeds 4 MFMAs (2 and 4 there), so the LDS A reads per MFMA halve and no two waves of a
// SIMD compete for its issue port; the operand prefetch (next slice's A reads + dequant behind the
// current slice's 16 MFMAs = 512 cycles) must hide the LDS latency on its own.  Same LDS images,
// k order, early barrier and stage ring as k_w4a16_b32e; per stage a wave issues 8 X pieces, 2 code
// pieces (+ 2 parameter pieces grouped).
// ---------------------------------------------------------------------------------------------
// SG: pin the interleave with sched_group_barrier (hipcc otherwise issues each A read right before
// its MFMAs and waits on it: ds_read -> lgkmcnt(0) -> MFMA, the LDS latency on the critical path):
// per slice, the next slice's 4 A reads first, then 16 x {1 MFMA, 3 VALU of the next slice's
// dequant}; after the barrier, the next stage's code/A reads, 4 bare MFMAs (cover the code read),
// then 12 x {1 MFMA, 4 VALU}.
template <bool GROUPED, bool FACTOR, bool SG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_w4a16_w4e(PrefillArgs a) {
  static_assert(!(GROUPED && FACTOR), "grouped scales change along k: no factoring");
  constexpr int STAGE = XS + CS + (GROUPED ? PS : 0);
  constexpr int PER_STAGE = 8 + 2 + (GROUPED ? 2 : 0);
  constexpr bool SCALE = !FACTOR;
  constexpr int MTL = 4, NTL = 4;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int nk = a.K / TK;
  const int64_t crow = a.K / 2;

  // X: slot 8 wid + i = rows 8 (8 wid + i) + [0, 8); lane = 8 (row % 8) + physical chunk.  Rows
  // 8 (8 wid + i) + lane / 8 = 64 wid + 8 i + lane / 8: one base pointer + i * 8 rows.
  const int xrow0 = wid * 64 + (lane >> 3);
  const int xgm0 = m0 + xrow0;
  const _Float16* xsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = xrow0 + 8 * i;
    const int gm = xgm0 + 8 * i < a.M ? xgm0 + 8 * i : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xswz(row)) << 3);
  }
  // codes: slots 2 wid, 2 wid + 1 = columns 64 wid + [0, 64)
  const uint8_t* csrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ccol = (2 * wid + i) * 32 + (lane >> 1);
    csrc[i] = a.codes + (int64_t)(n0 + ccol) * crow + (((lane & 1) ^ cswz(ccol)) << 4);
  }
  const _Float16* psrc_s = nullptr;
  const _Float16* psrc_z = nullptr;
  if constexpr (GROUPED) {
    psrc_s = a.scales + (int64_t)(n0 + wid * 64 + lane) * a.gpr;
    psrc_z = (a.zeros ? a.zeros : a.scales) + (int64_t)(n0 + wid * 64 + lane) * a.gpr;
  }
  auto issue = [&](int kt, int stg) {
    uint8_t* base = smem + stg * STAGE;
#pragma unroll
    for (int i = 0; i < 8; ++i) glds16(xsrc[i] + kt * TK, base + (wid * 8 + i) * 1024);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(csrc[i] + kt * (TK / 2), base + XS + (wid * 2 + i) * 1024);
    if constexpr (GROUPED) {
      glds2(psrc_s + (kt * TK) / a.group, base + XS + CS + wid * 256);
      glds2(psrc_z + (kt * TK) / a.group, base + XS + CS + (4 + wid) * 256);
    }
  };

  h2 sv[NTL], zz[NTL];
  float sf[NTL];
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) sf[nt] = 1.0f;
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      const int col = n0 + wn * 128 + nt * 32 + r32;
      const _Float16 sc = gp<_Float16>(a.scales)[col];
      const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
      sv[nt] = h2{sc, sc};
      sf[nt] = (float)sc;
      zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  uint32_t magic_v;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));

  auto read_params = [&](const uint8_t* xs) {
    if constexpr (GROUPED) {
      const uint32_t* ps = reinterpret_cast<const uint32_t*>(xs + XS + CS);
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt) {
        const int col = wn * 128 + nt * 32 + r32;
        const _Float16 sc = __builtin_bit_cast(_Float16, (uint16_t)ps[col]);
        const float zf = a.zeros ? (float)__builtin_bit_cast(_Float16, (uint16_t)ps[TN + col]) : a.zsym;
        sv[nt] = h2{sc, sc};
        zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
      }
    }
  };
  auto read_codes = [&](const uint8_t* xs, u32x4 (&wc)[NTL]) {
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      const int col = wn * 128 + nt * 32 + r32;
      wc[nt] = *reinterpret_cast<const u32x4*>(xs + XS + col * 32 + ((h ^ cswz(col)) << 4));
    }
  };
  auto read_a = [&](const uint8_t* xs, int s, h8 (&af)[MTL]) {
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt) {
      const int row = wm * 128 + mt * 32 + r32;
      af[mt] = *reinterpret_cast<const h8*>(xs + row * 128 + (((4 * h + s) ^ xswz(row)) << 4));
    }
  };

  f16x acc[MTL][NTL];
#pragma unroll
  for (int i = 0; i < MTL; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
#define IWQ_MFMA_SLICE4(AF, B0)                                                                  \
  _Pragma("unroll") for (int mt = 0; mt < MTL; ++mt)                                              \
  _Pragma("unroll") for (int nt = 0; nt < NTL; ++nt)                                              \
    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AF[mt], B0[nt], acc[mt][nt], 0, 0, 0);

  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STAGE) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (nk > 2) issue(2, 2);
  u32x4 wc[NTL];
  h8 af[MTL], bcur[NTL];
  read_params(smem);
  read_codes(smem, wc);
  read_a(smem, 0, af);
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) bcur[nt] = dq8<SCALE>(wc[nt][0], zz[nt], sv[nt], mask_s, magic_v);

#define IWQ_SLICES4_012(XS)                                                                       \
  _Pragma("unroll") for (int s = 0; s < 3; ++s) {                                                 \
    h8 an[MTL], bn[NTL];                                                                          \
    read_a(XS, s + 1, an);                                                                        \
    _Pragma("unroll") for (int nt = 0; nt < NTL; ++nt)                                            \
      bn[nt] = dq8<SCALE>(wc[nt][s + 1], zz[nt], sv[nt], mask_s, magic_v);                        \
    IWQ_MFMA_SLICE4(af, bcur)                                                                     \
    if constexpr (SG) {                                                                           \
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                                          \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                            \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                        \
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);                                        \
      }                                                                                           \
      __builtin_amdgcn_sched_barrier(0);                                                          \
    }                                                                                             \
    _Pragma("unroll") for (int mt = 0; mt < MTL; ++mt) af[mt] = an[mt];                          \
    _Pragma("unroll") for (int nt = 0; nt < NTL; ++nt) bcur[nt] = bn[nt];                        \
  }
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint8_t* xs = smem + (kt % NSTAGE) * STAGE;
    IWQ_SLICES4_012(xs)
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 3 < nk) issue(kt + 3, kt % NSTAGE);
    const uint8_t* xn = smem + ((kt + 1) % NSTAGE) * STAGE;
    h8 an[MTL], bn[NTL];
    u32x4 wn2[NTL];
    read_params(xn);
    read_codes(xn, wn2);
    read_a(xn, 0, an);
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) bn[nt] = dq8<SCALE>(wn2[nt][0], zz[nt], sv[nt], mask_s, magic_v);
    IWQ_MFMA_SLICE4(af, bcur)
    if constexpr (SG) {
      __builtin_amdgcn_sched_group_barrier(0x100, GROUPED ? 16 : 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt) af[mt] = an[mt];
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      bcur[nt] = bn[nt];
      wc[nt] = wn2[nt];
    }
  }
  {
    const uint8_t* xs = smem + ((nk - 1) % NSTAGE) * STAGE;
    IWQ_SLICES4_012(xs)
    IWQ_MFMA_SLICE4(af, bcur)
  }
#undef IWQ_SLICES4_012
#undef IWQ_MFMA_SLICE4

#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    const int col = n0 + wn * 128 + nt * 32 + r32;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < MTL; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = FACTOR ? opaque(acc[mt][nt][r] * sf[nt]) : acc[mt][nt][r];  // no fma_mix fold
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + b);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_b32w: 256 x 256 tile, 8 waves as 1 (M) x 8 (N): a wave owns ALL 256 rows x 32 columns
// (8 x 1 tiles of 32x32x16).  Against the 2 x 4 layout each weight is dequantized once per
// workgroup instead of twice (12 -> 6 dequant VALU per wave per MFMA slice... 96 -> 48 per K-step),
// for twice the LDS A bytes (256 KiB per K-step: 1 ds_read_b128 per MFMA gap, the array's 256 B/clk
// keeps up).  The per-SIMD issue budget is the limit of this loop (MFMA 8 of 32 cycles + ~4 per VALU,
// two waves per SIMD), which is what the halved VALU buys back.
// Hand-ordered stream: every LDS read is inline asm with hand-counted waits, every group pinned by
// sched_barrier (hipcc's waitcnt pass waits lgkmcnt(0) on reads it has just issued).  Per MFMA
// slice: MFMA mt then the rolling read of fragment mt of the next slice (7 MFMAs ahead of its use:
// before MFMA mt exactly 7 newer reads are outstanding -> lgkmcnt(7)); the next slice's dequant
// (4 pairs of 3, or 9 VALU with the NIB layout) between the MFMAs.  Early barrier as k_w4a16_b32e.
// Per channel (scale in the epilogue) only.
// ---------------------------------------------------------------------------------------------
template <int OFF>
__device__ __forceinline__ h8 lds_rd(uint32_t addr) {
  h8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ u32x4 lds_rd_u(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
// A value read by inline asm is only valid once its lgkmcnt wait has retired, which the compiler
// cannot see: passes before the scheduler (CSE, hoisting) may move a cheap use of it (a shift of a
// code dword) above the wait.  landed(v) after the wait re-defines v there (volatile asm keeps its
// order with the volatile wait), so every later use depends on the post-wait value.
template <class T>
__device__ __forceinline__ void landed(T& v) {
  asm volatile("" : "+v"(v));
}

template <int OFF>
__device__ __forceinline__ uint32_t lds_rd_d(uint32_t addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}

#define IWQ_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define IWQ_PIN() __builtin_amdgcn_sched_barrier(0)

// GROUPED (group % 64 == 0): each K-step lies in one group, so a lane needs ONE (s, z) per K-step;
// they ride with the stage (one more DMA piece per wave, b32e's parameter image) and the dequant
// applies s per weight (RN16((q - z) s), the reference's fp16 weight; no epilogue scale).
// SPLIT: one K range of a split-K launch (k_w4a16_b32e's SPLIT: tile / range from blockIdx, the raw
// accumulators to the workspace in b32e's 2 x 4 wave layout, so k_splitk_reduce is shared).
// PG (grouped only): the parameters change once per group, not per K-step -- a K-step stages, reads
// and converts them only when it starts a group (or is the range's first); the others keep the
// registers (one DMA piece, two LDS reads and the set_params VALU fewer per wave on every K-step
// that does not start a group: half of them at g = 128).  The vmcnt counts follow the pieces issued.
template <bool NIB, bool GROUPED = false, bool SPLIT = false, int EPI = 0, bool PG = false>
__global__ __launch_bounds__(THR) void k_w4a16_b32w(PrefillArgs a) {
  constexpr int STAGE = XS + CS + (GROUPED ? PS : 0);
  constexpr int PER_STAGE = GROUPED ? 6 : 5;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  int64_t t;
  int kbase = 0, nk = a.K / TK, split = 0;
  if constexpr (SPLIT) {
    const int64_t tiles = (int64_t)gridDim.x / a.nsplit;
    const int64_t b = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
    split = (int)(b / tiles);
    t = b - (int64_t)split * tiles;
    kbase = split * a.kps;
    nk = min(a.kps, nk - kbase);  // >= 1 by construction (prefill_splitk_count)
  } else {
    t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  }
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int64_t crow = a.K / 2;

  const _Float16* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + kbase * TK + (((lane & 7) ^ xswz(row)) << 3);
  }
  const int ccol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + ccol) * crow + kbase * (TK / 2) + (((lane & 1) ^ cswz(ccol)) << 4);
  // grouped: waves 0-3 stage the scales of columns 64 (wid & 3) + lane, waves 4-7 the zero points
  // (dword slots col / TN + col of the parameter image, as k_w4a16_b32e)
  const _Float16* psrc = nullptr;
  if constexpr (GROUPED) {
    const _Float16* arr = (wid < 4 || !a.zeros) ? a.scales : a.zeros;
    psrc = arr + (int64_t)(n0 + (wid & 3) * 64 + lane) * a.gpr;
  }
  // does K-step k of this range carry its group's parameters (wave-uniform)?
  auto hp = [&](int k) -> bool {
    if constexpr (!GROUPED) return false;
    else if constexpr (!PG) return true;
    else return k == 0 || ((kbase + k) * TK) % a.group == 0;
  };
  auto issue = [&](int kt, int stg) {
    uint8_t* base = smem + stg * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
    if constexpr (GROUPED) {
      if (hp(kt)) glds2(psrc + ((kbase + kt) * TK) / a.group, base + XS + CS + wid * 256);
    }
  };
  // one DMA piece (i < 4: X rows, 4: codes, 5: parameters) of K-step kt into stage stg
  auto issue1 = [&](int kt, int stg, int i) {
    uint8_t* base = smem + stg * STAGE;
    if (i < 4) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    else if (i == 4) glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
    else if constexpr (GROUPED) {
      if (hp(kt)) glds2(psrc + ((kbase + kt) * TK) / a.group, base + XS + CS + wid * 256);
    }
  };

  // this lane's column and its parameters (per channel: once; grouped: per K-step, set_params)
  const int col = n0 + wid * 32 + r32;
  float sfl = 1.0f;
  h2 s2{}, zz{}, zl{}, zh{};
  auto set_params = [&](_Float16 sc, float zf) {
    sfl = (float)sc;
    s2 = h2{sc, sc};
    zz = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  };
  if constexpr (!GROUPED)
    set_params(gp<_Float16>(a.scales)[col], a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym);
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  // LDS byte addresses: A fragment (stage st, slice s, tile mt) = la[s] + st * STAGE + 4096 mt
  // (row = 32 mt + r32, and (row >> 1) & 7 does not depend on mt); codes of this lane's column
  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) la[s] = lbase + (uint32_t)(r32 * 128 + (((4 * h + s) ^ xswz(r32)) << 4));
  const int ccl = wid * 32 + r32;
  const uint32_t lc = lbase + XS + (uint32_t)(ccl * 32 + ((h ^ cswz(ccl)) << 4));
  const uint32_t lp = lbase + XS + CS + (uint32_t)(ccl * 4);  // grouped: scale slot (zero: + 4 TN)
  uint32_t psv = 0, pzv = 0;                                   // grouped: the raw parameter dwords
  auto params_landed = [&]() {
    if constexpr (GROUPED) {
      landed(psv);
      landed(pzv);
      set_params(__builtin_bit_cast(_Float16, (uint16_t)psv),
                 a.zeros ? (float)__builtin_bit_cast(_Float16, (uint16_t)pzv) : a.zsym);
    }
  };

  // dequant pair j (weights 2j, 2j+1 of the 8 in code dword w), natural k order
  auto dqp = [&](uint32_t w, uint32_t t8, int j) -> h2 {
    h2 d;
    if constexpr (NIB) {
      if (j == 0) d = as_h2(and_or(w, m0_s, mg64)) - zl;
      else if (j == 1) d = as_h2(and_or(w, m1_s, mg54)) - zh;
      else if (j == 2) d = as_h2(and_or(t8, m0_s, mg64)) - zl;
      else d = as_h2(and_or(t8, m1_s, mg54)) - zh;
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      d = as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz;
    }
    if constexpr (GROUPED) d = d * s2;  // RN16((q - z) s)
    return d;
  };

  f16x acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
  h8 af[8];
  h8 bcur;
  u32x4 wc;

#define IWQ_RD_A(MT, ADDR) af[MT] = lds_rd<(MT) * 4096>(ADDR)
#define IWQ_MF(MT) acc[MT] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[MT], bcur, acc[MT], 0, 0, 0)
  // one MFMA slice: MFMA mt, then the read of fragment mt of the next slice at address NADDR, the
  // next slice's dequant (dword W) interleaved; WAITA: the lgkmcnt(7) before each MFMA
#define IWQ_SLICE(NADDR, W, WAITA)                                                                 \
  {                                                                                               \
    const uint32_t wq = (W);                                                                      \
    uint32_t t8 = 0;                                                                              \
    h2 p0, p1, p2, p3;                                                                            \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(0); IWQ_RD_A(0, NADDR); p0 = dqp(wq, t8, 0); IWQ_PIN();                     \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(1); IWQ_RD_A(1, NADDR); if (NIB) t8 = wq >> 8; IWQ_PIN();                   \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(2); IWQ_RD_A(2, NADDR); p1 = dqp(wq, t8, 1); IWQ_PIN();                     \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(3); IWQ_RD_A(3, NADDR); IWQ_PIN();                                          \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(4); IWQ_RD_A(4, NADDR); p2 = dqp(wq, t8, 2); IWQ_PIN();                     \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(5); IWQ_RD_A(5, NADDR); IWQ_PIN();                                          \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(6); IWQ_RD_A(6, NADDR); p3 = dqp(wq, t8, 3); IWQ_PIN();                     \
    if (WAITA) IWQ_LGKM(7);                                                                       \
    IWQ_PIN(); IWQ_MF(7); IWQ_RD_A(7, NADDR); IWQ_PIN();                                          \
    bcur = h8{p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y};                                    \
  }

  // prologue: stages 0, 1, 2 (K-steps clamped to nk - 1: re-loads of stages nobody reads again)
  issue(0, 0);
  issue(nk > 1 ? 1 : 0, 1);
  if (hp(nk > 1 ? 1 : 0)) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  issue(nk > 2 ? 2 : nk - 1, 2);
  IWQ_PIN();
  wc = lds_rd_u<0>(lc);
  if constexpr (GROUPED) {
    psv = lds_rd_d<0>(lp);
    pzv = lds_rd_d<TN * 4>(lp);
  }
  IWQ_RD_A(0, la[0]); IWQ_RD_A(1, la[0]); IWQ_RD_A(2, la[0]); IWQ_RD_A(3, la[0]);
  IWQ_RD_A(4, la[0]); IWQ_RD_A(5, la[0]); IWQ_RD_A(6, la[0]); IWQ_RD_A(7, la[0]);
  IWQ_LGKM(0);
  landed(wc);
  params_landed();
  IWQ_PIN();
  {
    const uint32_t t8 = NIB ? wc[0] >> 8 : 0u;
    const h2 p0 = dqp(wc[0], t8, 0), p1 = dqp(wc[0], t8, 1), p2 = dqp(wc[0], t8, 2), p3 = dqp(wc[0], t8, 3);
    bcur = h8{p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y};
  }
  // the last K-step is peeled (no branch in the loop body: acc / af need no merge copies)
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt % NSTAGE) * STAGE);
    IWQ_SLICE(la[1] + so, wc[1], true)
    IWQ_SLICE(la[2] + so, wc[2], true)
    IWQ_SLICE(la[3] + so, wc[3], true)
    // stage kt+1 landed (this wave's part: only stage kt+2's 5 pieces -- 6 with the parameters -- may
    // still fly; near the end those are re-loads of the last K-step into a stage nobody reads again),
    // every read of stage kt retired
    if (hp(kt + 2 < nk ? kt + 2 : nk - 1)) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    IWQ_PIN();
    const int kd = kt + 3 < nk ? kt + 3 : nk - 1;  // DMA source K-step (clamped: see above)
    const int sd = kt % NSTAGE;
    const uint32_t sn = (uint32_t)(((kt + 1) % NSTAGE) * STAGE);
    u32x4 wn = lds_rd_u<0>(lc + sn);
    const bool newp = hp(kt + 1);
    if constexpr (GROUPED) {  // older than the 4 A reads below: retired by the same lgkmcnt(4)
      if (newp) {
        psv = lds_rd_d<0>(lp + sn);
        pzv = lds_rd_d<TN * 4>(lp + sn);
      }
    }
    // slice 3 of this stage; rolling reads of the next stage's slice 0; the refill of stage kt
    // spread one DMA piece per MFMA gap (each costs the issuing wave ~60-185 cycles: back to back
    // after the barrier they left the MFMA pipe idle); the next slice's dequant once the code read
    // (older than the 4 A reads before it) has landed
    const uint32_t na = la[0] + sn;
    h2 p0, p1, p2, p3;
    uint32_t t8 = 0;
    IWQ_PIN(); IWQ_MF(0); IWQ_RD_A(0, na); issue1(kd, sd, 0); IWQ_PIN();
    IWQ_PIN(); IWQ_MF(1); IWQ_RD_A(1, na); issue1(kd, sd, 1); IWQ_PIN();
    IWQ_PIN(); IWQ_MF(2); IWQ_RD_A(2, na); issue1(kd, sd, 2); IWQ_PIN();
    IWQ_PIN(); IWQ_MF(3); IWQ_RD_A(3, na); issue1(kd, sd, 3); IWQ_PIN();
    IWQ_LGKM(4);
    landed(wn);
    if (newp) params_landed();
    IWQ_PIN(); IWQ_MF(4); IWQ_RD_A(4, na); issue1(kd, sd, 4); p0 = dqp(wn[0], t8, 0); if (NIB) t8 = wn[0] >> 8; IWQ_PIN();
    IWQ_PIN(); IWQ_MF(5); IWQ_RD_A(5, na); if (GROUPED) issue1(kd, sd, 5); p1 = dqp(wn[0], t8, 1); IWQ_PIN();
    IWQ_PIN(); IWQ_MF(6); IWQ_RD_A(6, na); p2 = dqp(wn[0], t8, 2); IWQ_PIN();
    IWQ_PIN(); IWQ_MF(7); IWQ_RD_A(7, na); p3 = dqp(wn[0], t8, 3); IWQ_PIN();
    bcur = h8{p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y};
    wc = wn;
  }
  {
    const uint32_t so = (uint32_t)(((nk - 1) % NSTAGE) * STAGE);
    IWQ_SLICE(la[1] + so, wc[1], true)
    IWQ_SLICE(la[2] + so, wc[2], true)
    IWQ_SLICE(la[3] + so, wc[3], true)
    IWQ_LGKM(0);
    IWQ_PIN();
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) IWQ_MF(mt);
  }
  // no LDS-DMA may still be landing when the workgroup retires (the CU's next workgroup owns the LDS)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_SLICE
#undef IWQ_MF
#undef IWQ_RD_A

  if constexpr (SPLIT) {
    // tile mt of this wave = tile (mt % 4, wid % 2) of b32e's wave (mt / 4) * 4 + wid / 2
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const int we = (mt >> 2) * 4 + (wid >> 1);
      float* dst = a.ws + ((t * a.nsplit + split) * 8 + we) * 8192 + (((mt & 3) * 2 + (wid & 1)) * 16) * 64 + lane;
#pragma unroll
      for (int r = 0; r < 16; ++r) gp<float>(dst)[r * 64] = acc[mt][r];
    }
    return;
  }
  if constexpr (EPI == 9) {  // DIAGNOSTIC (A/B only, wrong results): no output stores
    float t0 = 0.f;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) t0 += acc[mt][r];
    if (t0 == 12345.678f) gp<_Float16>(a.y)[col] = (_Float16)t0;
    return;
  }
  const float bcol = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
  if constexpr (EPI == 1) {  // the first epilogue (A/B variant 73): per-store 64-bit address + row check
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = GROUPED ? acc[mt][r] : opaque(acc[mt][r] * sfl);
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + bcol);
      }
    }
    return;
  }
  auto out = [&](int mt, int r) {
    const float v = GROUPED ? acc[mt][r] : opaque(acc[mt][r] * sfl);
    return (_Float16)(v + bcol);
  };
  const int64_t ld2 = __builtin_amdgcn_readfirstlane((int)a.ldy) * (int64_t)2;  // row pitch, bytes
  if (EPI != 2 || (a.ldy & 3) || (reinterpret_cast<uintptr_t>(a.y) & 7)) {
    // default: one 2-B store per value from a per-lane row pointer, the row offsets uniform multiples
    // of the pitch (scalar), the row check only on the partial last M tile (measured: the first
    // epilogue's per-store 64-bit address math and exec-mask branches were its cost)
    char* yl = reinterpret_cast<char*>(a.y) + ((int64_t)(m0 + 4 * h) * a.ldy + col) * 2;
    if (m0 + TM <= a.M) {
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          *gp<_Float16>(static_cast<void*>(yl + (int64_t)(mt * 32 + (r & 3) + 8 * (r >> 2)) * ld2)) = out(mt, r);
    } else {
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = mt * 32 + (r & 3) + 8 * (r >> 2);
          if (m0 + rr + 4 * h < a.M) *gp<_Float16>(static_cast<void*>(yl + (int64_t)rr * ld2)) = out(mt, r);
        }
    }
    return;
  }
  // A/B variant 97 (measured 1-2 % SLOWER than the default, profiles/r02_ab_gemm_epilogue.jsonl):
  // each quad of lanes (4 consecutive columns) transposes its 4 x 4 blocks (rows
  // 8 g + 4 h + j, j = 0..3, of tile mt) in registers -- two quad DPP exchanges -- so lane i of the
  // quad holds row 8 g + 4 h + i, 4 consecutive columns: one 8-B store per 4 values instead of four
  // 2-B stores, from a per-lane row pointer with uniform (scalar) row offsets
  const int qi = lane & 3;
  char* yq = reinterpret_cast<char*>(a.y) + ((int64_t)(m0 + 4 * h + qi) * a.ldy + (col - qi)) * 2;
  const bool full = m0 + TM <= a.M;
  typedef uint32_t u32x2s __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint32_t p0 = as_u32(h2{out(mt, 4 * g), out(mt, 4 * g + 1)});      // rows 0, 1 at col qi
      const uint32_t p1 = as_u32(h2{out(mt, 4 * g + 2), out(mt, 4 * g + 3)});  // rows 2, 3
      // stage 1 (lanes qi ^ 2): lanes 0, 1 collect rows 0, 1 of cols qi, qi + 2; lanes 2, 3 rows 2, 3
      const uint32_t snd1 = qi < 2 ? p1 : p0;
      const uint32_t rcv1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)snd1, 0x4E, 0xF, 0xF, false);
      const uint32_t lo = qi < 2 ? p0 : rcv1, hi = qi < 2 ? rcv1 : p1;  // cols qi & 1 / (qi & 1) + 2
      // stage 2 (lanes qi ^ 1, 16-bit halves): even lanes keep the first row of the pair, odd the second
      const uint32_t snd2 = (qi & 1) ? __builtin_amdgcn_perm(hi, lo, 0x05040100u)   // (lo.x, hi.x)
                                     : __builtin_amdgcn_perm(hi, lo, 0x07060302u);  // (lo.y, hi.y)
      const uint32_t rcv2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)snd2, 0xB1, 0xF, 0xF, false);
      u32x2s d;
      if (qi & 1) {  // row qi: c0 = rcv2.x, c1 = lo.y, c2 = rcv2.y, c3 = hi.y
        d.x = __builtin_amdgcn_perm(lo, rcv2, 0x07060100u);
        d.y = __builtin_amdgcn_perm(hi, rcv2, 0x07060302u);
      } else {       // row qi: c0 = lo.x, c1 = rcv2.x, c2 = hi.x, c3 = rcv2.y
        d.x = __builtin_amdgcn_perm(rcv2, lo, 0x05040100u);
        d.y = __builtin_amdgcn_perm(rcv2, hi, 0x07060100u);
      }
      const int rr = mt * 32 + 8 * g;
      if (full || m0 + rr + 4 * h + qi < a.M)
        *gp<u32x2s>(static_cast<void*>(yq + (int64_t)rr * ld2)) = d;
    }
  }
}
#undef IWQ_LGKM
#undef IWQ_PIN

// ---------------------------------------------------------------------------------------------
// k_w4a16_b32s: k_w4a16_b32w on SHORT row tiles for prompt-sized M (16 < M <= 128): TMS = 32 MTW
// rows x 256 columns (MTW = 2 or 4 tiles of 32x32 per wave, 8 waves as 1 x 8), always split along K
// (the short tile alone would leave most CUs idle), partials in the workspace in this kernel's own
// layout [tile][split][wave][mt][reg][lane] for k_splitk_reduce_s.  Same hand-ordered stream,
// staging, swizzles and k order as 74 (fewer MFMAs per K-step: the dequant VALU per MFMA doubles at
// MTW = 4 and quadruples at MTW = 2).
// ---------------------------------------------------------------------------------------------
template <int MTW, bool GROUPED>
__global__ __launch_bounds__(THR) void k_w4a16_b32s(PrefillArgs a) {
  static_assert(MTW == 2 || MTW == 4, "64- or 128-row tiles");
  constexpr int TMS = 32 * MTW;
  constexpr int XSS = TMS * TK * 2;              // X bytes per stage
  constexpr int NXP = MTW / 2;                   // X DMA pieces per wave (8 rows x 128 B each)
  constexpr int STAGE = XSS + CS + (GROUPED ? PS : 0);
  constexpr int NPC = NXP + 1 + (GROUPED ? 1 : 0);  // DMA pieces per wave per stage
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  const int64_t tiles = (int64_t)gridDim.x / a.nsplit;
  const int64_t b = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int split = (int)(b / tiles);
  const int64_t t = b - (int64_t)split * tiles;
  const int kbase = split * a.kps;
  const int nk = min(a.kps, a.K / TK - kbase);  // >= 1 by construction
  const int m0 = (int)(t / tiles_n) * TMS, n0 = (int)(t % tiles_n) * TN;
  const int64_t crow = a.K / 2;

  const _Float16* xsrc[NXP];
#pragma unroll
  for (int i = 0; i < NXP; ++i) {
    const int row = (wid * NXP + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + kbase * TK + (((lane & 7) ^ xswz(row)) << 3);
  }
  const int ccol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + ccol) * crow + kbase * (TK / 2) + (((lane & 1) ^ cswz(ccol)) << 4);
  const _Float16* psrc = nullptr;
  if constexpr (GROUPED) {
    const _Float16* arr = (wid < 4 || !a.zeros) ? a.scales : a.zeros;
    psrc = arr + (int64_t)(n0 + (wid & 3) * 64 + lane) * a.gpr;
  }
  // DMA piece i of K-step kt into stage stg: i < NXP X rows, NXP codes, NXP + 1 parameters
  auto issue1 = [&](int kt, int stg, int i) {
    uint8_t* base = smem + stg * STAGE;
    if (i < NXP) glds16(xsrc[i] + kt * TK, base + (wid * NXP + i) * 1024);
    else if (i == NXP) glds16(csrc + kt * (TK / 2), base + XSS + wid * 1024);
    else if constexpr (GROUPED) glds2(psrc + ((kbase + kt) * TK) / a.group, base + XSS + CS + wid * 256);
  };
  auto issue = [&](int kt, int stg) {
#pragma unroll
    for (int i = 0; i < NPC; ++i) issue1(kt, stg, i);
  };

  h2 s2{}, zz{};
  auto set_params = [&](_Float16 sc, float zf) {
    s2 = h2{sc, sc};
    zz = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
  };
  const int col = n0 + wid * 32 + r32;
  if constexpr (!GROUPED)
    set_params(gp<_Float16>(a.scales)[col], a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym);
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  uint32_t magic_v;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));

  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[4];
#pragma unroll
  for (int s2i = 0; s2i < 4; ++s2i) la[s2i] = lbase + (uint32_t)(r32 * 128 + (((4 * h + s2i) ^ xswz(r32)) << 4));
  const int ccl = wid * 32 + r32;
  const uint32_t lc = lbase + XSS + (uint32_t)(ccl * 32 + ((h ^ cswz(ccl)) << 4));
  const uint32_t lp = lbase + XSS + CS + (uint32_t)(ccl * 4);
  uint32_t psv = 0, pzv = 0;
  auto params_landed = [&]() {
    if constexpr (GROUPED) {
      landed(psv);
      landed(pzv);
      set_params(__builtin_bit_cast(_Float16, (uint16_t)psv),
                 a.zeros ? (float)__builtin_bit_cast(_Float16, (uint16_t)pzv) : a.zsym);
    }
  };
  auto dqp = [&](uint32_t w, int j) -> h2 {
    const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
    h2 d = as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz;
    if constexpr (GROUPED) d = d * s2;
    return d;
  };

  f16x acc[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
  h8 af[MTW];
  h8 bcur;
  u32x4 wc;
  h2 p[4];

#define IWQ_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define IWQ_PIN() __builtin_amdgcn_sched_barrier(0)
#define IWQ_MF(MT) acc[MT] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[MT], bcur, acc[MT], 0, 0, 0)
#define IWQ_BSET() bcur = h8{p[0].x, p[0].y, p[1].x, p[1].y, p[2].x, p[2].y, p[3].x, p[3].y};
  // one slice: MFMA mt (its fragment landed: MTW - 1 newer reads outstanding), then the rolling read
  // of fragment mt of the next slice at NADDR; the next slice's 4 dequant pairs (dword W) spread
#define IWQ_SLICE(NADDR, W)                                                                        \
  {                                                                                                \
    const uint32_t wq = (W);                                                                       \
    _Pragma("unroll") for (int mt = 0; mt < MTW; ++mt) {                                           \
      if constexpr (MTW == 4) IWQ_LGKM(3); else IWQ_LGKM(1);                                       \
      IWQ_PIN();                                                                                   \
      IWQ_MF(mt);                                                                                  \
      af[mt] = lds_rd<0>((NADDR) + 4096u * (uint32_t)mt);                                          \
      _Pragma("unroll") for (int j = 0; j < 4 / MTW; ++j) p[mt * (4 / MTW) + j] = dqp(wq, mt * (4 / MTW) + j); \
      IWQ_PIN();                                                                                   \
    }                                                                                              \
    IWQ_BSET()                                                                                     \
  }

  issue(0, 0);
  issue(nk > 1 ? 1 : 0, 1);
  if constexpr (NPC == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (NPC == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  issue(nk > 2 ? 2 : nk - 1, 2);
  IWQ_PIN();
  wc = lds_rd_u<0>(lc);
  if constexpr (GROUPED) {
    psv = lds_rd_d<0>(lp);
    pzv = lds_rd_d<TN * 4>(lp);
  }
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) af[mt] = lds_rd<0>(la[0] + 4096u * (uint32_t)mt);
  IWQ_LGKM(0);
  landed(wc);
  params_landed();
  IWQ_PIN();
#pragma unroll
  for (int j = 0; j < 4; ++j) p[j] = dqp(wc[0], j);
  IWQ_BSET()
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt % NSTAGE) * STAGE);
    IWQ_SLICE(la[1] + so, wc[1])
    IWQ_SLICE(la[2] + so, wc[2])
    IWQ_SLICE(la[3] + so, wc[3])
    if constexpr (NPC == 2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
    else if constexpr (NPC == 3) asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    IWQ_PIN();
    const int kd = kt + 3 < nk ? kt + 3 : nk - 1;
    const int sd = kt % NSTAGE;
    const uint32_t sn = (uint32_t)(((kt + 1) % NSTAGE) * STAGE);
    u32x4 wn = lds_rd_u<0>(lc + sn);
    if constexpr (GROUPED) {
      psv = lds_rd_d<0>(lp + sn);
      pzv = lds_rd_d<TN * 4>(lp + sn);
    }
    // slice 3: rolling reads of the next stage's slice 0, the refill DMA spread over the steps, the
    // next slice's dequant once the code / parameter reads (older than the W A reads) have landed
    constexpr int W = MTW / 2;
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      if (mt == W) {
        if constexpr (W == 2) IWQ_LGKM(2); else IWQ_LGKM(1);
        landed(wn);
        params_landed();
      }
      IWQ_PIN();
      IWQ_MF(mt);
      af[mt] = lds_rd<0>(la[0] + sn + 4096u * (uint32_t)mt);
#pragma unroll
      for (int i = 0; i < NPC; ++i)
        if (i % MTW == mt) issue1(kd, sd, i);
      if (mt >= W) {
#pragma unroll
        for (int j = 0; j < 4 / (MTW - W); ++j) p[(mt - W) * (4 / (MTW - W)) + j] = dqp(wn[0], (mt - W) * (4 / (MTW - W)) + j);
      }
      IWQ_PIN();
    }
    IWQ_BSET()
    wc = wn;
  }
  {
    const uint32_t so = (uint32_t)(((nk - 1) % NSTAGE) * STAGE);
    IWQ_SLICE(la[1] + so, wc[1])
    IWQ_SLICE(la[2] + so, wc[2])
    IWQ_SLICE(la[3] + so, wc[3])
    IWQ_LGKM(0);
    IWQ_PIN();
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) IWQ_MF(mt);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_SLICE
#undef IWQ_BSET
#undef IWQ_MF
#undef IWQ_LGKM
#undef IWQ_PIN
  float* dst = a.ws + ((t * a.nsplit + split) * 8 + wid) * (MTW * 1024) + lane;
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) gp<float>(dst)[(mt * 16 + r) * 64] = acc[mt][r];
}

// sum of k_w4a16_b32s's split partials in range order + epilogue (FACTOR: per-channel scale)
template <bool FACTOR, int MTW>
__global__ __launch_bounds__(256) void k_splitk_reduce_s(PrefillArgs a) {
  constexpr int TE = MTW * 8192;  // partial-tile elements
  const int tiles_n = a.N / TN;
  const int64_t t = blockIdx.x;
  const int m0 = (int)(t / tiles_n) * (32 * MTW), n0 = (int)(t % tiles_n) * TN;
  const int e = (blockIdx.y * 256 + threadIdx.x) * 4;
  const int wave = e / (MTW * 1024), rem = e % (MTW * 1024);
  const int mt = rem >> 10, reg = (rem >> 6) & 15, lane0 = rem & 63;
  const int row = m0 + mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane0 >> 5);
  const int col = n0 + wave * 32 + (lane0 & 31);
  if (row >= a.M) return;
  const IWQ_GLOBAL f4* src = gp<f4>(a.ws + (t * a.nsplit) * TE + e);
  f4 sum = src[0];
  for (int sp = 1; sp < a.nsplit; ++sp) sum += src[(int64_t)sp * (TE / 4)];
  _Float16 o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float bb = a.bias ? (float)gp<_Float16>(a.bias)[col + j] : 0.0f;
    const float v = FACTOR ? opaque(sum[j] * (float)gp<_Float16>(a.scales)[col + j]) : sum[j];
    o[j] = (_Float16)(v + bb);
  }
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  *reinterpret_cast<IWQ_GLOBAL u32x2v*>(gp<_Float16>(a.y) + (int64_t)row * a.ldy + col) =
      u32x2v{as_u32(h2{o[0], o[1]}), as_u32(h2{o[2], o[3]})};
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_b32v: k_w4a16_b32w's hand-ordered stream on 8 waves as 2 (M) x 4 (N), 128 rows x 64
// columns per wave (4 x 2 tiles): half the LDS A reads of the 1 x 8 form (17 instead of 33
// ds_read_b128 per wave per K-step, each A fragment feeding 2 MFMAs) for twice the dequant VALU
// (each weight dequantized by 2 waves).  Same staging (LDS-DMA, 3 stages, early barrier), k order
// and accumulation order as 74: bit-identical.
// ---------------------------------------------------------------------------------------------
template <bool NIB>
__global__ __launch_bounds__(THR) void k_w4a16_b32v(PrefillArgs a) {
  constexpr int STAGE = XS + CS;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int nk = a.K / TK;
  const int64_t crow = a.K / 2;

  // staging exactly as k_w4a16_b32w (X rows / code columns per wave, lane-linear LDS destinations)
  const _Float16* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xswz(row)) << 3);
  }
  const int scol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + scol) * crow + (((lane & 1) ^ cswz(scol)) << 4);
  auto issue = [&](int kt, int stg) {
    uint8_t* base = smem + stg * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
  };
  auto issue1 = [&](int kt, int stg, int i) {
    uint8_t* base = smem + stg * STAGE;
    if (i < 4) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    else glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
  };

  // this lane's 2 MFMA columns and their per-channel parameters
  h2 zz[2], zl[2], zh[2];
  float sfl[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int col = n0 + wn * 64 + nt * 32 + r32;
    const _Float16 sc = gp<_Float16>(a.scales)[col];
    const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
    sfl[nt] = (float)sc;
    zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[4];
  const int arow = wm * 128 + r32;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) la[s2] = lbase + (uint32_t)(arow * 128 + (((4 * h + s2) ^ xswz(arow)) << 4));
  const int ccl = wn * 64 + r32;
  const uint32_t lc = lbase + XS + (uint32_t)(ccl * 32 + ((h ^ cswz(ccl)) << 4));  // + 1024 nt

  auto dqp = [&](uint32_t w, int j, int nt) -> h2 {
    if constexpr (NIB) {
      const uint32_t t8 = w >> 8;
      if (j == 0) return as_h2(and_or(w, m0_s, mg64)) - zl[nt];
      if (j == 1) return as_h2(and_or(w, m1_s, mg54)) - zh[nt];
      if (j == 2) return as_h2(and_or(t8, m0_s, mg64)) - zl[nt];
      return as_h2(and_or(t8, m1_s, mg54)) - zh[nt];
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      return as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz[nt];
    }
  };

  f16x acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  h8 af[4], bcur[2];
  u32x4 wc[2];
  h2 pn[2][4];

#define IWQ_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define IWQ_PIN() __builtin_amdgcn_sched_barrier(0)
#define IWQ_MF(I) \
  acc[(I) >> 1][(I) & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[(I) >> 1], bcur[(I) & 1], acc[(I) >> 1][(I) & 1], 0, 0, 0)
#define IWQ_BSET()                                                                                 \
  _Pragma("unroll") for (int nt = 0; nt < 2; ++nt)                                                  \
    bcur[nt] = h8{pn[nt][0].x, pn[nt][0].y, pn[nt][1].x, pn[nt][1].y, pn[nt][2].x, pn[nt][2].y,     \
                  pn[nt][3].x, pn[nt][3].y};
  // one slice: step i = MFMA (mt = i / 2, nt = i % 2); before each even step the A fragment mt has
  // landed (3 newer reads outstanding); after each odd step the rolling read of fragment mt of the
  // next slice (address NADDR); pair i of the next slice's dequant (code dwords wc[.][S1])
#define IWQ_SLICE(NADDR, S1)                                                                       \
  {                                                                                                \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                               \
      if ((i & 1) == 0) IWQ_LGKM(3);                                                               \
      IWQ_PIN();                                                                                   \
      IWQ_MF(i);                                                                                   \
      if (i & 1) af[i >> 1] = lds_rd<0>((NADDR) + 4096u * (uint32_t)(i >> 1));                     \
      pn[i >> 2][i & 3] = dqp(wc[i >> 2][S1], i & 3, i >> 2);                                      \
      IWQ_PIN();                                                                                   \
    }                                                                                              \
    IWQ_BSET()                                                                                     \
  }

  // prologue: stages 0, 1, 2 (K-steps clamped to nk - 1)
  issue(0, 0);
  issue(nk > 1 ? 1 : 0, 1);
  asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  issue(nk > 2 ? 2 : nk - 1, 2);
  IWQ_PIN();
  wc[0] = lds_rd_u<0>(lc);
  wc[1] = lds_rd_u<1024>(lc);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) af[mt] = lds_rd<0>(la[0] + 4096u * (uint32_t)mt);
  IWQ_LGKM(0);
  landed(wc[0]);
  landed(wc[1]);
  IWQ_PIN();
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) pn[nt][j] = dqp(wc[nt][0], j, nt);
  IWQ_BSET()
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt % NSTAGE) * STAGE);
    IWQ_SLICE(la[1] + so, 1)
    IWQ_SLICE(la[2] + so, 2)
    IWQ_SLICE(la[3] + so, 3)
    asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    IWQ_PIN();
    const int kd = kt + 3 < nk ? kt + 3 : nk - 1;
    const int sd = kt % NSTAGE;
    const uint32_t sn = (uint32_t)(((kt + 1) % NSTAGE) * STAGE);
    u32x4 wq[2];
    wq[0] = lds_rd_u<0>(lc + sn);
    wq[1] = lds_rd_u<1024>(lc + sn);
    const uint32_t na = la[0] + sn;
    // slice 3 of this stage: rolling reads of the next stage's slice 0 (after the 2 code reads),
    // the refill DMA one piece per step, the next slice's dequant once the codes have landed
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i == 2) {  // code reads older than the one A read issued since
        IWQ_LGKM(1);
        landed(wq[0]);
        landed(wq[1]);
      }
      IWQ_PIN();
      IWQ_MF(i);
      if (i & 1) af[i >> 1] = lds_rd<0>(na + 4096u * (uint32_t)(i >> 1));
      if (i < 5) issue1(kd, sd, i);
      if (i == 2 || i == 3) {
        const int q = (i - 2) * 2;
        pn[0][q] = dqp(wq[0][0], q, 0);
        pn[0][q + 1] = dqp(wq[0][0], q + 1, 0);
      } else if (i >= 4) {
        pn[1][i - 4] = dqp(wq[1][0], i - 4, 1);
      }
      IWQ_PIN();
    }
    IWQ_BSET()
    wc[0] = wq[0];
    wc[1] = wq[1];
  }
  {
    const uint32_t so = (uint32_t)(((nk - 1) % NSTAGE) * STAGE);
    IWQ_SLICE(la[1] + so, 1)
    IWQ_SLICE(la[2] + so, 2)
    IWQ_SLICE(la[3] + so, 3)
    IWQ_LGKM(0);
    IWQ_PIN();
#pragma unroll
    for (int i = 0; i < 8; ++i) IWQ_MF(i);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_SLICE
#undef IWQ_BSET
#undef IWQ_MF
#undef IWQ_LGKM
#undef IWQ_PIN

#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int col = n0 + wn * 64 + nt * 32 + r32;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = opaque(acc[mt][nt][r] * sfl[nt]);
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + b);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_h2v (round 3, variants 98 / 99): b32v's per-wave work (128 rows x 64 columns, 4 x 2 tiles of
// 32x32x16, the same hand-ordered slice stream, k order and accumulation order: bit-identical to 74)
// on a HALF-width workgroup: 4 waves as 2 (M) x 2 (N), 256 x 128 output tile, a 2-stage LDS-DMA ring
// of 36 KiB stages.  72 KiB of LDS and <= 256 registers per lane admit TWO workgroups per CU, so the
// CU's 8 waves form two independent barrier domains: while one workgroup's waves wait at their
// per-K-step barrier (or for a DMA), the other's keep the MFMA pipe busy (in 74 / b32v all 8 waves of
// the CU share one barrier).  The ring's refill of the K-step after next is issued right after each
// barrier and has a whole K-step to land (vmcnt(0) at the next barrier).  Per channel (scale in the
// epilogue), as 74.
// ---------------------------------------------------------------------------------------------
constexpr int H2_TN = 128, H2_THR = 256, H2_NSTAGE = 2;
constexpr int H2_CS = H2_TN * TK / 2;       // 4 KiB of codes per stage
constexpr int H2_STAGE = XS + H2_CS;        // 36 KiB

template <bool NIB>
__global__ __launch_bounds__(H2_THR, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_w4a16_h2v(PrefillArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[H2_NSTAGE * H2_STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / H2_TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * H2_TN;
  const int nk = a.K / TK;
  const int64_t crow = a.K / 2;

  // staging: 8 X pieces (8 rows of 128 B each) and 1 code piece (32 columns x 32 B) per wave per stage
  const _Float16* xsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = (wid * 8 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xswz(row)) << 3);
  }
  const int scol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + scol) * crow + (((lane & 1) ^ cswz(scol)) << 4);
  auto issue1 = [&](int kt, int stg, int i) {
    uint8_t* base = smem + stg * H2_STAGE;
    if (i < 8) glds16(xsrc[i] + kt * TK, base + (wid * 8 + i) * 1024);
    else glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
  };
  auto issue = [&](int kt, int stg) {
#pragma unroll
    for (int i = 0; i < 9; ++i) issue1(kt, stg, i);
  };

  h2 zz[2], zl[2], zh[2];
  float sfl[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int col = n0 + wn * 64 + nt * 32 + r32;
    const _Float16 sc = gp<_Float16>(a.scales)[col];
    const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
    sfl[nt] = (float)sc;
    zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[4];
  const int arow = wm * 128 + r32;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) la[s2] = lbase + (uint32_t)(arow * 128 + (((4 * h + s2) ^ xswz(arow)) << 4));
  const int ccl = wn * 64 + r32;
  const uint32_t lc = lbase + XS + (uint32_t)(ccl * 32 + ((h ^ cswz(ccl)) << 4));  // + 1024 nt

  auto dqp = [&](uint32_t w, int j, int nt) -> h2 {
    if constexpr (NIB) {
      const uint32_t t8 = w >> 8;
      if (j == 0) return as_h2(and_or(w, m0_s, mg64)) - zl[nt];
      if (j == 1) return as_h2(and_or(w, m1_s, mg54)) - zh[nt];
      if (j == 2) return as_h2(and_or(t8, m0_s, mg64)) - zl[nt];
      return as_h2(and_or(t8, m1_s, mg54)) - zh[nt];
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      return as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz[nt];
    }
  };

  f16x acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  h8 af[4], bcur[2];
  u32x4 wc[2];
  h2 pn[2][4];

#define IWQ_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define IWQ_PIN() __builtin_amdgcn_sched_barrier(0)
#define IWQ_MF(I) \
  acc[(I) >> 1][(I) & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[(I) >> 1], bcur[(I) & 1], acc[(I) >> 1][(I) & 1], 0, 0, 0)
#define IWQ_BSET()                                                                                 \
  _Pragma("unroll") for (int nt = 0; nt < 2; ++nt)                                                  \
    bcur[nt] = h8{pn[nt][0].x, pn[nt][0].y, pn[nt][1].x, pn[nt][1].y, pn[nt][2].x, pn[nt][2].y,     \
                  pn[nt][3].x, pn[nt][3].y};
#define IWQ_SLICE(NADDR, S1)                                                                       \
  {                                                                                                \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                               \
      if ((i & 1) == 0) IWQ_LGKM(3);                                                               \
      IWQ_PIN();                                                                                   \
      IWQ_MF(i);                                                                                   \
      if (i & 1) af[i >> 1] = lds_rd<0>((NADDR) + 4096u * (uint32_t)(i >> 1));                     \
      pn[i >> 2][i & 3] = dqp(wc[i >> 2][S1], i & 3, i >> 2);                                      \
      IWQ_PIN();                                                                                   \
    }                                                                                              \
    IWQ_BSET()                                                                                     \
  }

  // prologue: stages 0 and 1 (K-step clamped to nk - 1: a re-load nobody reads)
  issue(0, 0);
  issue(nk > 1 ? 1 : 0, 1);
  asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  IWQ_PIN();
  wc[0] = lds_rd_u<0>(lc);
  wc[1] = lds_rd_u<1024>(lc);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) af[mt] = lds_rd<0>(la[0] + 4096u * (uint32_t)mt);
  IWQ_LGKM(0);
  landed(wc[0]);
  landed(wc[1]);
  IWQ_PIN();
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) pn[nt][j] = dqp(wc[nt][0], j, nt);
  IWQ_BSET()
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt & 1) * H2_STAGE);
    IWQ_SLICE(la[1] + so, 1)
    IWQ_SLICE(la[2] + so, 2)
    IWQ_SLICE(la[3] + so, 3)
    // stage kt+1 landed (nothing else in flight: 2-stage ring), every read of stage kt retired
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    IWQ_PIN();
    const int kd = kt + 2 < nk ? kt + 2 : nk - 1;
    const int sd = kt & 1;
    const uint32_t sn = (uint32_t)(((kt + 1) & 1) * H2_STAGE);
    u32x4 wq[2];
    wq[0] = lds_rd_u<0>(lc + sn);
    wq[1] = lds_rd_u<1024>(lc + sn);
    const uint32_t na = la[0] + sn;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i == 2) {  // the code reads are older than the one A read issued since
        IWQ_LGKM(1);
        landed(wq[0]);
        landed(wq[1]);
      }
      IWQ_PIN();
      IWQ_MF(i);
      if (i & 1) af[i >> 1] = lds_rd<0>(na + 4096u * (uint32_t)(i >> 1));
      issue1(kd, sd, i);
      if (i == 7) issue1(kd, sd, 8);
      if (i == 2 || i == 3) {
        const int q = (i - 2) * 2;
        pn[0][q] = dqp(wq[0][0], q, 0);
        pn[0][q + 1] = dqp(wq[0][0], q + 1, 0);
      } else if (i >= 4) {
        pn[1][i - 4] = dqp(wq[1][0], i - 4, 1);
      }
      IWQ_PIN();
    }
    IWQ_BSET()
    wc[0] = wq[0];
    wc[1] = wq[1];
  }
  {
    const uint32_t so = (uint32_t)(((nk - 1) & 1) * H2_STAGE);
    IWQ_SLICE(la[1] + so, 1)
    IWQ_SLICE(la[2] + so, 2)
    IWQ_SLICE(la[3] + so, 3)
    IWQ_LGKM(0);
    IWQ_PIN();
#pragma unroll
    for (int i = 0; i < 8; ++i) IWQ_MF(i);
  }
  // no LDS-DMA may still be landing when the workgroup retires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_SLICE
#undef IWQ_BSET
#undef IWQ_MF
#undef IWQ_LGKM
#undef IWQ_PIN

  // epilogue (74's form): per-lane row pointer, row offsets uniform multiples of the pitch
  const int64_t ld2 = __builtin_amdgcn_readfirstlane((int)a.ldy) * (int64_t)2;
  const bool full = m0 + TM <= a.M;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int col = n0 + wn * 64 + nt * 32 + r32;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
    char* yl = reinterpret_cast<char*>(a.y) + ((int64_t)(m0 + wm * 128 + 4 * h) * a.ldy + col) * 2;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = mt * 32 + (r & 3) + 8 * (r >> 2);
        const _Float16 v = (_Float16)(opaque(acc[mt][nt][r] * sfl[nt]) + b);
        if (full || m0 + wm * 128 + rr + 4 * h < a.M) *gp<_Float16>(static_cast<void*>(yl + (int64_t)rr * ld2)) = v;
      }
    }
  }
}

template <bool NIB>
hipError_t launch_h2v(const PrefillArgs& a, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / H2_TN);
  hipLaunchKernelGGL((k_w4a16_h2v<NIB>), dim3((unsigned)blocks), dim3(H2_THR), 0, st, a);
  return hipGetLastError();
}

template <bool NIB>
hipError_t launch_v(const PrefillArgs& a, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_b32v<NIB>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
  return hipGetLastError();
}

template <bool NIB, bool GROUPED = false, bool PG = false>
hipError_t launch_w(const PrefillArgs& a, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_b32w<NIB, GROUPED, false, 0, PG>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
  return hipGetLastError();
}



// ---------------------------------------------------------------------------------------------
// k_w4a16_w4h: the 256 x 256 tile on FOUR waves (one per SIMD, 128 x 128 each: 4 x 4 tiles of
// 32x32x16, 256 fp32 accumulators per lane in AGPRs), with k_w4a16_b32w's hand-ordered stream.
// Against the 8-wave forms the LDS read traffic per K-step drops 3x (each A fragment feeds 4 MFMAs,
// each dequantized B fragment 4: 80 KiB per K-step per CU instead of 264) and no second wave shares
// a SIMD's issue port; the price is that nothing else covers this wave's stalls, so:
//  * X and codes are staged through REGISTERS (global_load_dwordx4 -> ds_write_b128: an LDS-DMA
//    instruction holds its issuing wave ~60-185 cycles, 10 per K-step would idle the MFMA pipe),
//    issued one K-step ahead of their LDS write, into a 2-stage ring (80 KiB);
//  * every LDS access is inline asm with hand-counted waits and every group is pinned by
//    sched_barrier; each MFMA gap holds at most one LDS read, one staged write + load and a
//    dequant pair;
//  * one barrier per K-step, before its last slice (its 16 MFMAs cover the next stage's first
//    reads).  The stage written in K-step kt is the one read in kt - 1, whose reads all retired
//    before that K-step's barrier.
// Same LDS images, k order and accumulation order as k_w4a16_b32w: bit-identical to 45 / 74
// (NIB: to 66 / 75 on NIB codes).  Per channel (scale in the epilogue) only.
// Measured (profiles/r02_ab_gemm_w4h.jsonl): 1-4 % behind 74 (76; NIB 77 at
// par); the loop with the staging removed runs 10-14 % faster than 76 (78 of the A/B log), with the
// staging reading one cache-resident K-step over and over 3-4 % -- so the staging's cost is mostly
// its issue and LDS-write traffic, not memory latency; DMA staging (79) is no better.  Kept for A/B.
// ---------------------------------------------------------------------------------------------
template <int OFF>
__device__ __forceinline__ void lds_wr(uint32_t addr, u32x4 v) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "n"(OFF) : "memory");
}

// WMW: waves along M -- 2: 2 x 2 waves of 128 x 128 (4 x 4 tiles); 1: 1 x 4 waves of 256 x 64
// (8 x 2 tiles: every weight dequantized once per workgroup, twice the A reads)
template <bool NIB, int WMW, bool DMA = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_w4a16_w4h(PrefillArgs a) {
  constexpr int STAGE = XS + CS;  // 40 KiB
  constexpr int NST = DMA ? 3 : 2;
  constexpr int MT = 8 / WMW, NT = 2 * WMW;  // 32 x 32 tiles per wave
  constexpr int P = 4 * NT;                  // dequant pairs per slice
  constexpr int PSTEP = 16 / P;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NST * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = WMW == 2 ? wid >> 1 : 0, wn = WMW == 2 ? wid & 1 : wid;
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int nk = a.K / TK;

  // staging sources as 32-bit byte offsets from uniform bases (the launcher checks the ranges):
  // X slot i of wave w = rows 64 w + 8 i + lane / 8; codes slots 2 w + i = columns 64 w + 32 i + lane / 2
  uint32_t xoff[8], coff[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wid * 64 + i * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xoff[i] = (uint32_t)(((int64_t)gm * a.lda + (((lane & 7) ^ xswz(row)) << 3)) * 2);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ccol = (2 * wid + i) * 32 + (lane >> 1);
    coff[i] = (uint32_t)((int64_t)(n0 + ccol) * (a.K / 2) + (((lane & 1) ^ cswz(ccol)) << 4));
  }
  const char* xg = reinterpret_cast<const char*>(a.x);
  const char* cg = reinterpret_cast<const char*>(a.codes);
  u32x4 g[10];
  auto gload = [&](int kt, int j) {
    if (j < 8) g[j] = *gp<u32x4>(xg + (int64_t)kt * (TK * 2) + xoff[j]);
    else g[j] = *gp<u32x4>(cg + (int64_t)kt * (TK / 2) + coff[j - 8]);
  };
  // DMA staging: piece j of K-step kt straight into stage stg (lane-linear destination)
  auto dma1 = [&](int kt, int stg, int j) {
    uint8_t* base = smem + stg * STAGE;
    if (j < 8) glds16(xg + (int64_t)kt * (TK * 2) + xoff[j], base + wid * 8192 + j * 1024);
    else glds16(cg + (int64_t)kt * (TK / 2) + coff[j - 8], base + XS + wid * 2048 + (j - 8) * 1024);
  };
  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  const uint32_t wx = lbase + (uint32_t)(wid * 8192 + lane * 16);            // + 1024 i
  const uint32_t wcd = lbase + XS + (uint32_t)(wid * 2048 + lane * 16);      // + 1024 i
#define IWQ_GWRITE(J, SO)                                              \
  do {                                                                 \
    if ((J) < 8) lds_wr<((J) < 8 ? (J) : 0) * 1024>(wx + (SO), g[J]);  \
    else lds_wr<((J) >= 8 ? (J) - 8 : 0) * 1024>(wcd + (SO), g[J]);    \
  } while (0)

  // per-channel parameters of this lane's NT columns
  h2 zz[NT], zl[NT], zh[NT];
  float sfl[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = n0 + wn * (NT * 32) + nt * 32 + r32;
    const _Float16 sc = gp<_Float16>(a.scales)[col];
    const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
    sfl[nt] = (float)sc;
    zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  // LDS read addresses: A fragment (slice s, tile mt) = la[s] + stage + 4096 mt; codes of tile nt
  // = lc + stage + 1024 nt
  uint32_t la[4];
  const int arow = wm * (MT * 32) + r32;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) la[s2] = lbase + (uint32_t)(arow * 128 + (((4 * h + s2) ^ xswz(arow)) << 4));
  const int ccl = wn * (NT * 32) + r32;
  const uint32_t lc = lbase + XS + (uint32_t)(ccl * 32 + ((h ^ cswz(ccl)) << 4));

  auto dqp = [&](uint32_t w, uint32_t t8, int j, int nt) -> h2 {
    if constexpr (NIB) {
      if (j == 0) return as_h2(and_or(w, m0_s, mg64)) - zl[nt];
      if (j == 1) return as_h2(and_or(w, m1_s, mg54)) - zh[nt];
      if (j == 2) return as_h2(and_or(t8, m0_s, mg64)) - zl[nt];
      return as_h2(and_or(t8, m1_s, mg54)) - zh[nt];
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      return as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz[nt];
    }
  };

  f16x acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  h8 A0[MT], A1[MT];
  h2 B0[NT][4], B1[NT][4];  // [nt][pair]
  u32x4 wc[NT], wq[NT];

#define IWQ_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define IWQ_PIN() __builtin_amdgcn_sched_barrier(0)
#define IWQ_BV(B, NT) (h8{B[NT][0].x, B[NT][0].y, B[NT][1].x, B[NT][1].y, B[NT][2].x, B[NT][2].y, B[NT][3].x, B[NT][3].y})
#define IWQ_MF(AC, BC, I) \
  acc[(I) / NT][(I) % NT] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AC[(I) / NT], IWQ_BV(BC, (I) % NT), acc[(I) / NT][(I) % NT], 0, 0, 0)
  // dequant pair (nt, j) of slice S2 from code dwords W[nt][S2] into BN; NIB keeps w >> 8 per nt
#define IWQ_DQ(BN, W, S2, NT, J)                                                   \
  {                                                                               \
    const uint32_t wv = W[NT][S2];                                                \
    BN[NT][J] = dqp(wv, NIB ? (wv >> 8) : 0u, J, NT);                             \
  }
  // one slice: 16 MFMAs on (AC, BC); step i also: i < MT the read of A fragment i of the next
  // slice (address NA) into AN; every PSTEP-th step one of the P dequant pairs of the next slice
  // (code dwords W, slice S2) into BN; STG: staged write + refill j = STG0 + (i - 5) / 2 for odd i
  // in [5, 15)
#define IWQ_SLICE(AC, BC, AN, BN, NA, W, S2, STG, STG0, SO, KD)                     \
  _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                \
    IWQ_PIN();                                                                    \
    IWQ_MF(AC, BC, i);                                                            \
    if (i < MT) AN[i % MT] = lds_rd<0>((NA) + 4096u * (uint32_t)(i % MT));         \
    if (i % PSTEP == 0) IWQ_DQ(BN, W, S2, ((i / PSTEP) >> 2), ((i / PSTEP) & 3));  \
    if (STG && i >= 5 && i < 15 && ((i - 5) & 1) == 0) {                          \
      const int jj = (STG0) + ((i - 5) >> 1);                                     \
      if constexpr (DMA) {                                                        \
        dma1(KD, (int)(SO), jj);                                                  \
      } else {                                                                    \
        IWQ_GWRITE_RT(jj, SO);                                                    \
        gload(KD, jj);                                                            \
      }                                                                           \
    }                                                                             \
    IWQ_PIN();                                                                    \
  }                                                                               \
  if (!DMA && STG) {                                                                              \
    if constexpr (MT == 8) IWQ_LGKM(4); /* writes at steps 7..13 follow the last read */          \
    else IWQ_LGKM(5);                   /* all 5 writes follow the reads */                       \
  } else {                                                                                        \
    IWQ_LGKM(0);                                                                                  \
  }

  // runtime-j staged write (j is a compile-time constant after unrolling)
#define IWQ_GWRITE_RT(J, SO)                  \
  switch (J) {                                \
    case 0: IWQ_GWRITE(0, SO); break;         \
    case 1: IWQ_GWRITE(1, SO); break;         \
    case 2: IWQ_GWRITE(2, SO); break;         \
    case 3: IWQ_GWRITE(3, SO); break;         \
    case 4: IWQ_GWRITE(4, SO); break;         \
    case 5: IWQ_GWRITE(5, SO); break;         \
    case 6: IWQ_GWRITE(6, SO); break;         \
    case 7: IWQ_GWRITE(7, SO); break;         \
    case 8: IWQ_GWRITE(8, SO); break;         \
    default: IWQ_GWRITE(9, SO); break;        \
  }

  // prologue: K-step 0 -> stage 0 (written), K-step 1 in flight in g (DMA: K-steps 0 and 1 into
  // stages 0 and 1, the first landed)
  if constexpr (DMA) {
#pragma unroll
    for (int j = 0; j < 10; ++j) dma1(0, 0, j);
#pragma unroll
    for (int j = 0; j < 10; ++j) dma1(nk > 1 ? 1 : 0, 1, j);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  } else {
#pragma unroll
    for (int j = 0; j < 10; ++j) gload(0, j);
#pragma unroll
    for (int j = 0; j < 10; ++j) IWQ_GWRITE_RT(j, 0u);
#pragma unroll
    for (int j = 0; j < 10; ++j) gload(nk > 1 ? 1 : 0, j);
  }
  IWQ_LGKM(0);
  __builtin_amdgcn_s_barrier();
  IWQ_PIN();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wc[nt] = lds_rd_u<0>(lc + 1024u * (uint32_t)nt);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) A0[mt] = lds_rd<0>(la[0] + 4096u * (uint32_t)mt);
  IWQ_LGKM(0);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) landed(wc[nt]);
  IWQ_PIN();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) IWQ_DQ(B0, wc, 0, nt, j);

  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt % NST) * STAGE);        // stage of K-step kt
    const uint32_t sn = (uint32_t)(((kt + 1) % NST) * STAGE);  // stage of K-step kt + 1
    const int kd = kt + 2 < nk ? kt + 2 : nk - 1;              // refill source (clamped: re-load)
    // refill target: registers -> stage kt+1 (written this K-step, K-step kt+2 loaded); DMA ->
    // stage kt+2 (the one read in K-step kt-1), landing before the barrier of K-step kt+1
    const uint32_t sw = DMA ? (uint32_t)((kt + 2) % NST) : sn;
    IWQ_SLICE(A0, B0, A1, B1, la[1] + so, wc, 1, true, 0, sw, kd)
    IWQ_SLICE(A1, B1, A0, B0, la[2] + so, wc, 2, true, 5, sw, kd)
    IWQ_SLICE(A0, B0, A1, B1, la[3] + so, wc, 3, false, 0, sw, kd)
    // stage kt+1 written / landed for every wave, every read of stage kt retired (lgkmcnt(0) above)
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    IWQ_PIN();
    // slice 3: codes of K-step kt+1 first, then its slice-0 A fragments; the dequant once the codes
    // have landed (MT younger A reads may still fly: lgkmcnt(MT)), PP pairs per step
    constexpr int S0 = NT + MT;
    constexpr int PP = (P + (16 - S0) - 1) / (16 - S0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      IWQ_PIN();
      IWQ_MF(A1, B1, i);
      if (i < NT) wq[i % NT] = lds_rd_u<0>(lc + sn + 1024u * (uint32_t)(i % NT));
      else if (i < S0) A0[(i - NT) % MT] = lds_rd<0>(la[0] + sn + 4096u * (uint32_t)((i - NT) % MT));
      if (i == S0) {
        if constexpr (MT == 8) IWQ_LGKM(8);
        else IWQ_LGKM(4);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) landed(wq[nt]);
      }
      if (i >= S0) {
#pragma unroll
        for (int u = 0; u < PP; ++u) {
          const int q = (i - S0) * PP + u;
          if (q < P) IWQ_DQ(B0, wq, 0, (q >> 2), (q & 3));
        }
      }
      IWQ_PIN();
    }
    IWQ_LGKM(0);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) wc[nt] = wq[nt];
  }
  {
    const uint32_t so = (uint32_t)(((nk - 1) % NST) * STAGE);
    IWQ_SLICE(A0, B0, A1, B1, la[1] + so, wc, 1, false, 0, so, 0)
    IWQ_SLICE(A1, B1, A0, B0, la[2] + so, wc, 2, false, 0, so, 0)
    IWQ_SLICE(A0, B0, A1, B1, la[3] + so, wc, 3, false, 0, so, 0)
    IWQ_PIN();
#pragma unroll
    for (int i = 0; i < 16; ++i) IWQ_MF(A1, B1, i);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_SLICE
#undef IWQ_DQ
#undef IWQ_MF
#undef IWQ_BV
#undef IWQ_GWRITE_RT
#undef IWQ_GWRITE
#undef IWQ_LGKM
#undef IWQ_PIN

#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = n0 + wn * (NT * 32) + nt * 32 + r32;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (MT * 32) + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = opaque(acc[mt][nt][r] * sfl[nt]);
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + b);
      }
    }
  }
}

// the 32-bit staging offsets of k_w4a16_w4h must cover X and the codes
bool w4h_fits(const PrefillArgs& a) {
  return (int64_t)a.M * a.lda * 2 < ((int64_t)1 << 31) && (int64_t)a.N * (a.K / 2) < ((int64_t)1 << 31);
}

template <bool NIB, int WMW, bool DMA = false>
hipError_t launch_w4h(const PrefillArgs& a, hipStream_t st) {
  if (!w4h_fits(a)) return launch_w<NIB>(a, st);
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_w4h<NIB, WMW, DMA>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_w4b: k_w4a16_w4h with the weight tile dequantized ONCE per workgroup into LDS: each lane
// stages its own column's codes (32 B per K-step) in registers, dequantizes them and writes the
// column's 64 fp16 weights (q - z, natural k order) as one 128-B row of a B image laid out like the
// X image; the MFMA loop then reads A and B fragments alike from LDS (hipBLASLt's structure plus a
// dequant pass).  Per wave and K-step: 96 dequant VALU (72 NIB) instead of 192, 32 fragment reads
// and 16 staged writes instead of 20 + 10.  Same k order / accumulation order as 74: bit-identical.
// ---------------------------------------------------------------------------------------------
template <bool NIB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_w4a16_w4b(PrefillArgs a) {
  constexpr int BS = TN * TK * 2;      // B image bytes per stage (32 KiB)
  constexpr int STAGE = XS + BS;       // 64 KiB
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int r32 = lane & 31, h = lane >> 5;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int nk = a.K / TK;

  uint32_t xoff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wid * 64 + i * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xoff[i] = (uint32_t)(((int64_t)gm * a.lda + (((lane & 7) ^ xswz(row)) << 3)) * 2);
  }
  const int dcol = wid * 64 + lane;  // the column this lane dequantizes
  const uint32_t coff = (uint32_t)((int64_t)(n0 + dcol) * (a.K / 2));
  const char* xg = reinterpret_cast<const char*>(a.x);
  const char* cg = reinterpret_cast<const char*>(a.codes);
  u32x4 gx[8], gc[2];
  auto ldx = [&](int kt, int j) { gx[j] = *gp<u32x4>(xg + (int64_t)kt * (TK * 2) + xoff[j]); };
  auto ldc = [&](int kt, int j) { gc[j] = *gp<u32x4>(cg + (int64_t)kt * (TK / 2) + coff + 16 * j); };
  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  const uint32_t wx = lbase + (uint32_t)(wid * 8192 + lane * 16);  // + 1024 i
  uint32_t bw[8];                                                  // B image chunk j of dcol
#pragma unroll
  for (int j = 0; j < 8; ++j) bw[j] = lbase + XS + (uint32_t)(dcol * 128 + ((j ^ xswz(dcol)) << 4));

  // zero point of the dequantized column; scales of this lane's 4 MFMA columns (epilogue)
  const float zfd = a.zeros ? (float)gp<_Float16>(a.zeros)[n0 + dcol] : a.zsym;
  const h2 zz = h2{(_Float16)(1024.0f + zfd), (_Float16)(64.0f + zfd)};
  const h2 zl = h2{(_Float16)(1024.0f + zfd), (_Float16)(1024.0f + zfd)};
  const h2 zh = h2{(_Float16)(64.0f + zfd), (_Float16)(64.0f + zfd)};
  float sfl[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) sfl[nt] = (float)gp<_Float16>(a.scales)[n0 + wn * 128 + nt * 32 + r32];
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));
  auto dqp = [&](uint32_t w, int j) -> h2 {
    if constexpr (NIB) {
      const uint32_t t8 = w >> 8;
      if (j == 0) return as_h2(and_or(w, m0_s, mg64)) - zl;
      if (j == 1) return as_h2(and_or(w, m1_s, mg54)) - zh;
      if (j == 2) return as_h2(and_or(t8, m0_s, mg64)) - zl;
      return as_h2(and_or(t8, m1_s, mg54)) - zh;
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      return as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz;
    }
  };

  // fragment read addresses: A (slice s, tile mt) = la[s] + stage + 4096 mt, B (slice s, tile nt) =
  // lb[s] + stage + 4096 nt
  uint32_t la[4], lb[4];
  const int arow = wm * 128 + r32, brow = wn * 128 + r32;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    la[s2] = lbase + (uint32_t)(arow * 128 + (((4 * h + s2) ^ xswz(arow)) << 4));
    lb[s2] = lbase + XS + (uint32_t)(brow * 128 + (((4 * h + s2) ^ xswz(brow)) << 4));
  }

  f16x acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  h8 A0[4], A1[4], B0[4], B1[4];
  h2 dq[4];

#define IWQ_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define IWQ_PIN() __builtin_amdgcn_sched_barrier(0)
#define IWQ_MF(AC, BC, I) \
  acc[(I) >> 2][(I) & 3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AC[(I) >> 2], BC[(I) & 3], acc[(I) >> 2][(I) & 3], 0, 0, 0)
#define IWQ_WRB(J, SO)                                                                              \
  {                                                                                                 \
    const h8 v = h8{dq[0].x, dq[0].y, dq[1].x, dq[1].y, dq[2].x, dq[2].y, dq[3].x, dq[3].y};        \
    lds_wr<0>(bw[J] + (SO), __builtin_bit_cast(u32x4, v));                                         \
  }
  // one slice: 16 MFMAs on (AC, BC); steps 0-7 read the next slice's fragments (A i, B i - 4) at
  // NS (slice offset: la/lb index, stage); STG: steps 0-15 dequantize 4 code dwords (one pair per
  // step; dword d = 4 H + step / 4, its B row chunk written after its last pair), even steps >= 8
  // write X piece 4 H + (step - 8) / 2 and refill it; the code piece H is refilled after its dwords
#define IWQ_SLICE(AC, BC, AN, BN, S2N, SOR, STG, H, SOW, KD)                                       \
  _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                                \
    IWQ_PIN();                                                                                    \
    IWQ_MF(AC, BC, i);                                                                            \
    if (i < 4) AN[i] = lds_rd<0>(la[S2N] + (SOR) + 4096u * (uint32_t)i);                           \
    else if (i < 8) BN[i - 4] = lds_rd<0>(lb[S2N] + (SOR) + 4096u * (uint32_t)(i - 4));            \
    if (STG) {                                                                                    \
      dq[i & 3] = dqp(gc[H][i >> 2], i & 3);                                                      \
      if ((i & 3) == 3) IWQ_WRB(4 * (H) + (i >> 2), SOW);                                         \
      if (i >= 8 && (i & 1) == 0) {                                                               \
        const int jx = 4 * (H) + ((i - 8) >> 1);                                                  \
        lds_wr<0>(wx + 1024u * (uint32_t)jx + (SOW), gx[jx]);                                     \
        ldx(KD, jx);                                                                              \
      }                                                                                           \
      if (i == 15) ldc(KD, H);                                                                    \
    }                                                                                             \
    IWQ_PIN();                                                                                    \
  }                                                                                               \
  if (STG) IWQ_LGKM(7); else IWQ_LGKM(0);  /* STG: 7 writes were issued after the last read */

  // prologue: K-step 0 staged into stage 0 (X copied, codes dequantized), K-step 1 in flight
#pragma unroll
  for (int j = 0; j < 8; ++j) ldx(0, j);
  ldc(0, 0);
  ldc(0, 1);
#pragma unroll
  for (int j = 0; j < 8; ++j) lds_wr<0>(wx + 1024u * (uint32_t)j, gx[j]);
#pragma unroll
  for (int d = 0; d < 8; ++d) {
#pragma unroll
    for (int p2 = 0; p2 < 4; ++p2) dq[p2] = dqp(gc[d >> 2][d & 3], p2);
    IWQ_WRB(d, 0u);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) ldx(nk > 1 ? 1 : 0, j);
  ldc(nk > 1 ? 1 : 0, 0);
  ldc(nk > 1 ? 1 : 0, 1);
  IWQ_LGKM(0);
  __builtin_amdgcn_s_barrier();
  IWQ_PIN();
#pragma unroll
  for (int i = 0; i < 4; ++i) A0[i] = lds_rd<0>(la[0] + 4096u * (uint32_t)i);
#pragma unroll
  for (int i = 0; i < 4; ++i) B0[i] = lds_rd<0>(lb[0] + 4096u * (uint32_t)i);
  IWQ_LGKM(0);
  IWQ_PIN();

  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt & 1) * STAGE);
    const uint32_t sn = (uint32_t)(((kt + 1) & 1) * STAGE);
    const int kd = kt + 2 < nk ? kt + 2 : nk - 1;
    IWQ_SLICE(A0, B0, A1, B1, 1, so, true, 0, sn, kd)
    IWQ_SLICE(A1, B1, A0, B0, 2, so, true, 1, sn, kd)
    IWQ_SLICE(A0, B0, A1, B1, 3, so, false, 0, sn, kd)
    // stage kt+1 complete (X and B written by every wave), every read of stage kt retired
    __builtin_amdgcn_s_barrier();
    IWQ_SLICE(A1, B1, A0, B0, 0, sn, false, 0, sn, kd)
  }
  {
    const uint32_t so = (uint32_t)(((nk - 1) & 1) * STAGE);
    IWQ_SLICE(A0, B0, A1, B1, 1, so, false, 0, so, 0)
    IWQ_SLICE(A1, B1, A0, B0, 2, so, false, 0, so, 0)
    IWQ_SLICE(A0, B0, A1, B1, 3, so, false, 0, so, 0)
    IWQ_PIN();
#pragma unroll
    for (int i = 0; i < 16; ++i) IWQ_MF(A1, B1, i);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_SLICE
#undef IWQ_WRB
#undef IWQ_MF
#undef IWQ_LGKM
#undef IWQ_PIN

#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = n0 + wn * 128 + nt * 32 + r32;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = opaque(acc[mt][nt][r] * sfl[nt]);
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + b);
      }
    }
  }
}

template <bool NIB>
hipError_t launch_w4b(const PrefillArgs& a, hipStream_t st) {
  if (!w4h_fits(a)) return launch_w<NIB>(a, st);
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_w4b<NIB>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <bool GROUPED, bool FACTOR, bool SG = false>
hipError_t launch_w4(const PrefillArgs& a, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_w4e<GROUPED, FACTOR, SG>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

// Split-K epilogue: y = RN16(s * sum_split partial + b) (per channel, FACTOR) or RN16(sum + b), the
// partials summed in split order 0..S-1 in fp32.  One thread per 4 consecutive lanes of one
// accumulator register = 4 consecutive columns of one output row (16-B loads, 8-B stores); the
// register -> (row, col) map is k_w4a16_b32e's (WM = 2: wave (wm, wn) owns rows 128 wm + [0, 128),
// columns 64 wn + [0, 64); 32x32 C layout).
template <bool FACTOR>
__global__ __launch_bounds__(256) void k_splitk_reduce(PrefillArgs a) {
  const int tiles_n = a.N / TN;
  const int64_t t = blockIdx.x;
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int e = (blockIdx.y * 256 + threadIdx.x) * 4;  // element of the tile's 65536, lane-aligned
  const int wave = e >> 13, rem = e & 8191;
  const int tl = rem >> 10, reg = (rem >> 6) & 15, lane0 = rem & 63;
  const int mt = tl >> 1, nt = tl & 1;  // MTL 4 x NTL 2
  const int wm = wave >> 2, wn = wave & 3;
  const int row = m0 + wm * 128 + mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane0 >> 5);
  const int col = n0 + wn * 64 + nt * 32 + (lane0 & 31);
  if (row >= a.M) return;
  const IWQ_GLOBAL f4* src = gp<f4>(a.ws + (t * a.nsplit) * 65536 + e);
  f4 sum = src[0];
  for (int sp = 1; sp < a.nsplit; ++sp) sum += src[(int64_t)sp * (65536 / 4)];
  _Float16 o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col + j] : 0.0f;
    const float v = FACTOR ? opaque(sum[j] * (float)gp<_Float16>(a.scales)[col + j]) : sum[j];
    o[j] = (_Float16)(v + b);
  }
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  *reinterpret_cast<IWQ_GLOBAL u32x2v*>(gp<_Float16>(a.y) + (int64_t)row * a.ldy + col) =
      u32x2v{as_u32(h2{o[0], o[1]}), as_u32(h2{o[2], o[3]})};
}

template <bool GROUPED, bool FACTOR, int WM = 2, bool PHI = false, bool NIB = false, bool SWAP = false>
hipError_t launch_e(const PrefillArgs& a, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_b32e<GROUPED, FACTOR, WM, PHI, NIB, SWAP>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
  return hipGetLastError();
}

// 16x16x32 form of the early-barrier kernel (k_w4a16_b16e).  MI355X_MICROARCH.md (DVFS item 7):
// on random data a 16x16x32 MFMA loop holds a ~13 % higher clock than a 32x32x16 loop at equal
// cycles per FLOP, so with the dequant trimmed to 12 VALU per 8 weights (factored scale) the
// smaller shape can come out ahead despite its 2-slot gaps.  Same tile, staging and barrier
// placement as k_w4a16_b32e; per wave 128 x 64 = 8 x 4 tiles of 16 x 16; k order: lane group q
// of slice s holds k = 16 q + 8 s + [0, 8), so a lane's codes for a K-step are ONE 8-byte piece of
// its column.  A K-step is 4 sub-steps (slice s, rows half) of 16 MFMAs; each sub-step's MFMAs
// run behind the next sub-step's A reads (and the next slice's dequant).
template <bool GROUPED, bool FACTOR>
__global__ __launch_bounds__(THR) void k_w4a16_b16e(PrefillArgs a) {
  static_assert(!(GROUPED && FACTOR), "grouped scales change along k: no factoring");
  constexpr int STAGE = XS + CS + (GROUPED ? PS : 0);
  constexpr int PER_STAGE = 4 + 1 + (GROUPED ? 1 : 0);
  constexpr bool SCALE = !FACTOR;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int r16 = lane & 15, q = lane >> 4;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int nk = a.K / TK;
  const int64_t crow = a.K / 2;

  const _Float16* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xswz(row)) << 3);
  }
  const int ccol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + ccol) * crow + (((lane & 1) ^ cswz(ccol)) << 4);
  const _Float16* psrc = nullptr;
  if constexpr (GROUPED) {
    const _Float16* arr = (wid < 4 || !a.zeros) ? a.scales : a.zeros;
    psrc = arr + (int64_t)(n0 + (wid & 3) * 64 + lane) * a.gpr;
  }
  auto issue = [&](int kt, int stg) {
    uint8_t* base = smem + stg * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
    if constexpr (GROUPED) glds2(psrc + (kt * TK) / a.group, base + XS + CS + wid * 256);
  };

  h2 sv[4], zz[4];
  float sf[4] = {1.0f, 1.0f, 1.0f, 1.0f};
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = n0 + wn * 64 + nt * 16 + r16;
      const _Float16 sc = gp<_Float16>(a.scales)[col];
      const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym;
      sv[nt] = h2{sc, sc};
      sf[nt] = (float)sc;
      zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  uint32_t magic_v;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));

  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  auto read_params = [&](const uint8_t* xs) {
    if constexpr (GROUPED) {
      const uint32_t* ps = reinterpret_cast<const uint32_t*>(xs + XS + CS);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int col = wn * 64 + nt * 16 + r16;
        const _Float16 sc = __builtin_bit_cast(_Float16, (uint16_t)ps[col]);
        const float zf = a.zeros ? (float)__builtin_bit_cast(_Float16, (uint16_t)ps[TN + col]) : a.zsym;
        sv[nt] = h2{sc, sc};
        zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
      }
    }
  };
  // lane's 8 code bytes of column col = k 16 q + [0, 16): logical chunk q >> 1, half q & 1
  auto read_codes = [&](const uint8_t* xs, u32x2 (&wc)[4]) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = wn * 64 + nt * 16 + r16;
      wc[nt] = *reinterpret_cast<const u32x2*>(xs + XS + col * 32 + ((((q >> 1) ^ cswz(col)) << 4) | ((q & 1) << 3)));
    }
  };
  // A fragments of slice s, row half hf (4 of the 8 16-row tiles)
  auto read_a = [&](const uint8_t* xs, int s, int hf, h8 (&af)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 128 + (hf * 4 + i) * 16 + r16;
      af[i] = *reinterpret_cast<const h8*>(xs + row * 128 + (((2 * q + s) ^ xswz(row)) << 4));
    }
  };

  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f4){0.f, 0.f, 0.f, 0.f};
#define IWQ_MFMA_HALF(AF, B0, HF)                                                                  \
  _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                   \
  _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                                                \
    acc[(HF) * 4 + i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AF[i], B0[nt], acc[(HF) * 4 + i][nt], 0, 0, 0);
#define IWQ_DQ_SLICE(DST, WC, S)                                                                   \
  _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                                                \
    DST[nt] = dq8<SCALE>(WC[nt][S], zz[nt], sv[nt], mask_s, magic_v);

  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    if constexpr (PER_STAGE == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (nk > 2) issue(2, 2);
  u32x2 wc[4];
  h8 af[4], bcur[4];
  read_params(smem);
  read_codes(smem, wc);
  read_a(smem, 0, 0, af);
  IWQ_DQ_SLICE(bcur, wc, 0)

  // sub-steps 0..2 of the stage at XS: (s 0, half 0), (0, 1), (1, 0); sub-step 3 = (1, 1)
#define IWQ_SUBSTEPS_012(XS)                                                                       \
  {                                                                                               \
    h8 an[4], bn[4];                                                                              \
    read_a(XS, 0, 1, an);                                                                         \
    IWQ_MFMA_HALF(af, bcur, 0)                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) af[i] = an[i];                                 \
    read_a(XS, 1, 0, an);                                                                         \
    IWQ_DQ_SLICE(bn, wc, 1)                                                                       \
    IWQ_MFMA_HALF(af, bcur, 1)                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) af[i] = an[i];                                 \
    _Pragma("unroll") for (int nt = 0; nt < 4; ++nt) bcur[nt] = bn[nt];                          \
    read_a(XS, 1, 1, an);                                                                         \
    IWQ_MFMA_HALF(af, bcur, 0)                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) af[i] = an[i];                                 \
  }
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint8_t* xs = smem + (kt % NSTAGE) * STAGE;
    IWQ_SUBSTEPS_012(xs)
    if (kt + 2 < nk) {
      if constexpr (PER_STAGE == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + 3 < nk) issue(kt + 3, kt % NSTAGE);
    const uint8_t* xn = smem + ((kt + 1) % NSTAGE) * STAGE;
    h8 an[4], bn[4];
    u32x2 wn2[4];
    read_params(xn);
    read_codes(xn, wn2);
    read_a(xn, 0, 0, an);
    IWQ_DQ_SLICE(bn, wn2, 0)
    IWQ_MFMA_HALF(af, bcur, 1)
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = an[i];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      bcur[nt] = bn[nt];
      wc[nt] = wn2[nt];
    }
  }
  {
    const uint8_t* xs = smem + ((nk - 1) % NSTAGE) * STAGE;
    IWQ_SUBSTEPS_012(xs)
    IWQ_MFMA_HALF(af, bcur, 1)
  }
#undef IWQ_SUBSTEPS_012
#undef IWQ_DQ_SLICE
#undef IWQ_MFMA_HALF

  // epilogue, 16x16 C layout: col = lane & 15, row = 4 (lane >> 4) + reg
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = n0 + wn * 64 + nt * 16 + r16;
    const float b = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 128 + mt * 16 + 4 * q + r;
        const float v = FACTOR ? opaque(acc[mt][nt][r] * sf[nt]) : acc[mt][nt][r];  // no fma_mix fold
        if (row < a.M) gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)(v + b);
      }
    }
  }
}

template <bool GROUPED, bool FACTOR>
hipError_t launch_16e(const PrefillArgs& a, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_b16e<GROUPED, FACTOR>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// k_w4a16_mid: 16 < M < 512 (batched decode, short prompts).  A 256 x 256 tile leaves most of the
// chip idle here (q_proj at M = 64: 16 workgroups) and the weight stream, not the MFMA, is the
// floor, so this is the decode GEMV's structure (k_w4a16_gemv_ct, iwq_gemm.hip) widened to MT
// tiles of 16 rows: a workgroup of S waves owns CT column tiles x MT row tiles; wave ks takes the
// 128-k steps ks, ks + S, ...; each wave keeps a ring of PF steps of code loads (CT x 16 B per lane)
// AND of X fragments (MT x 4 x 16 B per lane, read from L2 in natural k order -- no LDS image, no
// permutation) in flight; per step every dequantized B fragment feeds MT MFMAs (the dequant VALU
// per FLOP drops MT-fold vs the GEMV); the S partial tiles are summed through LDS in k-split order.
// k order: lane group q of slice s holds k = 32 q + 8 s + [0, 8) -- exactly the GEMV's code bytes
// (row-major or the decode tile layout), decoded in natural order (dq8).  grid = (N / (16 CT),
// ceil(M / (16 MT))): row tiles past M read row M-1 (discarded).
// ---------------------------------------------------------------------------------------------
// PST (grouped, round 5; as the decode GEMV's): the CT tiles' (s, z) rows staged into LDS once per
// workgroup -- one dword per group, rows padded to gpr + 1 dwords -- instead of 2 CT two-byte gathers
// per k-step on the in-order vmcnt behind the code and X loads.
// GF (group % 128 == 0, with PST): the scale factored per 128-k step as the decode GEMV's -- B =
// (q - z) exactly, each (row tile, column tile)'s four MFMAs of the step into a fresh accumulator,
// then acc += s_g * partial (A = I still gives W_deq bit for bit).
template <int PF, int S, int CT, int MT, bool FACTOR, bool TILED, bool PST = false, bool GF = false>
__global__ __launch_bounds__(S * 64) void k_w4a16_mid(PrefillArgs a) {
  static_assert(!GF || PST, "the factored scale reads the staged parameters");
  constexpr bool SCALE = !FACTOR;
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int lane = threadIdx.x & 63;
  const int ks = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int tile0 = blockIdx.x * CT;
  const int mrow0 = blockIdx.y * 16 * MT;
  const int nks = a.K / 128;
  const int nj = nks > ks ? (nks - ks + S - 1) / S : 0;
  const int64_t crow = a.K / 2;
  const int64_t tstride = TILED ? (int64_t)nks * 1024 : 16 * crow;  // code bytes between column tiles
  const uint8_t* cbase = TILED ? a.codes + (int64_t)tile0 * tstride + lane * 16
                               : a.codes + (int64_t)(tile0 * 16 + r16) * crow + q * 16;
  const _Float16* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int r = mrow0 + mt * 16 + r16;
    xrow[mt] = a.x + (int64_t)(r < a.M ? r : a.M - 1) * a.lda + 32 * q;
  }
  const bool perch = a.gpr == 1;
  h2 zz0[CT], sv0[CT];
  float sf[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int n = (tile0 + c) * 16 + r16;
    const _Float16 sc = perch ? gp<_Float16>(a.scales)[n] : (_Float16)1.0f;
    const float zf = perch ? (a.zeros ? (float)gp<_Float16>(a.zeros)[n] : a.zsym) : 0.0f;
    sv0[c] = h2{sc, sc};
    sf[c] = (FACTOR && perch) ? (float)sc : 1.0f;
    zz0[c] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  uint32_t magic_v;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));

  u32x4 bc[PF][CT];
  u32x4 xa[PF][MT][4];
  _Float16 sv[PF][CT], zv[PF][CT];
  auto load = [&](int j, int u) {
    const int kt = ks + j * S;
#pragma unroll
    for (int c = 0; c < CT; ++c)
      bc[u][c] = __builtin_nontemporal_load(gp<u32x4>(cbase + c * tstride + kt * (TILED ? 1024 : 64)));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[u][mt][s] = *gp<u32x4>(xrow[mt] + kt * 128 + 8 * s);
    if (!perch && !PST) {
      const int gk = (kt * 128 + 32 * q) / a.group;
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
  uint32_t* pst = reinterpret_cast<uint32_t*>(dsm);
  if constexpr (PST) {
    constexpr int PRE = 4, NT = S * 64;
    const int np = CT * 16 * a.gpr;
    const int64_t pbase = (int64_t)tile0 * 16 * a.gpr;
    const uint32_t zs = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a.zsym);
    uint32_t ps[PRE], pz[PRE];
#pragma unroll
    for (int r = 0; r < PRE; ++r) {  // issued together: one round of latency
      const int i = (int)threadIdx.x + r * NT;
      ps[r] = i < np ? (uint32_t)gp<uint16_t>(a.scales)[pbase + i] : 0u;
      pz[r] = i < np && a.zeros ? (uint32_t)gp<uint16_t>(a.zeros)[pbase + i] : zs;
    }
#pragma unroll
    for (int r = 0; r < PRE; ++r) {
      const int i = (int)threadIdx.x + r * NT;
      if (i < np) {
        const int c = i / a.gpr, g = i - c * a.gpr;
        pst[c * (a.gpr + 1) + g] = ps[r] | (pz[r] << 16);
      }
    }
    for (int i = (int)threadIdx.x + PRE * NT; i < np; i += NT) {
      const int c = i / a.gpr, g = i - c * a.gpr;
      const uint32_t sv16 = gp<uint16_t>(a.scales)[pbase + i];
      const uint32_t zv16 = a.zeros ? (uint32_t)gp<uint16_t>(a.zeros)[pbase + i] : zs;
      pst[c * (a.gpr + 1) + g] = sv16 | (zv16 << 16);
    }
    __syncthreads();
  }

  f4 acc[MT][CT], accs[GF ? MT : 1][GF ? CT : 1];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[mt][c] = f4{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nj; j0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int j = j0 + u;
      if (j >= nj) break;
      h2 s2[CT], z2[CT];
      float sf[CT];  // GF: the step's group scale per column tile
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        if (perch) {
          s2[c] = sv0[c];
          z2[c] = zz0[c];
        } else if constexpr (PST) {
          const int kt = ks + j * S;
          const uint32_t sz = pst[(c * 16 + r16) * (a.gpr + 1) + (kt * 128 + 32 * q) / a.group];
          const float zf = (float)__builtin_bit_cast(_Float16, (uint16_t)(sz >> 16));
          s2[c] = as_h2(__builtin_amdgcn_perm(sz, sz, 0x01000100u));
          z2[c] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
          sf[c] = (float)__builtin_bit_cast(_Float16, (uint16_t)(sz & 0xFFFFu));
        } else {
          const float zf = (float)zv[u][c];
          s2[c] = h2{sv[u][c], sv[u][c]};
          z2[c] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const h8 bf = ((perch && FACTOR) || GF) ? dq8<false>(bc[u][c][s], z2[c], s2[c], mask_s, magic_v)
                                                  : dq8<true>(bc[u][c][s], z2[c], s2[c], mask_s, magic_v);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            if constexpr (GF)
              accs[mt][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, xa[u][mt][s]), bf,
                                                                   s == 0 ? f4{0.f, 0.f, 0.f, 0.f} : accs[mt][c], 0, 0, 0);
            else
              acc[mt][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, xa[u][mt][s]), bf,
                                                                  acc[mt][c], 0, 0, 0);
          }
        }
      }
      if constexpr (GF) {  // a lane's 4 accumulators of a tile all belong to its column r16
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[mt][c][e] = __builtin_fmaf(sf[c], accs[mt][c][e], acc[mt][c][e]);
      }
      if (j + PF < nj) load(j + PF, u);
    }
  }
  (void)SCALE;
  if constexpr (PST) __syncthreads();  // the staged parameters are dead: the LDS holds the partial tiles
  float* red = reinterpret_cast<float*>(dsm);  // [S][MT * CT][256]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int c = 0; c < CT; ++c)
      *reinterpret_cast<f4*>(red + ((ks * MT + mt) * CT + c) * 256 + lane * 4) = acc[mt][c];
  __syncthreads();
  for (int o = threadIdx.x; o < MT * CT * 256; o += S * 64) {
    const int tc = o >> 8, e = o & 255;
    const int mt = tc / CT, c = tc % CT;
    const int ln = e >> 2, reg = e & 3;
    const int row = mrow0 + mt * 16 + 4 * (ln >> 4) + reg, col = (tile0 + c) * 16 + (ln & 15);
    if (row < a.M) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) v += red[(k * MT * CT + tc) * 256 + e];
      if (FACTOR && perch) v *= (float)gp<_Float16>(a.scales)[col];
      if (a.bias) v += (float)gp<_Float16>(a.bias)[col];
      gp<_Float16>(a.y)[(int64_t)row * a.ldy + col] = (_Float16)v;
    }
  }
}

template <int PF, int S, int CT, int MT>
hipError_t launch_mid(const PrefillArgs& a, bool tiled, hipStream_t st, bool mid_no_gf = false) {
  const dim3 grid((unsigned)(a.N / (16 * CT)), (unsigned)((a.M + 16 * MT - 1) / (16 * MT)));
  const size_t red = (size_t)S * MT * CT * 256 * 4;
  const size_t pbytes = (size_t)CT * 16 * (a.gpr + 1) * 4;
  const bool pst = a.gpr > 1 && pbytes <= 64 * 1024;  // grouped: parameters staged (PST)
  const bool gf = pst && a.group % 128 == 0 && !mid_no_gf;  // and the scale factored per k-step
  const size_t lds = pst && pbytes > red ? pbytes : red;
  if (gf) {
    if (tiled) hipLaunchKernelGGL((k_w4a16_mid<PF, S, CT, MT, true, true, true, true>), grid, dim3(S * 64), lds, st, a);
    else hipLaunchKernelGGL((k_w4a16_mid<PF, S, CT, MT, true, false, true, true>), grid, dim3(S * 64), lds, st, a);
  } else if (pst) {
    if (tiled) hipLaunchKernelGGL((k_w4a16_mid<PF, S, CT, MT, true, true, true>), grid, dim3(S * 64), lds, st, a);
    else hipLaunchKernelGGL((k_w4a16_mid<PF, S, CT, MT, true, false, true>), grid, dim3(S * 64), lds, st, a);
  } else if (tiled) {
    hipLaunchKernelGGL((k_w4a16_mid<PF, S, CT, MT, true, true>), grid, dim3(S * 64), red, st, a);
  } else {
    hipLaunchKernelGGL((k_w4a16_mid<PF, S, CT, MT, true, false>), grid, dim3(S * 64), red, st, a);
  }
  return hipGetLastError();
}

template <bool GROUPED, bool FACTOR, int SCHED, bool PRIO>
hipError_t launch(const PrefillArgs& a, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  hipLaunchKernelGGL((k_w4a16_b32<GROUPED, FACTOR, SCHED, PRIO>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
  return hipGetLastError();
}

}  // namespace

bool mid_supported(int64_t M, int64_t N, int64_t K, int gpr, int group) {
  return M >= 1 && N % 64 == 0 && K % 128 == 0 && (gpr == 1 || group % 32 == 0);
}

// variants: 50 MT 1 CT 2, 51 MT 2 CT 1, 52 MT 2 CT 2, 53 MT 2 CT 4, 54 MT 4 CT 1, 55 MT 4 CT 2;
// 0 = by M (interleaved A/B vs hipBLASLt on the Llama-2-7B shapes, profiles/r02_ab_mid*.jsonl:
// M <= 32 -> 50, M <= 64 -> 52, above -> 53)
hipError_t mid_launch(const PrefillArgs& a, int variant, bool tiled, hipStream_t st) {
#if IWQ_AB
  if (variant == 56) {  // the default's shapes with the grouped scale per weight (no GF; A/B)
    const int v = a.M <= 32 ? 50 : (a.M <= 64 ? 52 : 53);
    if (v == 50) return launch_mid<2, 8, 2, 1>(a, tiled, st, true);
    if (v == 53) return launch_mid<2, 8, 4, 2>(a, tiled, st, true);
    return launch_mid<2, 8, 2, 2>(a, tiled, st, true);
  }
#endif
  if (variant == 0) variant = a.M <= 32 ? 50 : (a.M <= 64 ? 52 : 53);
  switch (variant) {
    case 50: return launch_mid<2, 8, 2, 1>(a, tiled, st);
    case 53: return launch_mid<2, 8, 4, 2>(a, tiled, st);
#if IWQ_AB
    case 51: return launch_mid<2, 8, 1, 2>(a, tiled, st);
    case 54: return launch_mid<2, 8, 1, 4>(a, tiled, st);
    case 55: return launch_mid<2, 8, 2, 4>(a, tiled, st);
#endif
    default: return launch_mid<2, 8, 2, 2>(a, tiled, st);
  }
}

static int cu_count() {
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

// Split-count model (times in us, fitted to profiles/r02_ab_gemm_splitk_forced.jsonl on the Llama-2-7B
// shapes, M = 256..4096): one 512-thread workgroup per CU (120 KiB of LDS), so T x S workgroups run
// in ceil(T S / CUs) rounds of ceil(nk / S) K-steps at ~1.4 us each; a split adds the fp32 partial
// tiles (256 KiB per workgroup, written and read back: ~0.105 us per workgroup at ~5 TB/s) and the
// reduce launch (~4 us).  The smallest modelled time wins (S = 1 on ties).
static double splitk_model_us(int64_t tiles, int64_t nk, int64_t c) {
  const int64_t cus = cu_count();
  const double t = (double)((tiles * c + cus - 1) / cus) * (double)((nk + c - 1) / c) * 1.4;
  return c == 1 ? t : t + 4.0 + 0.105 * (double)(tiles * c);
}

int prefill_splitk_count(int64_t M, int64_t N, int64_t K, int force) {
  const int64_t tiles = ((M + TM - 1) / TM) * (N / TN);
  const int64_t nk = K / TK;
  int64_t s = 1;
  if (force > 1) {
    s = force;
  } else {
    auto model = [&](int64_t c) { return splitk_model_us(tiles, nk, c); };
    double best = model(1);
    for (int64_t c = 2; c <= 32 && c <= nk / 2; ++c) {
      const double tc = model(c);
      if (tc < best) {
        best = tc;
        s = c;
      }
    }
  }
  if (s > nk / 2) s = nk / 2;  // at least 2 K-steps per range
  if (s < 2) return 1;
  const int64_t kps = (nk + s - 1) / s;
  return (int)((nk + kps - 1) / kps);  // no empty range
}

// 16 < M < 256: the split 256 x 256 prefill (rows past M computed and dropped) against the mid-M
// weight-streaming kernel, modelled as ~6 us + 0.45 ns per weight element per 64-row block (fitted
// to profiles/r02_ab_midm_split.jsonl, M = 64 / 128 / 200 on the Llama-2-7B shapes: the mid kernel
// wins q_proj up to M = 128, the split kernel gate_proj from M = 128 and everything at M = 200)
bool prefill_split_preferred(int64_t M, int64_t N, int64_t K, int gpr, int group) {
  if (M <= 16 || !prefill_b32_supported(M, N, K, gpr, group)) return false;
  const int s = prefill_splitk_count(M, N, K, 0);
  if (s <= 1) return false;
  if (M >= 256) return true;
  const int64_t tiles = ((M + TM - 1) / TM) * (N / TN);
  const double split_us = splitk_model_us(tiles, K / TK, s);
  const double mid_us = 6.0 + 0.45e-6 * (double)((M + 63) / 64) * (double)N * (double)K;
  return split_us < mid_us;
}

// 16 < M < 256 where the mid kernel's modelled time exceeds ~24 us: the short-tile split (64-row
// tiles) with S = floor(256 / tiles) ranges (2..12, >= 4 K-steps each).  Fitted to profiles/
// r02_ab_gemm_short_split.jsonl (M = 32 / 64 / 128 on the Llama-2-7B shapes: every split form has a
// ~20 us floor -- two launches and the reduce -- so the mid kernel keeps q_proj; gate / down at
// M = 64: 39.1 / 31.6 -> 23.2 / 23.7 us, at M = 128: 38.2 / 37.5 -> 28 / 25 us).
// 128 < M < 256: the short split also wins where it stays under ~128 tiles (q / down: 20 % / 12 %
// over the 256-row split at M = 160-250, profiles/r02_ab_gemm_short_split_hi.jsonl); wider weights
// (gate) keep the 256-row split.
// Round 5: 64 < M < 256 on wide weights (N >= 8192: 7B gate/up, 70B gate/up/down) takes 128-row
// tiles (MTW 4: half the per-tile re-dequantization of the weights) with S = min(256 / tiles,
// K-steps / 16, 8) -- profiles/r05_ab_short_split128.jsonl, M = 96 / 128: 70B gate g128 168 -> 100 us,
// 70B down 139 -> 100, 7B gate 32.5 -> 28.8 (per channel 87 -> 79, 85 -> 68, 28.0 -> 26.5); past
// M = 128 while the 128-row tiles stay <= 128 (70B down M = 160-224: g128 208-259 -> 163-172 us,
// 7B gate neutral); more tiles (70B gate past 128 rows) keep the 256-row split, and the N = 4096
// shapes the 64-row form (q / down: the mid kernel or 64-row tiles measured faster).
bool prefill_short_split(int64_t M, int64_t N, int64_t K, int gpr, int group, int* ns_out, int* mtw_out) {
  if (M <= 16 || M >= 256 || !prefill_b32_supported(M, N, K, gpr, group)) return false;
  // grouped scales cost the mid kernel ~1.4x (profiles/r02_ab_gemm_g128_mid.jsonl); ~1.1x since
  // round 5 where the scale is factored per k-step, i.e. g % 128 == 0 (parameters staged in LDS:
  // profiles/r05_ab_mid_gf.jsonl, q_proj g128 M = 128 mid 20.3 us vs the short split's 21.9); other
  // groups (g = 64) still scale every weight: the measured 1.4x stands for them
  const double gfac = gpr == 1 ? 1.0 : (group % 128 == 0 ? 1.1 : 1.4);
  const double mid_us = (6.0 + 0.45e-6 * (double)((M + 63) / 64) * (double)N * (double)K) * gfac;
  if (mid_us < 24.0) return false;
  const int64_t nk = K / TK;
  const int64_t tiles128 = ((M + 127) / 128) * (N / TN);
  if (M > 64 && N >= 8192 && (M <= 128 || tiles128 <= 128)) {
    const int64_t tiles = tiles128;
    int64_t ns = 256 / tiles;
    if (ns > nk / 16) ns = nk / 16;  // >= 16 K-steps per range
    if (ns > 8) ns = 8;
    if (ns < 2) ns = 2;
    if (ns_out) *ns_out = (int)ns;
    if (mtw_out) *mtw_out = 4;
    return true;
  }
  const int64_t tiles = ((M + 63) / 64) * (N / TN);
  if (M > 128 && tiles > 128) return false;
  int64_t ns = 256 / tiles;  // at most ~256 workgroups: best or within ~7 % in every sweep
  if (ns > 12) ns = 12;
  if (ns > nk / 4) ns = nk / 4;
  if (ns < 2) ns = 2;
  if (ns_out) *ns_out = (int)ns;
  if (mtw_out) *mtw_out = 2;
  return true;
}

int64_t prefill_splitk_bytes(int64_t M, int64_t N, int nsplit) {
  if (nsplit <= 1) return 0;
  return ((M + TM - 1) / TM) * (N / TN) * (int64_t)nsplit * 65536 * 4;
}

hipError_t prefill_splitk_launch(const PrefillArgs& a0, hipStream_t st, bool legacy, bool nib) {
  PrefillArgs a = a0;
  const int64_t tiles = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  const int nk = a.K / TK;
  a.kps = (nk + a.nsplit - 1) / a.nsplit;
  const dim3 grid((unsigned)(tiles * a.nsplit));
  // the partials: 74's hand-ordered kernel (legacy: k_w4a16_b32e, the round-2 first version)
#if IWQ_AB
  if (legacy && a.gpr != 1) hipLaunchKernelGGL((k_w4a16_b32e<true, false, 2, false, false, false, true>), grid, dim3(THR), 0, st, a);
  else if (legacy) hipLaunchKernelGGL((k_w4a16_b32e<false, true, 2, false, false, false, true>), grid, dim3(THR), 0, st, a);
  else
#else
  if (legacy) return hipErrorInvalidValue;
#endif
  if (nib && a.gpr != 1) hipLaunchKernelGGL((k_w4a16_b32w<true, true, true>), grid, dim3(THR), 0, st, a);
  else if (nib) hipLaunchKernelGGL((k_w4a16_b32w<true, false, true>), grid, dim3(THR), 0, st, a);
  else if (a.gpr != 1) hipLaunchKernelGGL((k_w4a16_b32w<false, true, true>), grid, dim3(THR), 0, st, a);
  else hipLaunchKernelGGL((k_w4a16_b32w<false, false, true>), grid, dim3(THR), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const dim3 rgrid((unsigned)tiles, 65536 / 4 / 256);
  if (a.gpr != 1) hipLaunchKernelGGL((k_splitk_reduce<false>), rgrid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((k_splitk_reduce<true>), rgrid, dim3(256), 0, st, a);
  return hipGetLastError();
}

// short-tile split (k_w4a16_b32s): MTW 32-row tiles per wave (2 or 4), nsplit K ranges
int64_t prefill_splitk_bytes_s(int64_t M, int64_t N, int mtw, int nsplit) {
  return ((M + 32 * mtw - 1) / (32 * mtw)) * (N / TN) * (int64_t)nsplit * (mtw * 8192) * 4;
}

hipError_t prefill_splitk_launch_s(const PrefillArgs& a0, int mtw, hipStream_t st) {
  PrefillArgs a = a0;
  const int64_t tiles = ((int64_t)(a.M + 32 * mtw - 1) / (32 * mtw)) * (a.N / TN);
  const int nk = a.K / TK;
  a.kps = (nk + a.nsplit - 1) / a.nsplit;
  a.nsplit = (nk + a.kps - 1) / a.kps;  // no empty range
  const dim3 grid((unsigned)(tiles * a.nsplit));
  const bool grouped = a.gpr != 1;
  if (mtw == 2) {
    if (grouped) hipLaunchKernelGGL((k_w4a16_b32s<2, true>), grid, dim3(THR), 0, st, a);
    else hipLaunchKernelGGL((k_w4a16_b32s<2, false>), grid, dim3(THR), 0, st, a);
  } else {
    if (grouped) hipLaunchKernelGGL((k_w4a16_b32s<4, true>), grid, dim3(THR), 0, st, a);
    else hipLaunchKernelGGL((k_w4a16_b32s<4, false>), grid, dim3(THR), 0, st, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const dim3 rgrid((unsigned)tiles, (unsigned)(mtw * 8));
  if (mtw == 2) {
    if (grouped) hipLaunchKernelGGL((k_splitk_reduce_s<false, 2>), rgrid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_splitk_reduce_s<true, 2>), rgrid, dim3(256), 0, st, a);
  } else {
    if (grouped) hipLaunchKernelGGL((k_splitk_reduce_s<false, 4>), rgrid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_splitk_reduce_s<true, 4>), rgrid, dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

bool prefill_b32_supported(int64_t M, int64_t N, int64_t K, int gpr, int group) {
  return M >= 1 && N % TN == 0 && K % TK == 0 && K >= TK && (gpr == 1 || group % TK == 0);
}

// variants (flags bits 16..23 of iwq_w4a16_gemm, for A/B): 0 default = 74 (1 x 8 waves, hand-ordered
// stream, bit-identical to 45): per channel +1-5 % over 45 (profiles/r02_ab_gemm_w18*.jsonl), grouped
// (g % 64 == 0) +7-8 % (r02_ab_gemm_b32w_grouped.jsonl; interleaved A/B, Llama-2-7B shapes, M = 8192);
// 60-69, 74, 75: see DESIGN.md section 5 (round 2); per channel: 40 exact
// (scale per element), 41 factored, 42 factored + interleave, 43 factored + setprio,
// 44 exact + interleave, 45 early barrier factored, 46 early barrier exact, 47 / 48 the same on
// 16x16x32, 49 = 41; grouped: 40, 41 and 49 plain, 42/43 interleave / setprio, 45 early barrier,
// 47 16x16x32.
hipError_t prefill_b32_launch(const PrefillArgs& a, int variant, hipStream_t st, bool nib) {
  if (variant == 0) {
    // 74 on the 16x16x32 MFMA (iwq_prefill16.hip; NIB twins give the same bits): per channel with
    // waves 4-7 staggered half a K-step (151; round 4: +6-11 % over 74 on q / gate / down at
    // M = 8192, profiles/r04_ab_gemm_b16.jsonl) and, on NIB codes, the persistent one-wave-per-SIMD
    // form (172: 1-4.5 % over 153, profiles/r04_ab_gemm_b16p_saddr.jsonl); grouped on the 3-slot
    // ring (150 / 152: +6-8 % over 74 at g128, profiles/r04_ab_gemm_grouped16.jsonl)
    if (prefill16_supported(a.M, a.N, a.K, a.gpr, a.group))
      return prefill16_launch(a, a.gpr == 1 ? (nib ? 172 : 151) : (nib ? 152 : 150), st);
    if (a.gpr == 1) return nib ? launch_w<true>(a, st) : launch_w<false>(a, st);
    return nib ? launch_w<true, true>(a, st) : launch_w<false, true>(a, st);
  }
#if IWQ_AB
  if (nib) return hipErrorInvalidValue;
  if (variant >= 158 && variant <= 160) {  // A/B: grouped 150 / 157 / 151 reading group-major parameters
    if (a.gpr == 1 || !prefill16_supported(a.M, a.N, a.K, a.gpr, a.group)) return hipErrorInvalidValue;
    PrefillArgs b = a;
    b.pgm = 1;
    return prefill16_launch(b, variant == 158 ? 150 : (variant == 159 ? 157 : 151), st);
  }
  // 161 diagnostic (per channel; grouped: 151); 162 / 163 (164 / 165 interleaved): one wave per SIMD
  // (k_w4a16_b16q), NIB codes for the odd ones; 168 / 169 / 170: k_w4a16_b16r reading 4 / 6 / 6
  // groups ahead (NIB, NIB, row-major); 171 / 172: persistent k_w4a16_b16p (row-major / NIB)
  if ((variant == 161 || variant == 166 || variant == 167) && a.gpr != 1) variant = 151;  // diagnostics
  if (variant >= 161 && variant <= 172) {
    if (prefill16_supported(a.M, a.N, a.K, a.gpr, a.group)) return prefill16_launch(a, variant, st);
    const bool nibv = variant == 163 || variant == 165 || variant == 168 || variant == 169 || variant == 172;
    return nibv ? launch_w<true, true>(a, st) : launch_w<false, true>(a, st);
  }
  if (variant >= 150 && variant <= 157) {
    if (prefill16_supported(a.M, a.N, a.K, a.gpr, a.group)) return prefill16_launch(a, variant, st);  // iwq_prefill16.hip
    // grouped: 74 on the same code layout
    return (variant == 152 || variant == 153) ? launch_w<true, true>(a, st) : launch_w<false, true>(a, st);
  }
  if (a.gpr != 1) {
    switch (variant) {
      case 42: return launch<true, false, 1, false>(a, st);
      case 43: return launch<true, false, 0, true>(a, st);
      case 45: return launch_e<true, false>(a, st);
      case 47: return launch_16e<true, false>(a, st);
      case 49: return launch<true, false, 0, false>(a, st);
      case 60: return launch_e<true, false, 4>(a, st);
      case 62: return launch_e<true, false, 2, true>(a, st);
      case 63: return launch_w4<true, false>(a, st);
      case 65: return launch_w4<true, false, true>(a, st);
      case 66: return launch_e<true, false, 2, false, true>(a, st);
      case 68: return launch_e<true, false, 2, false, false, true>(a, st);
      case 69: return launch_e<true, false, 2, false, true, true>(a, st);
      case 74: return launch_w<false, true>(a, st);  // 1 x 8 waves, hand-ordered stream
      case 75: return launch_w<true, true>(a, st);   // the same on NIB codes
      case 79: return launch_w<false, true, true>(a, st);  // 74 with the parameters staged once per group
      default: return launch_w<false, true>(a, st);  // 74: +7-8 % over 45 (r02_ab_gemm_b32w_grouped.jsonl)
    }
  }
  switch (variant) {
    case 40: return launch<false, false, 0, false>(a, st);
    case 42: return launch<false, true, 1, false>(a, st);
    case 43: return launch<false, true, 0, true>(a, st);
    case 44: return launch<false, false, 1, false>(a, st);
    case 45: return launch_e<false, true>(a, st);
    case 46: return launch_e<false, false>(a, st);
    case 47: return launch_16e<false, true>(a, st);
    case 48: return launch_16e<false, false>(a, st);
    case 49: return launch<false, true, 0, false>(a, st);
    case 60: return launch_e<false, true, 4>(a, st);
    case 61: return launch_e<false, false, 4>(a, st);
    case 62: return launch_e<false, true, 2, true>(a, st);
    case 63: return launch_w4<false, true>(a, st);
    case 64: return launch_w4<false, false>(a, st);
    case 65: return launch_w4<false, true, true>(a, st);
    case 66: return launch_e<false, true, 2, false, true>(a, st);   // codes in the NIB layout
    case 67: return launch_e<false, false, 2, false, true>(a, st);  // NIB, exact
    case 68: return launch_e<false, true, 2, false, false, true>(a, st);  // C^T epilogue
    case 69: return launch_e<false, true, 2, false, true, true>(a, st);   // NIB + C^T epilogue
    case 74: return launch_w<false>(a, st);   // 1 x 8 waves, hand-ordered stream
    case 72: {  // DIAGNOSTIC: 74 without the output stores (wrong results; epilogue cost)
      const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
      hipLaunchKernelGGL((k_w4a16_b32w<false, false, false, 9>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
      return hipGetLastError();
    }
    case 97: {  // 74 with the quad-transposed 8-B store epilogue (A/B)
      const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
      hipLaunchKernelGGL((k_w4a16_b32w<false, false, false, 2>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
      return hipGetLastError();
    }
    case 73: {  // 74 with the first epilogue (A/B)
      const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
      hipLaunchKernelGGL((k_w4a16_b32w<false, false, false, 1>), dim3((unsigned)blocks), dim3(THR), 0, st, a);
      return hipGetLastError();
    }
    case 75: return launch_w<true>(a, st);    // 1 x 8 waves, hand-ordered stream, NIB codes
    case 76: return launch_w4h<false, 2>(a, st);  // 2 x 2 waves of 128^2, register-staged, hand-ordered
    case 77: return launch_w4h<true, 2>(a, st);   // the same on NIB codes
    case 78: return launch_w4h<false, 1>(a, st);        // 1 x 4 waves of 256 x 64
    case 79: return launch_w4h<false, 2, true>(a, st);  // 2 x 2, LDS-DMA staging (3 stages)
    case 70: return launch_v<false>(a, st);             // 2 x 4 waves, hand-ordered stream
    case 71: return launch_v<true>(a, st);              // the same on NIB codes
    case 98: return launch_h2v<false>(a, st);           // 2 x 2 waves of 128 x 64, 256 x 128 tiles, 2 WGs / CU
    case 99: return launch_h2v<true>(a, st);            // the same on NIB codes
    case 80: return launch_w4b<false>(a, st);           // 2 x 2, weights dequantized once into LDS
    case 81: return launch_w4b<true>(a, st);            // the same on NIB codes
    default: return launch_w<false>(a, st);
  }
#else
  return hipErrorInvalidValue;  // A/B variants: IWQ_AB builds only
#endif
}

}  // namespace iwq

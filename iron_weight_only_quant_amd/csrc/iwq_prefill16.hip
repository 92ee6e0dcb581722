// iwq_prefill16.hip — the prefill (large M) fused dequant -> GEMM of iwq_prefill.hip's 74
// (k_w4a16_b32w) on the 16x16x32 f16 MFMA instead of 32x32x16.
//
// Replaces QuantLinear.forward = F.linear(x, W_deq, b) (quant_linear.py:960-972) for weights held
// packed (include/iwq.h layout), per channel: y = RN16(s * sum_k x (q - z) + b).
//
// Why a second MFMA shape: both shapes do the same FLOP per cycle, but under load the chip holds a
// higher clock on the 16x16x32 loop (MI355X_MICROARCH.md 'DVFS give-back' item 7: ~1.12-1.15x the
// FLOP/s on random data with every operand re-read from LDS; hipBLASLt's own kernel for these
// shapes is MT256x256x64_MI16x16).  74's structure is kept: 256 x 256 tile per 512-thread workgroup,
// 8 waves as 1 (M) x 8 (N) so each weight is dequantized once per workgroup; a wave owns 256 rows x
// 32 columns = 16 x 2 tiles of 16x16; K-steps of 64 staged by LDS-DMA into a ring; one raw
// s_barrier per K-step placed early (its wait covers only reads that are already in registers).
//
// k order: MFMA slice s (0, 1) of a K-step gives lane group g = lane >> 4 the logical
// k = 16 g + 8 s + [0, 8) -- the same permutation on both operands -- so a lane's codes for the whole
// K-step are 8 contiguous bytes of its column (one ds_read_b64 per 16-column tile) and its A fragment
// of slice s is one 16-B piece of its X row.
// LDS images (the DMA writes lane-linearly; swizzles are applied to the per-lane SOURCE address):
//   X rows of 128 B, 16-B chunk c of row r at c ^ h(r), h(r) = ((r >> 1) & 1) | (((r >> 3) & 1) * 6):
//     a ds_read_b128 lane group reads 16 rows, 8 of them at chunk c and 8 at chunk c ^ 2 (lanes
//     0-3 / 12-15 vs 4-11 of a 16-row tile), and h makes the 16 (row, chunk) slots distinct.
//   codes: columns of 32 B, 16-B chunk c of column n at c ^ ((n >> 3) & 1) (74's image); the b64
//     read of unit g (bytes 8 g .. 8 g + 7) hits 32 distinct dword pairs per 32 lanes.
// STAGGER (4-slot ring, 160 KiB): waves 4-7 run half a K-step (16 MFMA pairs) behind waves 0-3 --
// their barrier sits between pairs 7 and 8 of slice 0, the others' between pairs 7 and 8 of slice 1
// -- so the two waves sharing a SIMD do not reach their DMA issue, code reads and barrier together
// (MI355X_MICROARCH.md 'Two waves per SIMD' item 9).  A slot is then refilled one barrier later
// (after every wave has left it), hence the fourth slot.
#include "iwq_common.cuh"
#include "iwq_prefill.h"

namespace iwq {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int TM = 256, TN = 256, TK = 64, THR = 512;
constexpr int XS = TM * TK * 2;  // X bytes per stage (32 KiB)
constexpr int CS = TN * TK / 2;  // code bytes per stage (8 KiB)
constexpr int PS = 2 * TN * 4;   // grouped: 256 scales + 256 zero points, one dword each (2 KiB)

__device__ __forceinline__ int xh(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) * 6); }
__device__ __forceinline__ int cswz(int n) { return (n >> 3) & 1; }

// row-major dequant (after a v_perm_b32): inline asm, the schedule measured best for 151
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t mask_s, uint32_t magic_v) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(mask_s), "v"(magic_v));
  return r;
}
// NIB dequant: the same instruction left to the compiler (it then tracks the hazard to the
// following v_pk_add instead of padding every inline-asm result with s_nop: 172 -0.7...-1.5 %,
// profiles/r04_ab_lib_and_or.jsonl)
__device__ __forceinline__ uint32_t and_or_c(uint32_t x, uint32_t mask_s, uint32_t magic_v) {
  return (x & mask_s) | magic_v;
}

__device__ __forceinline__ int64_t swizzled_block(int64_t bid, int64_t nblocks) {
  const int64_t xcd = bid % 8, i = bid / 8;
  const int64_t q = nblocks / 8, r = nblocks % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
}

__device__ __forceinline__ void glds16(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
// 2-byte LDS-DMA: lane l's halfword lands in dword l of the wave's 256-B slot
__device__ __forceinline__ void glds2(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 2, 0, 0);
}

template <int OFF>
__device__ __forceinline__ h8 lds_rd(uint32_t addr) {
  h8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ u32x2 lds_rd2(uint32_t addr) {
  u32x2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
// two dwords 64 B apart (grouped: the parameters of a lane's two columns)
__device__ __forceinline__ u32x2 lds_rd_pair(uint32_t addr) {
  u32x2 v;
  asm volatile("ds_read2_b32 %0, %1 offset0:0 offset1:16" : "=v"(v) : "v"(addr));
  return v;
}
// re-defines v after its wait (see iwq_prefill.hip: keeps post-wait uses below the wait)
template <class T>
__device__ __forceinline__ void landed(T& v) {
  asm volatile("" : "+v"(v));
}

// grouped parameters from their raw dwords (the halfword in bits 0-15): the value in both halves
// (one v_perm), and the zero point's dequant offsets 1024 + z / 64 + z as packed fp16 adds (one
// rounding, as the float sum's conversion) -- 5 VALU per column instead of a float round trip each
__device__ __forceinline__ h2 bcast_lo(uint32_t v) { return as_h2(__builtin_amdgcn_perm(v, v, 0x01000100u)); }
__device__ __forceinline__ void zero_offsets(h2 z2, h2& zz, h2& zl, h2& zh) {
  zz = z2 + h2{(_Float16)1024.0f, (_Float16)64.0f};
  zl = z2 + h2{(_Float16)1024.0f, (_Float16)1024.0f};
  zh = z2 + h2{(_Float16)64.0f, (_Float16)64.0f};
}
// K-step -> its parameter group ((kt * TK) / group, group % TK == 0) by a multiply-high, not a
// division per DMA issue (exact while kt * group / TK < 2^32)
struct KStepGroup {
  uint32_t d, mul;
  __device__ explicit KStepGroup(int group) : d((uint32_t)group / TK), mul(0xFFFFFFFFu / ((uint32_t)group / TK) + 1u) {}
  __device__ int operator()(int kt) const { return d == 1 ? kt : (int)__umulhi((uint32_t)kt, mul); }
};

#define IWQ_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define IWQ_PIN() __builtin_amdgcn_sched_barrier(0)

// NIB: codes in the NIB layout (iwq_nib_codes: nibble p of a code dword holds k offset
// (0, 2, 4, 6, 1, 3, 5, 7)[p]) -- 9 instead of 12 VALU per 8 weights, the same (q - z) values, so
// the same bits as the row-major form
// LAG (A/B): the staggered waves' barrier sits 16 MFMA pairs (half a K-step) or 8 pairs before the
// others'; PRIO (A/B): static s_setprio 1 for waves 4-7 (1) or 0-3 (2) (cdna_hip_programming.md T5)
// GROUPED (group % 64 == 0): each K-step lies in one group, so a lane needs one (s, z) per column per
// K-step; they ride with the stage (a sixth DMA piece per wave: the parameter image of iwq_prefill.hip's
// 74) and the dequant applies s per weight, RN16((q - z) s) -- the reference's fp16 weight -- with no
// epilogue scale.  Its stage is 42 KiB, so the staggered ring has 3 slots: a slot is refilled with the
// K-step two ahead (AHEAD = 2), the barrier then waits for every piece this wave issued (vmcnt(0)), and
// the late waves issue right after their own barrier (EARLY_ISSUE) for a full K-step of DMA lead.
// NOSTORE: DIAGNOSTIC (wrong results): the epilogue computes but stores almost nothing (its cost)
template <bool STAGGER, bool NIB = false, int LAG = 16, int PRIO = 0, bool GROUPED = false, bool EARLY_ISSUE = false,
          bool NOSTORE = false>
__global__ __launch_bounds__(THR) void k_w4a16_b16w(PrefillArgs a) {
  static_assert(LAG == 16 || LAG == 8, "barrier between pairs 7/8 or after pair 15 of slice 0");
  static_assert(!EARLY_ISSUE || STAGGER, "only the staggered waves issue early");
  constexpr int STAGE = XS + CS + (GROUPED ? PS : 0);
  constexpr int PIECES = GROUPED ? 6 : 5;                  // DMA pieces per wave per K-step
  constexpr int NST = (STAGGER && !GROUPED) ? 4 : 3;       // ring slots (160 / 126 / 120 KiB)
  constexpr int AHEAD = STAGGER ? NST - 1 : 3;             // K-step distance of a refill
  // vmcnt at a barrier: this wave's pieces of the stage being published have landed; the pieces of
  // K-steps issued after it (AHEAD - 2 of them) may still fly
  constexpr int VM_AHEAD = (AHEAD - 2) * PIECES;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NST * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool late = STAGGER && wid >= 4;  // wave-uniform: waves 4-7 run half a K-step behind
  const int r16 = lane & 15, g = lane >> 4;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int64_t crow = a.K / 2;
  const int nk = a.K / TK;

  // DMA sources: X rows (wid * 4 + i) * 8 + lane / 8, 16-B chunk lane % 8 from chunk (lane % 8) ^ h;
  // codes: column wid * 32 + lane / 2, chunk lane % 2 from chunk (lane % 2) ^ cswz
  const _Float16* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xh(row)) << 3);
  }
  const int ccol = wid * 32 + (lane >> 1);
  const uint8_t* csrc = a.codes + (int64_t)(n0 + ccol) * crow + (((lane & 1) ^ cswz(ccol)) << 4);
  // grouped: waves 0-3 stage the scales of columns 64 (wid & 3) + lane, waves 4-7 the zero points
  // (dword c of the parameter image: scale of column c; dword 256 + c: its zero point)
  const _Float16* psrc = nullptr;
  if constexpr (GROUPED) {
    const _Float16* arr = (wid < 4 || !a.zeros) ? a.scales : a.zeros;
    const int64_t c = n0 + (wid & 3) * 64 + lane;
    psrc = arr + (a.pgm ? c : c * a.gpr);
  }
  const int64_t pstep = a.pgm ? a.N : 1;  // parameter stride between groups
  const KStepGroup kgrp(GROUPED ? a.group : TK);
  auto issue1 = [&](int kt, int stg, int i) {
    uint8_t* base = smem + stg * STAGE;
    if (i < 4) glds16(xsrc[i] + kt * TK, base + (wid * 4 + i) * 1024);
    else if (i == 4) glds16(csrc + kt * (TK / 2), base + XS + wid * 1024);
    else if constexpr (GROUPED) glds2(psrc + kgrp(kt) * pstep, base + XS + CS + wid * 256);
  };
  auto issue = [&](int kt, int stg) {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) issue1(kt, stg, i);
  };

  // this lane's two columns (16-column tiles 0, 1 of the wave) and their parameters
  const int col0 = n0 + wid * 32 + r16;
  float sfl[2] = {1.0f, 1.0f};
  h2 s2[2], zz[2], zl[2], zh[2];
  const h2 zsym2 = {(_Float16)a.zsym, (_Float16)a.zsym};
  auto set_zero = [&](int nt, float zf) {
    zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  };
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int col = col0 + 16 * nt;
      sfl[nt] = (float)gp<_Float16>(a.scales)[col];
      set_zero(nt, a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym);
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  // LDS byte addresses: A fragment (stage st, slice s, tile mt) = la[s] + st * STAGE + 2048 mt;
  // codes of tile nt = lc + st * STAGE + 512 nt
  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) la[s] = lbase + (uint32_t)(r16 * 128 + (((2 * g + s) ^ xh(r16)) << 4));
  const int ccl = wid * 32 + r16;
  const uint32_t lc = lbase + XS + (uint32_t)(ccl * 32 + (((g >> 1) ^ cswz(ccl)) << 4) + ((g & 1) << 3));
  const uint32_t lps = lbase + XS + CS + (uint32_t)(ccl * 4);  // grouped: scales of col0, col0 + 16
  const uint32_t lpz = lps + TN * 4;                           // grouped: their zero points
  u32x2 psv{}, pzv{};                                          // grouped: the raw parameter dwords
  auto params_landed = [&]() {
    if constexpr (GROUPED) {
      landed(psv);
      landed(pzv);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        s2[nt] = bcast_lo(psv[nt]);
        zero_offsets(a.zeros ? bcast_lo(pzv[nt]) : zsym2, zz[nt], zl[nt], zh[nt]);
      }
    }
  };

  // weight pair j (k offsets 2j, 2j + 1) of code dword w, tile nt: (q - z) exactly (3 VALU; NIB:
  // 2, plus one shift per dword for pairs 2 and 3)
  auto dqp = [&](uint32_t w, int j, int nt) -> h2 {
    h2 d;
    if constexpr (NIB) {
      const uint32_t t = j >= 2 ? w >> 8 : w;
      d = (j & 1) ? as_h2(and_or_c(t, m1_s, mg54)) - zh[nt] : as_h2(and_or_c(t, m0_s, mg64)) - zl[nt];
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      d = as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz[nt];
    }
    if constexpr (GROUPED) d = d * s2[nt];  // RN16((q - z) s)
    return d;
  };
  auto frag = [](const h2* p) -> h8 { return h8{p[0].x, p[0].y, p[1].x, p[1].y, p[2].x, p[2].y, p[3].x, p[3].y}; };

  f4 acc[16][2];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 af[8];
  h8 b0, b1;    // B fragments of the running slice (tiles 0, 1)
  u32x2 wc0, wc1;  // the running K-step's code dwords (tile 0, 1): .x slice 0, .y slice 1

#define IWQ_RD(MT, ADDR) af[(MT) & 7] = lds_rd<((MT) & 15) * 2048>(ADDR)
#define IWQ_MF2(MT)                                                                        \
  acc[MT][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[(MT) & 7], b0, acc[MT][0], 0, 0, 0); \
  acc[MT][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[(MT) & 7], b1, acc[MT][1], 0, 0, 0)
  // pair MT of a slice: its two MFMAs, then the rolling read 8 pairs ahead (READ), VALU work (DQ)
#define IWQ_PAIR(MT, WAIT, READ, DQ) \
  {                                  \
    if (WAIT) IWQ_LGKM(7);           \
    IWQ_PIN();                       \
    IWQ_MF2(MT);                     \
    READ;                            \
    DQ;                              \
    IWQ_PIN();                       \
  }

  // slice 0 of a K-step (stage offset SO): rolling reads of frags 8..15 of slice 0 and 0..7 of
  // slice 1; slice 1's B fragments (the same code dwords' .y) dequantized on the way, one weight pair
  // per MFMA pair; MID runs between pairs 7 and 8, END after pair 15 (the staggered waves' barrier)
#define IWQ_SLICE0(SO, MID, END, ISS)                                                     \
  {                                                                                       \
    const uint32_t a0 = la[0] + (SO), a1 = la[1] + (SO);                                  \
    h2 p[8];                                                                              \
    IWQ_PAIR(0, true, IWQ_RD(8, a0), p[0] = dqp(wc0.y, 0, 0));                            \
    IWQ_PAIR(1, true, IWQ_RD(9, a0), p[1] = dqp(wc0.y, 1, 0));                            \
    IWQ_PAIR(2, true, IWQ_RD(10, a0), p[2] = dqp(wc0.y, 2, 0));                           \
    IWQ_PAIR(3, true, IWQ_RD(11, a0), p[3] = dqp(wc0.y, 3, 0));                           \
    IWQ_PAIR(4, true, IWQ_RD(12, a0), p[4] = dqp(wc1.y, 0, 1));                           \
    IWQ_PAIR(5, true, IWQ_RD(13, a0), p[5] = dqp(wc1.y, 1, 1));                           \
    IWQ_PAIR(6, true, IWQ_RD(14, a0), p[6] = dqp(wc1.y, 2, 1));                           \
    IWQ_PAIR(7, true, IWQ_RD(15, a0), p[7] = dqp(wc1.y, 3, 1));                           \
    MID;                                                                                  \
    IWQ_PAIR(8, true, IWQ_RD(0, a1), ISS(0));                                             \
    IWQ_PAIR(9, true, IWQ_RD(1, a1), ISS(1));                                             \
    IWQ_PAIR(10, true, IWQ_RD(2, a1), ISS(2));                                            \
    IWQ_PAIR(11, true, IWQ_RD(3, a1), ISS(3));                                            \
    IWQ_PAIR(12, true, IWQ_RD(4, a1), ISS(4));                                            \
    IWQ_PAIR(13, true, IWQ_RD(5, a1), ISS(5));                                            \
    IWQ_PAIR(14, true, IWQ_RD(6, a1), );                                                  \
    IWQ_PAIR(15, true, IWQ_RD(7, a1), );                                                  \
    END;                                                                                  \
    b0 = frag(p);                                                                         \
    b1 = frag(p + 4);                                                                     \
  }

  // prologue: K-steps 0 .. AHEAD - 1 into slots 0 .. AHEAD - 1 (clamped to nk - 1: re-loads nobody
  // reads again); the loop's K-step kt refills the next slot with K-step kt + AHEAD
  issue(0, 0);
  issue(nk > 1 ? 1 : 0, 1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (AHEAD == 3) issue(nk > 2 ? 2 : nk - 1, 2);
  IWQ_PIN();
  wc0 = lds_rd2<0>(lc);
  wc1 = lds_rd2<512>(lc);
  if constexpr (GROUPED) {
    psv = lds_rd_pair(lps);
    pzv = lds_rd_pair(lpz);
  }
  IWQ_RD(0, la[0]); IWQ_RD(1, la[0]); IWQ_RD(2, la[0]); IWQ_RD(3, la[0]);
  IWQ_RD(4, la[0]); IWQ_RD(5, la[0]); IWQ_RD(6, la[0]); IWQ_RD(7, la[0]);
  IWQ_LGKM(0);
  landed(wc0);
  landed(wc1);
  params_landed();
  IWQ_PIN();
  {
    h2 p[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] = dqp(wc0.x, j, 0);
      p[4 + j] = dqp(wc1.x, j, 1);
    }
    b0 = frag(p);
    b1 = frag(p + 4);
  }

  if constexpr (PRIO == 1) {
    if (late) __builtin_amdgcn_s_setprio(1);
  } else if constexpr (PRIO == 2) {
    if (STAGGER && !late) __builtin_amdgcn_s_setprio(1);
  }
  // the last K-step is peeled (a branch in the body made the compiler keep two register images)
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt % NST) * STAGE);
    const uint32_t sn = (uint32_t)(((kt + 1) % NST) * STAGE);
    // the slot refilled in this K-step and the K-step it receives (clamped: re-loads nobody reads)
    const int sd = STAGGER ? (kt + NST - 1) % NST : kt % NST;
    const int kd = kt + AHEAD < nk ? kt + AHEAD : nk - 1;
    // waves 4-7 (STAGGER): their barrier between pairs 7 and 8 of slice 0, 16 MFMA pairs before the
    // others' -- stage kt + 1 published; the slot a DMA may refill before the next barrier holds
    // stage kt - 1, whose reads this wave retired in K-step kt - 1
    // (EARLY_ISSUE: their refill right after it, pairs 8.. of slice 0)
#define IWQ_ISS_LATE(I) \
  if (EARLY_ISSUE && late && (I) < PIECES) issue1(kd, sd, I)
    IWQ_SLICE0(so, if (LAG == 16 && late) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_AHEAD) : "memory");
      __builtin_amdgcn_s_barrier();
    }, if (LAG == 8 && late) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_AHEAD) : "memory");
      __builtin_amdgcn_s_barrier();
    }, IWQ_ISS_LATE)
#undef IWQ_ISS_LATE
    // slice 1: pairs 0..7 read frags 8..15 of slice 1; pairs 8..15 read the next K-step's slice-0
    // frags 0..7 (after the barrier that publishes it), its codes, and issue this K-step's refill
    const uint32_t a1 = la[1] + so;
    IWQ_PAIR(0, true, IWQ_RD(8, a1), );
    IWQ_PAIR(1, true, IWQ_RD(9, a1), );
    IWQ_PAIR(2, true, IWQ_RD(10, a1), );
    IWQ_PAIR(3, true, IWQ_RD(11, a1), );
    IWQ_PAIR(4, true, IWQ_RD(12, a1), );
    IWQ_PAIR(5, true, IWQ_RD(13, a1), );
    IWQ_PAIR(6, true, IWQ_RD(14, a1), );
    IWQ_PAIR(7, true, IWQ_RD(15, a1), );
    if (!late) {
      // waves 0-3 (all waves without STAGGER): stage kt + 1 landed (this wave's part), and -- 3-slot
      // ring -- every read of stage kt retired (its slot is refilled right after)
      if constexpr (STAGGER) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_AHEAD) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(VM_AHEAD) : "memory");
      __builtin_amdgcn_s_barrier();
    }
    if constexpr (STAGGER) IWQ_LGKM(0);  // frags 8..15 of slice 1 in registers
    IWQ_PIN();
    // codes of stage kt + 1 (oldest of what follows), then the rolling reads of its slice 0
    u32x2 wn0 = lds_rd2<0>(lc + sn);
    u32x2 wn1 = lds_rd2<512>(lc + sn);
    if constexpr (GROUPED) {  // older than the 4 A reads below: retired by the same lgkmcnt(4)
      psv = lds_rd_pair(lps + sn);
      pzv = lds_rd_pair(lpz + sn);
    }
    const uint32_t na = la[0] + sn;
    const bool iss = !(EARLY_ISSUE && late);  // wave-uniform
    IWQ_PAIR(8, false, IWQ_RD(0, na), if (iss) issue1(kd, sd, 0));
    IWQ_PAIR(9, false, IWQ_RD(1, na), if (iss) issue1(kd, sd, 1));
    IWQ_PAIR(10, false, IWQ_RD(2, na), if (iss) issue1(kd, sd, 2));
    IWQ_PAIR(11, false, IWQ_RD(3, na), if (iss) issue1(kd, sd, 3));
    IWQ_LGKM(4);  // the code (and parameter) reads, older than the 4 A reads above, landed
    landed(wn0);
    landed(wn1);
    params_landed();
    h2 p[8];
    IWQ_PAIR(12, false, IWQ_RD(4, na), if (iss) issue1(kd, sd, 4); p[0] = dqp(wn0.x, 0, 0); p[1] = dqp(wn0.x, 1, 0));
    IWQ_PAIR(13, false, IWQ_RD(5, na), if (iss && GROUPED) issue1(kd, sd, 5); p[2] = dqp(wn0.x, 2, 0); p[3] = dqp(wn0.x, 3, 0));
    IWQ_PAIR(14, false, IWQ_RD(6, na), p[4] = dqp(wn1.x, 0, 1); p[5] = dqp(wn1.x, 1, 1));
    IWQ_PAIR(15, false, IWQ_RD(7, na), p[6] = dqp(wn1.x, 2, 1); p[7] = dqp(wn1.x, 3, 1));
    b0 = frag(p);
    b1 = frag(p + 4);
    wc0 = wn0;
    wc1 = wn1;
  }
  {
    // the last K-step: no next stage, no barrier
    const uint32_t so = (uint32_t)(((nk - 1) % NST) * STAGE);
#define IWQ_NOP(I)
    IWQ_SLICE0(so, , , IWQ_NOP)
#undef IWQ_NOP
    const uint32_t a1 = la[1] + so;
    IWQ_PAIR(0, true, IWQ_RD(8, a1), );
    IWQ_PAIR(1, true, IWQ_RD(9, a1), );
    IWQ_PAIR(2, true, IWQ_RD(10, a1), );
    IWQ_PAIR(3, true, IWQ_RD(11, a1), );
    IWQ_PAIR(4, true, IWQ_RD(12, a1), );
    IWQ_PAIR(5, true, IWQ_RD(13, a1), );
    IWQ_PAIR(6, true, IWQ_RD(14, a1), );
    IWQ_PAIR(7, true, IWQ_RD(15, a1), );
    IWQ_LGKM(0);
    IWQ_PIN();
    IWQ_MF2(8); IWQ_MF2(9); IWQ_MF2(10); IWQ_MF2(11);
    IWQ_MF2(12); IWQ_MF2(13); IWQ_MF2(14); IWQ_MF2(15);
  }
  // no LDS-DMA may still be landing when the workgroup retires (the CU's next workgroup owns the LDS)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_SLICE0
#undef IWQ_PAIR
#undef IWQ_MF2
#undef IWQ_RD

  // epilogue: lane holds rows 16 mt + 4 g + r of columns col0, col0 + 16
  const float bc0 = a.bias ? (float)gp<_Float16>(a.bias)[col0] : 0.0f;
  const float bc1 = a.bias ? (float)gp<_Float16>(a.bias)[col0 + 16] : 0.0f;
  const int64_t ld2 = __builtin_amdgcn_readfirstlane((int)a.ldy) * (int64_t)2;  // row pitch, bytes
  char* yl = reinterpret_cast<char*>(a.y) + ((int64_t)(m0 + 4 * g) * a.ldy + col0) * 2;
  const bool full = m0 + TM <= a.M;
#pragma unroll
  for (int mt = 0; mt < 16; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = mt * 16 + r;
      if constexpr (NOSTORE) {
        if (acc[mt][0][r] == 1.2345e-30f || acc[mt][1][r] == 1.2345e-30f) {
          auto p = gp<_Float16>(static_cast<void*>(yl + (int64_t)rr * ld2));
          p[0] = (_Float16)(opaque(acc[mt][0][r] * sfl[0]) + bc0);
          p[16] = (_Float16)(opaque(acc[mt][1][r] * sfl[1]) + bc1);
        }
      } else if (full || m0 + rr + 4 * g < a.M) {
        auto p = gp<_Float16>(static_cast<void*>(yl + (int64_t)rr * ld2));
        if constexpr (GROUPED) {
          p[0] = (_Float16)(acc[mt][0][r] + bc0);
          p[16] = (_Float16)(acc[mt][1][r] + bc1);
        } else {
          p[0] = (_Float16)(opaque(acc[mt][0][r] * sfl[0]) + bc0);
          p[16] = (_Float16)(opaque(acc[mt][1][r] * sfl[1]) + bc1);
        }
      }
    }
}

// k_w4a16_b16q: one wave per SIMD.  4 waves (256 threads), the same 256 x 256 tile; wave w owns all
// 256 rows x columns 64 w .. 64 w + 63 = 16 x 4 tiles of 16x16, so each A fragment feeds FOUR MFMAs
// (b16w: two) and the LDS reads per MFMA halve -- b16w's 8 waves read 256 KiB of A per K-step per CU
// (~1024 of the 2048 LDS-array cycles the K-step's MFMAs take at 256 B/clk); here 128 KiB.  Each
// weight is still dequantized once per workgroup (one pair of 2 per group of four MFMAs).  The 256
// accumulators per lane sit in AGPRs (hipBLASLt's MT256x256x64_MI16x16 kernel for these shapes runs the
// same one-wave-per-SIMD shape).
// Rings: X in 4 slots of 32 KiB, codes (+ grouped parameters) in 3 slots of 8 (10) KiB: 152 (158) KiB.
// The barrier sits early in slice 1 (after the group that consumes fragment 3) and publishes the next
// stage; after it the X slot of the stage before the running one and the code slot of the running
// one (its codes were read a K-step ago) are refilled with K-step kt + 3.
// Per K-step and wave: slice 0 -- 16 groups of (wait, 4 MFMAs, rolling A read 4 fragments ahead, one
// weight pair of slice 1's B); slice 1 -- groups 0-3, the barrier, the next stage's codes (and
// parameters), the DMA pieces spread one per group from group 4, the next stage's slice-0 B
// dequantized over groups 8-15.
// IL: the work of a group (rolling read, DMA piece, dequant pairs) placed between its four MFMAs (one
// slot after each) instead of after the fourth, so the MFMA pipe is not left idle while one wave
// issues it.
// GROUPED (group % 64 == 0): one (s, z) per column per K-step, staged with the codes (b16w's parameter
// image), applied per weight (RN16((q - z) s)), no epilogue scale.
// DIAG (DIAGNOSTIC, wrong results): 1 = no barrier in the loop (its cost), 2 = no dequant VALU (the
// code dwords go to the MFMA as they are)
template <bool NIB, bool IL = false, bool GROUPED = false, int DIAG = 0>
__global__ __launch_bounds__(256) void k_w4a16_b16q(PrefillArgs a) {
  constexpr int NSX = 4, NSC = 3;             // X / code ring slots
  constexpr int CST = CS + (GROUPED ? PS : 0);  // code slot bytes
  constexpr int CBASE = NSX * XS;             // code ring offset (128 KiB)
  constexpr int PIECES = GROUPED ? 12 : 10;   // DMA pieces per wave per K-step: 8 X, 2 codes, 2 parameters
  constexpr int VM_AHEAD = PIECES;  // at a barrier the pieces of the K-step after the published one fly
  constexpr int NCR = GROUPED ? 8 : 4;  // LDS reads of a stage's codes (+ parameters)
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSX * XS + NSC * CST];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int64_t crow = a.K / 2;
  const int nk = a.K / TK;

  // DMA sources: X rows (wid * 8 + i) * 8 + lane / 8, 16-B chunk lane % 8 from chunk (lane % 8) ^ h;
  // codes: column wid * 64 + 32 j + lane / 2, chunk lane % 2 from chunk (lane % 2) ^ cswz; grouped:
  // the scale and zero point of column wid * 64 + lane (dword c / 256 + c of the parameter image)
  const _Float16* xsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = (wid * 8 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xh(row)) << 3);
  }
  const uint8_t* csrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ccol = wid * 64 + 32 * j + (lane >> 1);
    csrc[j] = a.codes + (int64_t)(n0 + ccol) * crow + (((lane & 1) ^ cswz(ccol)) << 4);
  }
  const _Float16* psrc[2] = {nullptr, nullptr};
  int64_t pstep = 1;
  const KStepGroup kgrp(GROUPED ? a.group : TK);
  if constexpr (GROUPED) {
    const int64_t c = n0 + wid * 64 + lane;
    const int64_t off = a.pgm ? c : c * a.gpr;
    psrc[0] = a.scales + off;
    psrc[1] = (a.zeros ? a.zeros : a.scales) + off;
    pstep = a.pgm ? a.N : 1;
  }
  // piece i of K-step kt into X slot xs / code slot cs
  auto issue1 = [&](int kt, int xs, int cs, int i) {
    if (i < 8) {
      glds16(xsrc[i] + kt * TK, smem + xs * XS + (wid * 8 + i) * 1024);
    } else if (i < 10) {
      glds16(csrc[i - 8] + kt * (TK / 2), smem + CBASE + cs * CST + (wid * 2 + i - 8) * 1024);
    } else if constexpr (GROUPED) {
      glds2(psrc[i - 10] + kgrp(kt) * pstep, smem + CBASE + cs * CST + CS + (i - 10) * 1024 + wid * 256);
    }
  };
  auto issue = [&](int kt, int s) {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) issue1(kt, s, s, i);
  };

  // this lane's four columns (16-column tiles 0..3 of the wave) and their parameters
  const int col0 = n0 + wid * 64 + r16;
  float sfl[4] = {1.0f, 1.0f, 1.0f, 1.0f};
  h2 s2[4], zz[4], zl[4], zh[4];
  const h2 zsym2 = {(_Float16)a.zsym, (_Float16)a.zsym};
  auto set_zero = [&](int nt, float zf) {
    zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  };
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = col0 + 16 * nt;
      sfl[nt] = (float)gp<_Float16>(a.scales)[col];
      set_zero(nt, a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym);
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  // LDS byte addresses: A fragment (X slot st, slice s, tile mt) = la[s] + st * XS + 2048 mt;
  // codes of tile nt (code slot st) = lc + st * CST + 512 nt; grouped: scales of tiles (0, 1) / (2, 3)
  // at lps / lps + 128, zero points 1 KiB on
  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) la[s] = lbase + (uint32_t)(r16 * 128 + (((2 * g + s) ^ xh(r16)) << 4));
  const int ccl = wid * 64 + r16;
  const uint32_t lc = lbase + CBASE + (uint32_t)(ccl * 32 + (((g >> 1) ^ cswz(ccl)) << 4) + ((g & 1) << 3));
  const uint32_t lps = lbase + CBASE + CS + (uint32_t)(ccl * 4);
  u32x2 pv[4];  // grouped: raw parameter dwords (scales of tiles 0/1, 2/3; zero points of 0/1, 2/3)
  auto set_params = [&](int nt) {
    if constexpr (GROUPED) {
      s2[nt] = bcast_lo(pv[nt >> 1][nt & 1]);
      zero_offsets(a.zeros ? bcast_lo(pv[2 + (nt >> 1)][nt & 1]) : zsym2, zz[nt], zl[nt], zh[nt]);
    }
  };
  // the code (+ parameter) reads of code slot offset CO into W / pv, in this order
  auto read_codes = [&](u32x2* w, uint32_t co) {
    w[0] = lds_rd2<0>(lc + co);
    w[1] = lds_rd2<512>(lc + co);
    w[2] = lds_rd2<1024>(lc + co);
    w[3] = lds_rd2<1536>(lc + co);
    if constexpr (GROUPED) {
      pv[0] = lds_rd_pair(lps + co);
      pv[1] = lds_rd_pair(lps + co + 128);
      pv[2] = lds_rd_pair(lps + co + 1024);
      pv[3] = lds_rd_pair(lps + co + 1152);
    }
  };
  auto codes_landed = [&](u32x2* w) {
    landed(w[0]);
    landed(w[1]);
    landed(w[2]);
    landed(w[3]);
    if constexpr (GROUPED) {
      landed(pv[0]);
      landed(pv[1]);
      landed(pv[2]);
      landed(pv[3]);
    }
  };

  auto dqp = [&](uint32_t w, int j, int nt) -> h2 {
    h2 d;
    if constexpr (DIAG == 2) {
      return as_h2(j & 1 ? w >> 1 : w);
    } else if constexpr (NIB) {
      const uint32_t t = j >= 2 ? w >> 8 : w;
      d = (j & 1) ? as_h2(and_or_c(t, m1_s, mg54)) - zh[nt] : as_h2(and_or_c(t, m0_s, mg64)) - zl[nt];
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      d = as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz[nt];
    }
    if constexpr (GROUPED) d = d * s2[nt];  // RN16((q - z) s)
    return d;
  };
  auto frag = [](const h2* p) -> h8 { return h8{p[0].x, p[0].y, p[1].x, p[1].y, p[2].x, p[2].y, p[3].x, p[3].y}; };

  f4 acc[16][4];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 af[8];
  h8 b0[4], b1[4];  // B fragments of slice 0 / 1 (tiles 0..3)
  u32x2 wc[4];      // the running K-step's code dwords per tile: .x slice 0, .y slice 1

#define IWQ_RD(MT, ADDR) af[(MT) & 7] = lds_rd<((MT) & 15) * 2048>(ADDR)
#define IWQ_LGKMN(N) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory")
#define IWQ_MF1(MT, NT, B) \
  acc[MT][NT] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[(MT) & 7], B[NT], acc[MT][NT], 0, 0, 0)
  // group MT of a slice: the wait for its fragment (N newer LDS reads may stay in flight), its four
  // MFMAs and the work slots W0..W3 (in this order; IL: W_i right after MFMA i)
#define IWQ_GRP(MT, N, B, W0, W1, W2, W3) \
  {                                       \
    IWQ_LGKMN(N);                         \
    IWQ_PIN();                            \
    if constexpr (IL) {                   \
      IWQ_MF1(MT, 0, B);                  \
      W0;                                 \
      IWQ_PIN();                          \
      IWQ_MF1(MT, 1, B);                  \
      W1;                                 \
      IWQ_PIN();                          \
      IWQ_MF1(MT, 2, B);                  \
      W2;                                 \
      IWQ_PIN();                          \
      IWQ_MF1(MT, 3, B);                  \
      W3;                                 \
    } else {                              \
      IWQ_MF1(MT, 0, B);                  \
      IWQ_MF1(MT, 1, B);                  \
      IWQ_MF1(MT, 2, B);                  \
      IWQ_MF1(MT, 3, B);                  \
      W0;                                 \
      W1;                                 \
      W2;                                 \
      W3;                                 \
    }                                     \
    IWQ_PIN();                            \
  }
  // slice 0 (X slot offset SO): rolling reads of fragments 4..15 of slice 0 and 0..3 of slice 1;
  // slice 1's B (the same code dwords' .y) dequantized one pair per group
#define IWQ_QSLICE0(SO)                                                     \
  {                                                                         \
    const uint32_t a0 = la[0] + (SO), a1 = la[1] + (SO);                    \
    h2 p[16];                                                               \
    IWQ_GRP(0, 3, b0, IWQ_RD(4, a0), p[0] = dqp(wc[0].y, 0, 0), , );         \
    IWQ_GRP(1, 3, b0, IWQ_RD(5, a0), p[1] = dqp(wc[0].y, 1, 0), , );         \
    IWQ_GRP(2, 3, b0, IWQ_RD(6, a0), p[2] = dqp(wc[0].y, 2, 0), , );         \
    IWQ_GRP(3, 3, b0, IWQ_RD(7, a0), p[3] = dqp(wc[0].y, 3, 0), , );         \
    IWQ_GRP(4, 3, b0, IWQ_RD(8, a0), p[4] = dqp(wc[1].y, 0, 1), , );         \
    IWQ_GRP(5, 3, b0, IWQ_RD(9, a0), p[5] = dqp(wc[1].y, 1, 1), , );         \
    IWQ_GRP(6, 3, b0, IWQ_RD(10, a0), p[6] = dqp(wc[1].y, 2, 1), , );        \
    IWQ_GRP(7, 3, b0, IWQ_RD(11, a0), p[7] = dqp(wc[1].y, 3, 1), , );        \
    IWQ_GRP(8, 3, b0, IWQ_RD(12, a0), p[8] = dqp(wc[2].y, 0, 2), , );        \
    IWQ_GRP(9, 3, b0, IWQ_RD(13, a0), p[9] = dqp(wc[2].y, 1, 2), , );        \
    IWQ_GRP(10, 3, b0, IWQ_RD(14, a0), p[10] = dqp(wc[2].y, 2, 2), , );      \
    IWQ_GRP(11, 3, b0, IWQ_RD(15, a0), p[11] = dqp(wc[2].y, 3, 2), , );      \
    IWQ_GRP(12, 3, b0, IWQ_RD(0, a1), p[12] = dqp(wc[3].y, 0, 3), , );       \
    IWQ_GRP(13, 3, b0, IWQ_RD(1, a1), p[13] = dqp(wc[3].y, 1, 3), , );       \
    IWQ_GRP(14, 3, b0, IWQ_RD(2, a1), p[14] = dqp(wc[3].y, 2, 3), , );       \
    IWQ_GRP(15, 3, b0, IWQ_RD(3, a1), p[15] = dqp(wc[3].y, 3, 3), , );       \
    b1[0] = frag(p);                                                        \
    b1[1] = frag(p + 4);                                                    \
    b1[2] = frag(p + 8);                                                    \
    b1[3] = frag(p + 12);                                                   \
  }

  // prologue: K-steps 0, 1, 2 into slots 0, 1, 2 of both rings (clamped to nk - 1: re-loads nobody
  // reads again)
  issue(0, 0);
  issue(nk > 1 ? 1 : 0, 1);
  issue(nk > 2 ? 2 : nk - 1, 2);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PIECES) : "memory");
  __builtin_amdgcn_s_barrier();
  IWQ_PIN();
  read_codes(wc, 0);
  IWQ_RD(0, la[0]); IWQ_RD(1, la[0]); IWQ_RD(2, la[0]); IWQ_RD(3, la[0]);
  IWQ_LGKM(0);
  codes_landed(wc);
  IWQ_PIN();
  {
    h2 p[16];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      set_params(nt);
#pragma unroll
      for (int j = 0; j < 4; ++j) p[4 * nt + j] = dqp(wc[nt].x, j, nt);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b0[nt] = frag(p + 4 * nt);
  }

  // the last K-step is peeled (a branch in the body made the compiler keep two register images)
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt % NSX) * XS);
    const uint32_t sn = (uint32_t)(((kt + 1) % NSX) * XS);
    const uint32_t cn = (uint32_t)(((kt + 1) % NSC) * CST);
    // after the barrier: X slot of stage kt - 1 and code slot of stage kt get K-step kt + 3 (clamped:
    // re-loads nobody reads)
    const int xd = (kt + 3) % NSX, cd = kt % NSC;
    const int kd = kt + 3 < nk ? kt + 3 : nk - 1;
    IWQ_QSLICE0(so)
    const uint32_t a1 = la[1] + so;
    const uint32_t na = la[0] + sn;
    IWQ_GRP(0, 3, b1, IWQ_RD(4, a1), , , );
    IWQ_GRP(1, 3, b1, IWQ_RD(5, a1), , , );
    IWQ_GRP(2, 3, b1, IWQ_RD(6, a1), , , );
    IWQ_GRP(3, 3, b1, IWQ_RD(7, a1), , , );
    // stage kt + 1 landed (this wave's part; K-step kt + 2's pieces may fly): publish it
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_AHEAD) : "memory");
    if constexpr (DIAG != 1) __builtin_amdgcn_s_barrier();
    IWQ_PIN();
    u32x2 wn[4];
    // the code (+ parameter) reads of stage kt + 1 are older than fragment 8's: NCR more reads in
    // flight at groups 5-7
    IWQ_GRP(4, 3, b1, read_codes(wn, cn), IWQ_RD(8, a1), issue1(kd, xd, cd, 0), );
    IWQ_GRP(5, 3 + NCR, b1, IWQ_RD(9, a1), issue1(kd, xd, cd, 1), , );
    IWQ_GRP(6, 3 + NCR, b1, IWQ_RD(10, a1), issue1(kd, xd, cd, 2), , );
    IWQ_GRP(7, 3 + NCR, b1, IWQ_RD(11, a1), issue1(kd, xd, cd, 3), , );
    h2 p[16];
    IWQ_LGKM(3);  // fragment 8 and everything older (the code reads) landed
    codes_landed(wn);
    IWQ_GRP(8, 3, b1, IWQ_RD(12, a1), issue1(kd, xd, cd, 4); set_params(0), p[0] = dqp(wn[0].x, 0, 0),
            p[1] = dqp(wn[0].x, 1, 0));
    IWQ_GRP(9, 3, b1, IWQ_RD(13, a1), issue1(kd, xd, cd, 5), p[2] = dqp(wn[0].x, 2, 0), p[3] = dqp(wn[0].x, 3, 0));
    IWQ_GRP(10, 3, b1, IWQ_RD(14, a1), issue1(kd, xd, cd, 6); set_params(1), p[4] = dqp(wn[1].x, 0, 1),
            p[5] = dqp(wn[1].x, 1, 1));
    IWQ_GRP(11, 3, b1, IWQ_RD(15, a1), issue1(kd, xd, cd, 7), p[6] = dqp(wn[1].x, 2, 1), p[7] = dqp(wn[1].x, 3, 1));
    IWQ_GRP(12, 3, b1, IWQ_RD(0, na), issue1(kd, xd, cd, 8); set_params(2), p[8] = dqp(wn[2].x, 0, 2),
            p[9] = dqp(wn[2].x, 1, 2));
    IWQ_GRP(13, 3, b1, IWQ_RD(1, na), issue1(kd, xd, cd, 9), p[10] = dqp(wn[2].x, 2, 2), p[11] = dqp(wn[2].x, 3, 2));
    IWQ_GRP(14, 3, b1, IWQ_RD(2, na), issue1(kd, xd, cd, 10); set_params(3), p[12] = dqp(wn[3].x, 0, 3),
            p[13] = dqp(wn[3].x, 1, 3));
    IWQ_GRP(15, 3, b1, IWQ_RD(3, na), issue1(kd, xd, cd, 11), p[14] = dqp(wn[3].x, 2, 3), p[15] = dqp(wn[3].x, 3, 3));
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      b0[nt] = frag(p + 4 * nt);
      wc[nt] = wn[nt];
    }
  }
  {
    // the last K-step: no next stage, no barrier
    const uint32_t so = (uint32_t)(((nk - 1) % NSX) * XS);
    IWQ_QSLICE0(so)
    const uint32_t a1 = la[1] + so;
    IWQ_GRP(0, 3, b1, IWQ_RD(4, a1), , , );
    IWQ_GRP(1, 3, b1, IWQ_RD(5, a1), , , );
    IWQ_GRP(2, 3, b1, IWQ_RD(6, a1), , , );
    IWQ_GRP(3, 3, b1, IWQ_RD(7, a1), , , );
    IWQ_GRP(4, 3, b1, IWQ_RD(8, a1), , , );
    IWQ_GRP(5, 3, b1, IWQ_RD(9, a1), , , );
    IWQ_GRP(6, 3, b1, IWQ_RD(10, a1), , , );
    IWQ_GRP(7, 3, b1, IWQ_RD(11, a1), , , );
    IWQ_GRP(8, 3, b1, IWQ_RD(12, a1), , , );
    IWQ_GRP(9, 3, b1, IWQ_RD(13, a1), , , );
    IWQ_GRP(10, 3, b1, IWQ_RD(14, a1), , , );
    IWQ_GRP(11, 3, b1, IWQ_RD(15, a1), , , );
    IWQ_GRP(12, 3, b1, , , , );
    IWQ_GRP(13, 2, b1, , , , );
    IWQ_GRP(14, 1, b1, , , , );
    IWQ_GRP(15, 0, b1, , , , );
  }
  // no LDS-DMA may still be landing when the workgroup retires (the CU's next workgroup owns the LDS)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_QSLICE0
#undef IWQ_GRP
#undef IWQ_MF1
#undef IWQ_RD
#undef IWQ_LGKMN

  // epilogue: lane holds rows 16 mt + 4 g + r of columns col0 + 16 nt
  float bc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) bc[nt] = a.bias ? (float)gp<_Float16>(a.bias)[col0 + 16 * nt] : 0.0f;
  const int64_t ld2 = __builtin_amdgcn_readfirstlane((int)a.ldy) * (int64_t)2;  // row pitch, bytes
  char* yl = reinterpret_cast<char*>(a.y) + ((int64_t)(m0 + 4 * g) * a.ldy + col0) * 2;
  const bool full = m0 + TM <= a.M;
#pragma unroll
  for (int mt = 0; mt < 16; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = mt * 16 + r;
      if (full || m0 + rr + 4 * g < a.M) {
        auto p = gp<_Float16>(static_cast<void*>(yl + (int64_t)rr * ld2));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          if constexpr (GROUPED) p[16 * nt] = (_Float16)(acc[mt][nt][r] + bc[nt]);
          else p[16 * nt] = (_Float16)(opaque(acc[mt][nt][r] * sfl[nt]) + bc[nt]);
        }
      }
    }
}

// k_w4a16_b16p: k_w4a16_b16q (IL) as a PERSISTENT kernel: gridDim <= CUs workgroups, workgroup b
// takes tiles swizzled_block(b + j * gridDim) (the non-persistent grid's XCD placement), and the
// K-steps of its tiles form ONE stream through the rings: the DMA runs three K-steps ahead across tile
// boundaries, so a tile starts with its first stages already resident (no prologue wait) and the
// previous tile's epilogue overlaps the next tile's loads.  Grouped: the (s, z) of every K-step ride
// in the code ring (b16q).  Per channel: the next tile's scales / zero points are loaded (global,
// 8 per lane) in the last K-step of a tile, right after its barrier, and waited for (vmcnt past the
// 4 DMA pieces issued after them) before the next tile's first dequant; the running tile's scale
// moves to the epilogue then.  The issue cursor (tile, K-step, DMA source pointers, parameter
// group) is wave-uniform state advanced once per K-step; past the last step it re-loads the last
// step into the freed slot.
template <bool NIB, bool GROUPED>
__global__ __launch_bounds__(256) void k_w4a16_b16p(PrefillArgs a) {
  constexpr int NSX = 4, NSC = 3;
  constexpr int CST = CS + (GROUPED ? PS : 0);
  constexpr int CBASE = NSX * XS;
  constexpr int PIECES = GROUPED ? 12 : 10;
  constexpr int VM_AHEAD = PIECES;
  constexpr int NCR = GROUPED ? 8 : 4;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSX * XS + NSC * CST];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int tiles_n = a.N / TN;
  const int64_t ntiles = (int64_t)((a.M + TM - 1) / TM) * tiles_n;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int my_tiles = (int)((ntiles - b + G - 1) / G);
  const int64_t crow = a.K / 2;
  const int nk = a.K / TK;
  const int ksg = GROUPED ? a.group / TK : 1;  // K-steps per parameter group

  // ---- the DMA issue cursor: tile ij, K-step ikt (group ipg, ipr K-steps left in it), source pointers
  int ij = 0, ikt = 0, ipg = 0, ipr = ksg;
  // X / code sources as a wave-uniform tile base (SGPRs) + 32-bit lane offsets: the DMA then takes
  // the saddr form, no 64-bit address VALU per piece
  const char* xb = nullptr;
  const char* cb = nullptr;
  uint32_t xo[8], co[2];
  const _Float16* psrc[2] = {nullptr, nullptr};
  const int64_t pstep = (GROUPED && a.pgm) ? a.N : 1;
  auto set_issue_tile = [&](int j) {
    const int64_t t = swizzled_block(b + (int64_t)j * G, ntiles);
    const int m0i = (int)(t / tiles_n) * TM, n0i = (int)(t % tiles_n) * TN;
    xb = reinterpret_cast<const char*>(a.x + (int64_t)m0i * a.lda);
    cb = reinterpret_cast<const char*>(a.codes + (int64_t)n0i * crow);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = (wid * 8 + i) * 8 + (lane >> 3);
      const int gm = m0i + row < a.M ? row : a.M - 1 - m0i;
      xo[i] = (uint32_t)(((int64_t)gm * a.lda + (((lane & 7) ^ xh(row)) << 3)) * 2);
    }
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2) {
      const int ccol = wid * 64 + 32 * j2 + (lane >> 1);
      co[j2] = (uint32_t)((int64_t)ccol * crow + (((lane & 1) ^ cswz(ccol)) << 4));
    }
    if constexpr (GROUPED) {
      const int64_t c = n0i + wid * 64 + lane;
      const int64_t off = a.pgm ? c : c * a.gpr;
      psrc[0] = a.scales + off;
      psrc[1] = (a.zeros ? a.zeros : a.scales) + off;
    }
  };
  auto issue1 = [&](int xs, int cs, int i) {
    if (i < 8) {
      glds16(xb + ikt * (TK * 2) + xo[i], smem + xs * XS + (wid * 8 + i) * 1024);
    } else if (i < 10) {
      glds16(cb + ikt * (TK / 2) + co[i - 8], smem + CBASE + cs * CST + (wid * 2 + i - 8) * 1024);
    } else if constexpr (GROUPED) {
      glds2(psrc[i - 10] + ipg * pstep, smem + CBASE + cs * CST + CS + (i - 10) * 1024 + wid * 256);
    }
  };
  auto advance_issue = [&]() {
    if (ikt + 1 < nk) {
      ++ikt;
      if (--ipr == 0) {
        ++ipg;
        ipr = ksg;
      }
    } else if (ij + 1 < my_tiles) {
      ++ij;
      ikt = 0;
      ipg = 0;
      ipr = ksg;
      set_issue_tile(ij);
    }  // else: stay on the last K-step (re-loads into freed slots nobody reads)
  };

  // ---- the compute side
  int m0 = 0, n0 = 0;
  auto tile_mn = [&](int j, int& mm, int& nn) {
    const int64_t t = swizzled_block(b + (int64_t)j * G, ntiles);
    mm = (int)(t / tiles_n) * TM;
    nn = (int)(t % tiles_n) * TN;
  };
  float sepi[4] = {1.0f, 1.0f, 1.0f, 1.0f};
  h2 s2[4], zz[4], zl[4], zh[4];
  const h2 zsym2 = {(_Float16)a.zsym, (_Float16)a.zsym};
  auto set_zero = [&](int nt, float zf) {
    zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  };
  // per channel: the parameters of tile j's columns as raw halves (pcs scales, pcz zero points)
  uint16_t pcs[4] = {0, 0, 0, 0}, pcz[4] = {0, 0, 0, 0};
  auto load_pc = [&](int j) {
    int mm, nn;
    tile_mn(j, mm, nn);
    const int col = nn + wid * 64 + r16;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      pcs[nt] = gp<uint16_t>(a.scales)[col + 16 * nt];
      pcz[nt] = a.zeros ? gp<uint16_t>(a.zeros)[col + 16 * nt] : (uint16_t)0;
    }
  };
  auto use_pc = [&]() {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      landed(pcs[nt]);
      landed(pcz[nt]);
      sepi[nt] = (float)s2[nt].x;
      const _Float16 sc = __builtin_bit_cast(_Float16, pcs[nt]);
      s2[nt] = h2{sc, sc};
      set_zero(nt, a.zeros ? (float)__builtin_bit_cast(_Float16, pcz[nt]) : a.zsym);
    }
  };
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) la[s] = lbase + (uint32_t)(r16 * 128 + (((2 * g + s) ^ xh(r16)) << 4));
  const int ccl = wid * 64 + r16;
  const uint32_t lc = lbase + CBASE + (uint32_t)(ccl * 32 + (((g >> 1) ^ cswz(ccl)) << 4) + ((g & 1) << 3));
  const uint32_t lps = lbase + CBASE + CS + (uint32_t)(ccl * 4);
  u32x2 pv[4];
  auto set_params = [&](int nt) {  // grouped: the stage's (s, z)
    if constexpr (GROUPED) {
      s2[nt] = bcast_lo(pv[nt >> 1][nt & 1]);
      zero_offsets(a.zeros ? bcast_lo(pv[2 + (nt >> 1)][nt & 1]) : zsym2, zz[nt], zl[nt], zh[nt]);
    }
  };
  auto read_codes = [&](u32x2* w, uint32_t co) {
    w[0] = lds_rd2<0>(lc + co);
    w[1] = lds_rd2<512>(lc + co);
    w[2] = lds_rd2<1024>(lc + co);
    w[3] = lds_rd2<1536>(lc + co);
    if constexpr (GROUPED) {
      pv[0] = lds_rd_pair(lps + co);
      pv[1] = lds_rd_pair(lps + co + 128);
      pv[2] = lds_rd_pair(lps + co + 1024);
      pv[3] = lds_rd_pair(lps + co + 1152);
    }
  };
  auto codes_landed = [&](u32x2* w) {
    landed(w[0]);
    landed(w[1]);
    landed(w[2]);
    landed(w[3]);
    if constexpr (GROUPED) {
      landed(pv[0]);
      landed(pv[1]);
      landed(pv[2]);
      landed(pv[3]);
    }
  };
  auto dqp = [&](uint32_t w, int j, int nt) -> h2 {
    h2 d;
    if constexpr (NIB) {
      const uint32_t t = j >= 2 ? w >> 8 : w;
      d = (j & 1) ? as_h2(and_or_c(t, m1_s, mg54)) - zh[nt] : as_h2(and_or_c(t, m0_s, mg64)) - zl[nt];
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      d = as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz[nt];
    }
    if constexpr (GROUPED) d = d * s2[nt];
    return d;
  };
  auto frag = [](const h2* p) -> h8 { return h8{p[0].x, p[0].y, p[1].x, p[1].y, p[2].x, p[2].y, p[3].x, p[3].y}; };

  f4 acc[16][4];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 af[8];
  h8 b0[4], b1[4];
  u32x2 wc[4];

#define IWQ_RD(MT, ADDR) af[(MT) & 7] = lds_rd<((MT) & 15) * 2048>(ADDR)
#define IWQ_LGKMN(N) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory")
#define IWQ_MF1(MT, NT, B) \
  acc[MT][NT] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[(MT) & 7], B[NT], acc[MT][NT], 0, 0, 0)
#define IWQ_GRP(MT, N, B, W0, W1, W2, W3) \
  {                                       \
    IWQ_LGKMN(N);                         \
    IWQ_PIN();                            \
    IWQ_MF1(MT, 0, B);                    \
    W0;                                   \
    IWQ_PIN();                            \
    IWQ_MF1(MT, 1, B);                    \
    W1;                                   \
    IWQ_PIN();                            \
    IWQ_MF1(MT, 2, B);                    \
    W2;                                   \
    IWQ_PIN();                            \
    IWQ_MF1(MT, 3, B);                    \
    W3;                                   \
    IWQ_PIN();                            \
  }

  if (my_tiles <= 0) return;  // (gridDim <= tiles by construction)
  set_issue_tile(0);
  if constexpr (!GROUPED) {
    load_pc(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    use_pc();
  }
  // prologue: the stream's K-steps 0, 1, 2 into slots 0, 1, 2 of both rings
#pragma unroll
  for (int s0 = 0; s0 < 3; ++s0) {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) issue1(s0, s0, i);
    advance_issue();
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PIECES) : "memory");
  __builtin_amdgcn_s_barrier();
  IWQ_PIN();
  read_codes(wc, 0);
  IWQ_RD(0, la[0]); IWQ_RD(1, la[0]); IWQ_RD(2, la[0]); IWQ_RD(3, la[0]);
  IWQ_LGKM(0);
  codes_landed(wc);
  IWQ_PIN();
  {
    h2 p[16];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      set_params(nt);
#pragma unroll
      for (int j = 0; j < 4; ++j) p[4 * nt + j] = dqp(wc[nt].x, j, nt);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b0[nt] = frag(p + 4 * nt);
  }

  // ring slots of the running K-step: X sx (of 4), codes sc (of 3)
  int sx = 0, sc = 0;
  for (int j = 0; j < my_tiles; ++j) {
    tile_mn(j, m0, n0);
    for (int kt = 0; kt < nk; ++kt) {
      const int sxn = (sx + 1) & 3, scn = sc == 2 ? 0 : sc + 1;
      const uint32_t so = (uint32_t)(sx * XS);
      const uint32_t sn = (uint32_t)(sxn * XS);
      const uint32_t cn = (uint32_t)(scn * CST);
      const int xd = (sx + 3) & 3, cd = sc;  // refilled after the barrier with the cursor's K-step
      const bool last = kt + 1 == nk;         // wave-uniform: the next stage starts a tile (or re-loads)
      {
        const uint32_t a0 = la[0] + so, a1 = la[1] + so;
        h2 p[16];
        IWQ_GRP(0, 3, b0, IWQ_RD(4, a0), p[0] = dqp(wc[0].y, 0, 0), , );
        IWQ_GRP(1, 3, b0, IWQ_RD(5, a0), p[1] = dqp(wc[0].y, 1, 0), , );
        IWQ_GRP(2, 3, b0, IWQ_RD(6, a0), p[2] = dqp(wc[0].y, 2, 0), , );
        IWQ_GRP(3, 3, b0, IWQ_RD(7, a0), p[3] = dqp(wc[0].y, 3, 0), , );
        IWQ_GRP(4, 3, b0, IWQ_RD(8, a0), p[4] = dqp(wc[1].y, 0, 1), , );
        IWQ_GRP(5, 3, b0, IWQ_RD(9, a0), p[5] = dqp(wc[1].y, 1, 1), , );
        IWQ_GRP(6, 3, b0, IWQ_RD(10, a0), p[6] = dqp(wc[1].y, 2, 1), , );
        IWQ_GRP(7, 3, b0, IWQ_RD(11, a0), p[7] = dqp(wc[1].y, 3, 1), , );
        IWQ_GRP(8, 3, b0, IWQ_RD(12, a0), p[8] = dqp(wc[2].y, 0, 2), , );
        IWQ_GRP(9, 3, b0, IWQ_RD(13, a0), p[9] = dqp(wc[2].y, 1, 2), , );
        IWQ_GRP(10, 3, b0, IWQ_RD(14, a0), p[10] = dqp(wc[2].y, 2, 2), , );
        IWQ_GRP(11, 3, b0, IWQ_RD(15, a0), p[11] = dqp(wc[2].y, 3, 2), , );
        IWQ_GRP(12, 3, b0, IWQ_RD(0, a1), p[12] = dqp(wc[3].y, 0, 3), , );
        IWQ_GRP(13, 3, b0, IWQ_RD(1, a1), p[13] = dqp(wc[3].y, 1, 3), , );
        IWQ_GRP(14, 3, b0, IWQ_RD(2, a1), p[14] = dqp(wc[3].y, 2, 3), , );
        IWQ_GRP(15, 3, b0, IWQ_RD(3, a1), p[15] = dqp(wc[3].y, 3, 3), , );
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) b1[nt] = frag(p + 4 * nt);
      }
      const uint32_t a1 = la[1] + so;
      const uint32_t na = la[0] + sn;
      IWQ_GRP(0, 3, b1, IWQ_RD(4, a1), , , );
      IWQ_GRP(1, 3, b1, IWQ_RD(5, a1), , , );
      IWQ_GRP(2, 3, b1, IWQ_RD(6, a1), , , );
      IWQ_GRP(3, 3, b1, IWQ_RD(7, a1), , , );
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_AHEAD) : "memory");
      __builtin_amdgcn_s_barrier();
      IWQ_PIN();
      // per channel, last K-step of the tile: the next tile's parameters (before this step's DMA
      // pieces; the clamped cursor past the last tile re-reads the same tile's)
      if constexpr (!GROUPED) {
        if (last) load_pc(j + 1 < my_tiles ? j + 1 : j);
      }
      IWQ_PIN();
      u32x2 wn[4];
      IWQ_GRP(4, 3, b1, read_codes(wn, cn), IWQ_RD(8, a1), issue1(xd, cd, 0), );
      IWQ_GRP(5, 3 + NCR, b1, IWQ_RD(9, a1), issue1(xd, cd, 1), , );
      IWQ_GRP(6, 3 + NCR, b1, IWQ_RD(10, a1), issue1(xd, cd, 2), , );
      IWQ_GRP(7, 3 + NCR, b1, IWQ_RD(11, a1), issue1(xd, cd, 3), , );
      h2 p[16];
      IWQ_LGKM(3);
      codes_landed(wn);
      if constexpr (!GROUPED) {
        if (last) {  // the parameter loads and everything older landed (4 DMA pieces issued since)
          asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
          use_pc();
        }
      }
      IWQ_PIN();
      IWQ_GRP(8, 3, b1, IWQ_RD(12, a1), issue1(xd, cd, 4); set_params(0), p[0] = dqp(wn[0].x, 0, 0),
              p[1] = dqp(wn[0].x, 1, 0));
      IWQ_GRP(9, 3, b1, IWQ_RD(13, a1), issue1(xd, cd, 5), p[2] = dqp(wn[0].x, 2, 0), p[3] = dqp(wn[0].x, 3, 0));
      IWQ_GRP(10, 3, b1, IWQ_RD(14, a1), issue1(xd, cd, 6); set_params(1), p[4] = dqp(wn[1].x, 0, 1),
              p[5] = dqp(wn[1].x, 1, 1));
      IWQ_GRP(11, 3, b1, IWQ_RD(15, a1), issue1(xd, cd, 7), p[6] = dqp(wn[1].x, 2, 1), p[7] = dqp(wn[1].x, 3, 1));
      IWQ_GRP(12, 3, b1, IWQ_RD(0, na), issue1(xd, cd, 8); set_params(2), p[8] = dqp(wn[2].x, 0, 2),
              p[9] = dqp(wn[2].x, 1, 2));
      IWQ_GRP(13, 3, b1, IWQ_RD(1, na), issue1(xd, cd, 9), p[10] = dqp(wn[2].x, 2, 2), p[11] = dqp(wn[2].x, 3, 2));
      IWQ_GRP(14, 3, b1, IWQ_RD(2, na), issue1(xd, cd, 10); set_params(3), p[12] = dqp(wn[3].x, 0, 3),
              p[13] = dqp(wn[3].x, 1, 3));
      IWQ_GRP(15, 3, b1, IWQ_RD(3, na), issue1(xd, cd, 11), p[14] = dqp(wn[3].x, 2, 3), p[15] = dqp(wn[3].x, 3, 3));
      advance_issue();
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        b0[nt] = frag(p + 4 * nt);
        wc[nt] = wn[nt];
      }
      sx = sxn;
      sc = scn;
    }
    // epilogue of tile j (the stream's next stages are in flight / landed meanwhile)
    const int col0 = n0 + wid * 64 + r16;
    float bc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bc[nt] = a.bias ? (float)gp<_Float16>(a.bias)[col0 + 16 * nt] : 0.0f;
    const int64_t ld2 = __builtin_amdgcn_readfirstlane((int)a.ldy) * (int64_t)2;
    char* yl = reinterpret_cast<char*>(a.y) + ((int64_t)(m0 + 4 * g) * a.ldy + col0) * 2;
    const bool full = m0 + TM <= a.M;
#pragma unroll
    for (int mt = 0; mt < 16; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = mt * 16 + r;
        if (full || m0 + rr + 4 * g < a.M) {
          auto q = gp<_Float16>(static_cast<void*>(yl + (int64_t)rr * ld2));
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            if constexpr (GROUPED) q[16 * nt] = (_Float16)(acc[mt][nt][r] + bc[nt]);
            else q[16 * nt] = (_Float16)(opaque(acc[mt][nt][r] * sepi[nt]) + bc[nt]);
          }
        }
      }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f4{0.f, 0.f, 0.f, 0.f};
  }
  // no LDS-DMA may still be landing when the workgroup retires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef IWQ_GRP
#undef IWQ_MF1
#undef IWQ_LGKMN
#undef IWQ_RD
}

// k_w4a16_b16r: k_w4a16_b16q (one wave per SIMD, IL work slots) with the rolling A reads D groups
// ahead instead of 4 (D - 1 reads in flight at every MFMA group; the fragment ring holds 8), written
// with compile-time group indices.  The next stage's slice-0 dequant then runs over groups D + 4 .. 15.
template <int I>
struct ic {
  static constexpr int v = I;
};
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(ic<B>{});
    sfor<B + 1, E>(f);
  }
}

template <bool NIB, int D, bool GROUPED = false>
__global__ __launch_bounds__(256) void k_w4a16_b16r(PrefillArgs a) {
  static_assert(D >= 2 && D <= 7, "fragment ring of 8");
  constexpr int NSX = 4, NSC = 3;
  constexpr int CST = CS + (GROUPED ? PS : 0);
  constexpr int CBASE = NSX * XS;
  constexpr int PIECES = GROUPED ? 12 : 10;
  constexpr int VM_AHEAD = PIECES;
  constexpr int NCR = GROUPED ? 8 : 4;
  static_assert(4 + PIECES <= 16, "DMA pieces fit groups 4..15");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NSX * XS + NSC * CST];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int tiles_n = a.N / TN;
  const int64_t t = swizzled_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * TM, n0 = (int)(t % tiles_n) * TN;
  const int64_t crow = a.K / 2;
  const int nk = a.K / TK;

  const _Float16* xsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = (wid * 8 + i) * 8 + (lane >> 3);
    const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
    xsrc[i] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ xh(row)) << 3);
  }
  const uint8_t* csrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ccol = wid * 64 + 32 * j + (lane >> 1);
    csrc[j] = a.codes + (int64_t)(n0 + ccol) * crow + (((lane & 1) ^ cswz(ccol)) << 4);
  }
  const _Float16* psrc[2] = {nullptr, nullptr};
  int64_t pstep = 1;
  const KStepGroup kgrp(GROUPED ? a.group : TK);
  if constexpr (GROUPED) {
    const int64_t c = n0 + wid * 64 + lane;
    const int64_t off = a.pgm ? c : c * a.gpr;
    psrc[0] = a.scales + off;
    psrc[1] = (a.zeros ? a.zeros : a.scales) + off;
    pstep = a.pgm ? a.N : 1;
  }
  auto issue1 = [&](int kt, int xs, int cs, int i) {
    if (i < 8) {
      glds16(xsrc[i] + kt * TK, smem + xs * XS + (wid * 8 + i) * 1024);
    } else if (i < 10) {
      glds16(csrc[i - 8] + kt * (TK / 2), smem + CBASE + cs * CST + (wid * 2 + i - 8) * 1024);
    } else if constexpr (GROUPED) {
      glds2(psrc[i - 10] + kgrp(kt) * pstep, smem + CBASE + cs * CST + CS + (i - 10) * 1024 + wid * 256);
    }
  };
  auto issue = [&](int kt, int s) {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) issue1(kt, s, s, i);
  };

  const int col0 = n0 + wid * 64 + r16;
  float sfl[4] = {1.0f, 1.0f, 1.0f, 1.0f};
  h2 s2[4], zz[4], zl[4], zh[4];
  const h2 zsym2 = {(_Float16)a.zsym, (_Float16)a.zsym};
  auto set_zero = [&](int nt, float zf) {
    zz[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(64.0f + zf)};
    zl[nt] = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    zh[nt] = h2{(_Float16)(64.0f + zf), (_Float16)(64.0f + zf)};
  };
  if constexpr (!GROUPED) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = col0 + 16 * nt;
      sfl[nt] = (float)gp<_Float16>(a.scales)[col];
      set_zero(nt, a.zeros ? (float)gp<_Float16>(a.zeros)[col] : a.zsym);
    }
  }
  const uint32_t mask_s = __builtin_amdgcn_readfirstlane(0x00F0000Fu);
  const uint32_t m0_s = __builtin_amdgcn_readfirstlane(0x000F000Fu);
  const uint32_t m1_s = __builtin_amdgcn_readfirstlane(0x00F000F0u);
  uint32_t magic_v, mg64, mg54;
  asm volatile("v_mov_b32 %0, 0x54006400" : "=v"(magic_v));
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(mg64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(mg54));

  const uint32_t lbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(smem));
  uint32_t la[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) la[s] = lbase + (uint32_t)(r16 * 128 + (((2 * g + s) ^ xh(r16)) << 4));
  const int ccl = wid * 64 + r16;
  const uint32_t lc = lbase + CBASE + (uint32_t)(ccl * 32 + (((g >> 1) ^ cswz(ccl)) << 4) + ((g & 1) << 3));
  const uint32_t lps = lbase + CBASE + CS + (uint32_t)(ccl * 4);
  u32x2 pv[4];
  auto set_params = [&](int nt) {
    if constexpr (GROUPED) {
      s2[nt] = bcast_lo(pv[nt >> 1][nt & 1]);
      zero_offsets(a.zeros ? bcast_lo(pv[2 + (nt >> 1)][nt & 1]) : zsym2, zz[nt], zl[nt], zh[nt]);
    }
  };
  auto read_codes = [&](u32x2* w, uint32_t co) {
    w[0] = lds_rd2<0>(lc + co);
    w[1] = lds_rd2<512>(lc + co);
    w[2] = lds_rd2<1024>(lc + co);
    w[3] = lds_rd2<1536>(lc + co);
    if constexpr (GROUPED) {
      pv[0] = lds_rd_pair(lps + co);
      pv[1] = lds_rd_pair(lps + co + 128);
      pv[2] = lds_rd_pair(lps + co + 1024);
      pv[3] = lds_rd_pair(lps + co + 1152);
    }
  };
  auto codes_landed = [&](u32x2* w) {
    landed(w[0]);
    landed(w[1]);
    landed(w[2]);
    landed(w[3]);
    if constexpr (GROUPED) {
      landed(pv[0]);
      landed(pv[1]);
      landed(pv[2]);
      landed(pv[3]);
    }
  };
  auto dqp = [&](uint32_t w, int j, int nt) -> h2 {
    h2 d;
    if constexpr (NIB) {
      const uint32_t t = j >= 2 ? w >> 8 : w;
      d = (j & 1) ? as_h2(and_or_c(t, m1_s, mg54)) - zh[nt] : as_h2(and_or_c(t, m0_s, mg64)) - zl[nt];
    } else {
      const uint32_t sel = j == 0 ? 0x0C000C00u : (j == 1 ? 0x0C010C01u : (j == 2 ? 0x0C020C02u : 0x0C030C03u));
      d = as_h2(and_or(__builtin_amdgcn_perm(w, w, sel), mask_s, magic_v)) - zz[nt];
    }
    if constexpr (GROUPED) d = d * s2[nt];
    return d;
  };
  auto frag = [](const h2* p) -> h8 { return h8{p[0].x, p[0].y, p[1].x, p[1].y, p[2].x, p[2].y, p[3].x, p[3].y}; };

  f4 acc[16][4];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 af[8];
  h8 b0[4], b1[4];
  u32x2 wc[4];

  // fragment F (0..31: slice F / 16) of the stage at X offset SO into the ring
  auto rd = [&](auto fc, uint32_t so) __attribute__((always_inline)) {
    constexpr int F = decltype(fc)::v;
    af[F & 7] = lds_rd<(F & 15) * 2048>(la[F >> 4] + so);
  };
  // group MT: wait until N newer LDS reads remain, then MFMA nt / work slot nt for nt = 0..3
  auto grp = [&](auto mc, auto nc, h8* B, auto&& w0, auto&& w1, auto&& w2, auto&& w3) __attribute__((always_inline)) {
    constexpr int MT = decltype(mc)::v;
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(decltype(nc)::v) : "memory");
    IWQ_PIN();
    acc[MT][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[MT & 7], B[0], acc[MT][0], 0, 0, 0);
    w0();
    IWQ_PIN();
    acc[MT][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[MT & 7], B[1], acc[MT][1], 0, 0, 0);
    w1();
    IWQ_PIN();
    acc[MT][2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[MT & 7], B[2], acc[MT][2], 0, 0, 0);
    w2();
    IWQ_PIN();
    acc[MT][3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[MT & 7], B[3], acc[MT][3], 0, 0, 0);
    w3();
    IWQ_PIN();
  };
  auto nop = []() __attribute__((always_inline)) {};

  // slice 0: group MT reads fragment MT + D (slice 1's first D at MT >= 16 - D); slice 1's B
  // dequantized one pair per group
  auto slice0 = [&](uint32_t so) __attribute__((always_inline)) {
    h2 p[16];
    sfor<0, 16>([&](auto mc) __attribute__((always_inline)) {
      constexpr int MT = decltype(mc)::v;
      grp(mc, ic<D - 1>{}, b0, [&]() __attribute__((always_inline)) { rd(ic<MT + D>{}, so); },
          [&]() __attribute__((always_inline)) { p[MT] = dqp(wc[MT >> 2].y, MT & 3, MT >> 2); }, nop, nop);
    });
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b1[nt] = frag(p + 4 * nt);
  };

  issue(0, 0);
  issue(nk > 1 ? 1 : 0, 1);
  issue(nk > 2 ? 2 : nk - 1, 2);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PIECES) : "memory");
  __builtin_amdgcn_s_barrier();
  IWQ_PIN();
  read_codes(wc, 0);
  sfor<0, D>([&](auto fc) __attribute__((always_inline)) { rd(fc, 0u); });
  IWQ_LGKM(0);
  codes_landed(wc);
  IWQ_PIN();
  {
    h2 p[16];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      set_params(nt);
#pragma unroll
      for (int j = 0; j < 4; ++j) p[4 * nt + j] = dqp(wc[nt].x, j, nt);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b0[nt] = frag(p + 4 * nt);
  }

  constexpr int G0 = D + 4;  // first group with the next stage's codes landed
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const uint32_t so = (uint32_t)((kt % NSX) * XS);
    const uint32_t sn = (uint32_t)(((kt + 1) % NSX) * XS);
    const uint32_t cn = (uint32_t)(((kt + 1) % NSC) * CST);
    const int xd = (kt + 3) % NSX, cd = kt % NSC;
    const int kd = kt + 3 < nk ? kt + 3 : nk - 1;
    slice0(so);
    // slice 1: group MT reads fragment 16 + MT + D of this stage, or (MT + D >= 16) the next stage's
    // slice-0 fragment MT + D - 16 (after the barrier)
    auto rd1 = [&](auto mc) __attribute__((always_inline)) {
      constexpr int F = decltype(mc)::v + D;
      if constexpr (F < 16) rd(ic<16 + F>{}, so);
      else rd(ic<F - 16>{}, sn);
    };
    sfor<0, 4>([&](auto mc) __attribute__((always_inline)) {
      grp(mc, ic<D - 1>{}, b1, [&]() __attribute__((always_inline)) { rd1(mc); }, nop, nop, nop);
    });
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_AHEAD) : "memory");
    __builtin_amdgcn_s_barrier();
    IWQ_PIN();
    u32x2 wn[4];
    h2 p[16];
    sfor<4, 16>([&](auto mc) __attribute__((always_inline)) {
      constexpr int MT = decltype(mc)::v;
      // newer reads than fragment MT's: D - 1 fragments, plus the code reads (group 4, before its
      // fragment read) while they are younger than fragment MT (MT < D + 4)
      constexpr int N = (MT >= 5 && MT < G0) ? D - 1 + NCR : D - 1;
      // this group's share of the next stage's 16 dequant pairs (groups G0..15)
      constexpr int NG = 16 - G0;
      constexpr int PB = MT >= G0 ? (16 * (MT - G0)) / NG : 0;
      constexpr int PE = MT >= G0 ? (16 * (MT - G0 + 1)) / NG : 0;
      constexpr int PM = (PB + PE) / 2;
      auto dq = [&](auto bc, auto ec) __attribute__((always_inline)) {
        sfor<decltype(bc)::v, decltype(ec)::v>([&](auto qc) __attribute__((always_inline)) {
          constexpr int Q = decltype(qc)::v;
          if constexpr ((Q & 3) == 0) set_params(Q >> 2);
          p[Q] = dqp(wn[Q >> 2].x, Q & 3, Q >> 2);
        });
      };
      grp(mc, ic<N>{}, b1,
          [&]() __attribute__((always_inline)) {
            if constexpr (MT == 4) read_codes(wn, cn);
            if constexpr (MT == G0) codes_landed(wn);
            rd1(mc);
          },
          [&]() __attribute__((always_inline)) {
            if constexpr (MT - 4 < PIECES) issue1(kd, xd, cd, MT - 4);
          },
          [&]() __attribute__((always_inline)) { dq(ic<PB>{}, ic<PM>{}); },
          [&]() __attribute__((always_inline)) { dq(ic<PM>{}, ic<PE>{}); });
    });
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      b0[nt] = frag(p + 4 * nt);
      wc[nt] = wn[nt];
    }
  }
  {
    const uint32_t so = (uint32_t)(((nk - 1) % NSX) * XS);
    slice0(so);
    sfor<0, 16>([&](auto mc) __attribute__((always_inline)) {
      constexpr int MT = decltype(mc)::v;
      constexpr int N = (D - 1 < 15 - MT) ? D - 1 : 15 - MT;
      grp(mc, ic<N>{}, b1,
          [&]() __attribute__((always_inline)) {
            if constexpr (MT + D < 16) rd(ic<16 + MT + D>{}, so);
          },
          nop, nop, nop);
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  float bc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) bc[nt] = a.bias ? (float)gp<_Float16>(a.bias)[col0 + 16 * nt] : 0.0f;
  const int64_t ld2 = __builtin_amdgcn_readfirstlane((int)a.ldy) * (int64_t)2;
  char* yl = reinterpret_cast<char*>(a.y) + ((int64_t)(m0 + 4 * g) * a.ldy + col0) * 2;
  const bool full = m0 + TM <= a.M;
#pragma unroll
  for (int mt = 0; mt < 16; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = mt * 16 + r;
      if (full || m0 + rr + 4 * g < a.M) {
        auto p = gp<_Float16>(static_cast<void*>(yl + (int64_t)rr * ld2));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          if constexpr (GROUPED) p[16 * nt] = (_Float16)(acc[mt][nt][r] + bc[nt]);
          else p[16 * nt] = (_Float16)(opaque(acc[mt][nt][r] * sfl[nt]) + bc[nt]);
        }
      }
    }
}

#undef IWQ_LGKM
#undef IWQ_PIN

}  // namespace

// 16x16x32 forms of 74: variants 150 (3-slot ring), 151 (4-slot ring, waves 4-7 staggered half a
// K-step: the per-channel default since round 4), 152 / 153 the same on NIB codes; grouped weights
// (group % 64 == 0): 150 / 152 the 3-slot ring, 151 / 153 staggered on 3 slots with the late waves
// issuing early, 157 staggered issuing in slice 1 (A/B)
// CUs of the current device (one persistent workgroup each: 152-158 KiB of LDS)
static int persistent_cus() {
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

bool prefill16_supported(int64_t M, int64_t N, int64_t K, int gpr, int group) {
  return M >= 1 && N % TN == 0 && K % TK == 0 && K >= TK && (gpr == 1 || (group % TK == 0 && K % group == 0));
}

hipError_t prefill16_launch(const PrefillArgs& a, int variant, hipStream_t st) {
  const int64_t blocks = ((int64_t)(a.M + TM - 1) / TM) * (a.N / TN);
  const dim3 grid((unsigned)blocks), blk(THR);
  // the product forms: per channel 151 (staggered, 4-slot ring) / 172 (NIB codes, persistent one wave
  // per SIMD), grouped 150 / 152 (3-slot ring)
  if (a.gpr == 1 && (variant == 151 || variant == 153)) {
    if (variant == 153) hipLaunchKernelGGL((k_w4a16_b16w<true, true>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((k_w4a16_b16w<true>), grid, blk, 0, st, a);
    return hipGetLastError();
  }
  if (a.gpr == 1 && variant == 172) {  // NIB codes: the persistent form (same bits as 151 / 153)
    const dim3 pg((unsigned)(blocks < persistent_cus() ? blocks : persistent_cus()));
    hipLaunchKernelGGL((k_w4a16_b16p<true, false>), pg, dim3(256), 0, st, a);
    return hipGetLastError();
  }
  if (a.gpr != 1 && (variant == 150 || variant == 152)) {
    if (variant == 152) hipLaunchKernelGGL((k_w4a16_b16w<false, true, 16, 0, true>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((k_w4a16_b16w<false, false, 16, 0, true>), grid, blk, 0, st, a);
    return hipGetLastError();
  }
#if IWQ_AB
  if (a.gpr != 1) {
    switch (variant) {
      case 150: hipLaunchKernelGGL((k_w4a16_b16w<false, false, 16, 0, true>), grid, blk, 0, st, a); break;
      case 152: hipLaunchKernelGGL((k_w4a16_b16w<false, true, 16, 0, true>), grid, blk, 0, st, a); break;
      case 153: hipLaunchKernelGGL((k_w4a16_b16w<true, true, 16, 0, true, true>), grid, blk, 0, st, a); break;
      case 157: hipLaunchKernelGGL((k_w4a16_b16w<true, false, 16, 0, true, false>), grid, blk, 0, st, a); break;
      case 162: hipLaunchKernelGGL((k_w4a16_b16q<false, false, true>), grid, dim3(256), 0, st, a); break;
      case 163: hipLaunchKernelGGL((k_w4a16_b16q<true, false, true>), grid, dim3(256), 0, st, a); break;
      case 164: hipLaunchKernelGGL((k_w4a16_b16q<false, true, true>), grid, dim3(256), 0, st, a); break;
      case 165: hipLaunchKernelGGL((k_w4a16_b16q<true, true, true>), grid, dim3(256), 0, st, a); break;
      case 171:
      case 172: {
        const dim3 pg((unsigned)(blocks < persistent_cus() ? blocks : persistent_cus()));
        if (variant == 172) hipLaunchKernelGGL((k_w4a16_b16p<true, true>), pg, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((k_w4a16_b16p<false, true>), pg, dim3(256), 0, st, a);
        break;
      }
      case 168: hipLaunchKernelGGL((k_w4a16_b16r<true, 4, true>), grid, dim3(256), 0, st, a); break;
      case 169: hipLaunchKernelGGL((k_w4a16_b16r<true, 6, true>), grid, dim3(256), 0, st, a); break;
      case 170: hipLaunchKernelGGL((k_w4a16_b16r<false, 6, true>), grid, dim3(256), 0, st, a); break;
      default: hipLaunchKernelGGL((k_w4a16_b16w<true, false, 16, 0, true, true>), grid, blk, 0, st, a); break;
    }
    return hipGetLastError();
  }
  switch (variant) {
    case 150: hipLaunchKernelGGL((k_w4a16_b16w<false>), grid, blk, 0, st, a); break;
    case 152: hipLaunchKernelGGL((k_w4a16_b16w<false, true>), grid, blk, 0, st, a); break;
    case 154: hipLaunchKernelGGL((k_w4a16_b16w<true, false, 8>), grid, blk, 0, st, a); break;
    case 155: hipLaunchKernelGGL((k_w4a16_b16w<true, false, 16, 1>), grid, blk, 0, st, a); break;
    case 156: hipLaunchKernelGGL((k_w4a16_b16w<true, false, 16, 2>), grid, blk, 0, st, a); break;
    case 162: hipLaunchKernelGGL((k_w4a16_b16q<false>), grid, dim3(256), 0, st, a); break;
    case 163: hipLaunchKernelGGL((k_w4a16_b16q<true>), grid, dim3(256), 0, st, a); break;
    case 164: hipLaunchKernelGGL((k_w4a16_b16q<false, true>), grid, dim3(256), 0, st, a); break;
    case 165: hipLaunchKernelGGL((k_w4a16_b16q<true, true>), grid, dim3(256), 0, st, a); break;
    case 171:
    case 172: {  // persistent one-wave-per-SIMD (k_w4a16_b16p), row-major / NIB
      const dim3 pg((unsigned)(blocks < persistent_cus() ? blocks : persistent_cus()));
      if (variant == 172) hipLaunchKernelGGL((k_w4a16_b16p<true, false>), pg, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((k_w4a16_b16p<false, false>), pg, dim3(256), 0, st, a);
      break;
    }
    case 168: hipLaunchKernelGGL((k_w4a16_b16r<true, 4>), grid, dim3(256), 0, st, a); break;
    case 169: hipLaunchKernelGGL((k_w4a16_b16r<true, 6>), grid, dim3(256), 0, st, a); break;
    case 170: hipLaunchKernelGGL((k_w4a16_b16r<false, 6>), grid, dim3(256), 0, st, a); break;
    case 166: hipLaunchKernelGGL((k_w4a16_b16q<true, true, false, 1>), grid, dim3(256), 0, st, a); break;  // DIAG
    case 167: hipLaunchKernelGGL((k_w4a16_b16q<true, true, false, 2>), grid, dim3(256), 0, st, a); break;  // DIAG
    case 161:  // DIAGNOSTIC: 151 without the output stores
      hipLaunchKernelGGL((k_w4a16_b16w<true, false, 16, 0, false, false, true>), grid, blk, 0, st, a);
      break;
    default: hipLaunchKernelGGL((k_w4a16_b16w<true>), grid, blk, 0, st, a); break;
  }
  return hipGetLastError();
#else
  return hipErrorInvalidValue;  // A/B forms: IWQ_AB builds only
#endif
}

}  // namespace iwq

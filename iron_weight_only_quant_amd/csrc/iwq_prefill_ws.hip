// iwq_prefill_ws.hip -- WARP-SPECIALISED form of the prefill fused dequant -> GEMM (round 6, A/B:
// iwq_w4a16_gemm variants 180-183, IWQ_AB builds).  The question it answers:
// the product prefill kernels (k_w4a16_b16w / b32w, iwq_prefill16.hip / iwq_prefill.hip) dequantize
// the packed codes on the MFMA waves themselves -- 12 VALU per 8 weights co-issued with the MFMA
// stream (PMC: SQ_VALU_MFMA_COEXEC_CYCLES 68-103 M vs hipBLASLt's 2.8 M, MFMA busy 0.66-0.74 vs
// 0.76-0.86).  Here producer waves turn the codes into an fp16 B image in LDS once per K-step and the
// consumer waves run a dequant-free MFMA loop on A (X) and B images, as hipBLASLt's fp16 kernel does.
//
// Replaces QuantLinear.forward = F.linear(x, W_deq, b) (/root/reference/quant_linear.py:960-972) for
// weights held packed, per channel: y = RN16(s * sum_k x (q - z) + b) -- the product kernels' numerics.
//
// Workgroup: 8 waves (512 threads, one workgroup per CU), a 128 (M) x 256 (N) output tile, K-steps of 64:
//   waves 0-3  CONSUMERS, 2 (M) x 2 (N): 64 rows x 128 columns each = 4 x 8 tiles of
//              v_mfma_f32_16x16x32_f16, 128 accumulators; per K-step 2 slices x (4 A + 8 B) ds_read_b128
//   waves 4-7  PRODUCERS: issue the K-step's LDS-DMA AHEAD K-steps ahead (X: 4 x 1 KiB per wave, codes:
//              2 x 1 KiB per wave); thread t owns column t of the tile -- its 32 code bytes (two ds_read_b128)
//              become 64 fp16 (q - z) (perm + and_or + pk_add per pair), written as 8 ds_write_b128
// LDS (160 KiB): A (X) ring of 4 slots x 16 KiB (rows of 128 B, chunk q of row r at q ^ xh(r), as b16w);
// codes ring of 4 slots x 8 KiB (half h of column c at 1024 (c / 32) + 512 h + 16 (c % 32)); B ring of
// 2 slots x 32 KiB (256 columns of 128 B, chunk q = k 8q .. 8q + 7 of column c at q ^ bz(c)).
// k order: slice s of a K-step gives lane group g = lane >> 4 the logical k = 16 g + 8 s + [0, 8), i.e.
// chunk 2 g + s of an A row and of a B column -- the same permutation on both operands.
// One s_barrier per K-step for all 8 waves, placed EARLY for the consumers: after slice 0's MFMAs and
// after every read of the stage has landed, before slice 1's MFMAs, so the next stage's slice-0 reads
// are covered by 32 MFMAs.  Between barriers B_kt and B_kt+1 the producers fill stage kt + 1 (B slot
// (kt + 1) % 2: read in K-step kt - 1, retired before B_kt) and issue the DMA / code loads of K-step
// kt + AHEAD (A slot (kt + AHEAD) % 4: stage kt - 1's, free since B_kt).
// Variants: 180 = AHEAD 3; 181 = AHEAD 2; 182 = 180 with the producers at s_setprio 1; 183 = 180 with
// DIAGNOSTIC producers that write constant B (no dequant VALU: wrong results; the sync + LDS skeleton).
#include "iwq_common.cuh"
#include "iwq_prefill.h"

namespace iwq {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int WS_TM = 128, WS_TN = 256, WS_TK = 64;
[[maybe_unused]] constexpr int WS_THR = 512;
constexpr int WS_AS = WS_TM * WS_TK * 2;  // 16 KiB of X per stage
constexpr int WS_BS = WS_TN * WS_TK * 2;  // 32 KiB of fp16 B per stage
constexpr int WS_CS = WS_TN * WS_TK / 2;  // 8 KiB of packed codes per stage
constexpr int WS_NA = 4, WS_NB = 2;       // ring slots (the codes ring has WS_NA slots too)
[[maybe_unused]] constexpr int WS_LDS = WS_NA * (WS_AS + WS_CS) + WS_NB * WS_BS;  // 160 KiB

__device__ __forceinline__ int ws_xh(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) * 6); }
// B column c's chunk q sits at slot q ^ bz(c), bz(c) = (c & 7) ^ ((c >> 3) & 1): conflict-free for both
// accesses of the image (MI355X_MICROARCH.md §LDS) -- the producers' ds_write_b128 (8 groups of 8
// contiguous lanes on 32 banks: bz is a permutation on every 8 aligned columns) and the consumers'
// ds_read_b128 (16-lane groups {0-3, 12-15, 20-27}, ... mixing lane groups g and g ^ 1: chunks 2 g + s of
// 16 columns on 64 banks).  The forms measured before it: (c >> 1) & 7 (2-way on the reads, 4-way on
// the writes) and the A rows' xh (reads clean, writes 2-way) -- profiles/r06_pmc_prefill_ws.txt
__device__ __forceinline__ int ws_bz(int c) { return (c & 7) ^ ((c >> 3) & 1); }

__device__ __forceinline__ int64_t ws_block(int64_t bid, int64_t nblocks) {  // XCD-contiguous tile order
  const int64_t xcd = bid % 8, i = bid / 8;
  const int64_t q = nblocks / 8, r = nblocks % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + i;
}

// the workgroup barrier as a compiler barrier for memory too (a bare s_barrier builtin lets LLVM move
// LDS accesses across it)
__device__ __forceinline__ void ws_barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ void ws_glds16(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

#if IWQ_AB  // an A/B form: the product library carries no instance of it
template <int AHEAD, int PRIO, bool DIAG>
__global__ __launch_bounds__(WS_THR) void k_w4a16_ws(PrefillArgs a) {
  static_assert(AHEAD >= 1 && AHEAD <= WS_NA - 1, "A ring: AHEAD stages in flight + the one being read");
  __shared__ __attribute__((aligned(16))) uint8_t smem[WS_LDS];
  uint8_t* const sa = smem;                   // A ring
  uint8_t* const sb = smem + WS_NA * WS_AS;   // B ring
  uint8_t* const sc = sb + WS_NB * WS_BS;     // codes ring
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = a.N / WS_TN;
  const int64_t t = ws_block(blockIdx.x, (int64_t)gridDim.x);
  const int m0 = (int)(t / tiles_n) * WS_TM, n0 = (int)(t % tiles_n) * WS_TN;
  const int nk = a.K / WS_TK;
  const int64_t crow = a.K / 2;

  if (wid >= 4) {
    // ------------------------------------------------------------------ producers
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
    const int pw = wid - 4;
    const int c = tid - 256;  // this thread's column of the tile
    // X DMA: wave pw issues instructions i = 4 pw .. 4 pw + 3 of a stage: rows 8 i + lane / 8, LDS
    // chunk lane % 8 holding logical chunk (lane % 8) ^ xh(row)
    const _Float16* xsrc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = (pw * 4 + j) * 8 + (lane >> 3);
      const int gm = m0 + row < a.M ? m0 + row : a.M - 1;
      xsrc[j] = a.x + (int64_t)gm * a.lda + (((lane & 7) ^ ws_xh(row)) << 3);
    }
    // codes DMA: wave pw issues instructions j = 0, 1 of a stage: columns (2 pw + j) 32 + lane % 32,
    // 16-B half lane / 32 -- half h of column c lands at codes-slot byte 1024 (c / 32) + 512 h + 16 (c % 32),
    // so a half's ds_read_b128 covers 16 distinct slots in every lane group (column-major 32 c was 2-way)
    const uint8_t* csrc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) csrc[j] = a.codes + (int64_t)(n0 + (pw * 2 + j) * 32 + (lane & 31)) * crow + (lane >> 5) * 16;
    const float zf = a.zeros ? (float)gp<_Float16>(a.zeros)[n0 + c] : a.zsym;
    const h2 zz = h2{(_Float16)(1024.0f + zf), (_Float16)(1024.0f + zf)};
    uint8_t* const bcol = sb + c * 128;
    const int bzc = ws_bz(c);
    const uint32_t cread = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)(sc + (c >> 5) * 1024 + (c & 31) * 16));
    // Everything the producers move goes through LDS-DMA (X and codes) and inline-asm LDS reads /
    // writes: the compiler then tracks no VMEM result in a register and inserts no vmcnt wait of its
    // own (a register-loaded code ring made it wait for every load in flight at loop-carried uses);
    // the waits below are the protocol's.
    auto issue = [&](int kt) {  // kt clamped: re-loads nobody reads keep the vmcnt counts static
      const int kc = kt < nk ? kt : nk - 1;
      uint8_t* abase = sa + (kt % WS_NA) * WS_AS;
      uint8_t* cbase = sc + (kt % WS_NA) * WS_CS;
#pragma unroll
      for (int j = 0; j < 4; ++j) ws_glds16(xsrc[j] + kc * WS_TK, abase + (pw * 4 + j) * 1024);
#pragma unroll
      for (int j = 0; j < 2; ++j) ws_glds16(csrc[j] + kc * 32, cbase + (pw * 2 + j) * 1024);
    };
    auto fill = [&](int kt) {  // the codes of K-step kt (landed) -> fp16 (q - z) into B slot kt % 2
      u32x4 cw[2];
      asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:512\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(cw[0]), "=&v"(cw[1])
                   : "v"(cread + (uint32_t)((kt % WS_NA) * WS_CS))
                   : "memory");
      uint8_t* bdst = bcol + (kt % WS_NB) * WS_BS;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t w = cw[q >> 2][q & 3];
        u32x4 o;
        if constexpr (DIAG) {
          o = (u32x4){w | 0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u};
        } else {
          const uint32_t w4 = w >> 4;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const uint32_t sel = 0x0C000C00u | ((uint32_t)(4 + p) << 16) | (uint32_t)p;
            const uint32_t v = (__builtin_amdgcn_perm(w4, w, sel) & 0x000F000Fu) | 0x64006400u;
            o[p] = as_u32(as_h2(v) - zz);  // (1024 + q) - (1024 + z) = q - z exactly
          }
        }
        const uint32_t la_ = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)(bdst + ((q ^ bzc) << 4)));
        asm volatile("ds_write_b128 %0, %1" ::"v"(la_), "v"(o) : "memory");
      }
    };
    // prologue: K-steps 0 .. AHEAD - 1 in flight; stage 0 filled before B_0
#pragma unroll
    for (int k = 0; k < AHEAD; ++k) issue(k);
    // in flight (oldest first): step 0's 6 DMA, then AHEAD - 1 more steps: 6 (AHEAD - 1) younger
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * (AHEAD - 1)) : "memory");
    fill(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ws_barrier();  // B_0
    for (int kt = 0; kt < nk; ++kt) {
      // between B_kt and B_kt+1: the DMA of K-step kt + AHEAD (its A / codes slots held stage kt - 1,
      // retired before B_kt), then stage kt + 1
      issue(kt + AHEAD);
      // oldest in flight: step kt + 1; younger: steps kt + 2 .. kt + AHEAD
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * (AHEAD - 1)) : "memory");
      if (kt + 1 < nk) fill(kt + 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ws_barrier();  // B_kt+1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup retires
    return;
  }

  // -------------------------------------------------------------------- consumers
  const int wm = wid >> 1, wn = wid & 1;
  const int r16 = lane & 15, g = lane >> 4;
  // A fragment (slice s, tile mt) of stage slot st: row wm 64 + 16 mt + r16, chunk 2 g + s
  uint32_t la[2], lb[2];
  const uint32_t abase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(sa));
  const uint32_t bbase = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)(sb));
  const int arow = wm * 64 + r16;  // + 16 mt: xh depends on r & 15 only, so one swizzle serves all mt
  const int bcol0 = wn * 128 + r16;  // + 16 nt: bz depends on c & 15 only
#pragma unroll
  for (int s = 0; s < 2; ++s) la[s] = abase + (uint32_t)(arow * 128 + (((2 * g + s) ^ ws_xh(arow)) << 4));
#pragma unroll
  for (int s = 0; s < 2; ++s) lb[s] = bbase + (uint32_t)(bcol0 * 128);
  int bq[2][8];  // B chunk offsets per (slice, nt): the column swizzle changes with nt
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) bq[s][nt] = nt * 16 * 128 + (((2 * g + s) ^ ws_bz(bcol0 + 16 * nt)) << 4);
  (void)bq;
  f4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 af0[4], bf0[8], af1[4], bf1[8];
  typedef __attribute__((address_space(3))) const h8 lds_h8;
  auto rd = [](uint32_t addr) -> h8 { return *(lds_h8*)(uintptr_t)addr; };
  auto read_slice = [&](int kt, int s, h8 (&af)[4], h8 (&bf)[8]) {
    const uint32_t ao = (uint32_t)((kt % WS_NA) * WS_AS), bo = (uint32_t)((kt % WS_NB) * WS_BS);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) af[mt] = rd(la[s] + ao + mt * 16 * 128);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) bf[nt] = rd(lb[s] + bo + (uint32_t)bq[s][nt]);
  };
  auto mma = [&](const h8 (&af)[4], const h8 (&bf)[8]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mt], bf[nt], acc[mt][nt], 0, 0, 0);
  };
  ws_barrier();  // B_0: stage 0 published
  read_slice(0, 0, af0, bf0);
  read_slice(0, 1, af1, bf1);
  for (int kt = 0; kt < nk; ++kt) {
    mma(af0, bf0);                                        // slice 0 of stage kt
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // every read of stage kt landed
    ws_barrier();                                         // B_kt+1: stage kt + 1 published
    if (kt + 1 < nk) read_slice(kt + 1, 0, af0, bf0);     // covered by slice 1's MFMAs
    mma(af1, bf1);                                        // slice 1 of stage kt
    if (kt + 1 < nk) read_slice(kt + 1, 1, af1, bf1);
  }
  // epilogue: lane holds rows wm 64 + 16 mt + 4 g + r of columns n0 + wn 128 + 16 nt + r16
  const int64_t ld = a.ldy;
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    const int col = n0 + wn * 128 + nt * 16 + r16;
    const float sc = (float)gp<_Float16>(a.scales)[col];
    const float bc = a.bias ? (float)gp<_Float16>(a.bias)[col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + mt * 16 + 4 * g + r;
        if (row < a.M) a.y[(int64_t)row * ld + col] = (_Float16)(opaque(acc[mt][nt][r] * sc) + bc);
      }
  }
}

#endif  // IWQ_AB

}  // namespace

bool prefill_ws_supported(int64_t M, int64_t N, int64_t K, int gpr, int group) {
  (void)group;
  return M >= 1 && N % WS_TN == 0 && K % WS_TK == 0 && K >= WS_TK && gpr == 1;
}

hipError_t prefill_ws_launch(const PrefillArgs& a, int variant, hipStream_t st) {
#if IWQ_AB
  const int64_t blocks = ((int64_t)(a.M + WS_TM - 1) / WS_TM) * (a.N / WS_TN);
  const dim3 grid((unsigned)blocks), blk(WS_THR);
  switch (variant) {
    case 180: hipLaunchKernelGGL((k_w4a16_ws<3, 0, false>), grid, blk, 0, st, a); break;
    case 181: hipLaunchKernelGGL((k_w4a16_ws<2, 0, false>), grid, blk, 0, st, a); break;
    case 182: hipLaunchKernelGGL((k_w4a16_ws<3, 1, false>), grid, blk, 0, st, a); break;
    case 183: hipLaunchKernelGGL((k_w4a16_ws<3, 0, true>), grid, blk, 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
#else
  (void)a;
  (void)variant;
  (void)st;
  return hipErrorInvalidValue;
#endif
}

}  // namespace iwq

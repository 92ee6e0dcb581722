// iwq_prefill.h — host-side interface of the prefill (large-M) fused dequant -> GEMM kernel on
// 32x32x16 MFMA (iwq_prefill.hip), called by iwq_w4a16_gemm (iwq_gemm.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace iwq {

struct PrefillArgs {
  const _Float16* x;       // [M, K] fp16, row stride lda (multiple of 8 elements, 16-B aligned)
  int64_t lda;
  const uint8_t* codes;    // [N, K/2] row-major packed 4-bit codes (low nibble = even k)
  const _Float16* scales;  // [N * gpr] fp16 (per channel: gpr = 1)
  const _Float16* zeros;   // [N * gpr] fp16, or null (symmetric: zsym)
  const _Float16* bias;    // [N] fp16 or null
  _Float16* y;             // [M, N] fp16, row stride ldy
  int64_t ldy;
  int M, N, K;
  int gpr;                 // scale groups per row (K / group)
  int group;               // group length along K
  float zsym;              // symmetric code offset 2^(b-1)
  float* ws = nullptr;     // split-K: fp32 partial tiles (prefill_splitk_bytes), else unused
  int nsplit = 1;          // split-K: number of K ranges
  int kps = 0;             // split-K: 64-k steps per range
  int pgm = 0;             // grouped, 16x16x32 forms: scales / zeros held group-major, [gpr, N] (IWQ_FLAG_GROUP_MAJOR)
};

// mid-size M (k_w4a16_mid): N % 64 == 0, K % 128 == 0, per-channel or group % 32 == 0; codes
// row-major or (tiled) in the decode tile layout
bool mid_supported(int64_t M, int64_t N, int64_t K, int gpr, int group);
hipError_t mid_launch(const PrefillArgs& a, int variant, bool tiled, hipStream_t st);

// N % 256 == 0, K % 64 == 0, per-channel or group % 64 == 0
bool prefill_b32_supported(int64_t M, int64_t N, int64_t K, int gpr, int group);
// variant: 0 = default; A/B variants documented at the dispatch in iwq_prefill.hip
// nib: codes in the NIB layout (variant 0 only)
hipError_t prefill_b32_launch(const PrefillArgs& a, int variant, hipStream_t st, bool nib = false);

// split-K form of the prefill kernel for M where the 256 x 256 tiles leave CUs idle: number of K
// ranges for the problem (1 = no split; force > 1 overrides the rule), the fp32 workspace it needs,
// and the launch (partial tiles to a.ws, then one reduce kernel: fixed split order, deterministic)
int prefill_splitk_count(int64_t M, int64_t N, int64_t K, int force);
int64_t prefill_splitk_bytes(int64_t M, int64_t N, int nsplit);
// nib: codes in the NIB layout (iwq_nib_codes), partials from 74's NIB twin
hipError_t prefill_splitk_launch(const PrefillArgs& a, hipStream_t st, bool legacy = false, bool nib = false);
// split prefill preferred over the mid-M kernel (M >= 256: whenever a split helps)
bool prefill_split_preferred(int64_t M, int64_t N, int64_t K, int gpr, int group);
// short-tile split prefill (k_w4a16_b32s, mtw 2 or 4 tiles of 32 rows per wave)
int64_t prefill_splitk_bytes_s(int64_t M, int64_t N, int mtw, int nsplit);
hipError_t prefill_splitk_launch_s(const PrefillArgs& a, int mtw, hipStream_t st);
// default plan for 16 < M < 256: the short-tile split (64-row tiles, *ns ranges) or not
bool prefill_short_split(int64_t M, int64_t N, int64_t K, int gpr, int group, int* ns, int* mtw);

// 16x16x32 form of the prefill kernel (iwq_prefill16.hip), per channel: A/B variants 150 / 151
bool prefill16_supported(int64_t M, int64_t N, int64_t K, int gpr, int group);
hipError_t prefill16_launch(const PrefillArgs& a, int variant, hipStream_t st);

// warp-specialised prefill (iwq_prefill_ws.hip, round 6 A/B variants 180-183): per channel, N % 256 == 0,
// K % 64 == 0
bool prefill_ws_supported(int64_t M, int64_t N, int64_t K, int gpr, int group);
hipError_t prefill_ws_launch(const PrefillArgs& a, int variant, hipStream_t st);

}  // namespace iwq

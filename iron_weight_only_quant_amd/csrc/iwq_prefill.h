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
};

// mid-size M (k_w4a16_mid): N % 64 == 0, K % 128 == 0, per-channel or group % 32 == 0; codes
// row-major or (tiled) in the decode tile layout
bool mid_supported(int64_t M, int64_t N, int64_t K, int gpr, int group);
hipError_t mid_launch(const PrefillArgs& a, int variant, bool tiled, hipStream_t st);

// N % 256 == 0, K % 64 == 0, per-channel or group % 64 == 0
bool prefill_b32_supported(int64_t M, int64_t N, int64_t K, int gpr, int group);
// variant: 0 = default; A/B variants documented at the dispatch in iwq_prefill.hip
hipError_t prefill_b32_launch(const PrefillArgs& a, int variant, hipStream_t st);

}  // namespace iwq

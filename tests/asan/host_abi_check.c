/*
 * Host-side checks of the C-ABI (include/iwq.h) under AddressSanitizer + UndefinedBehaviorSanitizer
 * (SURVEY.md §5 "Race detection / sanitizers": host ASan/UBSan on the C-ABI CPU paths).
 *
 * Built by tests/asan/Makefile from the library's own sources, host side only (--offload-host-only,
 * -Xarch_host -fsanitize=...): the plan / validation / dispatch code every entry point runs before a
 * kernel launch.  No GPU is needed: device pointers are fake (never dereferenced on the host), valid
 * calls end at the launch with IWQ_ERR_HIP (no device), invalid ones must return the documented
 * status without touching anything.  Any sanitizer report aborts the program (halt_on_error).
 * Run by tests/test_cpu_host.py::test_host_abi_under_asan_ubsan.
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/iwq.h"

static int failures = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    if (!(cond)) {                                                               \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);           \
      ++failures;                                                                \
    }                                                                            \
  } while (0)

#define DEV(x) ((void*)(uintptr_t)(0x10000000ull + (uint64_t)(x) * 0x1000000ull))

static void fill(iwq_batch_entry* e, int n, const int64_t (*shapes)[2], int codes) {
  memset(e, 0, sizeof(*e) * (size_t)n);
  for (int i = 0; i < n; ++i) {
    e[i].w = DEV(4 * i);
    e[i].out_deq = DEV(4 * i + 1);
    e[i].out_codes = codes ? DEV(4 * i + 2) : NULL;
    e[i].out_scales = DEV(4 * i + 3);
    e[i].out_zeros = DEV(4 * i + 3);
    e[i].rows = shapes[i][0];
    e[i].cols = shapes[i][1];
  }
}

static void check_batch_plans(void) {
  const int64_t llama[7][2] = {{4096, 4096}, {4096, 4096}, {4096, 4096}, {4096, 4096},
                               {11008, 4096}, {11008, 4096}, {4096, 11008}};
  iwq_batch_entry e[7];
  int64_t total = -1, glen = -1;
  fill(e, 7, llama, 1);
  CHECK(iwq_batch_plan(e, 7, IWQ_F16, 4, 128, &total) == IWQ_OK);
  int64_t want = 0;
  for (int i = 0; i < 7; ++i) {
    CHECK(e[i].unit_begin == want);
    want += llama[i][0] * llama[i][1] / 512;
  }
  CHECK(total == want);
  CHECK(iwq_batch_plan(NULL, 7, IWQ_F16, 4, 128, &total) == IWQ_ERR_ARG);
  CHECK(iwq_batch_plan(e, 0, IWQ_F16, 4, 128, &total) == IWQ_ERR_ARG);
  CHECK(iwq_batch_plan(e, 7, 7, 4, 128, &total) == IWQ_ERR_DTYPE);
  CHECK(iwq_batch_plan(e, 7, IWQ_F16, 9, 128, &total) == IWQ_ERR_BITS);
  CHECK(iwq_batch_plan(e, 7, IWQ_F16, 4, 96, &total) == IWQ_ERR_GROUP_MODE);
  e[3].w = (const void*)((uintptr_t)e[3].w + 2);
  CHECK(iwq_batch_plan(e, 7, IWQ_F16, 4, 128, &total) == IWQ_ERR_ARG);  /* unaligned */
  fill(e, 7, llama, 1);
  e[2].cols = 4095;
  CHECK(iwq_batch_plan(e, 7, IWQ_F16, 4, 128, &total) == IWQ_ERR_GROUP);
  e[2].cols = 8192;  /* divisible: fine */
  CHECK(iwq_batch_plan(e, 7, IWQ_F16, 4, 128, &total) == IWQ_OK);

  /* the _ex modes */
  fill(e, 7, llama, 0);
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 4, 128, 0, &total, &glen) == IWQ_OK && glen == 128 && total == want);
  fill(e, 4, llama, 0);  /* per channel, one row length */
  CHECK(iwq_batch_plan_ex(e, 4, IWQ_F16, 8, IWQ_GROUP_PER_CHANNEL, 0, &total, &glen) == IWQ_OK);
  CHECK(glen == 4096 && total == 4 * 4096 && e[3].unit_begin == 3 * 4096);
  fill(e, 7, llama, 0);  /* mixed row lengths in one table: bucket by length */
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 8, IWQ_GROUP_PER_CHANNEL, 0, &total, &glen) == IWQ_ERR_ARG);
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 4, IWQ_GROUP_PER_TENSOR, 0, &total, &glen) == IWQ_OK && total == want);
  CHECK(iwq_batch_workspace_bytes(7, IWQ_GROUP_PER_TENSOR, 0) >= 7 * 8);
  CHECK(iwq_batch_workspace_bytes(7, 128, 0) == 0);
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 4, 128, 1, &total, &glen) == IWQ_OK);  /* quant_dim 1 */
  CHECK(e[1].unit_begin == (4096 / 256) * (4096 / 128));
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_BF16, 4, 64, 1, &total, &glen) == IWQ_OK);
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 4, 1024, 0, &total, &glen) == IWQ_ERR_GROUP);  /* 11008 % 1024 */
  CHECK(iwq_batch_plan_ex(e, 4, IWQ_F16, 4, 1024, 0, &total, &glen) == IWQ_OK && glen == 1024);  /* long group */
  CHECK(total == 4 * 4096 * 4);
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 4, 96, 0, &total, &glen) == IWQ_ERR_GROUP);  /* 4096 % 96 */
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 4, 0, 0, &total, &glen) == IWQ_ERR_GROUP_MODE);
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 0, 128, 0, &total, &glen) == IWQ_ERR_BITS);
  CHECK(iwq_batch_plan_ex(e, 7, IWQ_F16, 4, 128, 2, &total, &glen) == IWQ_ERR_ARG);
  const int64_t wide[1][2] = {{8192, 28672}};  /* 28672-element rows: beyond the register-resident row kernel */
  fill(e, 1, wide, 0);
  CHECK(iwq_batch_plan_ex(e, 1, IWQ_F16, 4, IWQ_GROUP_PER_CHANNEL, 0, &total, &glen) == IWQ_ERR_ARG);
}

static void check_quantize_validation(void) {
  void* w = DEV(1);
  void* out = DEV(2);
  void* s = DEV(3);
  uint32_t* flag = (uint32_t*)DEV(5);
  /* every invalid argument returns its status before any launch */
  CHECK(iwq_quantize_minmax(w, 64, 128, 128, 9, 4, 128, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_DTYPE);
  CHECK(iwq_quantize_minmax(NULL, 64, 128, 128, IWQ_F16, 4, 128, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_quantize_minmax(w, 0, 128, 128, IWQ_F16, 4, 128, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_SHAPE);
  CHECK(iwq_quantize_minmax(w, 64, 128, 100, IWQ_F16, 4, 128, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_SHAPE);
  CHECK(iwq_quantize_minmax(w, 64, 128, 128, IWQ_F16, 0, 128, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_BITS);
  CHECK(iwq_quantize_minmax(w, 64, 128, 128, IWQ_F16, 1, 128, 1, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_BITS);
  CHECK(iwq_quantize_minmax(w, 64, 100, 100, IWQ_F16, 4, 128, 0, 0, out, 100, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_GROUP);
  CHECK(iwq_quantize_minmax(w, 64, 128, 128, IWQ_F16, 4, -3, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_GROUP_MODE);
  CHECK(iwq_quantize_minmax(w, 64, 128, 128, IWQ_F16, 4, 128, 0, 2, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_quantize_minmax(w, 64, 128, 128, IWQ_F16, 9, 128, 0, 0, out, 128, DEV(6), s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_CODES);
  CHECK(iwq_quantize_minmax(w, 64, 127, 127, IWQ_F16, 4, -2, 0, 0, out, 127, DEV(6), s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_CODES);
  /* per-tensor and universal paths ask for a workspace before launching anything */
  CHECK(iwq_quantize_minmax(w, 64, 128, 128, IWQ_F16, 4, -1, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_WORKSPACE);
  CHECK(iwq_quantize_minmax(w, 48, 100, 100, IWQ_F16, 4, 24, 0, 1, out, 100, NULL, s, s, NULL, 0, flag, 0, NULL) == IWQ_ERR_WORKSPACE);
  CHECK(iwq_workspace_bytes(64, 128, -1, 0) > 0);
  CHECK(iwq_workspace_bytes(48, 100, 24, 1) >= 8 * (100 * 48 / 24));
  CHECK(iwq_workspace_bytes(0, 128, 128, 0) == 0);
  /* a valid call reaches the launch: without a GPU that is IWQ_ERR_HIP, never a crash */
  int st = iwq_quantize_minmax(w, 64, 128, 128, IWQ_F16, 4, 128, 0, 0, out, 128, NULL, s, s, NULL, 0, flag, 0, NULL);
  CHECK(st == IWQ_ERR_HIP || st == IWQ_OK);
  iwq_batch_entry e[1];
  const int64_t sh[1][2] = {{64, 128}};
  fill(e, 1, sh, 0);
  CHECK(iwq_quantize_minmax_batched_ex(NULL, 1, 16, 0, IWQ_F16, 4, 128, 0, 0, NULL, 0, flag, 0, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_quantize_minmax_batched_ex((const iwq_batch_entry*)DEV(9), 1, 16, 0, IWQ_F16, 4, -1, 0, 0, NULL, 0, flag, 0,
                                       NULL) == IWQ_ERR_WORKSPACE);
  CHECK(iwq_quantize_minmax_batched_ex((const iwq_batch_entry*)DEV(9), 1, 16, 100, IWQ_F16, 4, -2, 0, 0, NULL, 0, flag, 0,
                                       NULL) == IWQ_ERR_ARG);  /* row length not a multiple of 8 */
  CHECK(iwq_quantize_minmax_batched_ex((const iwq_batch_entry*)DEV(9), 1, 16, 0, IWQ_F16, 4, 128, 0, 0, NULL, 0, flag,
                                       IWQ_FLAG_FORCE_GENERIC, NULL) == IWQ_ERR_ARG);
}

static void check_gemm_validation(void) {
  void* x = DEV(1);
  void* c = DEV(2);
  void* s = DEV(3);
  void* y = DEV(4);
  CHECK(iwq_w4a16_gemm(NULL, 8, 4096, 4096, c, s, NULL, 4, 128, 4096, NULL, y, 4096, 0, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_w4a16_gemm(x, 8, 4000, 4000, c, s, NULL, 4, 128, 4096, NULL, y, 4096, 0, NULL) == IWQ_ERR_SHAPE);
  CHECK(iwq_w4a16_gemm(x, 8, 4096, 4096, c, s, NULL, 5, 128, 4096, NULL, y, 4096, 0, NULL) == IWQ_ERR_BITS);
  CHECK(iwq_w4a16_gemm(x, 8, 4096, 4096, c, s, NULL, 4, 48, 4096, NULL, y, 4096, 0, NULL) == IWQ_ERR_GROUP);
  CHECK(iwq_w4a16_gemm((char*)x + 2, 8, 4096, 4096, c, s, NULL, 4, 128, 4096, NULL, y, 4096, 0, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_w4a16_gemm_ws(x, 8, 4096, 4096, c, s, NULL, 4, 128, 4096, NULL, y, 4096, NULL, 64, 0, NULL) == IWQ_ERR_ARG);
  /* NIB codes: M >= 256 only, no variant / tiled / generic */
  CHECK(iwq_w4a16_gemm(x, 128, 4096, 4096, c, s, NULL, 4, -2, 4096, NULL, y, 4096, IWQ_FLAG_NIB_CODES, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_w4a16_gemm(x, 17, 4096, 4096, c, s, NULL, 4, -2, 4096, NULL, y, 4096, IWQ_FLAG_TILED_CODES, NULL) == IWQ_ERR_ARG);
  /* group-major parameters: grouped weights, M >= 256, no variant / TILED / FORCE_GENERIC */
  CHECK(iwq_w4a16_gemm(x, 512, 4096, 4096, c, s, NULL, 4, -2, 4096, NULL, y, 4096, IWQ_FLAG_GROUP_MAJOR, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_w4a16_gemm(x, 255, 4096, 4096, c, s, NULL, 4, 128, 4096, NULL, y, 4096, IWQ_FLAG_GROUP_MAJOR, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_w4a16_gemm(x, 512, 4096, 4096, c, s, NULL, 4, 128, 4096, NULL, y, 4096,
                       IWQ_FLAG_GROUP_MAJOR | IWQ_FLAG_FORCE_GENERIC, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_w4a16_gemm(x, 512, 4096, 4096, c, s, NULL, 4, 32, 4096, NULL, y, 4096, IWQ_FLAG_GROUP_MAJOR, NULL) == IWQ_ERR_ARG);
  for (int64_t m = 1; m <= 8192; m *= 2) {
    CHECK(iwq_w4a16_gemm_workspace_bytes(m, 4096, 4096, -2) >= 0);
    CHECK(iwq_w4a16_gemm_workspace_bytes(m, 28672, 8192, 128) >= 0);
  }
  /* misaligned y / workspace: the split paths are dropped (the call still reaches a launch) */
  int st = iwq_w4a16_gemm_ws(x, 512, 4096, 4096, c, s, NULL, 4, -2, 4096, NULL, (char*)y + 2, 4096, DEV(8),
                             1 << 30, 0, NULL);
  CHECK(st == IWQ_ERR_HIP || st == IWQ_OK);
}

static void check_fp_validation(void) {
  void* w = DEV(1);
  void* out = DEV(2);
  void* s = DEV(3);
  uint32_t* flag = (uint32_t*)DEV(5);
  /* E5M2's fp_max (114688) overflows fp16: the reference's torch.clamp raises */
  CHECK(iwq_quantize_fp(w, 64, 128, 128, IWQ_F16, 5, 2, 128, 1, 0, out, 128, NULL, s, NULL, NULL, 0, flag, 0, NULL) ==
        IWQ_ERR_FORMAT);
  CHECK(iwq_quantize_fp(w, 64, 100, 100, IWQ_F16, 4, 3, 128, 1, 0, out, 100, NULL, s, NULL, NULL, 0, flag, 0, NULL) ==
        IWQ_ERR_GROUP);
  CHECK(iwq_quantize_bfp(w, 64, 128, 128, IWQ_F16, 4, -1, 0, out, 128, 0, NULL) == IWQ_ERR_GROUP_MODE);
  CHECK(iwq_quantize_bfp(w, 64, 128, 128, IWQ_F16, 0, 128, 0, out, 128, 0, NULL) == IWQ_ERR_BITS);
  CHECK(iwq_fp4_grid(w, 64, 100, 128, 0, out, s, NULL, 0, flag, 0, NULL) != IWQ_OK);
  CHECK(iwq_approx_workspace_bytes(64, 128, 4, 3, 128, 0, 1) >= 0);
  CHECK(iwq_quantize_fp_approx(w, 64, 128, 128, IWQ_F16, 4, 3, -2, 0, 12, 15, 1, 0, out, 128, s, NULL, 0, flag, 0, NULL) ==
        IWQ_ERR_GROUP_MODE);
  /* product library: an A/B variant of the double-approximate decode is refused before any launch */
  CHECK(iwq_quantize_fp_approx(w, 64, 128, 128, IWQ_F16, 4, 3, 128, 0, 12, 15, 1, 1, out, 128, s, NULL, 0, flag,
                               2u << 16, NULL) == IWQ_ERR_ARG);
  CHECK(iwq_quantize_fp_approx(w, 64, 128, 128, IWQ_F16, 4, 3, 128, 0, 12, 15, 1, 0, out, 128, s, NULL, 0, flag,
                               1u << 16, NULL) == IWQ_ERR_ARG);
  /* the table paths (a decode table given): every format's table-argument setup up to the launch --
   * E4M3 / E3M2 / E2M1 embed the codes in the entries, E3M4 does not; with and without packed codes,
   * sym / asym, plus the batched form and the approximate decode */
  void* lut = DEV(6);
  void* codes = DEV(7);
  void* z = DEV(8);
  const int fmts[4][2] = {{4, 3}, {3, 2}, {2, 1}, {3, 4}};
  for (int i = 0; i < 4; ++i)
    for (int sym = 0; sym <= 1; ++sym)
      for (int wc = 0; wc <= 1; ++wc) {
        const int st = iwq_quantize_fp_lut(w, 64, 128, 128, IWQ_F16, fmts[i][0], fmts[i][1], 128, sym, 0, out, 128,
                                           wc ? codes : NULL, s, sym ? NULL : z, NULL, 0, flag, 0, NULL, lut);
        CHECK(st == IWQ_ERR_HIP || st == IWQ_OK);
      }
  int st = iwq_quantize_fp_approx_lut(w, 64, 128, 128, IWQ_F16, 4, 3, 128, 0, 12, 15, 1, 0, out, 128, s, NULL, 0, flag,
                                      0, NULL, lut);
  CHECK(st == IWQ_ERR_HIP || st == IWQ_OK);
  st = iwq_fp4_grid_packed(w, 64, 128, 128, 0, out, codes, s, NULL, 0, flag, 0, NULL, lut);
  CHECK(st == IWQ_ERR_HIP || st == IWQ_OK);
}

int main(void) {
  for (int st = 0; st <= 11; ++st) CHECK(iwq_status_string(st) != NULL && strlen(iwq_status_string(st)) > 0);
  CHECK(strstr(iwq_build_info(), "gfx950") != NULL);
  check_batch_plans();
  check_quantize_validation();
  check_gemm_validation();
  check_fp_validation();
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("host ABI checks passed under ASan/UBSan\n");
  return 0;
}

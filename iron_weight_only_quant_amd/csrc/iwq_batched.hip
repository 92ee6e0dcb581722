// iwq_batched.hip -- gfx950 batched-table launches of the row / column / per-tensor min-max kernels
// (iwq_batch_plan_ex / iwq_quantize_minmax_batched_ex, include/iwq.h): quant_wrapper.py:52-82's
// RTN loop as a few launches for per-channel (-2), per-tensor (-1), quant_dim 1 and groups outside
// the power-of-two 8..512 range that k_group's one-launch walk covers (iwq_minmax.hip).  Kernels:
// iwq_minmax.cuh (k_rowwave_b, k_column_b, k_keys_init / k_tensor_reduce_b / k_tensor_apply_b).
#include "iwq_minmax.cuh"

namespace {

// ---- batched row / column / per-tensor launches (iwq_quantize_minmax_batched_ex) ----
enum BatchMode { BM_GROUP = 0, BM_ROW = 1, BM_COL = 2, BM_TENSOR = 3 };
int batch_mode(int64_t group, int quant_dim) {
  if (group == IWQ_GROUP_PER_TENSOR) return BM_TENSOR;
  if (quant_dim == 1) return BM_COL;
  if (group >= 8 && group <= 512 && is_pow2(group)) return BM_GROUP;
  return BM_ROW;
}
// quant_dim-1 block shape (the single-tensor default's rule, launch_col_v variant 0):
// 0 = 32 x 8 generic body (any g: per-channel g = rows differs per entry), 1 = 32 x 8 with the
// rows in registers (g 64 / 128, or 32 for bf16 / fp32), 2 = 64 x 4 (fp16 g 32), 3 = 16 x 16 (g 256)
int col_shape(int dt, int64_t group) {
  if (group == 32) return dt == IWQ_F16 ? 2 : 1;
  if (group == 64 || group == 128) return 1;
  if (group == 256) return 3;
  return 0;
}
int64_t col_tx(int shape) { return shape == 2 ? 64 : (shape == 3 ? 16 : 32); }

template <int DT, int CPL, bool SYM, int CODES>
hipError_t launch_row_b_k(const BatchExArgs& b, hipStream_t st) {
  constexpr bool PF = CPL <= 8 && DT != DT_F32;  // launch_row_t's register budget for two images
  static int cache[64] = {0};
  auto kern = k_rowwave_b<DT, CPL, SYM, CODES, PF>;
  int64_t blocks = (b.total_units + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  const int64_t cap = (int64_t)device_cu_count() * resident_blocks_per_cu(kern, cache);
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(BLOCK), 0, st, b);
  return hipGetLastError();
}
template <int DT, int CPL, bool SYM>
hipError_t launch_row_b_c(int codes, const BatchExArgs& b, hipStream_t st) {
  if (codes == 0) return launch_row_b_k<DT, CPL, SYM, 0>(b, st);
  if (codes == 4) return launch_row_b_k<DT, CPL, SYM, 4>(b, st);
  return launch_row_b_k<DT, CPL, SYM, 8>(b, st);
}
template <int DT, bool SYM>
hipError_t launch_row_b_l(int64_t L, int codes, const BatchExArgs& b, hipStream_t st) {
  const int64_t chunks = L / 8;  // launch_row_c's register classes
  if (chunks <= 64 * 1) return launch_row_b_c<DT, 1, SYM>(codes, b, st);
  if (chunks <= 64 * 2) return launch_row_b_c<DT, 2, SYM>(codes, b, st);
  if (chunks <= 64 * 4) return launch_row_b_c<DT, 4, SYM>(codes, b, st);
  if (chunks <= 64 * 8) return launch_row_b_c<DT, 8, SYM>(codes, b, st);
  if (chunks <= 64 * 12) return launch_row_b_c<DT, 12, SYM>(codes, b, st);
  if (chunks <= 64 * 16) return launch_row_b_c<DT, 16, SYM>(codes, b, st);
  if (chunks <= 64 * 24) return launch_row_b_c<DT, 24, SYM>(codes, b, st);
  return launch_row_b_c<DT, 32, SYM>(codes, b, st);
}
hipError_t launch_row_b(int dt, bool sym, int64_t L, int codes, const BatchExArgs& b, hipStream_t st) {
  if (dt == IWQ_F16) return sym ? launch_row_b_l<DT_F16, true>(L, codes, b, st) : launch_row_b_l<DT_F16, false>(L, codes, b, st);
  if (dt == IWQ_BF16) return sym ? launch_row_b_l<DT_BF16, true>(L, codes, b, st) : launch_row_b_l<DT_BF16, false>(L, codes, b, st);
  return sym ? launch_row_b_l<DT_F32, true>(L, codes, b, st) : launch_row_b_l<DT_F32, false>(L, codes, b, st);
}

template <int DT, bool SYM, int CODES>
hipError_t launch_col_b_k(int shape, const BatchExArgs& b, hipStream_t st) {
  const dim3 grid((unsigned)b.total_units);
  if (shape == 2) hipLaunchKernelGGL((k_column_b<DT, SYM, CODES, 64, 4, 8>), grid, dim3(256), 0, st, b);
  else if (shape == 3) hipLaunchKernelGGL((k_column_b<DT, SYM, CODES, 16, 16, 16>), grid, dim3(256), 0, st, b);
  else if (shape == 1 && b.group == 32) hipLaunchKernelGGL((k_column_b<DT, SYM, CODES, 32, 8, 4>), grid, dim3(256), 0, st, b);
  else if (shape == 1 && b.group == 64) hipLaunchKernelGGL((k_column_b<DT, SYM, CODES, 32, 8, 8>), grid, dim3(256), 0, st, b);
  else if (shape == 1) hipLaunchKernelGGL((k_column_b<DT, SYM, CODES, 32, 8, 16>), grid, dim3(256), 0, st, b);
  else hipLaunchKernelGGL((k_column_b<DT, SYM, CODES, 32, 8, 0>), grid, dim3(256), 0, st, b);
  return hipGetLastError();
}
template <int DT, bool SYM>
hipError_t launch_col_b_c(int codes, int shape, const BatchExArgs& b, hipStream_t st) {
  if (codes == 0) return launch_col_b_k<DT, SYM, 0>(shape, b, st);
  if (codes == 4) return launch_col_b_k<DT, SYM, 4>(shape, b, st);
  return launch_col_b_k<DT, SYM, 8>(shape, b, st);
}
hipError_t launch_col_b(int dt, bool sym, int codes, int shape, const BatchExArgs& b, hipStream_t st) {
  if (dt == IWQ_F16) return sym ? launch_col_b_c<DT_F16, true>(codes, shape, b, st) : launch_col_b_c<DT_F16, false>(codes, shape, b, st);
  if (dt == IWQ_BF16) return sym ? launch_col_b_c<DT_BF16, true>(codes, shape, b, st) : launch_col_b_c<DT_BF16, false>(codes, shape, b, st);
  return sym ? launch_col_b_c<DT_F32, true>(codes, shape, b, st) : launch_col_b_c<DT_F32, false>(codes, shape, b, st);
}

template <int DT, bool SYM, int CODES>
hipError_t launch_tensor_b_k(const GroupArgs& a, int32_t* keys, hipStream_t st) {
  static int cache_r[64] = {0}, cache_a[64] = {0};
  hipLaunchKernelGGL(k_keys_init, dim3((unsigned)((a.n_entries + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, keys,
                     a.n_entries);
  const int64_t waves_needed = (a.total_units + 3) / 4;
  const int64_t want = (waves_needed + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  auto kr = k_tensor_reduce_b<DT, SYM>;
  auto ka = k_tensor_apply_b<DT, SYM, CODES>;
  int64_t br = (int64_t)device_cu_count() * resident_blocks_per_cu(kr, cache_r);
  int64_t ba = (int64_t)device_cu_count() * resident_blocks_per_cu(ka, cache_a);
  if (br > want) br = want;
  if (ba > want) ba = want;
  hipLaunchKernelGGL(kr, dim3((unsigned)(br < 1 ? 1 : br)), dim3(BLOCK), 0, st, a, keys);
  hipLaunchKernelGGL(ka, dim3((unsigned)(ba < 1 ? 1 : ba)), dim3(BLOCK), 0, st, a, static_cast<const int32_t*>(keys));
  return hipGetLastError();
}
template <int DT, bool SYM>
hipError_t launch_tensor_b_c(int codes, const GroupArgs& a, int32_t* keys, hipStream_t st) {
  if (codes == 0) return launch_tensor_b_k<DT, SYM, 0>(a, keys, st);
  if (codes == 4) return launch_tensor_b_k<DT, SYM, 4>(a, keys, st);
  return launch_tensor_b_k<DT, SYM, 8>(a, keys, st);
}
hipError_t launch_tensor_b(int dt, bool sym, int codes, const GroupArgs& a, int32_t* keys, hipStream_t st) {
  if (dt == IWQ_F16) return sym ? launch_tensor_b_c<DT_F16, true>(codes, a, keys, st) : launch_tensor_b_c<DT_F16, false>(codes, a, keys, st);
  if (dt == IWQ_BF16) return sym ? launch_tensor_b_c<DT_BF16, true>(codes, a, keys, st) : launch_tensor_b_c<DT_BF16, false>(codes, a, keys, st);
  return sym ? launch_tensor_b_c<DT_F32, true>(codes, a, keys, st) : launch_tensor_b_c<DT_F32, false>(codes, a, keys, st);
}

}  // namespace

extern "C" {

int iwq_batch_plan_ex(iwq_batch_entry* h_entries, int32_t n_entries, int dtype, int n_bits, int64_t group,
                      int quant_dim, int64_t* h_total_units, int64_t* h_group_len) {
  if (!h_entries || n_entries <= 0 || !h_total_units) return IWQ_ERR_ARG;
  if (dtype != IWQ_F16 && dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (n_bits < 1 || n_bits > 8) return IWQ_ERR_BITS;
  if (quant_dim != 0 && quant_dim != 1) return IWQ_ERR_ARG;
  if (!(group > 0 || group == IWQ_GROUP_PER_TENSOR || group == IWQ_GROUP_PER_CHANNEL)) return IWQ_ERR_GROUP_MODE;
  const int mode = batch_mode(group, quant_dim);
  if (mode == BM_GROUP) {
    if (n_bits < 2) return IWQ_ERR_BITS;
    if (h_group_len) *h_group_len = group;
    return iwq_batch_plan(h_entries, n_entries, dtype, n_bits, group, h_total_units);
  }
  const int eb = elem_bytes(dtype);
  int64_t u = 0, len = 0;
  for (int32_t i = 0; i < n_entries; ++i) {
    iwq_batch_entry& e = h_entries[i];
    if (!e.w || e.rows <= 0 || e.cols <= 0) return IWQ_ERR_SHAPE;
    if (!aligned16(e.w) || (e.out_deq && !aligned16(e.out_deq)) || (e.out_codes && !aligned16(e.out_codes)))
      return IWQ_ERR_ARG;
    if (e.out_codes && n_bits <= 4 && (e.cols & 1)) return IWQ_ERR_CODES;
    e.unit_begin = u;
    if (mode == BM_TENSOR) {
      if ((e.rows * e.cols) % 8 != 0) return IWQ_ERR_ARG;
      u += (e.rows * e.cols + UNIT - 1) / UNIT;
    } else if (mode == BM_ROW) {
      const int64_t L = group > 0 ? group : e.cols;
      if (group > 0 && e.cols % group != 0) return IWQ_ERR_GROUP;
      if (L % 8 != 0 || L > ROW_MAX_L || (e.cols * eb) % 16 != 0) return IWQ_ERR_ARG;
      if (len != 0 && L != len) return IWQ_ERR_ARG;  // one register class per launch: bucket by L
      len = L;
      u += e.rows * (e.cols / L);
    } else {  // BM_COL
      const int64_t g = group > 0 ? group : e.rows;
      if (e.rows % g != 0) return IWQ_ERR_GROUP;
      if (e.cols % 8 != 0) return IWQ_ERR_ARG;
      const int64_t tx = col_tx(col_shape(dtype, group > 0 ? group : 0));
      u += ((e.cols + 8 * tx - 1) / (8 * tx)) * (e.rows / g);
    }
  }
  if (mode == BM_COL && u > 0x7FFFFFFF) return IWQ_ERR_SHAPE;
  *h_total_units = u;
  if (h_group_len) *h_group_len = len;
  return IWQ_OK;
}

int64_t iwq_batch_workspace_bytes(int32_t n_entries, int64_t group, int quant_dim) {
  (void)quant_dim;
  if (group != IWQ_GROUP_PER_TENSOR || n_entries <= 0) return 0;
  return ((8 * (int64_t)n_entries + 255) / 256) * 256;
}

int iwq_quantize_minmax_batched_ex(const iwq_batch_entry* d_entries, int32_t n_entries, int64_t total_units,
                                   int64_t group_len, int dtype, int n_bits, int64_t group, int symmetric,
                                   int quant_dim, void* workspace, int64_t workspace_bytes, uint32_t* nan_flag,
                                   unsigned flags, void* stream) {
  if (!d_entries || n_entries <= 0 || total_units <= 0) return IWQ_ERR_ARG;
  if (dtype != IWQ_F16 && dtype != IWQ_BF16 && dtype != IWQ_F32) return IWQ_ERR_DTYPE;
  if (n_bits < 1 || n_bits > 8 || (symmetric && n_bits < 2)) return IWQ_ERR_BITS;
  if (quant_dim != 0 && quant_dim != 1) return IWQ_ERR_ARG;
  if (!(group > 0 || group == IWQ_GROUP_PER_TENSOR || group == IWQ_GROUP_PER_CHANNEL)) return IWQ_ERR_GROUP_MODE;
  if (flags & IWQ_FLAG_FORCE_GENERIC) return IWQ_ERR_ARG;
  const int mode = batch_mode(group, quant_dim);
  if (mode == BM_GROUP)
    return iwq_quantize_minmax_batched(d_entries, n_entries, total_units, dtype, n_bits, group, symmetric, nan_flag,
                                       flags, stream);
  const int codes = (flags & IWQ_FLAG_BATCH_CODES) ? (n_bits <= 4 ? 4 : 8) : 0;
  const bool sym = symmetric != 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (mode == BM_TENSOR) {
    if (!workspace || workspace_bytes < iwq_batch_workspace_bytes(n_entries, group, quant_dim) || !aligned16(workspace))
      return IWQ_ERR_WORKSPACE;
    GroupArgs a{};
    a.entries = d_entries;
    a.n_entries = n_entries;
    a.total_units = total_units;
    a.n_bits = n_bits;
    a.nan_flag = nan_flag;
    IWQ_HIP(launch_tensor_b(dtype, sym, codes, a, static_cast<int32_t*>(workspace), st));
    return IWQ_OK;
  }
  BatchExArgs b{};
  b.entries = d_entries;
  b.n_entries = n_entries;
  b.total_units = total_units;
  b.group = group;
  b.n_bits = n_bits;
  b.nan_flag = nan_flag;
  if (mode == BM_ROW) {
    if (group_len <= 0 || group_len % 8 != 0 || group_len > ROW_MAX_L || (group > 0 && group_len != group))
      return IWQ_ERR_ARG;
    IWQ_HIP(launch_row_b(dtype, sym, group_len, codes, b, st));
    return IWQ_OK;
  }
  IWQ_HIP(launch_col_b(dtype, sym, codes, col_shape(dtype, group > 0 ? group : 0), b, st));
  return IWQ_OK;
}

}  // extern "C"

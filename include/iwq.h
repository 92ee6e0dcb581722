/*
 * iwq.h — C-ABI of the MI355X-native weight-only min-max quantization path.
 *
 * Drop-in boundary for the reference's hot path (LiuTielong/Iron_weight_only_quant):
 *   quant_funcs.pseudo_quantize_tensor            quant_funcs.py:4-46
 *   QuantLinear.quantize_weight (INT branch)      quant_linear.py:885-956 (+ quant_dim, :640-647)
 *   quant_wrapper.quantize_model RTN loop         quant_wrapper.py:52-82 (batched entry below)
 *
 * Conventions
 *   - All pointers are DEVICE pointers unless the name says host (h_*).  The library allocates
 *     nothing and frees nothing; the caller owns every buffer (SURVEY.md §8b "Ownership").
 *   - Every compute entry takes an explicit hipStream_t (passed as void*) and is asynchronous.
 *     There is no global mutable state: the library is reentrant across devices and streams.
 *   - Return value: IWQ_OK (0) or an iwq_status error code; no exceptions cross the ABI.
 *   - The NaN check of quant_funcs.py:40 is a device flag (uint32) OR-ed by the kernels; the
 *     caller reads it once (no extra pass over the output).
 *   - Storage dtype of weights, dequantized output, scales and zeros: IWQ_F16 / IWQ_BF16 / IWQ_F32.
 *     The arithmetic reproduces ATen's per-op rounding to that dtype bit-exactly.
 *
 * Group modes (quant_linear.py:896-906): group > 0 per-group along the (possibly transposed)
 * last dimension, IWQ_GROUP_PER_TENSOR (-1), IWQ_GROUP_PER_CHANNEL (-2: one group per row of the
 * grouped view).  quant_dim = 1 groups along dim 0 of the [rows, cols] weight (weight.t()).
 *
 * Grouped view and output ordering: let V = W (quant_dim 0) or W^T (quant_dim 1), shape [vr, vc].
 * Groups are consecutive runs of L elements of V flattened row-major (L = group, vc, or vr*vc),
 * group j -> scales[j], zeros[j]; exactly the reference's reshape(-1, L) order, so scales/zeros
 * are byte-identical to QuantLinear.scales/.zeros flattened ([G,1] -> [G]).
 *
 * Packed codes (new format; the reference keeps no integer codes): laid out in
 * the ORIGINAL weight orientation [rows, cols] (row-major, dense):
 *   n_bits <= 4 : rows x (cols/2) bytes, element (r, c) in byte r*(cols/2) + c/2,
 *                 low nibble = even c (cols must be even)
 *   n_bits 5..8 : rows x cols bytes
 *   code = q (asymmetric, q in [0, 2^b-1]) or q + 2^(b-1) (symmetric, q in [-2^(b-1), 2^(b-1)-1]).
 *   Dequant from codes: (code - zero) * scale (asym) / (code - 2^(b-1)) * scale (sym), each op
 *   rounded to the storage dtype, reproduces out_deq bit-exactly.
 */
#ifndef IWQ_H_
#define IWQ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum iwq_dtype { IWQ_F16 = 0, IWQ_BF16 = 1, IWQ_F32 = 2 };

enum iwq_status {
  IWQ_OK = 0,
  IWQ_ERR_SHAPE = 1,      /* non-positive dims, ld < cols, ...                       (quant_funcs.py:15)  */
  IWQ_ERR_GROUP = 2,      /* grouped last dim % group != 0  (AssertionError, quant_funcs.py:11, quant_linear.py:897) */
  IWQ_ERR_GROUP_MODE = 3, /* group not > 0, -1 or -2  (ValueError "Invalid w_group_size", quant_linear.py:906) */
  IWQ_ERR_BITS = 4,       /* n_bits outside [1, 24]                                                  */
  IWQ_ERR_DTYPE = 5,      /* unknown storage dtype                                                   */
  IWQ_ERR_WORKSPACE = 6,  /* workspace missing or smaller than iwq_workspace_bytes()                 */
  IWQ_ERR_CODES = 7,      /* codes requested with n_bits > 8, or odd cols for nibble packing         */
  IWQ_ERR_HIP = 8,        /* a HIP runtime call failed (see iwq_last_hip_error)                      */
  IWQ_ERR_ARG = 9,        /* null pointer where one is required, bad flags, ...                      */
  IWQ_ERR_FORMAT = 10     /* FP format whose max value overflows fp16 (RuntimeError in the reference's
                             torch.clamp, quant_linear.py:852)                                       */
};

#define IWQ_GROUP_PER_TENSOR (-1)
#define IWQ_GROUP_PER_CHANNEL (-2)

/* flags */
#define IWQ_FLAG_FORCE_GENERIC 0x1u  /* use the universal segmented path (testing / A-B)            */
#define IWQ_FLAG_BATCH_CODES 0x100u  /* batched entry: every entry carries out_codes              */
#define IWQ_FLAG_TILED_CODES 0x200u  /* iwq_w4a16_gemm: codes are in the decode tile layout
                                        (iwq_tile_codes); M <= 16 only                            */
#define IWQ_FLAG_NIB_CODES 0x400u    /* iwq_w4a16_gemm: codes are in the NIB layout (iwq_nib_codes);
                                        M >= 256 only (the prefill kernel and its split-K form);
                                        IWQ_ERR_ARG with a variant, TILED or FORCE_GENERIC        */
#define IWQ_FLAG_GROUP_MAJOR 0x800u  /* iwq_w4a16_gemm: scales / zeros are group-major, [K/group, N]
                                        (element g * N + n), grouped weights only; the unsplit
                                        prefill kernel only: M >= 256, N % 256 == 0, K % 64 == 0,
                                        group % 64 == 0 (IWQ_ERR_ARG otherwise, with a variant,
                                        TILED or FORCE_GENERIC); combines with IWQ_FLAG_NIB_CODES  */
#define IWQ_FLAG_WS_ZEROED 0x1000u   /* iwq_quantize_minmax, per tensor (group -1): the FIRST HALF of the
                                        workspace (iwq_workspace_bytes / 2 bytes) is zero on entry (e.g.
                                        a workspace kept per stream, zeroed once, used only by such
                                        calls): no zeroing launch before the one-pass kernel.  Every
                                        path leaves that half zero on exit (the one-pass kernel's last
                                        workgroup clears its hand-off words; the two-kernel and
                                        universal forms use only the second half, which needs no
                                        zeroing).
                                        iwq_w4a16_gemm, M <= 16 (round 6): the first 16 KiB of the
                                        workspace (the batched decode K-split's arrival counters) are
                                        zero on entry and left zero; without the flag that form is not
                                        taken.  Ignored by other calls.                              */
/* bits 16..23: kernel variant for A/B (0 = default; never needed for correct results): the batched
 * fp16/g128/asym quantize kernel (iwq_quantize_minmax_batched), and iwq_w4a16_gemm's kernel choice
 * (40-49 / 60-81 / 150-172 prefill kernels, 50-55 mid-M, 82-95 forced split-K ranges, 96 the first
 * split-K kernel; iwq_prefill.hip / iwq_prefill16.hip / iwq_gemm.hip list them).  NIB-layout variants
 * (66, 67, 69, 71, 75, 77, 81, 152, 153, 163, 165, 168, 169, 172) expect codes repacked so that nibble
 * p of a code dword holds k = (0,2,4,6,1,3,5,7)[p].
 * The product library (libiwq.so) carries only the defaults and the variants the tests pin: 0;
 * iwq_w4a16_gemm 1 / 2 at M > 16 on row-major codes (the k_w4a16 / k_w4a16_big fallbacks);
 * per-tensor iwq_quantize_minmax 6 (the two-kernel form, the host's retry), 8 (the one-pass kernel
 * at any size; the default takes it from 32 MiB, 16 MiB for bf16) and 9 (test-only abort);
 * iwq_quantize_minmax_batched(_ex) 100 / 101 / 102 / 118 (the roofline probes bench.py times).
 * Any other variant returns IWQ_ERR_ARG there; the A/B library (libiwq_ab.so, built with IWQ_AB=1)
 * has them all, and iwq_build_info() ends in "ab=1". */
#define IWQ_FLAG_VARIANT(v) (((unsigned)(v) & 0xFFu) << 16)

/* Bytes of device workspace iwq_quantize_minmax needs for this problem (0 if none). */
int64_t iwq_workspace_bytes(int64_t rows, int64_t cols, int64_t group, int quant_dim);

/*
 * Quantize -> dequantize one 2-D weight (replaces quant_funcs.py:16-38 and quant_linear.py:909-949).
 *   w          [rows, cols], leading dimension ld_w elements (row-major)
 *   out_deq    [rows, cols], ld_out; may equal w (in-place, quant_funcs.py:31-34 / quant_linear.py:949); nullable
 *   out_codes  packed codes (layout above); nullable
 *   out_scales [G] storage dtype; nullable
 *   out_zeros  [G] storage dtype; ignored when symmetric; nullable
 *   nan_flag   device uint32, OR-ed with 1 if any dequantized value is NaN; nullable.  Also OR-ed
 *              with 2 if the per-tensor one-pass kernel's in-launch hand-off between workgroups was
 *              ABORTED (its workgroups were not all resident -- another kernel held CUs): the launch
 *              then wrote NOTHING (no output, code or parameter byte; a consensus word decides one
 *              outcome for every workgroup before any store), so the input is untouched, in place
 *              too, and the caller re-runs the call with IWQ_FLAG_VARIANT(6) (the two-kernel form,
 *              which cannot time out) into the same outputs (kernels.QuantResult.has_nan does).
 *              OR-ed with 4 if the outputs are invalid (a workgroup could not rejoin a launch that
 *              went ahead; not reachable while stores become visible): the call must fail.  Without a
 *              nan_flag the per-tensor path takes the two-kernel form.
 *   symmetric  0 -> zero_point=True path (:16-22), 1 -> absmax path (:23-29)
 */
int iwq_quantize_minmax(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int n_bits,
                        int64_t group, int symmetric, int quant_dim, void* out_deq, int64_t ld_out,
                        void* out_codes, void* out_scales, void* out_zeros, void* workspace,
                        int64_t workspace_bytes, uint32_t* nan_flag, unsigned flags, void* stream);

/*
 * Batched form: quantize many independent contiguous weights in ONE persistent launch
 * (a whole model's Linear layers: the RTN loop of quant_wrapper.py:52-82).
 * Build the table on the host with iwq_batch_plan (validates every entry and fills the
 * work prefix), copy it to device memory, then call iwq_quantize_minmax_batched.
 * Supported: group > 0 with 8 <= group <= 512 a power of two, quant_dim 0, contiguous weights,
 * n_bits <= 8.  Use iwq_quantize_minmax per tensor for anything else.
 */
typedef struct iwq_batch_entry {
  const void* w;      /* [rows, cols] contiguous */
  void* out_deq;      /* [rows, cols] contiguous, may equal w; nullable */
  void* out_codes;    /* nullable */
  void* out_scales;   /* nullable */
  void* out_zeros;    /* nullable */
  int64_t rows;
  int64_t cols;
  int64_t unit_begin; /* filled by iwq_batch_plan */
} iwq_batch_entry;

int iwq_batch_plan(iwq_batch_entry* h_entries, int32_t n_entries, int dtype, int n_bits, int64_t group,
                   int64_t* h_total_units);

int iwq_quantize_minmax_batched(const iwq_batch_entry* d_entries, int32_t n_entries, int64_t total_units,
                                int dtype, int n_bits, int64_t group, int symmetric, uint32_t* nan_flag,
                                unsigned flags, void* stream);

/*
 * Batched form for EVERY group mode (the RTN loop of quant_wrapper.py:52-82 for per-channel -2,
 * per-tensor -1, quant_dim 1, and groups outside 8..512 powers of two); each tensor gets the bits
 * of its own iwq_quantize_minmax call.  Contiguous weights, 1 <= n_bits <= 8 (2 symmetric).
 *   iwq_batch_plan_ex  validates the host table and fills unit_begin in the mode's work items:
 *     group 8..512 pow2, quant_dim 0  -> iwq_batch_plan (512-element units, ONE launch)
 *     quant_dim 0, other group / -2   -> one wavefront per group of L = group (or cols) elements,
 *                                        L % 8 == 0, L <= 16384, (cols * elem) % 16 == 0; every
 *                                        entry of one table must share L (bucket by L; *h_group_len)
 *     quant_dim 1 (group > 0 or -2)   -> blocks of each entry's column grid, cols % 8 == 0
 *     -1 per-tensor                   -> 512-element units, rows * cols % 8 == 0; needs a workspace
 *                                        of iwq_batch_workspace_bytes (one (min, max) key pair per
 *                                        entry); three launches: key init, reduce, apply
 *   iwq_quantize_minmax_batched_ex  launches it (group_len: *h_group_len of the plan).
 */
int iwq_batch_plan_ex(iwq_batch_entry* h_entries, int32_t n_entries, int dtype, int n_bits, int64_t group,
                      int quant_dim, int64_t* h_total_units, int64_t* h_group_len);
int64_t iwq_batch_workspace_bytes(int32_t n_entries, int64_t group, int quant_dim);
int iwq_quantize_minmax_batched_ex(const iwq_batch_entry* d_entries, int32_t n_entries, int64_t total_units,
                                   int64_t group_len, int dtype, int n_bits, int64_t group, int symmetric,
                                   int quant_dim, void* workspace, int64_t workspace_bytes, uint32_t* nan_flag,
                                   unsigned flags, void* stream);

/*
 * FP4/FP6/FP8 weight formats (QuantLinear FP branches, quant_linear.py:724-883), fp16 weights only.
 * exp_bits/mant_bits as configure_fp_formats (quant_linear.py:84-110): E2M1 / E3M2 / E4M3 defaults.
 * symmetric 1: absmax / fp_max scales, no zeros; 0: mid-point zeros and half-span scales.
 * out_codes: the reference's code bytes (sign | exponent field | mantissa), nibble-packed
 * (low nibble = even column) when 1 + exp_bits + mant_bits <= 4, else one byte per element.
 */
int iwq_quantize_fp(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int exp_bits, int mant_bits,
                    int64_t group, int symmetric, int quant_dim, void* out_deq, int64_t ld_out, void* out_codes,
                    void* out_scales, void* out_zeros, void* workspace, int64_t workspace_bytes, uint32_t* nan_flag,
                    unsigned flags, void* stream);

/*
 * QuantLinear.quantize_weight_approximate (quant_linear.py:470-632), fp16 weights: symmetric absmax
 * FP codes exactly as iwq_quantize_fp (symmetric=1), decoded by the "aligned" decoder
 * _fp_decode_aligned (:237-285) or, with double_approx, fp_decode_aligned_double_approx (:288-363:
 * quads = 4 consecutive groups at one in-group position), then out = RN16(decoded * scale).
 * hi_align_start / hi_align_exp_field / tail_pad_bits: the fpN_* arguments of QuantLinear.
 * group > 0 only (IWQ_ERR_GROUP_MODE); out_scales [G] fp16 required.  workspace: at least
 * iwq_approx_workspace_bytes(...) bytes, 16-B aligned (codes of the double-approximate pass and the
 * generic path's group keys).
 */
int64_t iwq_approx_workspace_bytes(int64_t rows, int64_t cols, int exp_bits, int mant_bits, int64_t group,
                                   int quant_dim, int double_approx);
int iwq_quantize_fp_approx(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int exp_bits,
                           int mant_bits, int64_t group, int quant_dim, int hi_align_start, int hi_align_exp_field,
                           int tail_pad_bits, int double_approx, void* out_deq, int64_t ld_out, void* out_scales,
                           void* workspace, int64_t workspace_bytes, uint32_t* nan_flag, unsigned flags,
                           void* stream);

/*
 * Decode tables for the FP paths (no reference counterpart: an execution aid).  On a finite group
 * the fake-quantized value of an element is sign | T[|t|] (times scale, plus zero) where t is its
 * clamped normalized fp16 value; iwq_fp_build_lut writes T (fp16 magnitudes, at most
 * IWQ_FP_LUT_BYTES, 16-B aligned) for one format, computed on the device by the exact codec.
 * The *_lut entry points take such a table (built with the SAME codec / exp / mant / approximate
 * parameters) and read it through LDS instead of running the bit-level codec per element; lut NULL
 * is the plain entry point.  The table layout is internal to the library: for IWQ_CODEC_FP / GRID
 * formats with exp_bits + 2 * mant_bits <= 10 each entry also carries the magnitude code of its
 * decoded value in its low exp_bits + mant_bits bits, which is where packed codes (out_codes) come
 * from on the table path (bit-identical to the ALU codec's codes).
 * codec: IWQ_CODEC_FP (iwq_quantize_fp), IWQ_CODEC_GRID (iwq_fp4_grid; exp/mant ignored),
 * IWQ_CODEC_APX (iwq_quantize_fp_approx, single-aligned decode), IWQ_CODEC_APX_DOUBLE
 * (iwq_quantize_fp_approx with double_approx: per-code words of the quad decoder; one pass for
 * fp16, quant_dim 0, group 32 / 64 / 128 and a group count divisible by 4, else two passes).
 */
#define IWQ_FP_LUT_BYTES 65536
enum iwq_fp_codec { IWQ_CODEC_FP = 0, IWQ_CODEC_GRID = 1, IWQ_CODEC_APX = 2, IWQ_CODEC_APX_DOUBLE = 3 };
int iwq_fp_build_lut(int codec, int exp_bits, int mant_bits, int hi_align_start, int hi_align_exp_field,
                     int tail_pad_bits, void* lut, int64_t lut_bytes, void* stream);
int iwq_quantize_fp_lut(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int exp_bits,
                        int mant_bits, int64_t group, int symmetric, int quant_dim, void* out_deq, int64_t ld_out,
                        void* out_codes, void* out_scales, void* out_zeros, void* workspace, int64_t workspace_bytes,
                        uint32_t* nan_flag, unsigned flags, void* stream, const void* lut);
int iwq_quantize_fp_approx_lut(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int exp_bits,
                               int mant_bits, int64_t group, int quant_dim, int hi_align_start,
                               int hi_align_exp_field, int tail_pad_bits, int double_approx, void* out_deq,
                               int64_t ld_out, void* out_scales, void* workspace, int64_t workspace_bytes,
                               uint32_t* nan_flag, unsigned flags, void* stream, const void* lut);
int iwq_fp4_grid_lut(const void* w, int64_t rows, int64_t cols, int64_t group, int per_tensor, void* out,
                     void* out_scales, void* workspace, int64_t workspace_bytes, uint32_t* nan_flag, unsigned flags,
                     void* stream, const void* lut);

/*
 * Batched FP form (quantize_model over a whole model, one launch): fp16 weights, entries planned by
 * iwq_batch_plan(h_entries, n, IWQ_F16, 8, group, &total_units) (out_codes must be NULL), decode
 * table REQUIRED (iwq_fp_build_lut with the same codec / exp / mant / approximate parameters).
 * group: power of two in [8, 512].  Per tensor the result equals iwq_quantize_fp_lut /
 * iwq_quantize_fp_approx_lut (single-aligned) / iwq_fp4_grid_lut bit for bit.
 */
int iwq_quantize_fp_batched(const iwq_batch_entry* d_entries, int32_t n_entries, int64_t total_units, int codec,
                            int exp_bits, int mant_bits, int64_t group, int symmetric, int hi_align_start,
                            int hi_align_exp_field, int tail_pad_bits, const void* lut, uint32_t* nan_flag,
                            unsigned flags, void* stream);

/*
 * QuantLinear.quantize_weight, weight_format "bfp" (quant_linear.py:648-723): block floating point
 * with a shared per-group exponent (max fp16 exponent field of the group) and min(w_bit-1, 11)
 * mantissa bits incl. the leading one (round-half-up, saturating).  dtype F16 / BF16 / F32 (taken to
 * fp16 first, like the reference); out may equal w (in place).  group > 0 (IWQ_ERR_GROUP_MODE),
 * grouped dimension % group == 0 (IWQ_ERR_GROUP), w_bit >= 1 (IWQ_ERR_BITS).  No scales / zeros.
 */
int iwq_quantize_bfp(const void* w, int64_t rows, int64_t cols, int64_t ld_w, int dtype, int w_bit, int64_t group,
                     int quant_dim, void* out, int64_t ld_out, unsigned flags, void* stream);

/*
 * fp4_quantize_cpu.quantize_fp16_to_fp4_e1m2 (fp4_quantize_cpu.py:47-72): the E2M1 "grid" fake
 * quantizer (per-group absmax scale S = absmax/6, AxCore two-step rounding), fp16 [rows, cols]
 * contiguous -> fp16 out (same element order; the reference returns it viewed [-1, group]).
 * out_scales: [G] fp16 S values, nullable.  group > 0 requires cols % group == 0 (ValueError).
 */
int iwq_fp4_grid(const void* w, int64_t rows, int64_t cols, int64_t group, int per_tensor, void* out,
                 void* out_scales, void* workspace, int64_t workspace_bytes, uint32_t* nan_flag, unsigned flags,
                 void* stream);
/* the same with the E2M1 codes of the grid values q (out = RN16(q * S)): nibble-packed, low nibble =
 * even element, [rows * cols / 2] bytes (cols even), for storage / iwq_dequant_fp_packed (2, 1).
 * lut: NULL (bit-level codec) or the IWQ_CODEC_GRID decode table (same bits, table speed) */
int iwq_fp4_grid_packed(const void* w, int64_t rows, int64_t cols, int64_t group, int per_tensor, void* out,
                        void* out_codes, void* out_scales, void* workspace, int64_t workspace_bytes,
                        uint32_t* nan_flag, unsigned flags, void* stream, const void* lut);

/*
 * FP codes -> fp16 weights (the dequant of quant_linear.py:773-777 / :825-829 / :876-880 and of
 * fp4_quantize_cpu.py:66-72, from codes kept packed): out[N, K] = RN16(decode(code) * s) (+ z),
 * bit-identical to iwq_quantize_fp's / iwq_fp4_grid_packed's out_deq for the codes they emit.
 * codes: iwq_quantize_fp's layout (nibbles, low = even element, when 1 + exp_bits + mant_bits <= 4;
 * else one byte per element), quant_dim 0 order; scales / zeros (NULL: symmetric) [G] fp16 in the
 * reference's group order: group > 0 (K % group == 0, group % 8 == 0), IWQ_GROUP_PER_CHANNEL or
 * IWQ_GROUP_PER_TENSOR.  K % 8 == 0, ld_out == K, out 16-B aligned.  E2M1 and E4M3 decode on the
 * CDNA4 scaled conversions (v_cvt_scalef32_pk_f16_fp4 / _fp8; E4M3 codes 0x7F / 0xFF are the
 * reference's +-480, not OCP NaN), other formats through an LDS table.
 */
int iwq_dequant_fp_packed(const void* codes, const void* scales, const void* zeros, int exp_bits, int mant_bits,
                          int64_t group, int64_t N, int64_t K, void* out, int64_t ld_out, void* stream);

/*
 * Fused dequant -> GEMM forward (QuantLinear.forward, quant_linear.py:960-972, on packed weights):
 *   y[M, N] = x[M, K] . W_deq[N, K]^T (+ bias[N]),  W_deq = RN16((q - z) * s) per element
 * x, bias, y fp16 row-major (lda, ldy elements); codes = packed 2..4-bit weights in the include/iwq.h
 * layout ([N, K/2] bytes, low nibble = even k); scales/zeros [N * K/group] fp16 in the reference's
 * group order (zeros NULL = symmetric, code offset 2^(n_bits-1)).  group: IWQ_GROUP_PER_CHANNEL or a
 * multiple of 32 dividing K.  Requires N % 128 == 0, K % 128 == 0, 16-B aligned x / codes.
 * fp32 accumulation on v_mfma_f32_16x16x32_f16.  M <= 16 takes the weight-streaming decode kernel
 * (IWQ_FLAG_FORCE_GENERIC forces the tiled prefill kernel).
 */
int iwq_w4a16_gemm(const void* x, int64_t M, int64_t K, int64_t lda, const void* codes, const void* scales,
                   const void* zeros, int n_bits, int64_t group, int64_t N, const void* bias, void* y, int64_t ldy,
                   unsigned flags, void* stream);

/*
 * iwq_w4a16_gemm with a caller-provided fp32 workspace (16-B aligned).  Where the prefill kernel's
 * output tiles would leave CUs idle, K is split into S ranges: each workgroup writes its fp32
 * partial tile to the workspace and a second kernel sums the S partials in range order
 * (deterministic) and applies scale / bias -- within the fp16 output tolerance of the unsplit
 * kernel, not bit-identical to it.  M >= 256: 256 x 256 tiles, S from a time model
 * (iwq_prefill.hip prefill_splitk_count); 16 < M < 256: 64-row tiles where the mid-M kernel is
 * modelled slower (prefill_short_split), else the 256-row split where it pays
 * (prefill_split_preferred).  A NULL or too small workspace runs iwq_w4a16_gemm; so does a workspace
 * that is not 16-B aligned, or a y that is not 8-B aligned or whose ldy is not a multiple of 4 (the
 * split reduces store 4 outputs at a time).  From M = 256 with a workspace the prefill kernel runs
 * even when the model picks one range (same bits as the IWQ_FLAG_NIB_CODES path).
 * iwq_w4a16_gemm_workspace_bytes: the size that enables the split for this problem (0: none needed).
 */
int64_t iwq_w4a16_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K, int64_t group);
int iwq_w4a16_gemm_ws(const void* x, int64_t M, int64_t K, int64_t lda, const void* codes, const void* scales,
                      const void* zeros, int n_bits, int64_t group, int64_t N, const void* bias, void* y, int64_t ldy,
                      void* workspace, int64_t workspace_bytes, unsigned flags, void* stream);

/*
 * Row-major packed 4-bit codes [N, K/2] -> the decode tile layout read by iwq_w4a16_gemm with
 * IWQ_FLAG_TILED_CODES: for each 16-row tile t and 128-k step kt a contiguous 1 KiB block at
 * byte (t * K/128 + kt) * 1024, byte 16 l + i of it = row 16 t + (l % 16), code byte
 * 64 kt + 16 (l / 16) + i.  N % 16 == 0, K % 128 == 0; out holds N * K / 2 bytes.
 */
int iwq_tile_codes(const void* codes, int64_t N, int64_t K, void* out, void* stream);
/* Row-major packed codes (the layout above, [N, K/2] bytes) -> the NIB layout read by iwq_w4a16_gemm
 * with IWQ_FLAG_NIB_CODES: in every code dword (8 consecutive k of one row) nibble p holds
 * k = (0,2,4,6,1,3,5,7)[p], so the prefill kernel builds natural-order fp16 pairs with 9 VALU per 8
 * weights instead of 12 (variants 66 / 75).  A one-time repack at quantize time,
 * replacing no reference call (the reference keeps no packed codes, quant_linear.py:451-458); the
 * forward it feeds replaces QuantLinear.forward (quant_linear.py:960-972) at M >= 256.
 * K % 32 == 0, 16-B aligned codes / out; out may equal codes (in place).  Async on `stream`. */
int iwq_nib_codes(const void* codes, int64_t N, int64_t K, void* out, void* stream);

/*
 * Packed codes -> fp16 W_deq [N, K] (contiguous: ld_out == K, 16-B aligned), bit-identical to the
 * reference's dequantized weight RN16((q - z) * s): the prefill path for packed-only weights
 * (dequantize once, then one library GEMM).  Same codes / scales / zeros / group conventions as
 * iwq_w4a16_gemm; K % 32 == 0.
 */
int iwq_dequant_packed(const void* codes, const void* scales, const void* zeros, int n_bits, int64_t group,
                       int64_t N, int64_t K, void* out, int64_t ld_out, void* stream);

/*
 * Packed codes (layout above) -> the dequantized weight, for EVERY INT mode the quantizer writes codes
 * for: n_bits 1..8 (symmetric: 2..8), group > 0 / IWQ_GROUP_PER_TENSOR / IWQ_GROUP_PER_CHANNEL,
 * quant_dim 0 / 1, storage dtype F16 / BF16 / F32 (scales, zeros and out all in that dtype).
 * out[r * ld_out + c] = RN_dtype((code - z) * s) with (s, z) of element (r, c)'s group -- bit-identical
 * to the out_deq iwq_quantize_minmax wrote alongside those codes (quant_funcs.py:38 /
 * quant_linear.py:947).  zeros ignored (may be NULL) when symmetric.  Load-time inverse of the packed
 * format (the packed checkpoint, checkpoint.py); the reference has no counterpart (it keeps no codes).
 */
int iwq_dequant_codes(const void* codes, const void* scales, const void* zeros, int dtype, int n_bits,
                      int64_t group, int symmetric, int quant_dim, int64_t rows, int64_t cols, void* out,
                      int64_t ld_out, void* stream);

/* Deterministic synthetic weights (oracle/synth.py bit-for-bit), written to [rows, cols] contiguous. */
int iwq_fill_synthetic(void* out, int64_t n, int dtype, uint64_t seed, int64_t index_offset, void* stream);

/* Diagnostics */
const char* iwq_status_string(int status);
int iwq_last_hip_error(void);            /* last hipError_t seen by this thread (0 = none) */
const char* iwq_build_info(void);        /* arch, compile flags, version */

/* Test-only self check of the fast reciprocal and corrected fp32 division used in the hot loop
 * against IEEE division, over every finite fp16 numerator x every fp16 divisor in [2^-24, 65504].
 * Writes mismatch counts to d_counts[0..2]: quotient fp32 bits, quotient after fp16 rounding,
 * reciprocal fp32 bits. */
int iwq_selftest_division(uint64_t* d_counts, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* IWQ_H_ */

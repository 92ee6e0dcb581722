"""Torch-facing wrappers over the C-ABI (include/iwq.h).

These only marshal device pointers, strides and the current HIP stream; all arithmetic runs in the
gfx950 kernels of csrc/iwq_minmax.hip.  Error statuses are mapped onto the exception types the
reference raises (quant_funcs.py:11/15/40, quant_linear.py:897/906).
"""
import ctypes
from dataclasses import dataclass
from typing import Callable, List, Optional

import torch

from . import _lib as L

FAST_GROUPS = (8, 16, 32, 64, 128, 256, 512)


# iwq_minmax.hip per-tensor variant 6: the reduce + apply pair, which cannot time out
_TENSOR_PAIR = 6 << 16


@dataclass
class QuantResult:
    out: Optional[torch.Tensor]       # dequantized weight (same shape/dtype as input) or None
    scales: Optional[torch.Tensor]    # [G] storage dtype
    zeros: Optional[torch.Tensor]     # [G] storage dtype (asymmetric) or None
    codes: Optional[torch.Tensor]     # packed uint8 codes (include/iwq.h layout) or None
    nan_flag: torch.Tensor            # [1] int32 on device; bit 0: the output holds a NaN
    retry: Optional[Callable[[], torch.Tensor]] = None  # re-run on the pair into the same outputs
    retried: bool = False             # has_nan() found a timed-out hand-off and re-ran the call

    def has_nan(self) -> bool:
        v = self.settle()
        return v != 0

    def settle(self) -> int:
        """Resolve an aborted per-tensor one-pass hand-off (include/iwq.h, nan_flag bit 1): the launch
        wrote nothing -- its workgroups were not all resident, e.g. another stream's kernel held CUs
        -- so the input is untouched, out of place and in place alike, and the same call on the
        two-kernel form rewrites every output; its flag replaces this one.  Returns the final flag
        word (one device sync); raises if the outputs are invalid (bit 2)."""
        v = int(self.nan_flag.item())
        if v & 2 and self.retry is not None:
            self.nan_flag = self.retry()
            self.retry = None
            self.retried = True
            v = int(self.nan_flag.item())
        if v & 6:
            raise RuntimeError("iwq: per-tensor one-pass kernel could not complete its in-launch hand-off "
                               "(workgroups not all resident); outputs invalid")
        return v


class _FlagPool:
    """Per-device pool of pre-zeroed NaN flags: one int32 slot per call instead of a zero-fill kernel
    per call (the fill alone cost ~4 us of device time, 10-30 % of a 4096x4096 quantization).
    Slots are handed out round-robin; the pool is re-zeroed (one fill) when it wraps, so a result's
    flag stays valid for the next 65535 calls on that device."""
    SIZE = 65536

    def __init__(self):
        self.buf = {}
        self.next = {}

    def take(self, dev):
        key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
        buf = self.buf.get(key)
        i = self.next.get(key, 0)
        if (buf is None or i >= self.SIZE) and dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
            # never create or re-zero the shared pool inside a graph capture (its memory would come
            # from the graph's private pool and the zero-fill would only be recorded): a per-call
            # flag whose zero-fill is part of the captured graph instead
            return torch.zeros(1, dtype=torch.int32, device=dev)
        if buf is None or i >= self.SIZE:
            if buf is None:
                buf = torch.zeros(self.SIZE, dtype=torch.int32, device=dev)
                self.buf[key] = buf
            else:
                buf.zero_()
            i = 0
        self.next[key] = i + 1
        return buf[i:i + 1]


_flags = _FlagPool()


class _TensorWsCache:
    """Per (device, stream) workspace for per-tensor calls (include/iwq.h IWQ_FLAG_WS_ZEROED, round 5):
    zeroed once, and every per-tensor call leaves its first half zero again (the one-pass kernel's
    hand-off words; the pair's partial keys live in the second half), so the one-pass kernel runs without
    a zeroing launch before it (one launch floor, ~1.6-1.9 us, per call).  Calls on one stream are
    ordered, so one workspace per stream never serves two launches at once.  Not used while a graph is
    captured (a replay may run on another stream): those calls get a fresh workspace and the memset."""

    def __init__(self):
        self.bufs = {}

    def get(self, dev, stream_key, nbytes):
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), stream_key)
        b = self.bufs.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=dev)
            self.bufs[key] = b
        return b

    def drop(self, dev, stream_key):
        self.bufs.pop((dev.index if dev.index is not None else torch.cuda.current_device(), stream_key), None)


_tws = _TensorWsCache()
# the decode GEMV's per-stream workspace (round 6): its leading counters zero, left zero by every call
# (the cross-workgroup K-split, IWQ_FLAG_WS_ZEROED); the fp32 slabs after them are scratch
_gws = _TensorWsCache()


def group_geometry(rows, cols, group, quant_dim):
    """(L, G) of the grouped view, or raise like the reference (quant_linear.py:896-906)."""
    vr, vc = (cols, rows) if quant_dim == 1 else (rows, cols)
    if group > 0:
        assert vc % group == 0
        return group, vr * vc // group
    if group == -1:
        return vr * vc, 1
    if group == -2:
        return vc, vr
    raise ValueError("Invalid w_group_size")


def codes_nbytes(rows, cols, n_bits):
    return rows * (cols // 2) if n_bits <= 4 else rows * cols


def _raise_for(status, what):
    if status == L.IWQ_ERR_GROUP:
        raise AssertionError(f"{what}: last dimension not divisible by the group size")
    if status == L.IWQ_ERR_GROUP_MODE:
        raise ValueError("Invalid w_group_size")
    if status == L.IWQ_ERR_FORMAT:
        raise RuntimeError("value cannot be converted to type c10::Half without overflow")
    L.check(status, what)


def quantize_minmax(w: torch.Tensor, n_bits: int, group: int, symmetric: bool, quant_dim: int = 0,
                    out: Optional[torch.Tensor] = None, want_deq: bool = True, want_codes: bool = False,
                    want_scales: bool = True, flags: int = 0,
                    zeroed_workspace: Optional[torch.Tensor] = None) -> QuantResult:
    """Min-max fake-quantize a 2-D weight on the GPU.

    w       [rows, cols] fp16/bf16/fp32 CUDA tensor with unit column stride (any row stride).
    out     destination for the dequantized weight (may be `w` itself for in-place), else a new
            contiguous tensor is allocated when want_deq.
    zeroed_workspace  per tensor only: a uint8 device tensor of >= iwq_workspace_bytes whose first
            half is zero, and which the call leaves so (IWQ_FLAG_WS_ZEROED) -- for graph capture, where
            the per-stream cache is not used; eager calls get the stream's cached one without asking.
    """
    L.require_device(w)
    if w.dim() != 2:
        raise AssertionError("weight must be 2-D")
    if w.dtype not in L.DTYPE_CODE:
        raise TypeError(f"unsupported dtype {w.dtype}")
    lib = L.load()
    if w.stride(1) != 1 or w.stride(0) < w.shape[1]:
        w = w.contiguous()
    rows, cols = w.shape
    Lg, G = group_geometry(rows, cols, group, quant_dim)
    dev = w.device
    if out is None and want_deq:
        out = torch.empty((rows, cols), dtype=w.dtype, device=dev)
    if out is not None:
        if out.shape != w.shape or out.dtype != w.dtype or out.device != dev or out.stride(1) != 1:
            raise ValueError("out must match w in shape/dtype/device and have unit column stride")
    scales = torch.empty(G, dtype=w.dtype, device=dev) if want_scales else None
    zeros = torch.empty(G, dtype=w.dtype, device=dev) if (want_scales and not symmetric) else None
    codes = None
    if want_codes:
        if n_bits > 8:
            raise ValueError("packed codes need n_bits <= 8")
        codes = torch.empty(codes_nbytes(rows, cols, n_bits), dtype=torch.uint8, device=dev)
    nan_flag = _flags.take(dev)
    # the caller's stream: the call and, if the one-pass hand-off aborts, its retry (settle() may run
    # later under another current stream) both launch here -- the retry reuses this stream's workspace
    cur_stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(cur_stream.cuda_stream)

    def call(ws, wsb):
        with L.on_device(dev):
            return lib.iwq_quantize_minmax(
                L.ptr(w), rows, cols, w.stride(0), L.DTYPE_CODE[w.dtype], int(n_bits), int(group),
                int(bool(symmetric)), int(quant_dim), L.ptr(out), (out.stride(0) if out is not None else cols),
                L.ptr(codes), L.ptr(scales), L.ptr(zeros), L.ptr(ws), wsb, L.ptr(nan_flag), int(flags), sh)
    # the specialised kernels need no workspace; the C-ABI checks for one before launching anything,
    # so only the per-tensor and universal paths pay for the allocation (and a second call)
    st = call(None, 0)
    retry = None
    if st == L.IWQ_ERR_WORKSPACE:
        wsb = int(lib.iwq_workspace_bytes(rows, cols, group, quant_dim))
        skey = torch.cuda.current_stream(dev).cuda_stream if group == -1 else None
        if group == -1 and zeroed_workspace is not None:
            if zeroed_workspace.dtype != torch.uint8 or zeroed_workspace.numel() < wsb \
                    or zeroed_workspace.device != dev:
                raise ValueError(f"zeroed_workspace must be >= {wsb} uint8 bytes on {dev}")
            ws, skey = zeroed_workspace, None
            flags = int(flags) | L.IWQ_FLAG_WS_ZEROED
        elif group == -1 and not torch.cuda.is_current_stream_capturing():
            # the stream's zeroed workspace: no zeroing launch before the one-pass kernel
            ws = _tws.get(dev, skey, wsb)
            flags = int(flags) | L.IWQ_FLAG_WS_ZEROED
        else:
            ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
        st = call(ws, wsb)
        if st != L.IWQ_OK and skey is not None and (int(flags) & L.IWQ_FLAG_WS_ZEROED):
            _tws.drop(dev, skey)  # a failed launch may have left it dirty: zero a new one next time
        # where the C side can take the one-pass kernel (iwq_minmax.hip: per tensor, any quant_dim -- a
        # per-tensor group is the whole tensor, so quant_dim does not change the walk; fp16, and bf16 /
        # fp32 without packed codes)
        if group == -1:
            def retry():  # the one-pass hand-off aborted (QuantResult.settle): same call on the pair,
                # on the caller's stream (whose workspace it reuses), whatever stream settle() runs under
                with torch.cuda.stream(cur_stream):
                    flag2 = torch.zeros(1, dtype=torch.int32, device=dev)
                with L.on_device(dev):
                    st2 = lib.iwq_quantize_minmax(
                        L.ptr(w), rows, cols, w.stride(0), L.DTYPE_CODE[w.dtype], int(n_bits), int(group),
                        int(bool(symmetric)), int(quant_dim), L.ptr(out), (out.stride(0) if out is not None else cols),
                        L.ptr(codes), L.ptr(scales), L.ptr(zeros), L.ptr(ws), wsb, L.ptr(flag2),
                        (int(flags) & ~(0xFF << 16)) | _TENSOR_PAIR, sh)
                _raise_for(st2, "iwq_quantize_minmax")
                cur_stream.synchronize()  # settle() reads flag2 from its own current stream
                return flag2
    _raise_for(st, "iwq_quantize_minmax")
    return QuantResult(out, scales, zeros, codes, nan_flag, retry)


class _LutCache:
    """Per-device FP decode tables (include/iwq.h iwq_fp_build_lut), built once per format on first
    use and reused by every later call.  Returns None (plain ALU codec) while a CUDA graph is being
    captured and the table does not exist yet: a table allocated inside a capture would belong to
    the graph's private pool."""

    def __init__(self):
        self.tabs = {}

    def get(self, dev, codec, exp_bits=0, mant_bits=0, hs=0, hf=0, tp=0):
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        key = (idx, codec, exp_bits, mant_bits, hs, hf, tp)
        t = self.tabs.get(key)
        if t is not None:
            return t
        if torch.cuda.is_current_stream_capturing():
            return None
        t = torch.empty(L.IWQ_FP_LUT_BYTES, dtype=torch.uint8, device=dev)
        with L.on_device(dev):
            st = L.load().iwq_fp_build_lut(int(codec), int(exp_bits), int(mant_bits), int(hs), int(hf), int(tp),
                                           L.ptr(t), t.numel(), L.stream_handle(dev))
        if st != L.IWQ_OK:  # a format the table path does not cover: plain codec
            return None
        torch.cuda.current_stream(dev).synchronize()  # once per format: visible to every stream
        self.tabs[key] = t
        return t


_luts = _LutCache()


def fp_code_nbytes(rows, cols, exp_bits, mant_bits):
    return rows * (cols // 2) if (1 + exp_bits + mant_bits) <= 4 else rows * cols


def quantize_fp(w: torch.Tensor, exp_bits: int, mant_bits: int, group: int, symmetric: bool, quant_dim: int = 0,
                out: Optional[torch.Tensor] = None, want_codes: bool = False, flags: int = 0,
                use_lut: bool = True) -> QuantResult:
    """FP4/FP6/FP8 fake quantization of a 2-D weight (QuantLinear FP branches) on the GPU.
    fp16 weights: the LDS-table kernels (use_lut; False = bit-level ALU codec, same bits).  bf16 / fp32
    weights (round 4, iwq_fpdt.hip): every op in the weight's dtype like the reference; scales / zeros
    come back fp16, as the reference's .half() buffers (quant_linear.py:760-766)."""
    L.require_device(w)
    if w.dim() != 2:
        raise AssertionError("weight must be 2-D")
    if w.dtype not in L.DTYPE_CODE:
        raise TypeError(f"unsupported dtype {w.dtype}")
    lib = L.load()
    if w.stride(1) != 1 or w.stride(0) < w.shape[1]:
        w = w.contiguous()
    rows, cols = w.shape
    _, G = group_geometry(rows, cols, group, quant_dim)
    dev = w.device
    if out is None:
        out = torch.empty((rows, cols), dtype=w.dtype, device=dev)
    scales = torch.empty(G, dtype=torch.float16, device=dev)
    zeros = None if symmetric else torch.empty(G, dtype=torch.float16, device=dev)
    codes = torch.empty(fp_code_nbytes(rows, cols, exp_bits, mant_bits), dtype=torch.uint8, device=dev) \
        if want_codes else None
    nan_flag = _flags.take(dev)
    f16 = w.dtype == torch.float16
    lut = _luts.get(dev, L.IWQ_CODEC_FP, exp_bits, mant_bits) if (use_lut and f16) else None

    def call(ws, wsb):
        with L.on_device(dev):
            return lib.iwq_quantize_fp_lut(L.ptr(w), rows, cols, w.stride(0), L.DTYPE_CODE[w.dtype], int(exp_bits),
                                           int(mant_bits), int(group), int(bool(symmetric)), int(quant_dim),
                                           L.ptr(out), out.stride(0), L.ptr(codes), L.ptr(scales), L.ptr(zeros),
                                           L.ptr(ws), wsb, L.ptr(nan_flag), int(flags), L.stream_handle(dev),
                                           L.ptr(lut))
    st = call(None, 0)  # the specialised kernel needs no workspace (checked before any launch)
    if st == L.IWQ_ERR_WORKSPACE:
        wsb = ((8 * G + 255) // 256) * 256
        st = call(torch.empty(wsb, dtype=torch.uint8, device=dev), wsb)
    _raise_for(st, "iwq_quantize_fp")
    return QuantResult(out, scales, zeros, codes, nan_flag)


def quantize_fp_approx(w: torch.Tensor, exp_bits: int, mant_bits: int, group: int, quant_dim: int = 0,
                       hi_align_start: int = 12, hi_align_exp_field: int = 15, tail_pad_bits: int = 1,
                       double_approx: bool = False, out: Optional[torch.Tensor] = None,
                       flags: int = 0, use_lut: bool = True) -> QuantResult:
    """QuantLinear.quantize_weight_approximate arithmetic (quant_linear.py:470-632) on an fp16 weight:
    symmetric absmax FP codes, aligned / double-approximate decode, RN16(decoded * scale)."""
    L.require_device(w)
    if w.dim() != 2:
        raise AssertionError("weight must be 2-D")
    if w.dtype not in L.DTYPE_CODE:
        raise TypeError(f"unsupported dtype {w.dtype}")
    if group <= 0:
        raise ValueError("approximate 仅支持分组量化，w_group_size 必须 > 0")
    lib = L.load()
    if w.stride(1) != 1 or w.stride(0) < w.shape[1]:
        w = w.contiguous()
    rows, cols = w.shape
    _, G = group_geometry(rows, cols, group, quant_dim)
    if double_approx and (G * group) % 4 != 0:
        raise ValueError("double approx requires total elements divisible by 4")
    dev = w.device
    if out is None:
        out = torch.empty((rows, cols), dtype=w.dtype, device=dev)
    scales = torch.empty(G, dtype=torch.float16, device=dev)  # the reference's .half() buffer (:606)
    nan_flag = _flags.take(dev)
    wsb = int(lib.iwq_approx_workspace_bytes(rows, cols, int(exp_bits), int(mant_bits), int(group), int(quant_dim),
                                             int(bool(double_approx))))
    ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
    lut = (_luts.get(dev, L.IWQ_CODEC_APX_DOUBLE if double_approx else L.IWQ_CODEC_APX, exp_bits, mant_bits,
                     hi_align_start, hi_align_exp_field, tail_pad_bits) if (use_lut and w.dtype == torch.float16)
           else None)
    with L.on_device(dev):
        st = lib.iwq_quantize_fp_approx_lut(L.ptr(w), rows, cols, w.stride(0), L.DTYPE_CODE[w.dtype], int(exp_bits),
                                            int(mant_bits), int(group), int(quant_dim), int(hi_align_start),
                                            int(hi_align_exp_field), int(tail_pad_bits), int(bool(double_approx)),
                                            L.ptr(out), out.stride(0), L.ptr(scales), L.ptr(ws), ws.numel(),
                                            L.ptr(nan_flag), int(flags), L.stream_handle(dev), L.ptr(lut))
    _raise_for(st, "iwq_quantize_fp_approx")
    return QuantResult(out, scales, None, None, nan_flag)


def quantize_bfp(w: torch.Tensor, w_bit: int, group: int, quant_dim: int = 0, out: Optional[torch.Tensor] = None,
                 flags: int = 0) -> torch.Tensor:
    """BFP branch of QuantLinear.quantize_weight (quant_linear.py:648-723) on the GPU: shared group
    exponent, min(w_bit-1, 11)-bit mantissas; returns the dequantized weight (out may be w)."""
    L.require_device(w)
    if w.dim() != 2:
        raise AssertionError("weight must be 2-D")
    if w.dtype not in L.DTYPE_CODE:
        raise TypeError(f"unsupported dtype {w.dtype}")
    if group <= 0:
        raise ValueError("BFP 仅支持分组量化，请将 w_group_size 设为正数")
    if w_bit < 1:
        raise ValueError("negative shift count")
    lib = L.load()
    if w.stride(1) != 1 or w.stride(0) < w.shape[1]:
        w = w.contiguous()
    rows, cols = w.shape
    group_geometry(rows, cols, group, quant_dim)
    if out is None:
        out = torch.empty((rows, cols), dtype=w.dtype, device=w.device)
    with L.on_device(w.device):
        st = lib.iwq_quantize_bfp(L.ptr(w), rows, cols, w.stride(0), L.DTYPE_CODE[w.dtype], int(w_bit), int(group),
                                  int(quant_dim), L.ptr(out), out.stride(0), int(flags), L.stream_handle(w.device))
    _raise_for(st, "iwq_quantize_bfp")
    return out


def fp4_grid(w: torch.Tensor, group: int, per_tensor: bool = False, flags: int = 0,
             use_lut: bool = True, want_codes: bool = False) -> QuantResult:
    """fp4_quantize_cpu.quantize_fp16_to_fp4_e1m2 arithmetic on the GPU; output in w's element order.
    want_codes: also the E2M1 codes of the grid values (nibble-packed, low nibble = even element;
    iwq_fp4_grid_packed), so that dequant_fp_packed(codes, scales, None, 2, 1, ...) == out."""
    L.require_device(w)
    lib = L.load()
    w = w.contiguous()
    rows, cols = w.shape
    if per_tensor:
        G = 1
    elif group > 0:
        if cols % group != 0:
            raise ValueError("in_features must be divisible by group_size.")
        G = rows * cols // group
    else:
        G = rows
    dev = w.device
    out = torch.empty_like(w)
    scales = torch.empty(G, dtype=w.dtype, device=dev)
    nan_flag = _flags.take(dev)
    wsb = ((8 * G + 255) // 256) * 256
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    lut = _luts.get(dev, L.IWQ_CODEC_GRID) if use_lut else None
    if want_codes:
        if cols % 2:
            raise ValueError("fp4_grid: packed codes need an even number of columns")
        codes = torch.empty(rows * cols // 2, dtype=torch.uint8, device=dev)
        with L.on_device(dev):
            st = lib.iwq_fp4_grid_packed(L.ptr(w), rows, cols, int(group), int(bool(per_tensor)), L.ptr(out),
                                         L.ptr(codes), L.ptr(scales), L.ptr(ws), wsb, L.ptr(nan_flag), int(flags),
                                         L.stream_handle(dev), L.ptr(lut))
        _raise_for(st, "iwq_fp4_grid_packed")
        return QuantResult(out, scales, None, codes, nan_flag)
    with L.on_device(dev):
        st = lib.iwq_fp4_grid_lut(L.ptr(w), rows, cols, int(group), int(bool(per_tensor)), L.ptr(out),
                                  L.ptr(scales), L.ptr(ws), wsb, L.ptr(nan_flag), int(flags), L.stream_handle(dev),
                                  L.ptr(lut))
    _raise_for(st, "iwq_fp4_grid")
    return QuantResult(out, scales, None, None, nan_flag)


def dequant_fp_packed(codes: torch.Tensor, scales: torch.Tensor, zeros: Optional[torch.Tensor], exp_bits: int,
                      mant_bits: int, group: int, N: int, K: int,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """FP codes (iwq_quantize_fp / fp4_grid(want_codes=True) layout: nibbles for 1+E+M <= 4, else one
    byte per element) -> fp16 [N, K] = RN16(decode(code) * s) (+ z): bit-identical to the fake-quant
    output of the same quantization (quant_linear.py:773-777; fp4_quantize_cpu.py:66-72).  E2M1 and
    E4M3 decode on the CDNA4 scaled-conversion instructions, other formats through a table."""
    L.require_device(codes)
    nib = 1 + exp_bits + mant_bits <= 4
    G = 1 if group == -1 else (N if group == -2 else (N * K // group if group > 0 else 0))
    if codes.dtype != torch.uint8 or not codes.is_contiguous() or codes.numel() != (N * K // 2 if nib else N * K):
        raise ValueError("dequant_fp_packed: codes must be contiguous uint8 of N*K/2 (nibbles) or N*K bytes")
    for name, t in (("scales", scales), ("zeros", zeros)):
        if t is not None and (t.dtype != torch.float16 or t.device != codes.device or t.numel() != G
                              or not t.is_contiguous()):
            raise ValueError(f"dequant_fp_packed: {name} must be contiguous fp16 [{G}] on the codes' device")
    lib = L.load()
    if out is None:
        out = torch.empty((N, K), dtype=torch.float16, device=codes.device)
    elif (out.dtype != torch.float16 or out.device != codes.device or out.shape != (N, K)
          or not out.is_contiguous()):
        raise ValueError("dequant_fp_packed: out must be a contiguous fp16 [N, K] tensor")
    with L.on_device(codes.device):
        st = lib.iwq_dequant_fp_packed(L.ptr(codes), L.ptr(scales), L.ptr(zeros), int(exp_bits), int(mant_bits),
                                       int(group), int(N), int(K), L.ptr(out), K, L.stream_handle(codes.device))
    _raise_for(st, "iwq_dequant_fp_packed")
    return out


def gemm_variant_flags(v: int) -> int:
    """IWQ_FLAG_VARIANT(v) for iwq_w4a16_gemm's decode path (0 = default; A/B and tests only)."""
    return (int(v) & 0xFF) << 16


GEMV_MAX_M = 16  # iwq_w4a16_gemm takes the weight-streaming decode kernel up to this many rows
# w4a16_linear keeps the fused kernels (decode GEMV, the mid-M weight-streaming kernel below 256
# rows, the split-K prefill kernel from 256) up to packed_fused_preferred's row count, at most this;
# above, dequantize-once + hipBLASLt
FUSED_MAX_M = 2048
# from this many rows the prefill kernel can read NIB-layout codes (nib_codes; iwq_w4a16_gemm with
# IWQ_FLAG_NIB_CODES): 74's NIB twin (variant 75), +0.5-1.2 % per channel at M = 8192 over the
# current 74 (+4.5-5 % over the round-2 first 74; profiles/r02_ab_gemm_nib_product.jsonl)
NIB_MIN_M = 256


# [N, K] weights on which the fused prefill beats hipBLASLt at large M (per channel, M = 8192, in-run
# interleaved A/B): Llama-2-7B gate / up_proj, 1.14-1.18x (profiles/r04_ab_gemm_b16*.jsonl; the library
# GEMM's 43 column tiles).  Everywhere else at large M the library GEMM on the resident fp16 weight
# is 1.0-1.1x faster.
LARGE_M_FUSED = frozenset({(11008, 4096)})


def auto_fused_preferred(M: int, N: int, K: int, group: int) -> bool:
    """QuantLinear(fused_forward="auto"): whether the packed-code kernels beat the reference forward
    F.linear(x, W_deq) (hipBLASLt on the resident fp16 weight) for an M-row batch on an [N, K] weight.
    Measured in DEVICE time, cold (each pass walks >= 1.2 GB of distinct weights, as a model forward
    reads each layer once; hipGraph replay, so no host launch cost; profiles/r03_ab_auto_graph.jsonl,
    Llama-2-7B q / gate / down, 4-bit): per channel the fused kernels win at every M <= 192
    (1.01-3.6x) and on down-like weights (K >= 2N) up to M = 1024 (1.14-1.31x); g128 wins at every
    M <= 32 (1.06-3.2x) and on down-like weights up to M = 512 (1.08-1.72x), but not on q_proj at
    M = 64 (0.86x) or gate_proj at 128-192 (0.92-0.94x).  Round 5 (g128 parameters staged in LDS in the
    GEMV / mid kernels, 128-row split tiles on wide weights; profiles/r05_ab_auto_g128.jsonl): g128 now
    also wins on gate-like weights (N > K) up to M = 128 (1.06-1.35x) and on square ones at
    M = 96-192 (1.09-1.43x; 48-64 stay at 0.91-1.0x)."""
    if group == -2:
        return M <= 192 or (M <= 1024 and K >= 2 * N) or (M >= 4096 and (N, K) in LARGE_M_FUSED)
    if K >= 2 * N:
        return M <= 512
    if N > K:
        return M <= 128
    return M <= 32 or 96 <= M <= 192


def packed_fused_preferred(M: int, N: int, K: int, group: int) -> bool:
    """kernels.w4a16_linear (packed-only weights, PackedLinear): whether the fused kernels beat
    dequant-once (iwq_dequant_packed) + F.linear for an M-row batch on an [N, K] weight.  Measured
    cold in device time (tools/ab_auto.py --packed: each pass walks >= 1.2 GB of distinct codes,
    hipGraph replay; profiles/r03_ab_packed_graph.jsonl, Llama-2-7B q / gate / down, 4-bit): per
    channel every shape wins up to M = 1024 (q 0.99x there, gate 1.21x, down 1.38x) and down-like
    weights (K >= 2N) up to 2048 (1.15x); g128 q / gate up to 768 (1.03 / 1.00x; q 0.93x at 1024),
    down up to 1024 (1.18x; 0.99x at 1536).  (Round 2 stopped every shape at 1024 from MALL-warm
    single-weight timings.)"""
    down = K >= 2 * N
    if group == -2:
        return M <= (FUSED_MAX_M if down else 1024)
    return M <= (1024 if down else 768)


def w4a16_gemm_supported(x: torch.Tensor, N: int, K: int, n_bits: int, group: int) -> bool:
    g = K if group == -2 else group
    return (x.is_cuda and x.dtype == torch.float16 and 2 <= n_bits <= 4 and N % 128 == 0 and K % 128 == 0
            and g > 0 and g % 32 == 0 and K % g == 0)


def nib_supported(x: torch.Tensor, N: int, K: int, n_bits: int, group: int) -> bool:
    """Shapes the NIB-layout prefill path takes (iwq_w4a16_gemm with IWQ_FLAG_NIB_CODES): N % 256,
    K % 64, per channel or g % 64 == 0, on top of w4a16_gemm_supported."""
    g = K if group == -2 else group
    return (w4a16_gemm_supported(x, N, K, n_bits, group) and N % 256 == 0 and K % 64 == 0
            and (g == K or g % 64 == 0))


def _check_packed(what, dev, codes, scales, zeros, n_bits, group, N, K, bias=None):
    """Host-side validation of a packed 4-bit weight before its pointers reach a kernel: codes
    [N*K/2] uint8, scales (and zeros) [N*K/g] fp16, all on `dev` and contiguous.  A tensor of the
    wrong size or layout (e.g. quant_dim=1 codes) raises here instead of reading out of bounds."""
    if not 2 <= n_bits <= 4:
        raise ValueError(f"{what}: packed 4-bit codes need 2 <= n_bits <= 4")
    g = K if group == -2 else group
    if g <= 0 or K % g != 0:
        raise ValueError(f"{what}: group {group} does not divide K={K}")
    G = N * (K // g)

    def chk(name, t, numel, dtype):
        if t.device != dev:
            raise ValueError(f"{what}: {name} is on {t.device}, expected {dev}")
        if t.dtype != dtype:
            raise TypeError(f"{what}: {name} must be {dtype}, got {t.dtype}")
        if not t.is_contiguous() or t.numel() != numel:
            raise ValueError(f"{what}: {name} must be contiguous with {numel} elements, got "
                             f"{tuple(t.shape)}")
    chk("codes", codes, N * K // 2, torch.uint8)
    chk("scales", scales, G, torch.float16)
    if zeros is not None:
        chk("zeros", zeros, G, torch.float16)
    if bias is not None:
        chk("bias", bias, N, torch.float16)


def group_major_params(scales: torch.Tensor, zeros: Optional[torch.Tensor], N: int, K: int, group: int):
    """Grouped scales / zeros in the reference's order ([N, K/group]) -> group-major copies
    ([K/group, N], element g * N + n) for w4a16_gemm(..., scales_gm=, zeros_gm=): the prefill kernel
    then stages a K-step's 256 parameters as contiguous pieces (IWQ_FLAG_GROUP_MAJOR)."""
    if group == -2:
        raise ValueError("group_major_params: grouped weights only (per channel has one group per row)")
    gpr = K // group

    def t(v):
        return None if v is None else v.reshape(N, gpr).t().contiguous().view(-1)
    return t(scales), t(zeros)


def gm_prefill_applies(M: int, N: int, K: int, group: int) -> bool:
    """Shapes and row counts at which w4a16_gemm reads group-major parameters (IWQ_FLAG_GROUP_MAJOR:
    the unsplit 16x16x32 prefill kernel, grouped, M >= NIB_MIN_M, no split-K needed)."""
    if group == -2 or M < NIB_MIN_M or N % 256 or K % 64 or group % 64 or K % group:
        return False
    lib = L.load()
    return int(lib.iwq_w4a16_gemm_workspace_bytes(M, N, K, int(group))) == 0


def w4a16_gemm(x: torch.Tensor, codes: torch.Tensor, scales: torch.Tensor, zeros: Optional[torch.Tensor],
               n_bits: int, group: int, N: int, bias: Optional[torch.Tensor] = None, flags: int = 0,
               tiled: bool = False, out: Optional[torch.Tensor] = None, nib: bool = False,
               scales_gm: Optional[torch.Tensor] = None, zeros_gm: Optional[torch.Tensor] = None,
               zeroed_workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ W_deq^T (+ bias) with W_deq dequantized in registers from packed codes (MFMA).
    tiled: `codes` is in the decode tile layout (tile_codes), M <= 16 only.
    nib: `codes` is in the NIB layout (nib_codes), M >= NIB_MIN_M only (the prefill kernel).
    scales_gm / zeros_gm: optional group-major copies of the grouped parameters
    (group_major_params), read where gm_prefill_applies (same bits; scales / zeros elsewhere).
    out: optional contiguous fp16 [M, N] destination (rows of x flattened).
    zeroed_workspace: M <= 16 only, for graph capture: a uint8 device tensor of >= gemm_workspace_bytes
    whose first gemm_counter_bytes are zero and which the call leaves so (IWQ_FLAG_WS_ZEROED: the
    batched decode's cross-workgroup K-split); eager calls use a per-stream one without asking, calls
    captured without one take the unsplit kernels."""
    if tiled:
        flags |= L.IWQ_FLAG_TILED_CODES
    if nib:
        flags |= L.IWQ_FLAG_NIB_CODES
    L.require_device(x)
    if x.dtype != torch.float16:
        raise TypeError(f"w4a16_gemm: x must be float16, got {x.dtype}")
    K = x.shape[-1]
    _check_packed("w4a16_gemm", x.device, codes, scales, zeros, n_bits, group, N, K, bias)
    lib = L.load()
    x2 = x.reshape(-1, K)
    if x2.stride(-1) != 1 or x2.data_ptr() % 16 or x2.stride(0) % 8:
        x2 = x2.contiguous()
    M = x2.shape[0]
    if out is None:
        y = torch.empty((M, N), dtype=torch.float16, device=x.device)
    else:
        if (out.dtype != torch.float16 or out.device != x.device or not out.is_contiguous()
                or out.numel() != M * N):
            raise ValueError("w4a16_gemm: out must be a contiguous fp16 tensor of M*N elements on x's device")
        y = out.view(M, N)
    # split-K workspace (prefill kernel with fewer 256 x 256 tiles than CUs; variants 82-95 force 2-15
    # K ranges for A/B): fp32 partial tiles, from torch's caching allocator
    if nib and M < NIB_MIN_M:
        raise ValueError(f"w4a16_gemm: NIB-layout codes need M >= {NIB_MIN_M} rows, got {M}")
    with L.on_device(x.device):
        # the size depends on the CU count of the device it is queried on: ask x's device
        # (M <= 16: the K-split decode's fp32 slabs where it applies, tile layout or row-major)
        ws_bytes = int(lib.iwq_w4a16_gemm_workspace_bytes(M, N, K, int(group))) if (not tiled or M <= 16) else 0
        v = (int(flags) >> 16) & 0xFF
        if 81 < v < 96 and N % 256 == 0:
            ws_bytes = max(ws_bytes, ((M + 255) // 256) * (N // 256) * (v - 80) * 65536 * 4)
        if 110 <= v < 150 and N % 256 == 0:  # short-tile split (A/B): 128- / 64-row tiles, S ranges
            mtw, ns = (4, v - 108) if v < 130 else (2, v - 128)
            ws_bytes = max(ws_bytes, ((M + 32 * mtw - 1) // (32 * mtw)) * (N // 256) * ns * mtw * 8192 * 4)
        if (scales_gm is not None and not tiled and v == 0 and not (flags & L.IWQ_FLAG_FORCE_GENERIC)
                and ws_bytes == 0 and gm_prefill_applies(M, N, K, group)):
            _check_packed("w4a16_gemm", x.device, codes, scales_gm, zeros_gm, n_bits, group, N, K, bias)
            if (zeros_gm is None) != (zeros is None):
                raise ValueError("w4a16_gemm: zeros_gm must accompany zeros (and only zeros)")
            flags |= L.IWQ_FLAG_GROUP_MAJOR
            scales, zeros = scales_gm, zeros_gm
        if v == 31 and M <= 16:  # A/B: the K-split decode with a reduce launch (KS <= 16 slabs)
            ws_bytes = max(ws_bytes, 16 * M * N * 4)
        if 200 <= v < 260:  # A/B: the K-split decode forced to (CT, KS) (iwq_gemm.hip)
            ksn = 1 + (v - 200) % 20
            ws_bytes = max(ws_bytes, 16384 + ksn * M * N * 4)  # GEMV_KSX_CNT_BYTES + slabs
        gkey = None
        if M <= 16 and ws_bytes:
            if zeroed_workspace is not None:
                if (zeroed_workspace.dtype != torch.uint8 or zeroed_workspace.numel() < ws_bytes
                        or zeroed_workspace.device != x.device):
                    raise ValueError(f"w4a16_gemm: zeroed_workspace must be >= {ws_bytes} uint8 bytes on {x.device}")
                ws = zeroed_workspace
                flags |= L.IWQ_FLAG_WS_ZEROED
            elif not torch.cuda.is_current_stream_capturing():
                gkey = torch.cuda.current_stream(x.device).cuda_stream
                ws = _gws.get(x.device, gkey, ws_bytes)
                flags |= L.IWQ_FLAG_WS_ZEROED
            else:
                ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
        else:
            ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=x.device) if ws_bytes else None
        st = lib.iwq_w4a16_gemm_ws(L.ptr(x2), M, K, x2.stride(0), L.ptr(codes), L.ptr(scales), L.ptr(zeros),
                                   int(n_bits), int(group), N, L.ptr(bias), L.ptr(y), N, L.ptr(ws), ws_bytes,
                                   int(flags), L.stream_handle(x.device))
        if st != L.IWQ_OK and gkey is not None:
            _gws.drop(x.device, gkey)  # a failed launch may have left its counters dirty
    _raise_for(st, "iwq_w4a16_gemm")
    return y.reshape(*x.shape[:-1], N)


def gemm_workspace_bytes(M: int, N: int, K: int, group: int, flags: int = 0) -> int:
    """Workspace w4a16_gemm uses for this call (0: none); for a zeroed_workspace at M <= 16."""
    lib = L.load()
    n = int(lib.iwq_w4a16_gemm_workspace_bytes(M, N, K, int(group)))
    v = (int(flags) >> 16) & 0xFF
    if M <= 16 and v == 31:
        n = max(n, 16 * M * N * 4)
    if M <= 16 and 200 <= v < 260:
        ksn = 1 + (v - 200) % 20
        n = max(n, 16384 + ksn * M * N * 4)  # GEMV_KSX_CNT_BYTES + slabs
    return n


def tile_codes(codes: torch.Tensor, N: int, K: int) -> torch.Tensor:
    """Row-major packed 4-bit codes -> the decode tile layout (iwq_tile_codes): each 1 KiB a GEMV
    wave loads is contiguous.  Use with w4a16_gemm(..., tiled=True) for M <= 16."""
    L.require_device(codes)
    if codes.dtype != torch.uint8 or not codes.is_contiguous() or codes.numel() != N * K // 2:
        raise ValueError(f"tile_codes: codes must be contiguous uint8 with N*K/2 = {N * K // 2} elements")
    lib = L.load()
    out = torch.empty(N * K // 2, dtype=torch.uint8, device=codes.device)
    with L.on_device(codes.device):
        st = lib.iwq_tile_codes(L.ptr(codes), int(N), int(K), L.ptr(out), L.stream_handle(codes.device))
    _raise_for(st, "iwq_tile_codes")
    return out


def nib_codes(codes: torch.Tensor, N: int, K: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row-major packed 4-bit codes -> the NIB layout (iwq_nib_codes: nibble p of each code dword holds
    k = (0,2,4,6,1,3,5,7)[p]) read by w4a16_gemm(..., nib=True) at M >= NIB_MIN_M: the prefill
    kernel's dequant takes 9 instead of 12 VALU per 8 weights.  out may be `codes` (in place)."""
    L.require_device(codes)
    if codes.dtype != torch.uint8 or not codes.is_contiguous() or codes.numel() != N * K // 2 or K % 32:
        raise ValueError(f"nib_codes: codes must be contiguous uint8 with N*K/2 = {N * K // 2} elements, K % 32 == 0")
    if out is None:
        out = torch.empty(N * K // 2, dtype=torch.uint8, device=codes.device)
    elif out.dtype != torch.uint8 or not out.is_contiguous() or out.numel() != N * K // 2 or out.device != codes.device:
        raise ValueError("nib_codes: out must be contiguous uint8 of N*K/2 elements on codes' device")
    lib = L.load()
    with L.on_device(codes.device):
        st = lib.iwq_nib_codes(L.ptr(codes), int(N), int(K), L.ptr(out), L.stream_handle(codes.device))
    _raise_for(st, "iwq_nib_codes")
    return out.view(codes.shape)


def dequant_packed(codes: torch.Tensor, scales: torch.Tensor, zeros: Optional[torch.Tensor], n_bits: int,
                   group: int, N: int, K: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed codes -> fp16 W_deq [N, K], bit-identical to the reference's dequantized weight."""
    L.require_device(codes)
    _check_packed("dequant_packed", codes.device, codes, scales, zeros, n_bits, group, N, K)
    lib = L.load()
    if out is None:
        out = torch.empty((N, K), dtype=torch.float16, device=codes.device)
    elif (out.dtype != torch.float16 or out.device != codes.device or out.shape != (N, K)
          or out.stride(1) != 1):
        raise ValueError("dequant_packed: out must be an fp16 [N, K] tensor with unit column stride")
    with L.on_device(codes.device):
        st = lib.iwq_dequant_packed(L.ptr(codes), L.ptr(scales), L.ptr(zeros), int(n_bits), int(group), int(N),
                                    int(K), L.ptr(out), out.stride(0), L.stream_handle(codes.device))
    _raise_for(st, "iwq_dequant_packed")
    return out


def dequant_codes(codes: torch.Tensor, scales: torch.Tensor, zeros: Optional[torch.Tensor], n_bits: int,
                  group: int, symmetric: bool, quant_dim: int, rows: int, cols: int,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed codes of any INT mode (include/iwq.h layout) -> the dequantized [rows, cols] weight in
    the scales' dtype, bit-identical to what quantize_minmax(..., want_codes=True) returned as `out`
    next to those codes (iwq_dequant_codes)."""
    L.require_device(codes)
    dev, dt = codes.device, scales.dtype
    if dt not in L.DTYPE_CODE:
        raise TypeError(f"dequant_codes: unsupported parameter dtype {dt}")
    if not 1 <= n_bits <= 8:
        raise ValueError("dequant_codes: codes exist for 1 <= n_bits <= 8")
    _, G = group_geometry(rows, cols, group, quant_dim)
    if codes.dtype != torch.uint8 or not codes.is_contiguous() or codes.numel() != codes_nbytes(rows, cols, n_bits):
        raise ValueError(f"dequant_codes: codes must be contiguous uint8 of {codes_nbytes(rows, cols, n_bits)} bytes")
    for name, t in (("scales", scales), ("zeros", None if symmetric else zeros)):
        if name == "zeros" and t is None and not symmetric:
            raise ValueError("dequant_codes: asymmetric codes need zeros")
        if t is not None and (t.device != dev or t.dtype != dt or not t.is_contiguous() or t.numel() != G):
            raise ValueError(f"dequant_codes: {name} must be {G} contiguous {dt} values on {dev}")
    if out is None:
        out = torch.empty((rows, cols), dtype=dt, device=dev)
    elif out.dtype != dt or out.device != dev or out.shape != (rows, cols) or out.stride(1) != 1:
        raise ValueError("dequant_codes: out must be a [rows, cols] tensor of the scales' dtype, unit column stride")
    lib = L.load()
    with L.on_device(dev):
        st = lib.iwq_dequant_codes(L.ptr(codes), L.ptr(scales), None if symmetric else L.ptr(zeros),
                                   L.DTYPE_CODE[dt], int(n_bits), int(group), int(bool(symmetric)), int(quant_dim),
                                   int(rows), int(cols), L.ptr(out), out.stride(0), L.stream_handle(dev))
    _raise_for(st, "iwq_dequant_codes")
    return out


def w4a16_linear(x: torch.Tensor, codes: torch.Tensor, scales: torch.Tensor, zeros: Optional[torch.Tensor],
                 n_bits: int, group: int, N: int, bias: Optional[torch.Tensor] = None,
                 tiled_codes: Optional[torch.Tensor] = None,
                 nib_codes: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Forward on packed-only weights, fastest path per batch size: the weight-streaming GEMV for
    decode batches (M <= GEMV_MAX_M; on `tiled_codes` = tile_codes(codes) when given), the mid-M
    weight-streaming kernel and the split-K prefill kernel up to packed_fused_preferred's rows
    (1024 / 2048 per channel, 768 / 1024 g128), dequant-once + hipBLASLt (F.linear) above,
    where the library GEMM on a freshly dequantized weight beats the fused kernels.
    nib_codes: the same codes in the NIB layout (nib_codes(codes)), read by the prefill kernel at
    M >= NIB_MIN_M."""
    K = x.shape[-1]
    M = x.numel() // K
    if packed_fused_preferred(M, N, K, group) and w4a16_gemm_supported(x, N, K, n_bits, group):
        if tiled_codes is not None and M <= GEMV_MAX_M:
            return w4a16_gemm(x, tiled_codes, scales, zeros, n_bits, group, N, bias, tiled=True)
        if nib_codes is not None and M >= NIB_MIN_M and nib_supported(x, N, K, n_bits, group):
            return w4a16_gemm(x, nib_codes, scales, zeros, n_bits, group, N, bias, nib=True)
        return w4a16_gemm(x, codes, scales, zeros, n_bits, group, N, bias)
    w = dequant_packed(codes, scales, zeros, n_bits, group, N, K)
    return torch.nn.functional.linear(x, w, bias)


def batch_supported(w: torch.Tensor, n_bits: int, group: int, quant_dim: int = 0) -> bool:
    """Whether one weight can be an entry of a batched whole-model launch (BatchPlan) for this
    configuration (include/iwq.h iwq_batch_plan_ex); otherwise quantize it with its own call."""
    if not (w.is_cuda and w.dim() == 2 and w.is_contiguous() and w.dtype in L.DTYPE_CODE
            and w.data_ptr() % 16 == 0 and 1 <= n_bits <= 8 and quant_dim in (0, 1)):
        return False
    rows, cols = w.shape
    eb = w.element_size()
    if group == -1:
        return rows * cols % 8 == 0
    if quant_dim == 1:
        g = rows if group == -2 else group
        return g > 0 and rows % g == 0 and cols % 8 == 0
    if group in FAST_GROUPS:
        return n_bits >= 2 and cols % group == 0
    Lg = cols if group == -2 else group
    return Lg > 0 and cols % Lg == 0 and Lg % 8 == 0 and Lg <= 16384 and (cols * eb) % 16 == 0


class BatchPlan:
    """Device-resident work table for quantizing many weights in one launch (quant_wrapper.py:52-82).

    Every group mode and quant_dim (include/iwq.h iwq_batch_plan_ex): per-group (power of two
    8..512, quant_dim 0) is ONE persistent launch over all weights; per-channel / long groups run one
    launch per distinct group length (one register class each: 2 for a Llama-2-7B), quant_dim 1 one
    launch, per-tensor one key-init + reduce + apply triple.  Each weight gets exactly the bits of its
    own quantize_minmax call.  Built once per set of tensors; `run()` may be replayed (e.g. by
    bench.py) without host work beyond the launches."""

    def __init__(self, weights: List[torch.Tensor], n_bits: int, group: int, symmetric: bool,
                 outs: Optional[List[torch.Tensor]] = None, want_scales: bool = True, want_codes: bool = False,
                 quant_dim: int = 0):
        if not weights:
            raise ValueError("empty batch")
        lib = L.load()
        dev = weights[0].device
        dt = weights[0].dtype
        for w in weights:
            L.require_device(w)
            if w.device != dev or w.dtype != dt or w.dim() != 2 or not w.is_contiguous():
                raise ValueError("batched weights must be contiguous 2-D tensors of one dtype on one device")
            group_geometry(w.shape[0], w.shape[1], group, quant_dim)  # the reference's errors first
            if not batch_supported(w, n_bits, group, quant_dim):
                raise ValueError(f"weight {tuple(w.shape)} cannot join a batched launch for group {group}, "
                                 f"quant_dim {quant_dim}, n_bits {n_bits} (kernels.batch_supported)")
        self.device, self.dtype = dev, dt
        self.n_bits, self.group, self.symmetric = int(n_bits), int(group), bool(symmetric)
        self.quant_dim = int(quant_dim)
        self.weights = weights
        self.outs = outs if outs is not None else [torch.empty_like(w) for w in weights]
        sizes = [group_geometry(w.shape[0], w.shape[1], group, quant_dim)[1] for w in weights]
        self.scales = _param_views(sizes, dt, dev) if want_scales else [None] * len(weights)
        self.zeros = (_param_views(sizes, dt, dev) if (want_scales and not symmetric)
                      else [None] * len(weights))
        self.codes = [torch.empty(codes_nbytes(w.shape[0], w.shape[1], n_bits), dtype=torch.uint8, device=dev)
                      if want_codes else None for w in weights]
        self.want_codes = want_codes
        # launches: per-channel / long groups need one register class per launch -> bucket by length
        if quant_dim == 0 and group not in FAST_GROUPS and group != -1:
            buckets = {}
            for i, w in enumerate(weights):
                buckets.setdefault(w.shape[1] if group == -2 else group, []).append(i)
            index_sets = [buckets[k] for k in sorted(buckets)]
        else:
            index_sets = [list(range(len(weights)))]
        self.launches = []
        for idx in index_sets:
            table = (L.IwqBatchEntry * len(idx))()
            for k, i in enumerate(idx):
                table[k].w = weights[i].data_ptr()
                table[k].out_deq = self.outs[i].data_ptr() if self.outs[i] is not None else None
                table[k].out_codes = self.codes[i].data_ptr() if self.codes[i] is not None else None
                table[k].out_scales = self.scales[i].data_ptr() if self.scales[i] is not None else None
                table[k].out_zeros = self.zeros[i].data_ptr() if self.zeros[i] is not None else None
                table[k].rows, table[k].cols = weights[i].shape
            total, glen = ctypes.c_int64(0), ctypes.c_int64(0)
            _raise_for(lib.iwq_batch_plan_ex(table, len(idx), L.DTYPE_CODE[dt], self.n_bits, self.group,
                                             self.quant_dim, ctypes.byref(total), ctypes.byref(glen)),
                       "iwq_batch_plan_ex")
            wsb = int(lib.iwq_batch_workspace_bytes(len(idx), self.group, self.quant_dim))
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev) if wsb else None
            d_table = torch.frombuffer(bytearray(bytes(table)), dtype=torch.uint8).to(dev)
            self.launches.append((d_table, len(idx), total.value, glen.value, ws, wsb))
        self.d_table, self.n, self.total_units = self.launches[0][0], len(weights), self.launches[0][2]
        self.nan_flag = torch.zeros(1, dtype=torch.int32, device=dev)
        self.numel = sum(w.numel() for w in weights)

    def run(self, stream=None, variant=0):
        lib = L.load()
        flags = (L.IWQ_FLAG_BATCH_CODES if self.want_codes else 0) | ((int(variant) & 0xFF) << 16)
        sh = ctypes.c_void_p(stream.cuda_stream) if stream is not None else L.stream_handle(self.device)
        with L.on_device(self.device):
            for d_table, n, total, glen, ws, wsb in self.launches:
                st = lib.iwq_quantize_minmax_batched_ex(L.ptr(d_table), n, total, glen, L.DTYPE_CODE[self.dtype],
                                                        self.n_bits, self.group, int(self.symmetric), self.quant_dim,
                                                        L.ptr(ws), wsb, L.ptr(self.nan_flag), flags, sh)
                _raise_for(st, "iwq_quantize_minmax_batched_ex")


def fill_synthetic(t: torch.Tensor, seed: int, index_offset: int = 0):
    """Fill a contiguous tensor with oracle/synth.py's deterministic weights (bit-identical)."""
    L.require_device(t)
    assert t.is_contiguous() and t.dtype in L.DTYPE_CODE
    lib = L.load()
    with L.on_device(t.device):
        st = lib.iwq_fill_synthetic(L.ptr(t), t.numel(), L.DTYPE_CODE[t.dtype], int(seed), int(index_offset),
                                    L.stream_handle(t.device))
    L.check(st, "iwq_fill_synthetic")
    return t


def selftest_division(device="cuda"):
    """(quotient fp32 mismatches, quotient fp16 mismatches, reciprocal mismatches) of the hot loop's
    fast division vs IEEE division, exhaustive over fp16 operands."""
    lib = L.load()
    counts = torch.zeros(3, dtype=torch.int64, device=device)
    with L.on_device(counts.device):
        L.check(lib.iwq_selftest_division(L.ptr(counts), L.stream_handle(counts.device)), "iwq_selftest_division")
    return tuple(int(x) for x in counts.cpu())


def _param_views(sizes, dtype, dev):
    """Per-tensor [G] parameter vectors (sizes[i] elements each) as views of ONE allocation (one
    caching-allocator call instead of one per layer: 224 / 560 for a 7B / 70B model); each view is
    contiguous."""
    return list(torch.empty(sum(sizes), dtype=dtype, device=dev).split(sizes))


class FpBatchPlan:
    """Whole-model FP fake quantization in ONE launch (quantize_model's loop for weight_format
    fp4/fp6/fp8, approximate single-aligned decode, or the E2M1 grid): fp16 contiguous weights,
    power-of-two groups in [8, 512], decode table path (iwq_quantize_fp_batched).  Per tensor the
    result is bit-identical to quantize_fp / quantize_fp_approx / fp4_grid."""

    def __init__(self, weights: List[torch.Tensor], codec: int, exp_bits: int, mant_bits: int, group: int,
                 symmetric: bool, hs: int = 0, hf: int = 0, tp: int = 0,
                 outs: Optional[List[torch.Tensor]] = None):
        if not weights:
            raise ValueError("empty batch")
        lib = L.load()
        dev = weights[0].device
        for w in weights:
            L.require_device(w)
            if w.device != dev or w.dtype != torch.float16 or w.dim() != 2 or not w.is_contiguous():
                raise ValueError("batched FP weights must be contiguous 2-D fp16 tensors on one device")
        if group not in FAST_GROUPS:
            raise ValueError("batched FP path supports power-of-two groups 8..512")
        self.device = dev
        self.codec, self.exp_bits, self.mant_bits = int(codec), int(exp_bits), int(mant_bits)
        self.group, self.symmetric = int(group), bool(symmetric) or codec != L.IWQ_CODEC_FP
        self.hs, self.hf, self.tp = int(hs), int(hf), int(tp)
        self.lut = _luts.get(dev, codec, exp_bits if codec != L.IWQ_CODEC_GRID else 0,
                             mant_bits if codec != L.IWQ_CODEC_GRID else 0, hs, hf, tp)
        if self.lut is None:
            raise RuntimeError("decode table unavailable for this format (or building it inside a graph capture)")
        self.weights = weights
        self.outs = outs if outs is not None else [torch.empty_like(w) for w in weights]
        sizes = [w.numel() // group for w in weights]
        self.scales = _param_views(sizes, torch.float16, dev)
        self.zeros = (_param_views(sizes, torch.float16, dev) if not self.symmetric
                      else [None] * len(weights))
        n = len(weights)
        table = (L.IwqBatchEntry * n)()
        for i, w in enumerate(weights):
            table[i].w = w.data_ptr()
            table[i].out_deq = self.outs[i].data_ptr()
            table[i].out_codes = None
            table[i].out_scales = self.scales[i].data_ptr()
            table[i].out_zeros = self.zeros[i].data_ptr() if self.zeros[i] is not None else None
            table[i].rows, table[i].cols = w.shape
        total = ctypes.c_int64(0)
        _raise_for(lib.iwq_batch_plan(table, n, L.IWQ_F16, 8, self.group, ctypes.byref(total)), "iwq_batch_plan")
        self.total_units = total.value
        self.d_table = torch.frombuffer(bytearray(bytes(table)), dtype=torch.uint8).to(dev)
        self.n = n
        self.nan_flag = torch.zeros(1, dtype=torch.int32, device=dev)
        self.numel = sum(w.numel() for w in weights)

    def run(self, stream=None):
        lib = L.load()
        sh = ctypes.c_void_p(stream.cuda_stream) if stream is not None else L.stream_handle(self.device)
        with L.on_device(self.device):
            st = lib.iwq_quantize_fp_batched(L.ptr(self.d_table), self.n, self.total_units, self.codec,
                                             self.exp_bits, self.mant_bits, self.group, int(self.symmetric),
                                             self.hs, self.hf, self.tp, L.ptr(self.lut), L.ptr(self.nan_flag), 0, sh)
        _raise_for(st, "iwq_quantize_fp_batched")

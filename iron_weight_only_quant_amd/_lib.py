"""Loader for the in-tree HIP library (include/iwq.h C-ABI) via ctypes.

The product path has NO CPU fallback: if the library is missing, or no ROCm GPU is
visible when a kernel is requested, these functions raise.  PyTorch is only the
allocator/stream provider; the C-ABI takes raw device pointers and a hipStream_t.
"""
import contextlib
import ctypes
import os
import threading

import torch  # imported first: torch's libamdhip64.so.7 becomes THE HIP runtime of the process

HERE = os.path.dirname(os.path.abspath(__file__))
# IWQ_AB=1: the A/B library (every kernel variant; iron_weight_only_quant_amd/build.py) instead of the
# product one
LIB_PATH = os.path.join(HERE, "_lib", "libiwq_ab.so" if os.environ.get("IWQ_AB", "0") == "1" else "libiwq.so")

IWQ_F16, IWQ_BF16, IWQ_F32 = 0, 1, 2
DTYPE_CODE = {torch.float16: IWQ_F16, torch.bfloat16: IWQ_BF16, torch.float32: IWQ_F32}

IWQ_OK = 0
IWQ_ERR_SHAPE, IWQ_ERR_GROUP, IWQ_ERR_GROUP_MODE, IWQ_ERR_BITS, IWQ_ERR_DTYPE = 1, 2, 3, 4, 5
IWQ_ERR_WORKSPACE, IWQ_ERR_CODES, IWQ_ERR_HIP, IWQ_ERR_ARG, IWQ_ERR_FORMAT = 6, 7, 8, 9, 10

IWQ_FLAG_FORCE_GENERIC = 0x1
IWQ_FLAG_BATCH_CODES = 0x100
IWQ_FLAG_TILED_CODES = 0x200
IWQ_FLAG_NIB_CODES = 0x400
IWQ_FLAG_GROUP_MAJOR = 0x800
IWQ_FLAG_WS_ZEROED = 0x1000

EXPORTS = (
    "iwq_workspace_bytes", "iwq_quantize_minmax", "iwq_batch_plan", "iwq_quantize_minmax_batched",
    "iwq_fill_synthetic", "iwq_status_string", "iwq_last_hip_error", "iwq_build_info",
    "iwq_selftest_division", "iwq_quantize_fp", "iwq_fp4_grid", "iwq_w4a16_gemm",
    "iwq_approx_workspace_bytes", "iwq_quantize_fp_approx", "iwq_quantize_bfp",
    "iwq_fp_build_lut", "iwq_quantize_fp_lut", "iwq_quantize_fp_approx_lut", "iwq_fp4_grid_lut",
    "iwq_dequant_packed", "iwq_dequant_codes", "iwq_quantize_fp_batched", "iwq_tile_codes", "iwq_nib_codes",
    "iwq_w4a16_gemm_workspace_bytes", "iwq_w4a16_gemm_ws", "iwq_fp4_grid_packed", "iwq_dequant_fp_packed",
    "iwq_batch_plan_ex", "iwq_batch_workspace_bytes", "iwq_quantize_minmax_batched_ex",
)

IWQ_CODEC_FP, IWQ_CODEC_GRID, IWQ_CODEC_APX, IWQ_CODEC_APX_DOUBLE = 0, 1, 2, 3
IWQ_FP_LUT_BYTES = 65536


class IwqBatchEntry(ctypes.Structure):
    """Mirror of `iwq_batch_entry` (include/iwq.h)."""
    _fields_ = [("w", ctypes.c_void_p), ("out_deq", ctypes.c_void_p), ("out_codes", ctypes.c_void_p),
                ("out_scales", ctypes.c_void_p), ("out_zeros", ctypes.c_void_p), ("rows", ctypes.c_int64),
                ("cols", ctypes.c_int64), ("unit_begin", ctypes.c_int64)]


_lock = threading.Lock()
_lib = None


class IwqError(RuntimeError):
    def __init__(self, status, what):
        self.status = status
        super().__init__(f"{what}: {status_string(status)} (status {status})")


def load():
    """Load libiwq.so (raises OSError if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise OSError(f"iwq HIP library not built: {LIB_PATH} missing (run `python -c 'import __graft_entry__ as g; "
                          f"g.build()'`; the A/B library: `IWQ_AB=1 python -m iron_weight_only_quant_amd.build --ab`)")
        lib = ctypes.CDLL(LIB_PATH)
        i64, i32, u32, vp, u64 = ctypes.c_int64, ctypes.c_int, ctypes.c_uint, ctypes.c_void_p, ctypes.c_uint64
        lib.iwq_workspace_bytes.argtypes = [i64, i64, i64, i32]
        lib.iwq_workspace_bytes.restype = i64
        lib.iwq_quantize_minmax.argtypes = [vp, i64, i64, i64, i32, i32, i64, i32, i32, vp, i64, vp, vp, vp, vp, i64,
                                            vp, u32, vp]
        lib.iwq_quantize_minmax.restype = i32
        lib.iwq_batch_plan.argtypes = [ctypes.POINTER(IwqBatchEntry), ctypes.c_int32, i32, i32, i64,
                                       ctypes.POINTER(i64)]
        lib.iwq_batch_plan.restype = i32
        lib.iwq_quantize_minmax_batched.argtypes = [vp, ctypes.c_int32, i64, i32, i32, i64, i32, vp, u32, vp]
        lib.iwq_quantize_minmax_batched.restype = i32
        lib.iwq_batch_plan_ex.argtypes = [ctypes.POINTER(IwqBatchEntry), ctypes.c_int32, i32, i32, i64, i32,
                                          ctypes.POINTER(i64), ctypes.POINTER(i64)]
        lib.iwq_batch_plan_ex.restype = i32
        lib.iwq_batch_workspace_bytes.argtypes = [ctypes.c_int32, i64, i32]
        lib.iwq_batch_workspace_bytes.restype = i64
        lib.iwq_quantize_minmax_batched_ex.argtypes = [vp, ctypes.c_int32, i64, i64, i32, i32, i64, i32, i32, vp, i64,
                                                       vp, u32, vp]
        lib.iwq_quantize_minmax_batched_ex.restype = i32
        lib.iwq_fill_synthetic.argtypes = [vp, i64, i32, u64, i64, vp]
        lib.iwq_fill_synthetic.restype = i32
        lib.iwq_status_string.argtypes = [i32]
        lib.iwq_status_string.restype = ctypes.c_char_p
        lib.iwq_last_hip_error.argtypes = []
        lib.iwq_last_hip_error.restype = i32
        lib.iwq_build_info.argtypes = []
        lib.iwq_build_info.restype = ctypes.c_char_p
        lib.iwq_quantize_fp.argtypes = [vp, i64, i64, i64, i32, i32, i32, i64, i32, i32, vp, i64, vp, vp, vp, vp,
                                        i64, vp, u32, vp]
        lib.iwq_quantize_fp.restype = i32
        lib.iwq_fp4_grid.argtypes = [vp, i64, i64, i64, i32, vp, vp, vp, i64, vp, u32, vp]
        lib.iwq_fp4_grid_packed.argtypes = [vp, i64, i64, i64, i32, vp, vp, vp, vp, i64, vp, u32, vp, vp]
        lib.iwq_fp4_grid_packed.restype = i32
        lib.iwq_dequant_fp_packed.argtypes = [vp, vp, vp, i32, i32, i64, i64, i64, vp, i64, vp]
        lib.iwq_dequant_fp_packed.restype = i32
        lib.iwq_fp4_grid.restype = i32
        lib.iwq_w4a16_gemm.argtypes = [vp, i64, i64, i64, vp, vp, vp, i32, i64, i64, vp, vp, i64, u32, vp]
        lib.iwq_w4a16_gemm.restype = i32
        lib.iwq_w4a16_gemm_workspace_bytes.argtypes = [i64, i64, i64, i64]
        lib.iwq_w4a16_gemm_workspace_bytes.restype = i64
        lib.iwq_w4a16_gemm_ws.argtypes = [vp, i64, i64, i64, vp, vp, vp, i32, i64, i64, vp, vp, i64, vp, i64, u32, vp]
        lib.iwq_w4a16_gemm_ws.restype = i32
        lib.iwq_approx_workspace_bytes.argtypes = [i64, i64, i32, i32, i64, i32, i32]
        lib.iwq_approx_workspace_bytes.restype = i64
        lib.iwq_quantize_fp_approx.argtypes = [vp, i64, i64, i64, i32, i32, i32, i64, i32, i32, i32, i32, i32, vp,
                                               i64, vp, vp, i64, vp, u32, vp]
        lib.iwq_quantize_fp_approx.restype = i32
        lib.iwq_quantize_bfp.argtypes = [vp, i64, i64, i64, i32, i32, i64, i32, vp, i64, u32, vp]
        lib.iwq_quantize_bfp.restype = i32
        lib.iwq_fp_build_lut.argtypes = [i32, i32, i32, i32, i32, i32, vp, i64, vp]
        lib.iwq_fp_build_lut.restype = i32
        lib.iwq_quantize_fp_lut.argtypes = lib.iwq_quantize_fp.argtypes + [vp]
        lib.iwq_quantize_fp_lut.restype = i32
        lib.iwq_fp4_grid_lut.argtypes = lib.iwq_fp4_grid.argtypes + [vp]
        lib.iwq_fp4_grid_lut.restype = i32
        lib.iwq_quantize_fp_approx_lut.argtypes = lib.iwq_quantize_fp_approx.argtypes + [vp]
        lib.iwq_quantize_fp_approx_lut.restype = i32
        lib.iwq_quantize_fp_batched.argtypes = [vp, ctypes.c_int32, i64, i32, i32, i32, i64, i32, i32, i32, i32, vp,
                                                vp, u32, vp]
        lib.iwq_quantize_fp_batched.restype = i32
        lib.iwq_tile_codes.argtypes = [vp, i64, i64, vp, vp]
        lib.iwq_tile_codes.restype = i32
        lib.iwq_nib_codes.argtypes = [vp, i64, i64, vp, vp]
        lib.iwq_nib_codes.restype = i32
        lib.iwq_dequant_packed.argtypes = [vp, vp, vp, i32, i64, i64, i64, vp, i64, vp]
        lib.iwq_dequant_packed.restype = i32
        lib.iwq_dequant_codes.argtypes = [vp, vp, vp, i32, i32, i64, i32, i32, i64, i64, vp, i64, vp]
        lib.iwq_dequant_codes.restype = i32
        lib.iwq_selftest_division.argtypes = [vp, vp]
        lib.iwq_selftest_division.restype = i32
        _lib = lib
        return lib


def ab_built():
    """True when the loaded library carries the A/B kernel variants (IWQ_AB build)."""
    return load().iwq_build_info().endswith(b"ab=1")


def status_string(status):
    try:
        return load().iwq_status_string(int(status)).decode()
    except OSError:
        return "unknown"


def check(status, what):
    if status != IWQ_OK:
        if status == IWQ_ERR_HIP:
            raise IwqError(status, f"{what} (hipError {load().iwq_last_hip_error()})")
        raise IwqError(status, what)


def require_device(t):
    """The HIP path only runs on ROCm devices: fail loudly instead of falling back to the CPU."""
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError("iron_weight_only_quant_amd: tensors must live on a ROCm GPU (device 'cuda'); "
                           "there is no CPU fallback — use oracle/ only as a test checker")
    if torch.version.hip is None:
        raise RuntimeError("iron_weight_only_quant_amd requires a ROCm build of PyTorch")


_NULL_CTX = contextlib.nullcontext()


def on_device(device):
    """torch.cuda.device(device), or a no-op when it already is the current device (the common case:
    saves the two device switches, ~2 us per call on the decode path)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _NULL_CTX if idx == torch.cuda.current_device() else torch.cuda.device(idx)


def stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None

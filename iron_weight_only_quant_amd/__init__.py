"""MI355X-native (gfx950) weight-only min-max quantization — drop-in for the hot path of
LiuTielong/Iron_weight_only_quant (quant_funcs / quant_linear / quant_wrapper).

Kernels: csrc/*.hip, C-ABI: include/iwq.h, built in-tree into _lib/libiwq.so (build.py)."""
from .build import build_library, library_path  # noqa: F401

__all__ = ["build_library", "library_path"]
__version__ = "0.1.0"

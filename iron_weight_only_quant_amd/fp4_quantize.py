"""Drop-in for the reference's fp4_quantize_cpu.py (`quantize_fp16_to_fp4_e1m2`, :47-72) on the GPU.

Same signature, grouping, errors and return value: the GROUPED view ([-1, group_size], or [1, numel]
per tensor) of the fake-quantized fp16 values.  `return_scales` is accepted and ignored, as in the
reference (fp4_quantize_cpu.py:47, :72); the per-group scales S = absmax / 6 (and the E2M1 codes) are
available from kernels.fp4_grid(w, group_size, per_tensor, want_codes=...)."""
import torch

from . import kernels


@torch.no_grad()
def quantize_fp16_to_fp4_e1m2(tensor, group_size=128, per_tensor=False, return_scales=False):
    if tensor.dtype != torch.float16:
        tensor = tensor.to(torch.float16)
    if tensor.dim() != 2:
        raise ValueError("Expected a 2D tensor of shape [out_features, in_features].")
    rows, cols = tensor.shape
    if group_size > 0 and cols % group_size != 0:
        raise ValueError("in_features must be divisible by group_size.")
    res = kernels.fp4_grid(tensor, group_size, per_tensor)
    out = res.out
    if group_size > 0:
        out = out.reshape(-1, group_size)
    if per_tensor:
        out = out.reshape(1, -1)
    return out

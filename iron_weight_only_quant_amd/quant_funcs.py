"""Drop-in for the reference's quant_funcs.py (same names, arguments, return values and errors).

pseudo_quantize_tensor            quant_funcs.py:4-46
quantize_weight_per_channel_absmax        :50-55
quantize_activation_per_token_absmax      :58-62
quantize_weight_per_tensor_absmax         :65-70
quantize_activation_per_tensor_absmax     :73-77

Every call runs the gfx950 kernels (csrc/iwq_minmax.hip); inputs must be on a ROCm GPU.
The reference's NaN assertion (:40) is kept: the kernel raises a device flag, read once here.
"""
import torch

from . import kernels


@torch.no_grad()
def pseudo_quantize_tensor(tensor, n_bits=8, zero_point=True, q_group_size=-1, per_tensor=False, inplace=False):
    """Min-max fake quantization (quantize -> dequantize), returns a tensor of the input's shape.

    Grouping follows the reference exactly: reshape(-1, q_group_size) when q_group_size > 0 (the
    last dim must divide, :11), then reshape(1, -1) when per_tensor, else the 2-D input's rows (:15).
    With inplace=True a contiguous input is overwritten (as the reference's in-place chain does
    through its reshape view, :31-34); a non-contiguous one is not (its reshape copied)."""
    org_shape = tensor.shape
    if q_group_size > 0:
        assert org_shape[-1] % q_group_size == 0
    if q_group_size > 0 or per_tensor:
        # the grouped view is a flat re-chunking; any 2-D factorisation whose row length is a
        # multiple of the group length produces identical groups
        cols = org_shape[-1] if len(org_shape) >= 1 else 1
        rows = tensor.numel() // max(cols, 1)
        group = -1 if per_tensor else q_group_size
        view_ok = tensor.is_contiguous()
        src = tensor.reshape(rows, cols) if view_ok else tensor.contiguous().view(rows, cols)
    else:
        assert tensor.dim() == 2
        rows, cols = org_shape
        group = -2
        src = tensor
    if inplace and (q_group_size > 0 or per_tensor) and not tensor.is_contiguous():
        inplace = False  # reference: reshape() copied, the caller's tensor is untouched
    if inplace and src.stride(-1) == 1:
        res = kernels.quantize_minmax(src, n_bits, group, not zero_point, 0, out=src, want_scales=False)
        out = src
    else:
        res = kernels.quantize_minmax(src, n_bits, group, not zero_point, 0, want_scales=False)
        out = res.out
        if inplace:
            src.copy_(out)
            out = src
    assert not res.has_nan()
    return out.reshape(org_shape)


@torch.no_grad()
def quantize_weight_per_channel_absmax(w, n_bits=8):
    return pseudo_quantize_tensor(w, n_bits=n_bits, zero_point=False, q_group_size=-1, per_tensor=False, inplace=False)


@torch.no_grad()
def quantize_activation_per_token_absmax(t, n_bits=8):
    t_shape = t.shape
    t = t.view(-1, t_shape[-1])
    t = pseudo_quantize_tensor(t, n_bits=n_bits, zero_point=True, q_group_size=-1, per_tensor=False, inplace=False)
    return t.reshape(t_shape)


@torch.no_grad()
def quantize_weight_per_tensor_absmax(w, n_bits=8):
    return pseudo_quantize_tensor(w, n_bits=n_bits, zero_point=False, q_group_size=-1, per_tensor=True, inplace=False)


@torch.no_grad()
def quantize_activation_per_tensor_absmax(t, n_bits=8):
    t_shape = t.shape
    t = t.view(-1, t_shape[-1])
    t = pseudo_quantize_tensor(t, n_bits=n_bits, zero_point=True, q_group_size=-1, per_tensor=True, inplace=False)
    return t.reshape(t_shape)

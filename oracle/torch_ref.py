"""CPU baseline: op-for-op torch-CPU restatement of the reference's quantizer.

TEST/BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests/).  This is the reference's
own arithmetic — the ATen op sequence of quant_funcs.py:16-38 (== quant_linear.py:909-947) on CPU
tensors of the storage dtype — restated so it can be timed on the GPU box's host cores, where
the reference itself does not exist.  Pinned bit-exactly against the reference's golden fixtures
in tests/test_oracle_golden.py::test_torch_restatement_matches_golden.
"""
import torch


@torch.no_grad()
def minmax_fake_quant_cpu(w: torch.Tensor, n_bits: int, zero_point: bool, group: int, per_tensor: bool = False):
    """Same arithmetic as quant_funcs.pseudo_quantize_tensor (out-of-place variant); CPU tensors."""
    shape = w.shape
    grouped = w
    if group > 0:
        assert shape[-1] % group == 0
        grouped = grouped.reshape(-1, group)
    if per_tensor:
        grouped = grouped.reshape(1, -1)
    assert grouped.dim() == 2
    if zero_point:
        hi_q = 2 ** n_bits - 1
        lo_q = 0
        vmax = grouped.amax(dim=1, keepdim=True)
        vmin = grouped.amin(dim=1, keepdim=True)
        step = (vmax - vmin).clamp(min=1e-5) / hi_q
        zp = (-torch.round(vmin / step)).clamp_(lo_q, hi_q)
    else:
        hi_q = 2 ** (n_bits - 1) - 1
        lo_q = -(2 ** (n_bits - 1))
        step = grouped.abs().amax(dim=1, keepdim=True).clamp(min=1e-5) / hi_q
        zp = 0
    q = torch.clamp(torch.round(grouped / step) + zp, lo_q, hi_q)
    deq = (q - zp) * step
    assert torch.isnan(deq).sum() == 0
    return deq.reshape(shape)

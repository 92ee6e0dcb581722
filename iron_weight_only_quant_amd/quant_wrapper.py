"""Drop-in for the reference's quant_wrapper.quantize_model (quant_wrapper.py:7-84), RTN branch.

Same contract: every nn.Linear whose qualified name contains neither 'lm_head' nor 'output_layer'
is replaced (setattr on its parent) by a QuantLinear that aliases and overwrites the original
weight storage; weight-only runs need 0 < w_bit < 16 and a_bit None or >= 16 (:10-11).

MI355X-first difference: instead of quantizing layer after layer (one ~16-op ATen chain plus an
empty_cache per layer, :52-82), all eligible layers that live on one GPU and share a dtype are
quantized by batched multi-tensor launches: INT in every group mode (kernels.BatchPlan: ONE launch
for power-of-two groups 8..512, one per distinct row length for per-channel / long groups, one for
quant_dim 1, three for per-tensor), FP4/FP6/FP8 and the single-aligned approximate decode on fp16
weights with power-of-two groups (kernels.FpBatchPlan, one launch).  Layers a batch cannot take
(strided, unaligned, rows longer than 16384 per channel, ...) use one launch per layer.
"""
import torch

from . import kernels
from .quant_linear import QuantLinear


def _eligible(name, module):
    return isinstance(module, torch.nn.Linear) and "lm_head" not in name and "output_layer" not in name


def _set_module(model, name, new):
    parent = model
    path = name.split(".")
    for p in path[:-1]:
        parent = getattr(parent, p)
    if path[-1] in parent._modules:  # replacing a registered child: skip nn.Module.__setattr__'s checks
        parent._modules[path[-1]] = new
    else:
        setattr(parent, path[-1], new)


def _qkw(args, w_format):
    return dict(
        w_bit=args.w_bit, w_group_size=args.w_group_size, symmetric=args.w_symmetric,
        mode=getattr(args, "mode", 0), weight_format=w_format, approximate=getattr(args, "approximate", False),
        quant_dim=getattr(args, "quant_dim", 0),
        fp8_hi_align_start=getattr(args, "fp8_hi_align_start", 12),
        fp8_hi_align_exp_field=getattr(args, "fp8_hi_align_exp_field", 15),
        fp8_tail_pad_bits=getattr(args, "fp8_tail_pad_bits", 1),
        double_approximate=getattr(args, "double_approximate", False),
        fp6_hi_align_start=getattr(args, "fp6_hi_align_start", 4),
        fp6_hi_align_exp_field=getattr(args, "fp6_hi_align_exp_field", 7),
        fp6_tail_pad_bits=getattr(args, "fp6_tail_pad_bits", 2),
        fp4_hi_align_start=getattr(args, "fp4_hi_align_start", 1),
        fp4_hi_align_exp_field=getattr(args, "fp4_hi_align_exp_field", 1),
        fp4_tail_pad_bits=getattr(args, "fp4_tail_pad_bits", 0),
        # MI355X additions (not in the reference's args): the packed-code forward of QuantLinear
        # (False = the reference's F.linear on the dequantized weight, "auto" = packed GEMV for
        # decode batches, True = always the fused kernels) and its opt-in NIB prefill layout
        fused_forward=getattr(args, "fused_forward", False),
        nib_prefill=getattr(args, "nib_prefill", False),
        keep_codes=getattr(args, "keep_codes", False),
    )


def _tied(layers):
    """Names of layers whose weight bytes overlap those of an EARLIER layer (tied weights: two
    Linear modules over one storage).  Such a pair must not be two entries of one in-place launch
    (a data race); the reference quantizes them one after the other, the later one on the earlier
    one's dequantized output, which the per-layer loop after the batch replays in layer order.
    One sort + sweep over byte intervals, so untied models pay O(n log n) host time."""
    iv = []
    for i, (n, m) in enumerate(layers):
        w = m.weight.data
        if w.numel():
            lo = w.data_ptr()
            iv.append((str(w.device), lo, lo + w.numel() * w.element_size(), i))
    iv.sort()
    tied, active = set(), []
    for dev, lo, hi, i in iv:
        active = [a for a in active if a[0] == dev and a[1] > lo]
        for _, _, j in active:
            tied.add(layers[max(i, j)][0])
        active.append((dev, hi, i))
    return tied


def quantize_model(model, args, quant_mix_gate=False, batched=True, verbose=True):
    if not ((args.w_bit is not None and args.w_bit < 16) and (args.a_bit is None or args.a_bit >= 16)):
        return model
    assert args.w_bit > 0 and args.w_bit < 16, \
        "Weight bitwidth should be an integer between [1, 16] for weigth-only quantization, please check."
    w_format = getattr(args, "w_format", "int").lower()
    is_bfp = w_format.startswith("bfp")
    if is_bfp and getattr(args, "w_group_size", -1) <= 0:
        raise ValueError("BFP quantization needs a positive w_group_size (e.g. 128)")
    if getattr(args, "gptq", False):
        raise NotImplementedError("GPTQ calibration is outside this build's hot path (SURVEY.md §2 #8)")
    if verbose:
        print("Using RTN (Round-to-Nearest) quantization")
    kw = _qkw(args, w_format)
    layers = [(n, m) for n, m in model.named_modules() if _eligible(n, m)]

    done = set()
    tied = _tied(layers) if batched else set()
    g = kw["w_group_size"]
    qd = kw["quant_dim"]
    if (batched and w_format == "int" and not kw["approximate"] and 1 <= kw["w_bit"] <= 8 and layers
            and (g > 0 or g in (-1, -2)) and qd in (0, 1) and not (kw["symmetric"] and kw["w_bit"] < 2)):
        buckets = {}
        for n, m in layers:
            w = m.weight.data
            if n not in tied and w.device.type == "cuda" and kernels.batch_supported(w, kw["w_bit"], g, qd):
                buckets.setdefault((w.device, w.dtype), []).append((n, m))
        want_codes = bool(kw["keep_codes"] or kw["fused_forward"])  # as QuantLinear.quantize_weight
        for (dev, dt), items in buckets.items():
            ws = [m.weight.data for _, m in items]
            plan = kernels.BatchPlan(ws, kw["w_bit"], g, bool(kw["symmetric"]), outs=ws, want_codes=want_codes,
                                     quant_dim=qd)
            plan.run()
            for i, (n, m) in enumerate(items):
                q = QuantLinear.from_linear(m, quantize=False, **kw)
                q._set_int_result(plan.scales[i], plan.zeros[i], plan.codes[i])
                _set_module(model, n, q)
                done.add(n)
    if (batched and w_format in ("fp4", "fp6", "fp8") and kw["quant_dim"] == 0 and g in kernels.FAST_GROUPS
            and not (kw["approximate"] and kw["double_approximate"]) and layers
            and not (kw["keep_codes"] or kw["fused_forward"])):  # FP codes: per-layer path keeps them
        _batched_fp(model, layers, kw, w_format, done, tied)
    for n, m in layers:
        if n in done:
            continue
        q = QuantLinear.from_linear(m, **kw)
        _set_module(model, n, q)
    return model


def _batched_fp(model, layers, kw, fmt, done, tied):
    """FP formats (and the single-aligned approximate decode) of every eligible fp16 layer on one
    GPU in one launch (kernels.FpBatchPlan); buffers as QuantLinear's FP branches set them."""
    from . import _lib as L
    from .quant_linear import _fp_bits
    e, m = _fp_bits(fmt)
    g = kw["w_group_size"]
    apx = bool(kw["approximate"])
    if apx and fmt == "fp4" and e not in (1, 2):
        return  # the per-layer path raises the reference's error
    hs, hf, tp = ((kw[f"{fmt}_hi_align_start"], kw[f"{fmt}_hi_align_exp_field"], kw[f"{fmt}_tail_pad_bits"])
                  if apx else (0, 0, 0))
    codec = L.IWQ_CODEC_APX if apx else L.IWQ_CODEC_FP
    sym = True if apx else bool(kw["symmetric"])
    buckets = {}
    for n, mod in layers:
        w = mod.weight.data
        if (n not in tied and w.device.type == "cuda" and w.dim() == 2 and w.is_contiguous()
                and w.shape[1] % g == 0 and w.dtype == torch.float16 and w.data_ptr() % 16 == 0):
            buckets.setdefault(w.device, []).append((n, mod))
    for dev, items in buckets.items():
        ws = [mod.weight.data for _, mod in items]
        try:
            plan = kernels.FpBatchPlan(ws, codec, e, m, g, sym, hs, hf, tp, outs=ws)
        except (RuntimeError, ValueError, AssertionError):
            continue  # e.g. E5M2 (fp_max overflows fp16): per-layer path raises like the reference
        plan.run()
        for i, (n, mod) in enumerate(items):
            q = QuantLinear.from_linear(mod, quantize=False, **kw)
            # weight_fp4/6/8 stay None (set so by __init__, as the FP branches leave them)
            q._buffers.update(scales=plan.scales[i].view(-1, 1),
                              zeros=plan.zeros[i].view(-1, 1) if plan.zeros[i] is not None else None)
            q.quantized.fill_(True)
            if apx:
                q.__dict__["approximate"] = True
            _set_module(model, n, q)
            done.add(n)

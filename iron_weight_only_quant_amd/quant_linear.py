"""Drop-in for the reference's QuantLinear (quant_linear.py:395-1033), INT weight format.

Same constructor signature, buffers (quantized / scales / zeros / weight_fp4/6/8 / weight_bfp_*),
`quantize_weight()`, `forward()` and `from_linear()` semantics:
  * `from_linear` aliases the original Linear's weight storage and overwrites it in place with the
    dequantized weight (:1021-1024, :949), scales/zeros become [G,1] buffers of the weight dtype
    (:924-932), w_bit >= 16 leaves the layer unquantized (:887-892).
  * Errors: ValueError for an unknown weight_format (:440-441) or group size (:906),
    AssertionError when the grouped dimension does not divide (:897).
Differences by design (documented in DESIGN.md):
  * the throw-away kaiming init of a fresh [out,in] weight that from_linear immediately replaces
    (:444, :464; 75 % of the reference's from_linear time) is skipped on that path;
  * quantization runs in the gfx950 kernels (no CPU path);
  * `keep_codes=True` additionally keeps the packed integer codes (`qweight`, include/iwq.h layout)
    for the fused dequant->GEMM forward.
FP4/FP6/FP8 (quant_linear.py:724-883) run the gfx950 FP codec on fp16, bf16 and fp32 weights (every
op in the weight's dtype, fp16 scales / zeros like the reference's .half() buffers), with the formats
set by the same module-level `configure_fp_formats` (:84-110).  The research formats run on the GPU
too, on fp16 / bf16 / fp32 weights: `approximate=True` (+ `double_approximate`) =
quantize_weight_approximate (:470-632) and weight_format "bfp" = the block-floating-point branch
(:648-723).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels

_FORMATS = {"int", "fp4", "fp6", "fp8", "bfp"}

# FP format configuration, module globals exactly like the reference (quant_linear.py:7-16, :84-110)
FP4_EXP_BITS = 2
FP4_MANTISSA_BITS = 1
FP4_EXP_BIAS = 2 ** (FP4_EXP_BITS - 1) - 1
FP6_EXP_BITS = 3
FP6_MANTISSA_BITS = 2
FP6_EXP_BIAS = 2 ** (FP6_EXP_BITS - 1) - 1
FP8_EXP_BITS = 4
FP8_MANTISSA_BITS = 3
FP8_EXP_BIAS = 2 ** (FP8_EXP_BITS - 1) - 1


def configure_fp_formats(fp4_exp_bits: int = 2, fp4_mantissa_bits: int = 1, fp6_exp_bits: int = 3,
                         fp6_mantissa_bits: int = 2, fp8_exp_bits: int = 4, fp8_mantissa_bits: int = 3):
    """quant_linear.py:84-110: set exponent/mantissa widths of FP4/FP6/FP8 (bias follows)."""
    global FP4_EXP_BITS, FP4_MANTISSA_BITS, FP4_EXP_BIAS, FP6_EXP_BITS, FP6_MANTISSA_BITS, FP6_EXP_BIAS
    global FP8_EXP_BITS, FP8_MANTISSA_BITS, FP8_EXP_BIAS
    FP4_EXP_BITS, FP4_MANTISSA_BITS = int(fp4_exp_bits), int(fp4_mantissa_bits)
    FP4_EXP_BIAS = 2 ** (FP4_EXP_BITS - 1) - 1
    FP6_EXP_BITS, FP6_MANTISSA_BITS = int(fp6_exp_bits), int(fp6_mantissa_bits)
    FP6_EXP_BIAS = 2 ** (FP6_EXP_BITS - 1) - 1
    FP8_EXP_BITS, FP8_MANTISSA_BITS = int(fp8_exp_bits), int(fp8_mantissa_bits)
    FP8_EXP_BIAS = 2 ** (FP8_EXP_BITS - 1) - 1


def _fp_bits(fmt):
    return {"fp4": (FP4_EXP_BITS, FP4_MANTISSA_BITS), "fp6": (FP6_EXP_BITS, FP6_MANTISSA_BITS),
            "fp8": (FP8_EXP_BITS, FP8_MANTISSA_BITS)}[fmt]


class QuantLinear(nn.Module):
    def __init__(self, in_features, out_features, bias=True, w_bit=4, w_group_size=128, symmetric=True, mode=0,
                 weight_format: str = "int", approximate: bool = False, quant_dim: int = 0,
                 fp8_hi_align_start: int = 12, fp8_hi_align_exp_field: int = 15, fp8_tail_pad_bits: int = 1,
                 double_approximate: bool = False, fp6_hi_align_start: int = 4, fp6_hi_align_exp_field: int = 7,
                 fp6_tail_pad_bits: int = 2, fp4_hi_align_start: int = 1, fp4_hi_align_exp_field: int = 1,
                 fp4_tail_pad_bits: int = 0, *, keep_codes: bool = False, fused_forward: bool = False,
                 nib_prefill: bool = False, _init_weight: bool = True):
        super().__init__()
        raw_format = weight_format.lower()
        fmt = "bfp" if raw_format.startswith("bfp") else raw_format
        if fmt not in _FORMATS:
            raise ValueError(f"Unsupported weight_format: {weight_format}")
        # plain attributes straight into __dict__ (nn.Module.__setattr__'s checks cost ~2 us each and
        # quantize_model builds one module per Linear: 224 for a 7B, 560 for a 70B)
        self.__dict__.update(
            in_features=in_features, out_features=out_features, w_bit=w_bit, w_group_size=w_group_size,
            symmetric=symmetric, mode=mode, quant_dim=quant_dim, weight_format=fmt, approximate=approximate,
            double_approximate=double_approximate, fp8_hi_align_start=fp8_hi_align_start,
            fp8_hi_align_exp_field=fp8_hi_align_exp_field, fp8_tail_pad_bits=fp8_tail_pad_bits,
            fp6_hi_align_start=fp6_hi_align_start, fp6_hi_align_exp_field=fp6_hi_align_exp_field,
            fp6_tail_pad_bits=fp6_tail_pad_bits, fp4_hi_align_start=fp4_hi_align_start,
            fp4_hi_align_exp_field=fp4_hi_align_exp_field, fp4_tail_pad_bits=fp4_tail_pad_bits,
            fused_forward=fused_forward, keep_codes=keep_codes or bool(fused_forward), nib_prefill=nib_prefill)

        if _init_weight:
            self.weight = nn.Parameter(torch.Tensor(out_features, in_features))
            if bias:
                self.bias = nn.Parameter(torch.Tensor(out_features))
            else:
                self.register_parameter("bias", None)
        else:
            self._parameters.update(weight=None, bias=None)

        # the reference's buffers (quant_linear.py:451-458), registered without the per-name checks
        self._buffers.update(quantized=torch.tensor(False), scales=None, zeros=None, weight_fp4=None,
                             weight_fp6=None, weight_fp8=None, weight_bfp_mantissa=None,
                             weight_bfp_exponent=None, qweight=None, qweight_tiled=None,
                             qweight_nib=None, scales_gm=None, zeros_gm=None)
        # the packed codes are a derived cache of (weight, scales, zeros), not part of the reference's
        # state: kept out of state_dict (a strict load of a reference checkpoint must match), and
        # dropped whenever a state_dict is loaded so the forward never runs on stale codes
        self._non_persistent_buffers_set.update(("qweight", "qweight_tiled", "qweight_nib", "scales_gm", "zeros_gm"))
        self.register_load_state_dict_post_hook(QuantLinear._drop_codes_after_load)
        if _init_weight:
            self.reset_parameters()

    @staticmethod
    def _drop_codes_after_load(module, incompatible_keys):
        module._buffers.update(qweight=None, qweight_tiled=None, qweight_nib=None, scales_gm=None, zeros_gm=None)

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.weight, a=5 ** 0.5)
        if self.bias is not None:
            fan_in, _ = nn.init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / fan_in ** 0.5
            nn.init.uniform_(self.bias, -bound, bound)

    # ------------------------------------------------------------------------------------------
    def _scale_shape(self, G):
        return (G, 1)

    def quantize_weight(self):
        """quant_linear.py:635-958 — INT branch on the GPU; in-place on self.weight."""
        with torch.no_grad():
            if self.approximate:
                return self.quantize_weight_approximate()
            if self.weight_format == "bfp":
                return self._quantize_weight_bfp()
            if self.weight_format in ("fp4", "fp6", "fp8"):
                return self._quantize_weight_fp()
            if self.w_bit >= 16:
                self.quantized.fill_(False)
                self.weight_fp4 = None
                self.weight_fp6 = None
                self.weight_fp8 = None
                return
            if self.w_group_size not in (-1, -2) and not self.w_group_size > 0:
                raise ValueError("Invalid w_group_size")
            w = self.weight.data
            res = kernels.quantize_minmax(w, self.w_bit, self.w_group_size, bool(self.symmetric), self.quant_dim,
                                          out=w if w.stride(1) == 1 and w.stride(0) >= w.shape[1] else None,
                                          want_codes=self.keep_codes and self.w_bit <= 8)
            if self.w_group_size == -1:
                # per tensor (any dtype / quant_dim): an aborted one-pass hand-off (another kernel
                # holding CUs) wrote nothing; settle() re-runs it on the two-kernel form (the reference
                # never fails here) and raises if the outputs are still invalid
                res.settle()
            if res.out is not w:
                w.copy_(res.out)
            self._set_int_result(res.scales, res.zeros, res.codes)

    def _set_int_result(self, scales, zeros, codes):
        """Install the INT branch's buffers (quant_linear.py:924-932) -- scales / zeros [G, 1] -- plus,
        when the packed codes were kept, the derived layouts the fused forward reads.  Shared by
        quantize_weight and quantize_model's batched launch."""
        rows, cols = self.out_features, self.in_features
        tiled = None
        if (self.fused_forward == "auto" and codes is not None and self.quant_dim == 0
                and self.w_bit <= 4 and rows % 16 == 0 and cols % 128 == 0):
            # decode batches read the codes in the GEMV tile layout (1 KiB contiguous per load)
            tiled = kernels.tile_codes(codes, rows, cols)
        nib = None
        if (self.fused_forward is True and self.nib_prefill and codes is not None
                and self.quant_dim == 0
                and 2 <= self.w_bit <= 4 and rows % 256 == 0 and cols % 64 == 0
                and (self.w_group_size == -2 or (self.w_group_size > 0 and self.w_group_size % 64 == 0))):
            # opt-in: prefill batches (M >= 256) read a NIB-layout copy (9 instead of 12 dequant
            # VALU per 8 weights; +0.5-1.2 % per channel, +-0 g128 at M = 8192, for 0.5 B per
            # weight more device memory: DESIGN.md section 5)
            nib = kernels.nib_codes(codes, rows, cols)
        sgm = zgm = None
        if (self.fused_forward is True and codes is not None and self.quant_dim == 0
                and 2 <= self.w_bit <= 4 and rows % 256 == 0 and cols % 64 == 0
                and self.w_group_size > 0 and self.w_group_size % 64 == 0 and cols % self.w_group_size == 0):
            # prefill batches read group-major copies of the grouped parameters (4 B per group and
            # row; the kernel then stages a K-step's 256 of them as contiguous pieces, +1.5-5 % at
            # g128, M = 8192: DESIGN.md section 5)
            sgm, zgm = kernels.group_major_params(scales.reshape(-1), None if zeros is None else zeros.reshape(-1),
                                                  rows, cols, self.w_group_size)
        # registered buffers (see __init__), written without nn.Module.__setattr__'s per-name checks
        self._buffers.update(scales=scales.view(-1, 1),
                             zeros=zeros.view(-1, 1) if zeros is not None else None,
                             qweight=codes, qweight_tiled=tiled, qweight_nib=nib, scales_gm=sgm, zeros_gm=zgm,
                             weight_fp4=None, weight_fp6=None, weight_fp8=None)
        self.quantized.fill_(True)

    def quantize_weight_approximate(self):
        """quant_linear.py:470-632 on the GPU: symmetric absmax FP codes per group of w_group_size,
        decoded by the aligned (or, with double_approximate, the quad-wise double-approximate)
        decoder; weight <- RN16(decoded * scales) in place, scales [G,1] fp16, zeros None."""
        with torch.no_grad():
            if self.w_group_size <= 0:
                raise ValueError("approximate 仅支持分组量化，w_group_size 必须 > 0")
            fmt = self.weight_format
            if fmt not in ("fp4", "fp6", "fp8"):
                raise NotImplementedError("approximate 目前仅支持 fp4/fp6/fp8")
            e, m = _fp_bits(fmt)
            hs, hf, tp = (getattr(self, f"{fmt}_hi_align_start"), getattr(self, f"{fmt}_hi_align_exp_field"),
                          getattr(self, f"{fmt}_tail_pad_bits"))
            if fmt == "fp4" and e not in (1, 2):
                # the reference's fp4 branch only decodes E1 / E2 layouts; `decoded` stays unbound
                raise UnboundLocalError("cannot access local variable 'decoded' where it is not associated "
                                        "with a value")
            double = bool(self.double_approximate) and not (fmt == "fp4" and e == 1)
            w = self.weight.data
            res = kernels.quantize_fp_approx(w, e, m, self.w_group_size, self.quant_dim, hs, hf, tp, double,
                                             out=w if w.stride(1) == 1 and w.stride(0) >= w.shape[1] else None)
            if res.out is not w:
                w.copy_(res.out)
            self.scales = res.scales.view(-1, 1).half()
            self.zeros = None
            for other in ("fp4", "fp6", "fp8"):
                if other != fmt:
                    setattr(self, f"weight_{other}", None)
            self.quantized.fill_(True)
            self.approximate = True

    def _quantize_weight_bfp(self):
        """BFP branch (quant_linear.py:648-723) on the GPU, in place on self.weight."""
        if self.w_group_size <= 0:
            raise ValueError("BFP 仅支持分组量化，请将 w_group_size 设为正数")
        w = self.weight.data
        out = kernels.quantize_bfp(w, self.w_bit, self.w_group_size, self.quant_dim,
                                   out=w if w.stride(1) == 1 and w.stride(0) >= w.shape[1] else None)
        if out is not w:
            w.copy_(out)
        self.weight_bfp_mantissa = None
        self.weight_bfp_exponent = None
        self.scales = None
        self.zeros = None
        self.weight_fp4 = None
        self.weight_fp6 = None
        self.weight_fp8 = None
        self.quantized.fill_(True)

    def _quantize_weight_fp(self):
        """FP4/FP6/FP8 branches (quant_linear.py:724-883) on the GPU, in place on self.weight."""
        if self.w_group_size not in (-1, -2) and not self.w_group_size > 0:
            raise ValueError("Invalid w_group_size")
        e, m = _fp_bits(self.weight_format)
        w = self.weight.data
        res = kernels.quantize_fp(w, e, m, self.w_group_size, bool(self.symmetric), self.quant_dim,
                                  out=w if w.stride(1) == 1 and w.stride(0) >= w.shape[1] else None,
                                  want_codes=self.keep_codes)
        if res.out is not w:
            w.copy_(res.out)
        upd = dict(scales=res.scales.view(-1, 1), zeros=res.zeros.view(-1, 1) if res.zeros is not None else None,
                   qweight=res.codes)
        upd.update({f"weight_{o}": None for o in ("fp4", "fp6", "fp8") if o != self.weight_format})
        self._buffers.update(upd)  # registered buffers (see __init__)
        self.quantized.fill_(True)

    def forward(self, input):
        """quant_linear.py:960-972: the dequantized weight already sits in self.weight.

        With fused_forward=True (INT, 2-4 bits, quant_dim 0) the GEMM reads the packed codes instead
        (kernels.w4a16_gemm, MFMA): same weights, fp32 accumulation in a different order.
        fused_forward="auto" takes the packed-weight kernels only where they are the faster ones
        (kernels.auto_fused_preferred, device time, cold): decode batches (M <= 16 rows: the
        weight-streaming GEMV on the tile-layout codes, 1.5-3.6x hipBLASLt) and prompt-sized
        batches up to 192 rows per channel / 32 grouped (more on down-like K >= 2N weights); other
        batches run F.linear on the resident dequantized weight, like the reference."""
        if not self.quantized:
            return F.linear(input, self.weight, self.bias)
        fused = self.fused_forward
        if fused == "auto":
            m = input.numel() // max(1, self.in_features)
            fused = kernels.auto_fused_preferred(m, self.out_features, self.in_features, self.w_group_size)
            if fused and m <= kernels.GEMV_MAX_M and self.qweight_tiled is not None and self._fused_ok(input):
                return kernels.w4a16_gemm(input, self.qweight_tiled, self.scales.view(-1),
                                          None if self.zeros is None else self.zeros.view(-1), self.w_bit,
                                          self.w_group_size, self.out_features, self.bias, tiled=True)
        if fused and self.qweight is not None and self._fused_ok(input):
            if (self.qweight_nib is not None and input.numel() // self.in_features >= kernels.NIB_MIN_M
                    and kernels.nib_supported(input, self.out_features, self.in_features, self.w_bit,
                                              self.w_group_size)):
                return kernels.w4a16_gemm(input, self.qweight_nib, self.scales.view(-1),
                                          None if self.zeros is None else self.zeros.view(-1), self.w_bit,
                                          self.w_group_size, self.out_features, self.bias, nib=True,
                                          scales_gm=self.scales_gm, zeros_gm=self.zeros_gm)
            return kernels.w4a16_gemm(input, self.qweight, self.scales.view(-1),
                                      None if self.zeros is None else self.zeros.view(-1), self.w_bit,
                                      self.w_group_size, self.out_features, self.bias,
                                      scales_gm=self.scales_gm, zeros_gm=self.zeros_gm)
        original_input_shape = input.shape
        weight = self.weight.to(input.dtype)
        out = F.linear(input, weight, self.bias)
        if input.dim() > 2:
            out = out.reshape(original_input_shape[:-1] + (self.out_features,))
        return out

    def _fused_ok(self, input):
        """The packed-code kernels read fp16 codes' parameters and fp16 activations: any other
        storage dtype (bf16/fp32 weights -> bf16/fp32 scales) takes the reference's
        F.linear(input, weight.to(input.dtype)) path instead of misreading the parameter bits."""
        return (self.weight_format == "int" and self.quant_dim == 0
                and self.scales is not None and self.scales.dtype == torch.float16
                and (self.zeros is None or self.zeros.dtype == torch.float16)
                and (self.bias is None or self.bias.dtype == torch.float16)
                and kernels.w4a16_gemm_supported(input, self.out_features, self.in_features, self.w_bit,
                                                 self.w_group_size))

    @classmethod
    def from_linear(cls, linear_layer, w_bit=4, w_group_size=128, symmetric=False, mode=0,
                    weight_format: str = "int", approximate: bool = False, quant_dim: int = 0,
                    fp8_hi_align_start: int = 12, fp8_hi_align_exp_field: int = 15, fp8_tail_pad_bits: int = 1,
                    double_approximate: bool = False, fp6_hi_align_start: int = 4, fp6_hi_align_exp_field: int = 7,
                    fp6_tail_pad_bits: int = 2, fp4_hi_align_start: int = 1, fp4_hi_align_exp_field: int = 1,
                    fp4_tail_pad_bits: int = 0, *, keep_codes: bool = False, fused_forward: bool = False,
                    nib_prefill: bool = False, quantize: bool = True):
        """quant_linear.py:974-1033.  `quantize=False` is used by the batched model transform,
        which has already quantized the weight in one multi-tensor launch."""
        assert isinstance(linear_layer, nn.Linear), "Input layer must be nn.Linear"
        q = cls(in_features=linear_layer.in_features, out_features=linear_layer.out_features,
                bias=linear_layer.bias is not None, w_bit=w_bit, w_group_size=w_group_size, symmetric=symmetric,
                mode=mode, weight_format=weight_format, approximate=approximate, quant_dim=quant_dim,
                fp8_hi_align_start=fp8_hi_align_start, fp8_hi_align_exp_field=fp8_hi_align_exp_field,
                fp8_tail_pad_bits=fp8_tail_pad_bits, double_approximate=double_approximate,
                fp6_hi_align_start=fp6_hi_align_start, fp6_hi_align_exp_field=fp6_hi_align_exp_field,
                fp6_tail_pad_bits=fp6_tail_pad_bits, fp4_hi_align_start=fp4_hi_align_start,
                fp4_hi_align_exp_field=fp4_hi_align_exp_field, fp4_tail_pad_bits=fp4_tail_pad_bits,
                keep_codes=keep_codes, fused_forward=fused_forward, nib_prefill=nib_prefill, _init_weight=False)
        # aliases the original storage (quant_linear.py:1021-1024); straight into _parameters
        q._parameters["weight"] = nn.Parameter(linear_layer.weight.data.detach(), requires_grad=False)
        if linear_layer.bias is not None:
            q._parameters["bias"] = nn.Parameter(linear_layer.bias.data.detach(), requires_grad=False)
        if quantize:
            q.quantize_weight()
        return q


class GPTQQuantLinear(nn.Module):
    """quant_linear.py:1035-1065 — holder for externally quantized weights; forward = F.linear."""

    def __init__(self, weight: torch.Tensor, bias=None):
        super().__init__()
        assert weight.dim() == 2, "Weight tensor must be 2-dimensional"
        self.out_features, self.in_features = weight.shape
        self.weight = nn.Parameter(weight.clone().detach(), requires_grad=False)
        if bias is not None:
            self.bias = nn.Parameter(bias.clone().detach(), requires_grad=False)
        else:
            self.register_parameter("bias", None)

    def forward(self, input):
        return F.linear(input, self.weight, self.bias)

    @classmethod
    def from_linear(cls, linear_layer):
        assert isinstance(linear_layer, nn.Linear), "Input layer must be nn.Linear"
        layer = cls(linear_layer.weight.data, linear_layer.bias.data if linear_layer.bias is not None else None)
        if getattr(linear_layer, "scales", None) is not None:
            layer.scales = linear_layer.scales.clone().detach()
        if getattr(linear_layer, "zeros", None) is not None:
            layer.zeros = linear_layer.zeros.clone().detach()
        return layer

"""Packed checkpoint of a quantized model, and the packed-only layer.

The reference never saves a quantized model: quantize_model rewrites every Linear's weight in place
with its fake-quantized fp16 values (quant_wrapper.py:52-82, quant_linear.py:949) and main.py
evaluates it in the same process (SURVEY.md §5 "Checkpoint / resume": optional next).  Storing that
state as fp16 costs the full model size; the quantizer's packed codes (include/iwq.h layout) plus the
reference's scales / zeros hold the same information in ~0.27x (4-bit, g=128):

    save_packed(model, path)
        every INT QuantLinear quantized with its codes kept (keep_codes / fused_forward, or
        quantize_model(args.keep_codes=True)) -> "<layer>.qweight" (uint8 codes), "<layer>.scales",
        "<layer>.zeros" (asymmetric), "<layer>.bias"; every other tensor of model.state_dict() as is.
        One safetensors file; per-layer settings in its metadata (format "iwq-packed-v1").
    load_packed(model, path, device, packed=False)
        model: the same architecture (e.g. built from its config; on the meta device only if every
        tensor it needs is in the checkpoint -- no non-persistent buffers).  packed=False
        rebuilds each quantized layer as the QuantLinear quantize_model made -- weight restored by
        iwq_dequant_codes, bit-identical to the fake-quantized weight that was saved, scales / zeros
        [G, 1], codes kept -- so the loaded model computes exactly what the saved one did.
        packed=True installs PackedLinear layers instead (no fp16 weight held).

PackedLinear: a Linear held only as codes + scales (+ zeros).  Forward: INT 2-4 bit quant_dim 0
fp16 -> kernels.w4a16_linear (the weight-streaming GEMV / fused MFMA kernels, or dequant-once +
library GEMM at large M); any other mode dequantizes the weight (iwq_dequant_codes) into a transient
buffer for F.linear.  Results equal F.linear on the fake-quantized weight up to fp32 accumulation
order (the fused kernels) or exactly (the dequant path)."""
import json

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels
from .quant_linear import QuantLinear
from .quant_wrapper import _set_module

FORMAT = "iwq-packed-v1"
_LAYER_FIELDS = ("in_features", "out_features", "w_bit", "w_group_size", "symmetric", "quant_dim")


class PackedLinear(nn.Module):
    """y = x W_deq^T + b with W_deq held only as packed codes (include/iwq.h) + scales (+ zeros)."""

    def __init__(self, in_features, out_features, w_bit, w_group_size, symmetric, quant_dim, qweight, scales,
                 zeros=None, bias=None):
        super().__init__()
        self.in_features, self.out_features = int(in_features), int(out_features)
        self.w_bit, self.w_group_size = int(w_bit), int(w_group_size)
        self.symmetric, self.quant_dim = bool(symmetric), int(quant_dim)
        if not 1 <= self.w_bit <= 8:
            raise ValueError("PackedLinear: packed codes exist for 1 <= w_bit <= 8")
        _, G = kernels.group_geometry(self.out_features, self.in_features, self.w_group_size, self.quant_dim)
        if qweight.numel() != kernels.codes_nbytes(self.out_features, self.in_features, self.w_bit):
            raise ValueError("PackedLinear: qweight size does not match the layer shape")
        if scales.numel() != G or (not self.symmetric and (zeros is None or zeros.numel() != G)):
            raise ValueError(f"PackedLinear: scales / zeros must hold {G} values")
        self.register_buffer("qweight", qweight.reshape(-1).contiguous())
        self.register_buffer("scales", scales.reshape(-1, 1).contiguous())
        self.register_buffer("zeros", None if self.symmetric else zeros.reshape(-1, 1).contiguous())
        self.bias = nn.Parameter(bias, requires_grad=False) if bias is not None else None
        # the decode tile layout of qweight: a derived cache, so a non-persistent buffer (module.to()
        # moves it, state_dict keys stay qweight / scales / zeros / bias) dropped on every state-dict
        # load (the new codes are copied into qweight; a stale tile copy would serve M <= 16 batches)
        self.register_buffer("_tiled", None, persistent=False)
        self.register_load_state_dict_post_hook(PackedLinear._drop_tiles_after_load)

    @staticmethod
    def _drop_tiles_after_load(module, incompatible_keys):
        module._buffers["_tiled"] = None

    @classmethod
    def from_quant_linear(cls, q):
        if q.qweight is None or not bool(q.quantized) or q.weight_format != "int" or q.approximate:
            raise ValueError("PackedLinear needs an INT QuantLinear quantized with its codes kept "
                             "(keep_codes=True or fused_forward)")
        return cls(q.in_features, q.out_features, q.w_bit, q.w_group_size, q.symmetric, q.quant_dim, q.qweight,
                   q.scales, q.zeros, None if q.bias is None else q.bias.data)

    def dequantize(self):
        """The fake-quantized weight [out, in] (bit-identical to QuantLinear.weight after quantize)."""
        return kernels.dequant_codes(self.qweight, self.scales.view(-1),
                                     None if self.zeros is None else self.zeros.view(-1), self.w_bit,
                                     self.w_group_size, self.symmetric, self.quant_dim, self.out_features,
                                     self.in_features)

    def _fused_ok(self, x):
        return (self.quant_dim == 0 and 2 <= self.w_bit <= 4 and self.scales.dtype == torch.float16
                and (self.bias is None or self.bias.dtype == torch.float16)
                and kernels.w4a16_gemm_supported(x, self.out_features, self.in_features, self.w_bit,
                                                 self.w_group_size))

    def forward(self, x):
        if self._fused_ok(x):
            m = x.numel() // self.in_features
            if (self._tiled is None and m <= kernels.GEMV_MAX_M and self.out_features % 16 == 0
                    and self.in_features % 128 == 0):
                self._buffers["_tiled"] = kernels.tile_codes(self.qweight, self.out_features, self.in_features)
            return kernels.w4a16_linear(x, self.qweight, self.scales.view(-1),
                                        None if self.zeros is None else self.zeros.view(-1), self.w_bit,
                                        self.w_group_size, self.out_features,
                                        None if self.bias is None else self.bias.data, tiled_codes=self._tiled)
        w = self.dequantize()
        return F.linear(x, w.to(x.dtype), None if self.bias is None else self.bias.to(x.dtype))

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, w_bit={self.w_bit}, "
                f"w_group_size={self.w_group_size}, symmetric={self.symmetric}, quant_dim={self.quant_dim}")


def _packed_layers(model):
    """name -> (settings, qweight, scales [G], zeros [G] or None, bias or None) of every layer that
    is saved packed; raises for an INT QuantLinear whose codes were not kept."""
    out = {}
    for name, m in model.named_modules():
        if isinstance(m, PackedLinear):
            out[name] = ({f: getattr(m, f) for f in _LAYER_FIELDS}, m.qweight, m.scales.view(-1),
                         None if m.zeros is None else m.zeros.view(-1), None if m.bias is None else m.bias.data)
        elif isinstance(m, QuantLinear) and bool(m.quantized) and m.weight_format == "int" and not m.approximate:
            if m.qweight is None:
                raise ValueError(f"save_packed: layer '{name}' was quantized without its codes; quantize with "
                                 f"keep_codes=True (or args.keep_codes / fused_forward) to save it packed")
            out[name] = ({f: getattr(m, f) for f in _LAYER_FIELDS}, m.qweight, m.scales.view(-1),
                         None if m.zeros is None else m.zeros.view(-1), None if m.bias is None else m.bias.data)
    return out


def _under(key, prefixes):
    return any(key.startswith(p) for p in prefixes)


def save_packed(model, path, metadata=None):
    """Write `model` (after quantize_model / QuantLinear with codes kept) as one safetensors file."""
    from safetensors.torch import save_file
    layers = _packed_layers(model)
    tensors, meta_layers = {}, {}
    for name, (cfg, qw, sc, zr, b) in layers.items():
        cfg = dict(cfg, symmetric=bool(cfg["symmetric"]), dtype=str(sc.dtype).replace("torch.", ""))
        meta_layers[name] = cfg
        tensors[f"{name}.qweight"] = qw.detach().reshape(-1).contiguous().cpu()
        tensors[f"{name}.scales"] = sc.detach().contiguous().cpu()
        if zr is not None:
            tensors[f"{name}.zeros"] = zr.detach().contiguous().cpu()
        if b is not None:
            tensors[f"{name}.bias"] = b.detach().contiguous().cpu()
    prefixes = tuple(n + "." for n in layers)
    aliases, seen = {}, {}
    for k, v in model.state_dict(keep_vars=False).items():
        if _under(k, prefixes) or v is None:
            continue
        ident = (v.data_ptr(), v.dtype, tuple(v.shape), tuple(v.stride()), str(v.device)) if v.numel() else None
        if ident is not None and ident in seen:  # tied weights: stored once, the other key an alias
            aliases[k] = seen[ident]
            continue
        if ident is not None:
            seen[ident] = k
        tensors[k] = v.detach().contiguous().cpu().clone()
    meta = {"format": FORMAT, "layers": json.dumps(meta_layers, sort_keys=True), "aliases": json.dumps(aliases)}
    if metadata:
        meta.update({str(k): str(v) for k, v in metadata.items()})
    save_file(tensors, str(path), metadata=meta)
    return path


def _owner(model, key):
    mod_name, _, attr = key.rpartition(".")
    return (model.get_submodule(mod_name) if mod_name else model), attr


def _retie(model, key, src):
    (dst_mod, dst_attr), (src_mod, src_attr) = _owner(model, key), _owner(model, src)
    if src_attr in src_mod._parameters and dst_attr in dst_mod._parameters:
        dst_mod._parameters[dst_attr] = src_mod._parameters[src_attr]
    elif src_attr in src_mod._buffers and dst_attr in dst_mod._buffers:
        dst_mod._buffers[dst_attr] = src_mod._buffers[src_attr]


def read_packed_metadata(path):
    from safetensors import safe_open
    with safe_open(str(path), framework="pt") as f:
        meta = f.metadata() or {}
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not an {FORMAT} checkpoint (format {meta.get('format')!r})")
    return json.loads(meta["layers"]), json.loads(meta.get("aliases", "{}")), meta


def load_packed(model, path, device="cuda", packed=False, fused_forward=False, strict=True):
    """Load a save_packed checkpoint into `model` (same architecture; may live on the meta device).
    Quantized layers are replaced (QuantLinear with the restored fake-quant weight, or PackedLinear
    when packed=True); every other tensor is assigned from the file on `device`."""
    from safetensors import safe_open
    layers, aliases, _ = read_packed_metadata(path)
    device = torch.device(device)
    modules = dict(model.named_modules())
    prefixes = tuple(n + "." for n in layers)
    with safe_open(str(path), framework="pt", device="cpu") as f:
        keys = set(f.keys())
        # the plain tensors first: QuantLinear drops its codes after any load_state_dict (a stale-code
        # guard), so the quantized layers are installed after this load
        rest = {k: f.get_tensor(k).to(device) for k in keys if not _under(k, prefixes)}
        for k, src in aliases.items():
            rest[k] = rest[src]
        res = model.load_state_dict(rest, strict=False, assign=True)
        if strict:
            missing = [k for k in res.missing_keys if not _under(k, prefixes)]
            if missing or res.unexpected_keys:
                raise RuntimeError(f"load_packed: missing keys {missing[:8]}, unexpected keys "
                                   f"{res.unexpected_keys[:8]}")
        del rest
        # assign=True wraps every key in its own Parameter: re-tie the aliases to their source object
        for k, src in aliases.items():
            _retie(model, k, src)

        def get(k):
            return f.get_tensor(k).to(device) if k in keys else None
        for name, cfg in layers.items():
            old = modules.get(name)
            if old is None:
                raise KeyError(f"load_packed: the model has no module '{name}'")
            if (getattr(old, "in_features", None), getattr(old, "out_features", None)) != (
                    cfg["in_features"], cfg["out_features"]):
                raise ValueError(f"load_packed: '{name}' is {getattr(old, 'out_features', None)}x"
                                 f"{getattr(old, 'in_features', None)}, the checkpoint holds "
                                 f"{cfg['out_features']}x{cfg['in_features']}")
            qw, sc, zr, b = get(f"{name}.qweight"), get(f"{name}.scales"), get(f"{name}.zeros"), get(f"{name}.bias")
            if packed:
                new = PackedLinear(cfg["in_features"], cfg["out_features"], cfg["w_bit"], cfg["w_group_size"],
                                   cfg["symmetric"], cfg["quant_dim"], qw, sc, zr, b)
            else:
                w = kernels.dequant_codes(qw, sc, zr, cfg["w_bit"], cfg["w_group_size"], cfg["symmetric"],
                                          cfg["quant_dim"], cfg["out_features"], cfg["in_features"])
                new = QuantLinear(cfg["in_features"], cfg["out_features"], bias=b is not None, w_bit=cfg["w_bit"],
                                  w_group_size=cfg["w_group_size"], symmetric=cfg["symmetric"],
                                  quant_dim=cfg["quant_dim"], keep_codes=True, fused_forward=fused_forward,
                                  _init_weight=False)
                new._parameters.update(weight=nn.Parameter(w, requires_grad=False),
                                       bias=nn.Parameter(b, requires_grad=False) if b is not None else None)
                new.quantized = new.quantized.to(device)
                new._set_int_result(sc, zr, qw)
            _set_module(model, name, new)
    left = [n for n, t in list(model.named_parameters()) + list(model.named_buffers()) if t is not None and t.is_meta]
    if left:
        raise RuntimeError(f"load_packed: {len(left)} tensors are still on the meta device (not in the checkpoint, "
                           f"e.g. non-persistent buffers: {left[:4]}); build the skeleton on the target device")
    return model

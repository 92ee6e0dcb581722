"""Fused decode projections: one packed-weight GEMV for sibling Linear layers that read the same input.

A decoder layer reads its attention input three times (q_proj, k_proj, v_proj) and its MLP input
twice (gate_proj, up_proj).  At decode batch sizes the packed GEMV is bound by the weight bytes plus
a per-launch ramp; one launch over the row-concatenated weight ([Nq + Nk + Nv, K]) streams the same
bytes with one ramp: Llama-2-7B q/k/v at M = 1 8.3 us instead of 3 x 5.2, gate+up 12.0 instead of
2 x 8.1 (profiles/r03_ab_auto_graph.jsonl, qkv_proj / gate_up_proj rows; device time, cold).

fuse_projections(model) finds every module holding all members of a group (default
("q_proj", "k_proj", "v_proj") and ("gate_proj", "up_proj"), the Llama / Mistral / Qwen2 names) whose
members are INT QuantLinear / PackedLinear layers with kept 2-4 bit codes, quant_dim 0, fp16 and one
(w_bit, group, symmetric) setting, registers one shared FusedProjection on that module (its buffers
are not persistent: state_dict keys are unchanged) and routes each member's forward through it.  The
members stay in place (same module objects, same parameters); unfuse_projections(model) restores
their own forward.  The reference has no such layer (its forward is one F.linear per Linear,
quant_linear.py:960-972); numerics are the packed GEMV's (fp32 accumulation, one rounding per
output), the same as each member's own fused_forward path.

Call protocol: the first member called with an input computes the whole concatenated output for that
input and keeps it; the other members called with the SAME tensor object (same storage version)
take their column slice of it.  Any other input, or a batch above the decode GEMV's rows, makes a
member run its own module's forward -- so a caller that does not follow the q, k, v order still gets
exact per-layer results.

Staleness: the concatenated copies are derived from the members' codes / scales / zeros / bias.
Every new input first compares the members' current tensors (object and in-place version) with the
ones the copies were built from; after a load_state_dict (QuantLinear drops its codes, PackedLinear
copies new ones in place) or a re-quantization the group is rebuilt from the members' new state, or
-- if a member can no longer take part -- retired, and every member runs its own forward.
"""
import torch
import torch.nn as nn

from . import kernels
from .checkpoint import PackedLinear
from .quant_linear import QuantLinear

DEFAULT_GROUPS = (("q_proj", "k_proj", "v_proj"), ("gate_proj", "up_proj"))


def _packed_view(m):
    """(codes [N*K/2] row-major, scales [G], zeros [G] or None, bias or None, w_bit, group, symmetric)
    of a member, or None if it cannot take part."""
    if isinstance(m, PackedLinear):
        codes, sc, zr = m.qweight, m.scales.view(-1), None if m.zeros is None else m.zeros.view(-1)
        bias = None if m.bias is None else m.bias.data
    elif (isinstance(m, QuantLinear) and bool(m.quantized) and m.weight_format == "int" and not m.approximate
          and m.qweight is not None):
        codes, sc, zr = m.qweight, m.scales.view(-1), None if m.zeros is None else m.zeros.view(-1)
        bias = None if m.bias is None else m.bias.data
    else:
        return None
    if not (2 <= m.w_bit <= 4 and m.quant_dim == 0 and sc.dtype == torch.float16 and codes.is_cuda
            and m.out_features % 16 == 0 and m.in_features % 128 == 0
            and (bias is None or bias.dtype == torch.float16)):
        return None
    return codes, sc, zr, bias, m.w_bit, m.w_group_size, bool(m.symmetric)


def _version(t):
    try:
        return t._version
    except RuntimeError:  # inference-mode tensors keep no version counter
        return -1


def _member_state(m):
    """Identity of the member tensors the fused copies are built from: (object, in-place version)."""
    ts = (m._buffers.get("qweight"), m._buffers.get("scales"), m._buffers.get("zeros"), m._parameters.get("bias"))
    return tuple(None if t is None else (id(t), _version(t), t.data_ptr()) for t in ts)


class FusedProjection(nn.Module):
    """Row-concatenated packed codes (decode tile layout) + parameters of sibling projections."""

    def __init__(self, members):
        super().__init__()
        # the members are not submodules of this one (they stay where the model holds them)
        self.__dict__["_members"] = list(members)
        self._dead = False
        self._build()
        self._key = None
        self._out = None

    def _build(self):
        members = self._members
        views = [_packed_view(m) for m in members]
        if any(v is None for v in views):
            raise ValueError("FusedProjection: every member must be an INT 2-4 bit quant_dim-0 fp16 layer with codes")
        cfg = {(v[4], v[5], v[6]) for v in views}
        ks = {m.in_features for m in members}
        if len(cfg) != 1 or len(ks) != 1:
            raise ValueError("FusedProjection: members differ in (w_bit, group, symmetric) or in_features")
        (self.w_bit, self.w_group_size, self.symmetric), = cfg
        self.in_features = ks.pop()
        self.sizes = [m.out_features for m in members]
        self.out_features = sum(self.sizes)
        codes = torch.cat([v[0].view(-1) for v in views])
        # derived copies of the members' state: not persistent (state_dict keys stay the model's own)
        self.register_buffer("qweight_tiled", kernels.tile_codes(codes, self.out_features, self.in_features),
                             persistent=False)
        self.register_buffer("scales", torch.cat([v[1] for v in views]), persistent=False)
        self.register_buffer("zeros", None if self.symmetric else torch.cat([v[2] for v in views]),
                             persistent=False)
        bias = None
        if any(v[3] is not None for v in views):
            bias = torch.cat([v[3] if v[3] is not None else torch.zeros(n, dtype=torch.float16, device=codes.device)
                              for v, n in zip(views, self.sizes)])
        self.register_buffer("bias", bias, persistent=False)
        self._state = [_member_state(m) for m in members]

    def _refresh(self):
        """Rebuild from the members' current state if it changed since the copies were made; False
        (and retired for good) if a member can no longer take part."""
        if self._dead:
            return False
        if [_member_state(m) for m in self._members] == self._state:
            return True
        try:
            self._build()
            return True
        except ValueError:
            self._dead = True
            self.qweight_tiled = self.scales = self.zeros = self.bias = None
            return False

    def usable(self, x):
        return (not self._dead and x.dtype == torch.float16 and x.shape[-1] == self.in_features
                and x.numel() // self.in_features <= kernels.GEMV_MAX_M
                and kernels.w4a16_gemm_supported(x, self.out_features, self.in_features, self.w_bit,
                                                 self.w_group_size))

    def output_for(self, x):
        """The concatenated [.., sum N] output for x, computed once per (tensor, storage version)."""
        key = (id(x), _version(x), x.data_ptr())
        if self._key != key or self._out is None:
            if not self._refresh():
                return None
            self._out = kernels.w4a16_gemm(x, self.qweight_tiled, self.scales, self.zeros, self.w_bit,
                                           self.w_group_size, self.out_features, self.bias, tiled=True)
            self._key = key
            self._x = x  # keeps id(x) from being reused while the key is live
        return self._out

    def release(self):
        self._key = self._out = None
        self._x = None


def _member_forward(member, fused, index):
    """The member's forward while fused: its columns of the shared decode GEMV, else its own."""
    own = type(member).forward.__get__(member)
    lo = sum(fused.sizes[:index])
    hi = lo + fused.sizes[index]
    last = index == len(fused.sizes) - 1

    def forward(x):
        if fused.usable(x):
            full = fused.output_for(x)
            if full is not None:  # None: the group was retired (a member changed; see _refresh)
                y = full[..., lo:hi]
                if last:
                    fused.release()  # the last member: drop the cached output
                return y
        return own(x)
    return forward


def fuse_projections(model, groups=DEFAULT_GROUPS, drop_member_tiles=True):
    """Install a FusedProjection for every eligible group; returns the number of groups fused.
    drop_member_tiles: the members' own decode tile copies (QuantLinear.qweight_tiled) are no longer
    read at M <= 16 -- free them (their row-major codes stay for larger batches)."""
    n = 0
    for parent in list(model.modules()):
        for names in groups:
            members = [getattr(parent, nm, None) for nm in names]
            if any(m is None for m in members) or any("_iwq_fused" in m.__dict__ for m in members):
                continue
            try:
                fused = FusedProjection(members)
            except ValueError:
                continue
            parent.add_module("iwq_fused_" + "_".join(nm.split("_")[0] for nm in names), fused)
            for j, m in enumerate(members):
                if drop_member_tiles and isinstance(m, QuantLinear):
                    m._buffers["qweight_tiled"] = None
                m.__dict__["_iwq_fused"] = (fused, j)
                m.__dict__["forward"] = _member_forward(m, fused, j)
            n += 1
    return n


def unfuse_projections(model):
    """Undo fuse_projections: members run their own forward again (their tile copies, if dropped,
    are rebuilt for QuantLinear(fused_forward="auto"))."""
    for parent in list(model.modules()):
        for name, child in list(parent._modules.items()):
            if isinstance(child, FusedProjection):
                del parent._modules[name]
        for m in parent.children():
            if "_iwq_fused" in m.__dict__:
                del m.__dict__["_iwq_fused"]
                del m.__dict__["forward"]
                if (isinstance(m, QuantLinear) and m.fused_forward == "auto" and m.qweight is not None
                        and m.qweight_tiled is None and m.w_bit <= 4 and m.quant_dim == 0
                        and m.out_features % 16 == 0 and m.in_features % 128 == 0):
                    m._buffers["qweight_tiled"] = kernels.tile_codes(m.qweight, m.out_features, m.in_features)

"""Fused decode projections (fused_proj.py) on a Llama-shaped model: one packed GEMV per (q, k, v) and
(gate, up) group at decode batch sizes, the members' own forward above; logits against the unfused
model, launch counts, state_dict keys unchanged, unfuse restores."""
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _model(group=128, seed=0):
    from transformers import LlamaConfig, LlamaForCausalLM

    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=512, max_position_embeddings=128)
    torch.manual_seed(seed)
    m = LlamaForCausalLM(cfg).half().to(DEV).eval()
    quantize_model(m, SimpleNamespace(w_bit=4, a_bit=16, w_group_size=group, w_symmetric=False, w_format="int",
                                      quant_dim=0, fused_forward="auto"), verbose=False)
    return cfg, m


@pytest.mark.parametrize("group", [128, -2])
def test_fused_projections_match_unfused(group, monkeypatch):
    from iron_weight_only_quant_amd import kernels
    from iron_weight_only_quant_amd.fused_proj import FusedProjection, fuse_projections, unfuse_projections
    cfg, m = _model(group)
    keys = list(m.state_dict())
    g = torch.Generator(DEV).manual_seed(3)
    decode = [torch.randint(0, cfg.vocab_size, (b, 1), device=DEV, generator=g) for b in (1, 4, 16)]
    prefill = torch.randint(0, cfg.vocab_size, (2, 24), device=DEV, generator=g)
    with torch.no_grad():
        ref = [m(ids).logits for ids in decode + [prefill]]
    assert fuse_projections(m) == 4  # (q, k, v) and (gate, up) in each of 2 layers
    assert sum(isinstance(x, FusedProjection) for x in m.modules()) == 4
    assert list(m.state_dict()) == keys  # derived buffers are not persistent
    calls = []
    real = kernels.w4a16_gemm
    monkeypatch.setattr(kernels, "w4a16_gemm", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        for ids, r in zip(decode, ref):
            calls.clear()
            got = m(ids).logits
            assert len(calls) == 2 * 4  # per layer: qkv, o, gate_up, down (was 7)
            torch.testing.assert_close(got.float(), r.float(), rtol=2e-2, atol=2e-2)
        got = m(prefill).logits  # M = 48 rows: every member runs its own forward, exactly as before
        assert torch.equal(got, ref[-1])
    unfuse_projections(m)
    assert not any(isinstance(x, FusedProjection) for x in m.modules())
    with torch.no_grad():
        calls.clear()
        assert torch.equal(m(decode[0]).logits, ref[0])
        assert len(calls) == 7 * 2


def test_fused_projection_cache_follows_the_input():
    """A member called with a different tensor (or after an in-place change) recomputes."""
    from iron_weight_only_quant_amd.fused_proj import fuse_projections
    _, m = _model()
    fuse_projections(m)
    attn = m.model.layers[0].self_attn
    x = torch.randn(1, 1, 256, device=DEV, dtype=torch.float16)
    y = torch.randn(1, 1, 256, device=DEV, dtype=torch.float16)
    with torch.no_grad():
        q_x = attn.q_proj(x)
        k_y = attn.k_proj(y)                      # not the cached input: k of y
        k_ref = type(attn.k_proj).forward(attn.k_proj, y)
        torch.testing.assert_close(k_y, k_ref, rtol=1e-2, atol=2e-3)
        attn.q_proj(x)
        x.mul_(2.0)                               # in place: the cached output is stale
        v_x = attn.v_proj(x)
        torch.testing.assert_close(v_x, type(attn.v_proj).forward(attn.v_proj, x), rtol=1e-2, atol=2e-3)
        assert q_x.shape[-1] == 256 and v_x.shape[-1] == 128


def test_fused_projections_on_packed_only_model(tmp_path):
    """A packed-only model (checkpoint.load_packed(packed=True): PackedLinear, no fp16 weights) fuses
    the same way; decode logits against the fp16-resident quantized model."""
    from transformers import LlamaForCausalLM

    from iron_weight_only_quant_amd.checkpoint import PackedLinear, load_packed, save_packed
    from iron_weight_only_quant_amd.fused_proj import fuse_projections
    cfg, m = _model()
    p = tmp_path / "m.safetensors"
    save_packed(m, p)
    with torch.device(DEV):
        pk = LlamaForCausalLM(cfg).half()
    load_packed(pk, p, device=DEV, packed=True)
    pk.eval()
    assert isinstance(pk.model.layers[0].self_attn.q_proj, PackedLinear)
    assert fuse_projections(pk) == 4
    ids = torch.randint(0, cfg.vocab_size, (3, 1), device=DEV, generator=torch.Generator(DEV).manual_seed(5))
    with torch.no_grad():
        torch.testing.assert_close(pk(ids).logits.float(), m(ids).logits.float(), rtol=2e-2, atol=2e-2)


def test_fused_projections_follow_state_dict_loads(tmp_path):
    """after fuse_projections, loading another state_dict (QuantLinear drops its codes,
    PackedLinear copies new codes in place) or re-quantizing a member must never leave decode batches
    on the old fused copies: the group is rebuilt from the members' new state or retired."""
    from transformers import LlamaForCausalLM

    from iron_weight_only_quant_amd.checkpoint import load_packed, save_packed
    from iron_weight_only_quant_amd.fused_proj import FusedProjection, fuse_projections
    cfg, m = _model()
    _, m2 = _model(seed=1)  # a second, different quantized model of the same shape
    ids = torch.randint(0, cfg.vocab_size, (2, 1), device=DEV, generator=torch.Generator(DEV).manual_seed(9))
    # fp16-resident QuantLinear: load m2's state (weights, scales, zeros; the codes are dropped)
    fuse_projections(m)
    with torch.no_grad():
        m(ids)
        m.load_state_dict(m2.state_dict())
        got = m(ids).logits
        ref = m2(ids).logits
    torch.testing.assert_close(got.float(), ref.float(), rtol=2e-2, atol=2e-2)
    assert all(f._dead for f in m.modules() if isinstance(f, FusedProjection))  # no codes left to fuse
    # re-quantizing a member (new codes): the group is rebuilt, not served stale
    _, m3 = _model()
    fuse_projections(m3)
    q = m3.model.layers[0].self_attn.q_proj
    with torch.no_grad():
        m3(ids)
        q.weight.data.mul_(-1.0)
        q.quantize_weight()
        x = torch.randn(1, 1, 256, device=DEV, dtype=torch.float16)
        y = q(x)
        y_own = type(q).forward(q, x)
    torch.testing.assert_close(y, y_own, rtol=1e-2, atol=2e-3)
    fp = [f for f in m3.model.layers[0].self_attn.modules() if isinstance(f, FusedProjection)]
    assert fp and not fp[0]._dead
    # packed-only model: load_state_dict copies new codes into the same buffers (in place)
    p1, p2 = tmp_path / "a.safetensors", tmp_path / "b.safetensors"
    _, ma = _model()
    save_packed(ma, p1)
    save_packed(m2, p2)
    with torch.device(DEV):
        pk, pk2 = LlamaForCausalLM(cfg).half(), LlamaForCausalLM(cfg).half()
    load_packed(pk, p1, device=DEV, packed=True)
    load_packed(pk2, p2, device=DEV, packed=True)
    pk.eval()
    pk2.eval()
    assert fuse_projections(pk) == 4
    with torch.no_grad():
        pk(ids)  # builds the members' and the groups' tile copies
        o_proj = pk.model.layers[0].self_attn.o_proj
        o_proj(torch.randn(1, 1, 256, device=DEV, dtype=torch.float16))  # PackedLinear's own decode tiles
        assert o_proj._tiled is not None
        pk.load_state_dict(pk2.state_dict())
        assert o_proj._tiled is None  # dropped on load
        torch.testing.assert_close(pk(ids).logits.float(), pk2(ids).logits.float(), rtol=2e-2, atol=2e-2)

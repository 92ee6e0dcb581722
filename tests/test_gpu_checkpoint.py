"""Packed codes -> weight (iwq_dequant_codes) for every INT mode, and the packed checkpoint round trip
(checkpoint.py) on a Llama-shaped model: bit-identical restored weights and logits, and the
packed-only layers' forward against F.linear on the fake-quantized weight."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import iwq_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
ORACLE_DT = {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}


def bits_equal(a, b):
    """Bit-exact equality of two float tensors (any device)."""
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    iv = torch.int16 if a.element_size() == 2 else torch.int32
    return torch.equal(a.contiguous().view(iv).cpu(), b.contiguous().view(iv).cpu())


def _np_bits(t):
    t = t.detach().contiguous().cpu()
    return t.view(torch.int16).numpy().view(np.uint16) if t.element_size() == 2 else t.view(torch.int32).numpy().view(np.uint32)


def _weight(rows, cols, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(rows, cols, generator=g) * 0.02
    w[0, : min(cols, 8)] = 0.0                    # a constant run (zero range)
    w[-1, -1] = 0.5                               # one outlier
    return w.to(dtype)


CASES = [  # rows, cols, bits, group, sym, quant_dim
    (128, 256, 4, 128, False, 0), (128, 256, 4, 128, True, 0), (96, 384, 3, 32, False, 0),
    (64, 512, 2, -2, False, 0), (64, 512, 8, -2, True, 0), (80, 256, 5, 64, False, 0),
    (64, 256, 4, -1, False, 0), (64, 256, 8, -1, True, 0), (256, 96, 4, 32, False, 1),
    (256, 128, 8, -2, False, 1), (192, 64, 4, -1, True, 1), (48, 36, 4, 12, False, 0),   # ragged: cols % 8
    (40, 20, 6, 20, False, 0), (30, 48, 1, 16, False, 0), (24, 72, 4, 24, True, 1),
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_dequant_codes_matches_quantizer_and_oracle(case, dtype):
    from iron_weight_only_quant_amd import kernels
    rows, cols, bits, group, sym, qd = case
    w = _weight(rows, cols, dtype, hash(case) & 0xFFFF)
    res = kernels.quantize_minmax(w.to(DEV), bits, group, sym, qd, want_codes=True)
    deq = kernels.dequant_codes(res.codes, res.scales, res.zeros, bits, group, sym, qd, rows, cols)
    assert bits_equal(deq, res.out), "codes -> weight differs from the quantizer's own dequant"
    # and from the oracle restatement of quant_linear.py:885-956 (codes through its own packer)
    wn = _np_bits(w) if dtype == torch.bfloat16 else w.numpy()
    r = O.quantlinear_int(wn, w_bit=bits, w_group_size=group, symmetric=sym, quant_dim=qd, dtype=ORACLE_DT[dtype])
    assert np.array_equal(res.codes.cpu().numpy().reshape(-1), O.pack_codes(r.codes, bits).reshape(-1))
    exp = np.ascontiguousarray(r.dequant)
    exp = exp.view(np.uint16) if exp.dtype.itemsize == 2 else exp.view(np.uint32)
    assert np.array_equal(_np_bits(deq), exp)


def test_dequant_codes_strided_out_and_errors():
    from iron_weight_only_quant_amd import kernels
    w = _weight(64, 256, torch.float16, 3).to(DEV)
    res = kernels.quantize_minmax(w, 4, 128, False, 0, want_codes=True)
    big = torch.full((64, 264), 7.0, dtype=torch.float16, device=DEV)
    out = big[:, 4:260]  # row stride 264, offset 8 bytes: not 16-B aligned
    kernels.dequant_codes(res.codes, res.scales, res.zeros, 4, 128, False, 0, 64, 256, out=out)
    assert bits_equal(out, res.out)
    assert (big[:, :4] == 7).all() and (big[:, 260:] == 7).all()  # nothing outside the view touched
    with pytest.raises(ValueError):
        kernels.dequant_codes(res.codes, res.scales, None, 4, 128, False, 0, 64, 256)  # asym without zeros
    with pytest.raises(ValueError):
        kernels.dequant_codes(res.codes[:-1], res.scales, res.zeros, 4, 128, False, 0, 64, 256)
    with pytest.raises(AssertionError):
        kernels.dequant_codes(res.codes, res.scales, res.zeros, 4, 96, False, 0, 64, 256)


def _tiny_llama():
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=4, vocab_size=512, max_position_embeddings=128)
    torch.manual_seed(0)
    return cfg, LlamaForCausalLM(cfg).half().to(DEV).eval()


def _args(**kw):
    base = dict(w_bit=4, a_bit=16, w_group_size=128, w_symmetric=False, w_format="int", quant_dim=0,
                keep_codes=True)
    base.update(kw)
    return SimpleNamespace(**base)


@pytest.mark.parametrize("kw", [dict(), dict(w_group_size=-2), dict(w_bit=8, w_group_size=-2, w_symmetric=True),
                                dict(quant_dim=1, w_group_size=64), dict(w_group_size=-1)],
                         ids=["g128", "perchannel", "w8sym", "qd1", "pertensor"])
def test_packed_checkpoint_round_trip(tmp_path, kw):
    from transformers import LlamaForCausalLM

    from iron_weight_only_quant_amd.checkpoint import PackedLinear, load_packed, save_packed
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    cfg, model = _tiny_llama()
    quantize_model(model, _args(**kw), verbose=False)
    ids = torch.randint(0, cfg.vocab_size, (2, 24), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
    with torch.no_grad():
        ref = model(ids).logits
    p = tmp_path / "llama_tiny.safetensors"
    save_packed(model, p)
    fp16_bytes = sum(t.numel() * t.element_size() for t in model.state_dict().values())
    import os
    assert os.path.getsize(p) < fp16_bytes  # the Linear weights shrink (embeddings stay fp16)

    with torch.device(DEV):  # rotary inv_freq is a non-persistent buffer: not in any checkpoint
        skel = LlamaForCausalLM(cfg).half()
    load_packed(skel, p, device=DEV)
    skel.eval()
    n = 0
    for name, m in model.named_modules():
        if isinstance(m, QuantLinear):
            q = skel.get_submodule(name)
            assert isinstance(q, QuantLinear) and bits_equal(q.weight, m.weight), name
            assert bits_equal(q.scales, m.scales) and torch.equal(q.qweight, m.qweight)
            n += 1
    assert n == 14  # 7 Linear layers per decoder block
    with torch.no_grad():
        assert torch.equal(skel(ids).logits, ref)

    with torch.device(DEV):
        skel2 = LlamaForCausalLM(cfg).half()
    load_packed(skel2, p, device=DEV, packed=True)
    skel2.eval()
    assert isinstance(skel2.model.layers[0].mlp.up_proj, PackedLinear)
    assert not any(k.endswith("proj.weight") for k in skel2.state_dict())
    x = torch.randn(5, 256, dtype=torch.float16, device=DEV)
    for name, m in model.named_modules():
        if isinstance(m, QuantLinear):
            pl = skel2.get_submodule(name)
            assert bits_equal(pl.dequantize(), m.weight), name
            y = pl(x if m.in_features == 256 else torch.randn(5, m.in_features, dtype=torch.float16, device=DEV))
            assert y.shape[-1] == m.out_features
    with torch.no_grad():
        got = skel2(ids).logits
    torch.testing.assert_close(got.float(), ref.float(), atol=2e-2, rtol=2e-2)

"""CPU checks of the packed checkpoint (checkpoint.py): file layout, metadata, tied tensors, the
packed-only layer's buffers, and the loud failures.  Codes / scales / zeros come from the oracle (the
checker; no kernel runs here).  GPU round trips: tests/test_gpu_checkpoint.py."""
import json

import numpy as np
import pytest
import torch
import torch.nn as nn

from iron_weight_only_quant_amd.checkpoint import FORMAT, PackedLinear, load_packed, read_packed_metadata, save_packed
from iron_weight_only_quant_amd.quant_linear import QuantLinear
from oracle import iwq_oracle as O


class Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        self.embed = nn.Embedding(32, 64)
        self.up = nn.Linear(64, 128, bias=False)
        self.down = nn.Linear(128, 64, bias=True)
        self.norm = nn.LayerNorm(64)
        self.lm_head = nn.Linear(64, 32, bias=False)
        self.lm_head.weight = self.embed.weight  # tied, as many HF models


def _oracle_quant_layer(lin, w_bit, group, sym, qd, seed):
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal(lin.weight.shape) * 0.02).astype(np.float16)
    r = O.quantlinear_int(w, w_bit=w_bit, w_group_size=group, symmetric=sym, quant_dim=qd)
    q = QuantLinear.from_linear(lin, w_bit=w_bit, w_group_size=group, symmetric=sym, quant_dim=qd, quantize=False,
                                keep_codes=True)
    q.weight.data = torch.from_numpy(r.dequant.view(np.float16).copy())
    codes = torch.from_numpy(O.pack_codes(r.codes, w_bit).reshape(-1).copy())
    zeros = None if r.zeros is None else torch.from_numpy(r.zeros.view(np.float16).reshape(-1).copy())
    q._set_int_result(torch.from_numpy(r.scales.view(np.float16).reshape(-1).copy()), zeros, codes)
    return q, r


def _quantized_tiny():
    torch.manual_seed(0)
    m = Tiny().half()
    up, r_up = _oracle_quant_layer(m.up, 4, 32, False, 0, 1)
    down, r_down = _oracle_quant_layer(m.down, 8, -2, True, 1, 2)
    m.up, m.down = up, down
    return m, r_up, r_down


def test_save_layout_and_metadata(tmp_path):
    from safetensors import safe_open
    m, r_up, r_down = _quantized_tiny()
    p = tmp_path / "tiny.safetensors"
    save_packed(m, p, metadata={"model": "tiny"})
    layers, aliases, meta = read_packed_metadata(p)
    assert meta["format"] == FORMAT and meta["model"] == "tiny"
    assert layers["up"] == dict(in_features=64, out_features=128, w_bit=4, w_group_size=32, symmetric=False,
                                quant_dim=0, dtype="float16")
    assert layers["down"]["quant_dim"] == 1 and layers["down"]["symmetric"] is True
    with safe_open(str(p), framework="pt") as f:
        keys = set(f.keys())
        assert f.get_tensor("up.qweight").dtype == torch.uint8 and f.get_tensor("up.qweight").numel() == 128 * 64 // 2
        assert f.get_tensor("down.qweight").numel() == 64 * 128  # 8-bit: one byte per code
        assert torch.equal(f.get_tensor("up.scales"), torch.from_numpy(r_up.scales.view(np.float16).reshape(-1)))
    # no fp16 weight of a packed layer, no zeros for the symmetric one, the tie stored once
    assert "up.weight" not in keys and "down.weight" not in keys and "down.zeros" not in keys
    assert "down.bias" in keys and "norm.weight" in keys
    assert len([k for k in ("embed.weight", "lm_head.weight") if k in keys]) == 1
    assert set(aliases.items()) == {("lm_head.weight", "embed.weight")}


def test_load_packed_only_layers_on_cpu(tmp_path):
    m, r_up, r_down = _quantized_tiny()
    p = tmp_path / "tiny.safetensors"
    save_packed(m, p)
    fresh = Tiny().half()
    load_packed(fresh, p, device="cpu", packed=True)
    assert isinstance(fresh.up, PackedLinear) and isinstance(fresh.down, PackedLinear)
    assert torch.equal(fresh.up.qweight, m.up.qweight) and torch.equal(fresh.up.scales, m.up.scales)
    assert torch.equal(fresh.up.zeros, m.up.zeros) and fresh.down.zeros is None
    assert torch.equal(fresh.down.bias, m.down.bias)
    assert torch.equal(fresh.norm.weight, m.norm.weight)
    assert fresh.lm_head.weight is fresh.embed.weight  # the tie survives
    assert torch.equal(fresh.embed.weight, m.embed.weight)
    # a second save of the packed-only model writes the same tensors
    p2 = tmp_path / "again.safetensors"
    save_packed(fresh, p2)
    assert read_packed_metadata(p2)[0] == read_packed_metadata(p)[0]


def test_meta_skeleton_and_packed_forward_needs_gpu(tmp_path):
    m, _, _ = _quantized_tiny()
    p = tmp_path / "tiny.safetensors"
    save_packed(m, p)
    with torch.device("meta"):
        skel = Tiny().half()
    load_packed(skel, p, device="cpu", packed=True)
    assert not any(t.is_meta for t in skel.state_dict().values())
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        skel.up(torch.zeros(2, 64, dtype=torch.float16))  # no CPU fallback


def test_loud_failures(tmp_path):
    torch.manual_seed(0)
    m = Tiny().half()
    q = QuantLinear.from_linear(m.up, w_bit=4, w_group_size=32, quantize=False)
    q.quantized.fill_(True)  # quantized without codes
    m.up = q
    with pytest.raises(ValueError, match="keep_codes"):
        save_packed(m, tmp_path / "x.safetensors")
    good, _, _ = _quantized_tiny()
    p = tmp_path / "tiny.safetensors"
    save_packed(good, p)
    with pytest.raises(RuntimeError, match="ROCm GPU"):  # the fp16 weight is restored by the HIP kernel
        load_packed(Tiny().half(), p, device="cpu", packed=False)

    class Other(Tiny):
        def __init__(self):
            super().__init__()
            self.up = nn.Linear(64, 96, bias=False)
    with pytest.raises(ValueError, match="checkpoint holds"):
        load_packed(Other().half(), p, device="cpu", packed=True)
    from safetensors.torch import save_file
    save_file({"a": torch.zeros(1)}, str(tmp_path / "plain.safetensors"), metadata={"format": "other"})
    with pytest.raises(ValueError, match="not an"):
        read_packed_metadata(tmp_path / "plain.safetensors")
    with pytest.raises(ValueError):
        PackedLinear(64, 128, 4, 32, False, 0, torch.zeros(10, dtype=torch.uint8), torch.zeros(256), torch.zeros(256))


def test_metadata_is_json(tmp_path):
    m, _, _ = _quantized_tiny()
    p = tmp_path / "tiny.safetensors"
    save_packed(m, p)
    from safetensors import safe_open
    with safe_open(str(p), framework="pt") as f:
        meta = f.metadata()
    assert json.loads(meta["layers"])["up"]["w_bit"] == 4

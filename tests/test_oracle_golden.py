"""Pin the CPU oracle (oracle/iwq_oracle.py) against golden vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only.

Bit-exact comparison of the dequantized weights, scales and zero-points, with
one documented relaxation: a stored zero-point whose value is zero is compared
by value (+0 == -0) only for groups that contain both +0 and -0 elements (ATen's
amin picks an order-dependent zero there; see oracle header)."""
import json
import os

import numpy as np
import pytest

from oracle import iwq_oracle as O
from oracle.synth import synth

from .golden_util import GOLD, bits_equal, load_small, load_edge, sha


def _mixed_zero_groups(x_groups):
    b = x_groups.view(np.uint16) if x_groups.dtype != np.float32 else x_groups.view(np.uint32)
    if x_groups.dtype == np.float32:
        pz = (b == 0).any(axis=1)
        nz = (b == 0x80000000).any(axis=1)
    else:
        pz = (b == 0).any(axis=1)
        nz = (b == 0x8000).any(axis=1)
    return pz & nz


def test_small_qf_all_modes():
    d = load_small()
    n = 0
    for key in d.files:
        if not key.startswith("qf/"):
            continue
        _, tag, dtype, bits, zp, g, pt = key.split("/")
        x = d[f"in/{tag}/{dtype}"]
        exp = d[key]
        kw = dict(n_bits=int(bits), zero_point=bool(int(zp)), q_group_size=int(g), per_tensor=bool(int(pt)))
        if exp.size == 0:
            with pytest.raises(AssertionError):
                O.pseudo_quantize_tensor(x, dtype=dtype, **kw)
            continue
        r = O.pseudo_quantize_tensor(x, dtype=dtype, **kw)
        assert bits_equal(r.dequant, exp), key
        n += 1
    assert n > 50


def test_small_ql_all_modes():
    d = load_small()
    n = 0
    for key in d.files:
        if not (key.startswith("ql/") and key.endswith("/deq")):
            continue
        _, tag, dtype, bits, sym, g, qd, _ = key.split("/")
        base = key[: -len("/deq")]
        x = d[f"in/{tag}/{dtype}"]
        r = O.quantlinear_int(x, w_bit=int(bits), w_group_size=int(g), symmetric=bool(int(sym)),
                              quant_dim=int(qd), dtype=dtype)
        assert bits_equal(r.dequant, d[key]), key
        assert bits_equal(r.scales, d[base + "/scales"]), key
        if base + "/zeros" in d.files:
            assert bits_equal(r.zeros, d[base + "/zeros"]), key
        else:
            assert r.zeros is None
        n += 1
    assert n > 50


def test_edge_rows():
    d = load_edge()
    e = d["in/edge"]
    fin = d["in/edge_finite_rows"]
    for bits in (2, 3, 4, 8):
        for zp in (True, False):
            exp = d[f"qf/edge/{bits}/{int(zp)}"]
            r = O.pseudo_quantize_tensor(e[fin], n_bits=bits, zero_point=zp, q_group_size=128)
            assert bits_equal(r.dequant, exp), (bits, zp)
            exp_all = d[f"qf/edge_all/{bits}/{int(zp)}"]
            if exp_all.size == 0:
                with pytest.raises(AssertionError):
                    O.pseudo_quantize_tensor(e, n_bits=bits, zero_point=zp, q_group_size=128)
            else:
                r = O.pseudo_quantize_tensor(e, n_bits=bits, zero_point=zp, q_group_size=128)
                assert bits_equal(r.dequant, exp_all)
            base = f"ql/edge_all/{bits}/{int(not zp)}"
            r = O.quantlinear_int(e, w_bit=bits, w_group_size=128, symmetric=not zp)
            assert bits_equal(r.dequant, d[base + "/deq"]), (bits, zp)
            assert bits_equal(r.scales, d[base + "/scales"]), (bits, zp)
            if zp:
                mixed = _mixed_zero_groups(e.reshape(-1, 128))
                zr, ze = r.zeros.reshape(-1), d[base + "/zeros"].reshape(-1)
                assert bits_equal(zr[~mixed], ze[~mixed])
                assert np.array_equal(zr[mixed].astype(np.float32), ze[mixed].astype(np.float32))


def test_nonfinite_inputs():
    d = load_edge()
    x = d["in/nonfinite"]
    for zp in (True, False):
        exp = d[f"qf/nonfinite/{int(zp)}"]
        assert exp.size == 0  # the reference asserts on the NaN it produces
        with pytest.raises(AssertionError):
            O.pseudo_quantize_tensor(x, n_bits=4, zero_point=zp, q_group_size=128)
        base = f"ql/nonfinite/{int(not zp)}"
        r = O.quantlinear_int(x, w_bit=4, w_group_size=128, symmetric=not zp)
        assert bits_equal(r.dequant, d[base + "/deq"], nan_equal=True)
        assert bits_equal(r.scales, d[base + "/scales"], nan_equal=True)


@pytest.mark.parametrize("case_idx", range(3))
def test_large_llama_shapes_sha(case_idx):
    """Full Llama-2-7B shapes through the oracle vs the reference's SHA-256 (CPU, a few seconds each)."""
    spec = json.load(open(os.path.join(GOLD, "int_large.json")))
    cases = [c for c in spec["cases"]]
    names = ["q_proj", "gate_proj", "down_proj"]
    name = names[case_idx]
    mine = [c for c in cases if c["name"] == name]
    inp = mine[0]
    x = synth(inp["seed"], tuple(inp["shape"]), "float16")
    assert sha(x) == inp["sha_input"]
    for c in mine[1:]:
        if c["kind"] == "qf":
            if c["n_bits"] != 4 or c["q_group_size"] != 128:
                continue
            r = O.pseudo_quantize_tensor(x, n_bits=4, zero_point=c["zero_point"], q_group_size=128)
            assert sha(r.dequant) == c["sha_deq"], c
        elif c["kind"] == "ql" and c["w_group_size"] == 128 and not c["symmetric"]:
            r = O.quantlinear_int(x, w_bit=4, w_group_size=128, symmetric=False)
            assert sha(r.dequant) == c["sha_deq"], c
            assert sha(r.scales) == c["sha_scales"], c
            assert sha(r.zeros) == c["sha_zeros"], c


def test_large_per_tensor_bf16_sha():
    """Per-tensor (-1) on a full 4096 x 4096 bf16 weight through the oracle vs the reference's SHA-256s
    (tests/golden/int_large_pt_dt.json, round 5: the fixtures the GPU one-pass bf16 / fp32 kernel is
    checked against)."""
    spec = json.load(open(os.path.join(GOLD, "int_large_pt_dt.json")))
    mine = [c for c in spec["cases"] if c["name"] == "q_proj" and c["dtype"] == "bfloat16"]
    inp = mine[0]
    x = synth(inp["seed"], tuple(inp["shape"]), "bfloat16")
    assert sha(x) == inp["sha_input"]
    for c in mine[1:]:
        if c["kind"] == "qf_pt":
            r = O.pseudo_quantize_tensor(x, n_bits=c["n_bits"], zero_point=c["zero_point"], q_group_size=-1,
                                         per_tensor=True, dtype="bfloat16")
            assert sha(r.dequant) == c["sha_deq"], c
        else:
            r = O.quantlinear_int(x, w_bit=c["w_bit"], w_group_size=-1, symmetric=c["symmetric"], dtype="bfloat16")
            assert sha(r.dequant) == c["sha_deq"], c
            assert sha(r.scales) == c["sha_scales"], c
            if c["sha_zeros"] is not None:
                assert sha(r.zeros) == c["sha_zeros"], c


def test_torch_restatement_matches_golden():
    """bench.py's CPU baseline (oracle/torch_ref.py) is pinned to the reference's outputs too."""
    import torch

    from oracle.torch_ref import minmax_fake_quant_cpu
    d = load_small()
    n = 0
    for key in d.files:
        if not (key.startswith("qf/") and "/float16/" in key):
            continue
        _, tag, dtype, bits, zp, g, pt = key.split("/")
        x = torch.from_numpy(d[f"in/{tag}/{dtype}"].copy())
        exp = d[key]
        if exp.size == 0:
            continue
        out = minmax_fake_quant_cpu(x, int(bits), bool(int(zp)), int(g), bool(int(pt)))
        assert bits_equal(out.numpy(), exp), key
        n += 1
    assert n > 30

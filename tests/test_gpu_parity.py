"""GPU parity: the gfx950 kernels (through the C-ABI) vs the golden fixtures the reference produced
and vs the CPU oracle.  Bit-exact for dequantized values, scales, zero-points and integer codes."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import iwq_oracle as O
from oracle.synth import synth

from .golden_util import GOLD, bits_equal, load_edge, load_small, sha

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
TD = {"float16": torch.float16, "bfloat16": torch.bfloat16, "float32": torch.float32}


def _ab_built():
    try:
        from iron_weight_only_quant_amd import _lib
        return _lib.ab_built()
    except OSError:
        return False


# The A/B kernel variants (flags bits 16..23 no default path takes) live in the IWQ_AB library only
# (IWQ_AB=1: iron_weight_only_quant_amd/build.py --ab, _lib/libiwq_ab.so); their bit-identity checks
# run there.  The product library refuses them (IWQ_ERR_ARG), tested below.
AB = _ab_built()
needs_ab = pytest.mark.skipif(not AB, reason="A/B kernel variants: IWQ_AB=1 library")


def abv(*vs):
    """The A/B variants vs, in an IWQ_AB build; none otherwise."""
    return tuple(vs) if AB else ()


def to_dev(a, dtype):
    a = np.ascontiguousarray(a)
    if dtype == "bfloat16":
        return torch.from_numpy(a.view(np.int16)).view(torch.bfloat16).to(DEV)
    return torch.from_numpy(a).to(DEV)


def to_np(t):
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


@pytest.fixture(scope="module")
def K():
    from iron_weight_only_quant_amd import kernels
    return kernels


def test_native_library_is_loaded(K):
    from iron_weight_only_quant_amd import _lib
    lib = _lib.load()
    assert os.path.exists(_lib.LIB_PATH)
    assert b"gfx950" in lib.iwq_build_info()


def test_product_library_refuses_ab_variants(K):
    """The product library answers an A/B variant with IWQ_ERR_ARG (no silent default); the pinned
    ones (gemm fallbacks 1 / 2 at M > 16, per-tensor 6 / 9) run."""
    if AB:
        pytest.skip("IWQ_AB library: every variant is built")
    from iron_weight_only_quant_amd import _lib as L
    w = torch.empty(256, 512, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 3)
    r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
    x = torch.randn(32, 512, device=DEV).half()
    for v in (3, 45, 74, 150, 162):
        with pytest.raises(L.IwqError) as e:
            K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, 256, flags=K.gemm_variant_flags(v))
        assert e.value.status == L.IWQ_ERR_ARG, v
    for v in (1, 2):
        K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, 256, flags=K.gemm_variant_flags(v))
    with pytest.raises(L.IwqError):
        K.quantize_minmax(w, 4, 128, False, 0, flags=K.gemm_variant_flags(3))
    for v in (6, 9):
        K.quantize_minmax(w, 4, -1, False, 0, flags=K.gemm_variant_flags(v)).settle()


def test_division_selftest(K):
    bad32, bad16, badrcp = K.selftest_division(DEV)
    assert badrcp == 0, badrcp
    assert bad16 == 0, bad16
    assert bad32 == 0, bad32


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
def test_synthetic_generator_matches_oracle(K, dtype):
    shape = (333, 1000)
    t = torch.empty(shape, dtype=TD[dtype], device=DEV)
    K.fill_synthetic(t, 11)
    exp = synth(11, shape, dtype)
    assert bits_equal(to_np(t), exp)


FLAG_SETS = [0, 1]  # 0: specialised kernels, 1: IWQ_FLAG_FORCE_GENERIC (universal path)


@pytest.mark.parametrize("flags", FLAG_SETS)
def test_golden_small_quant_funcs(K, flags):
    """Every pseudo_quantize_tensor case of the golden set; kernel called at C-ABI level."""
    d = load_small()
    n = 0
    for key in d.files:
        if not key.startswith("qf/"):
            continue
        _, tag, dtype, bits, zp, g, pt = key.split("/")
        exp = d[key]
        x = to_dev(d[f"in/{tag}/{dtype}"], dtype)
        g, pt = int(g), bool(int(pt))
        group = -1 if pt else (g if g > 0 else -2)
        res = K.quantize_minmax(x, int(bits), group, not bool(int(zp)), 0, flags=flags)
        if exp.size == 0:
            assert res.has_nan(), key
            continue
        assert not res.has_nan(), key
        assert bits_equal(to_np(res.out), exp), key
        n += 1
    assert n > 50


@pytest.mark.parametrize("flags", FLAG_SETS)
def test_golden_small_quantlinear(K, flags):
    d = load_small()
    n = 0
    for key in d.files:
        if not (key.startswith("ql/") and key.endswith("/deq")):
            continue
        _, tag, dtype, bits, sym, g, qd, _ = key.split("/")
        base = key[:-4]
        x = to_dev(d[f"in/{tag}/{dtype}"], dtype)
        res = K.quantize_minmax(x, int(bits), int(g), bool(int(sym)), int(qd), flags=flags)
        assert bits_equal(to_np(res.out), d[key]), key
        assert bits_equal(to_np(res.scales), d[base + "/scales"].reshape(-1)), key
        if base + "/zeros" in d.files:
            assert bits_equal(to_np(res.zeros), d[base + "/zeros"].reshape(-1)), key
        n += 1
    assert n > 50


def test_golden_small_python_face():
    """The drop-in Python API (quant_funcs / QuantLinear) reproduces the golden outputs."""
    from iron_weight_only_quant_amd.quant_funcs import pseudo_quantize_tensor
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    d = load_small()
    for key in d.files:
        if key.startswith("qf/") and "/float16/" in key:
            _, tag, dtype, bits, zp, g, pt = key.split("/")
            x = to_dev(d[f"in/{tag}/{dtype}"], dtype)
            kw = dict(n_bits=int(bits), zero_point=bool(int(zp)), q_group_size=int(g), per_tensor=bool(int(pt)))
            if d[key].size == 0:
                with pytest.raises(AssertionError):
                    pseudo_quantize_tensor(x, **kw)
                continue
            assert bits_equal(to_np(pseudo_quantize_tensor(x, **kw)), d[key]), key
            y = x.clone()
            r = pseudo_quantize_tensor(y, inplace=True, **kw)
            assert bits_equal(to_np(y), d[key]) and r.data_ptr() == y.data_ptr(), key
        if key.startswith("ql/") and key.endswith("/deq"):
            _, tag, dtype, bits, sym, g, qd, _ = key.split("/")
            base = key[:-4]
            x = to_dev(d[f"in/{tag}/{dtype}"], dtype)
            lin = torch.nn.Linear(x.shape[1], x.shape[0], bias=False).to(DEV)
            lin.weight.data = x
            q = QuantLinear.from_linear(lin, w_bit=int(bits), w_group_size=int(g), symmetric=bool(int(sym)),
                                        quant_dim=int(qd))
            assert q.weight.data.data_ptr() == x.data_ptr()  # aliases the Linear's storage
            assert bits_equal(to_np(x), d[key]), key
            assert bits_equal(to_np(q.scales), d[base + "/scales"]), key
            if base + "/zeros" in d.files:
                assert bits_equal(to_np(q.zeros), d[base + "/zeros"]), key
            else:
                assert q.zeros is None


@pytest.mark.parametrize("flags", FLAG_SETS)
def test_golden_edge_rows(K, flags):
    d = load_edge()
    e = d["in/edge"]
    fin = d["in/edge_finite_rows"]
    x_all = to_dev(e, "float16")
    x_fin = to_dev(e[fin], "float16")
    for bits in (2, 3, 4, 8):
        for zp in (True, False):
            r = K.quantize_minmax(x_fin, bits, 128, not zp, 0, flags=flags)
            assert not r.has_nan()
            assert bits_equal(to_np(r.out), d[f"qf/edge/{bits}/{int(zp)}"]), (bits, zp)
            r = K.quantize_minmax(x_all, bits, 128, not zp, 0, flags=flags)
            exp_all = d[f"qf/edge_all/{bits}/{int(zp)}"]
            assert r.has_nan() == (exp_all.size == 0)
            base = f"ql/edge_all/{bits}/{int(not zp)}"
            assert bits_equal(to_np(r.out), d[base + "/deq"], nan_equal=True), (bits, zp)
            assert bits_equal(to_np(r.scales), d[base + "/scales"].reshape(-1), nan_equal=True)
            if zp:
                zr = to_np(r.zeros)
                ze = d[base + "/zeros"].reshape(-1)
                ox = O.quantlinear_int(e, w_bit=bits, w_group_size=128, symmetric=False)
                assert bits_equal(zr, ox.zeros.reshape(-1), nan_equal=True)  # oracle's -0 < +0 convention
                assert np.array_equal(zr.astype(np.float32), ze.astype(np.float32), equal_nan=True)


@pytest.mark.parametrize("flags", FLAG_SETS)
def test_golden_nonfinite(K, flags):
    d = load_edge()
    x = to_dev(d["in/nonfinite"], "float16")
    for zp in (True, False):
        r = K.quantize_minmax(x, 4, 128, not zp, 0, flags=flags)
        assert r.has_nan()  # quant_funcs.py:40 would assert
        base = f"ql/nonfinite/{int(not zp)}"
        assert bits_equal(to_np(r.out), d[base + "/deq"], nan_equal=True)
        assert bits_equal(to_np(r.scales), d[base + "/scales"].reshape(-1), nan_equal=True)


def _large_cases():
    spec = json.load(open(os.path.join(GOLD, "int_large.json")))
    return spec["cases"]


@pytest.mark.parametrize("name", ["q_proj", "gate_proj", "down_proj"])
def test_llama_shapes_vs_reference_sha(K, name):
    """Full Llama-2-7B weight shapes: GPU-generated synthetic input -> kernels -> SHA-256 equal to
    the reference's own outputs on the same input (tests/golden/int_large.json)."""
    cases = [c for c in _large_cases() if c["name"] == name]
    inp = cases[0]
    x = torch.empty(tuple(inp["shape"]), dtype=torch.float16, device=DEV)
    K.fill_synthetic(x, inp["seed"])
    assert sha(to_np(x)) == inp["sha_input"]
    for c in cases[1:]:
        if c["kind"] == "qf":
            g = c["q_group_size"]
            r = K.quantize_minmax(x, c["n_bits"], g if g > 0 else -2, not c["zero_point"], 0)
            assert not r.has_nan()
            assert sha(to_np(r.out)) == c["sha_deq"], c
        else:
            r = K.quantize_minmax(x, c["w_bit"], c["w_group_size"], c["symmetric"], 0)
            assert sha(to_np(r.out)) == c["sha_deq"], c
            assert sha(to_np(r.scales).reshape(-1, 1)) == c["sha_scales"], c
            if c["sha_zeros"] is not None:
                assert sha(to_np(r.zeros).reshape(-1, 1)) == c["sha_zeros"], c


@pytest.mark.parametrize("bits", [2, 3, 4, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("mode", [(128, 0), (32, 0), (-2, 0), (-1, 0), (16, 1), (-2, 1)])
def test_codes_match_oracle(K, bits, sym, mode):
    g, qd = mode
    x_np = synth(21, (96, 512), "float16")
    x = to_dev(x_np, "float16")
    ref = O.quantlinear_int(x_np, w_bit=bits, w_group_size=g, symmetric=sym, quant_dim=qd)
    for flags in FLAG_SETS:
        r = K.quantize_minmax(x, bits, g, sym, qd, want_codes=True, flags=flags)
        assert bits_equal(to_np(r.out), ref.dequant)
        assert np.array_equal(r.codes.cpu().numpy(), O.pack_codes(ref.codes, bits).reshape(-1)), (flags,)


def test_batched_matches_single(K):
    shapes = [(256, 512), (128, 1024), (384, 256), (64, 2048), (8, 128)]
    ws = []
    for i, s in enumerate(shapes):
        t = torch.empty(s, dtype=torch.float16, device=DEV)
        K.fill_synthetic(t, 40 + i)
        ws.append(t)
    for sym in (False, True):
        plan = K.BatchPlan(ws, 4, 128, sym, want_codes=True)
        plan.run()
        torch.cuda.synchronize()
        assert plan.nan_flag.item() == 0
        for i, w in enumerate(ws):
            r = K.quantize_minmax(w, 4, 128, sym, 0, want_codes=True)
            assert torch.equal(plan.outs[i].view(torch.int16), r.out.view(torch.int16))
            assert torch.equal(plan.scales[i].view(torch.int16), r.scales.view(torch.int16))
            assert torch.equal(plan.codes[i], r.codes)
            if not sym:
                assert torch.equal(plan.zeros[i].view(torch.int16), r.zeros.view(torch.int16))


def test_quantize_model_drop_in(K):
    from types import SimpleNamespace

    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model

    torch.manual_seed(0)
    specs = {"l0": (384, 256, True), "l1": (256, 384, False), "lm_head": (1000, 256, False)}
    originals = {n: (torch.randn(o, i) * 0.02).half() for n, (o, i, _) in specs.items()}
    for batched in (True, False):
        m = torch.nn.Sequential()
        for n, (o, i, b) in specs.items():
            lin = torch.nn.Linear(i, o, bias=b).half().to(DEV)
            lin.weight.data.copy_(originals[n])
            m.add_module(n, lin)
        args = SimpleNamespace(w_bit=4, a_bit=16, w_group_size=128, w_symmetric=False, w_format="int", quant_dim=0)
        quantize_model(m, args, batched=batched, verbose=False)
        assert isinstance(m.l0, QuantLinear) and isinstance(m.l1, QuantLinear)
        assert isinstance(m.lm_head, torch.nn.Linear) and not isinstance(m.lm_head, QuantLinear)
        for n in ("l0", "l1"):
            ref = O.quantlinear_int(originals[n].numpy(), w_bit=4, w_group_size=128, symmetric=False)
            q = getattr(m, n)
            assert bits_equal(to_np(q.weight.data), ref.dequant), (n, batched)
            assert bits_equal(to_np(q.scales), ref.scales), (n, batched)
            assert bits_equal(to_np(q.zeros), ref.zeros), (n, batched)
        assert torch.equal(m.lm_head.weight.data.cpu(), originals["lm_head"])
        x = torch.randn(2, 5, 256, dtype=torch.float16, device=DEV)
        y = m.l0(x)
        torch.testing.assert_close(y, torch.nn.functional.linear(x, m.l0.weight, m.l0.bias))
        # state_dict round trip (batched scales/zeros are views of one allocation): same keys as the
        # reference's buffers, independent saved copies, loadable into a fresh quantized module
        sd = m.state_dict()
        for n in ("l0", "l1"):
            assert {f"{n}.scales", f"{n}.zeros", f"{n}.quantized"} <= set(sd), n
            assert sd[f"{n}.scales"].shape == (specs[n][0] * specs[n][1] // 128, 1)
        import io
        buf = io.BytesIO()
        torch.save(sd, buf)
        buf.seek(0)
        sd2 = torch.load(buf, weights_only=True)
        q2 = QuantLinear.from_linear(torch.nn.Linear(384, 256, bias=False).half().to(DEV), w_bit=4,
                                     w_group_size=128, symmetric=False)
        q2.load_state_dict({k[3:]: v for k, v in sd2.items() if k.startswith("l1.")})
        assert torch.equal(q2.scales, m.l1.scales) and torch.equal(q2.weight, m.l1.weight)


@pytest.mark.parametrize("fmt,sym,apx", [("fp8", False, False), ("fp8", True, False), ("fp6", False, False),
                                         ("fp4", False, False), ("fp8", True, True), ("fp4", True, True)])
def test_quantize_model_fp_batched(K, fmt, sym, apx):
    """quantize_model with FP formats: the one-launch batched path (kernels.FpBatchPlan) leaves
    every layer (weight, scales, zeros, buffers) bit-identical to the per-layer QuantLinear path."""
    from types import SimpleNamespace

    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model

    torch.manual_seed(1)
    specs = {"l0": (384, 256, True), "l1": (256, 384, False), "l2": (128, 512, True)}
    originals = {n: (torch.randn(o, i) * 0.02).half() for n, (o, i, _) in specs.items()}
    res = {}
    for batched in (True, False):
        m = torch.nn.Sequential()
        for n, (o, i, b) in specs.items():
            lin = torch.nn.Linear(i, o, bias=b).half().to(DEV)
            lin.weight.data.copy_(originals[n])
            m.add_module(n, lin)
        args = SimpleNamespace(w_bit=8, a_bit=16, w_group_size=128, w_symmetric=sym, w_format=fmt, quant_dim=0,
                               approximate=apx, double_approximate=False)
        quantize_model(m, args, batched=batched, verbose=False)
        res[batched] = m
    for n in specs:
        a, b = getattr(res[True], n), getattr(res[False], n)
        assert isinstance(a, QuantLinear) and isinstance(b, QuantLinear)
        assert torch.equal(a.weight.data.view(torch.int16), b.weight.data.view(torch.int16)), n
        assert torch.equal(a.scales.view(torch.int16), b.scales.view(torch.int16)), n
        assert (a.zeros is None) == (b.zeros is None), n
        if a.zeros is not None:
            assert torch.equal(a.zeros.view(torch.int16), b.zeros.view(torch.int16)), n
        assert bool(a.quantized) and a.approximate == b.approximate


def test_errors_match_reference(K):
    from iron_weight_only_quant_amd.quant_funcs import pseudo_quantize_tensor
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    x = torch.randn(8, 100, dtype=torch.float16, device=DEV)
    with pytest.raises(AssertionError):
        pseudo_quantize_tensor(x, n_bits=4, q_group_size=128)          # quant_funcs.py:11
    with pytest.raises(AssertionError):
        pseudo_quantize_tensor(torch.randn(2, 3, 4, device=DEV).half())  # quant_funcs.py:15
    lin = torch.nn.Linear(100, 8).half().to(DEV)
    with pytest.raises(ValueError):
        QuantLinear.from_linear(lin, w_bit=4, w_group_size=-3)          # quant_linear.py:906
    with pytest.raises(AssertionError):
        QuantLinear.from_linear(torch.nn.Linear(100, 8).half().to(DEV), w_bit=4, w_group_size=64)  # :897
    with pytest.raises(ValueError):
        QuantLinear(4, 4, weight_format="int3")                          # :440-441


def test_ragged_and_strided_inputs(K):
    """Unaligned / strided / odd shapes take the universal path and still match the oracle."""
    base_np = synth(77, (37, 262), "float16")
    base = to_dev(base_np, "float16")
    view = base[:, 3:259]            # row stride 262, 256 columns, not 16-B aligned
    v_np = np.ascontiguousarray(base_np[:, 3:259])
    for g in (128, 64, -2, -1):
        r = K.quantize_minmax(view, 4, g, False, 0)
        ref = O.quantlinear_int(v_np, w_bit=4, w_group_size=g, symmetric=False)
        assert bits_equal(to_np(r.out), ref.dequant), g
        assert bits_equal(to_np(r.scales), ref.scales.reshape(-1)), g
    odd_np = synth(78, (13, 7), "float16")
    r = K.quantize_minmax(to_dev(odd_np, "float16"), 3, -2, True, 0)
    assert bits_equal(to_np(r.out), O.quantlinear_int(odd_np, w_bit=3, w_group_size=-2, symmetric=True).dequant)
    for nb in (9, 12, 15):
        x_np = synth(79, (16, 256), "float16")
        r = K.quantize_minmax(to_dev(x_np, "float16"), nb, 128, False, 0)
        ref = O.quantlinear_int(x_np, w_bit=nb, w_group_size=128, symmetric=False)
        assert bits_equal(to_np(r.out), ref.dequant, nan_equal=True), nb


# ----------------------------------------------------------------------------------------------
# FP formats (config 5)
# ----------------------------------------------------------------------------------------------
FPF = {"e4m3": (4, 3), "e3m2": (3, 2), "e2m1": (2, 1), "e5m2": (5, 2)}


@pytest.fixture(scope="module")
def FPD():
    return np.load(os.path.join(GOLD, "fp_small.npz"))


@pytest.mark.parametrize("fmt", ["e4m3", "e3m2", "e2m1"])
def test_fp_exhaustive_encode_decode(K, FPD, fmt):
    """Every finite fp16 value in [-fp_max, fp_max] through the kernel's encoder: rows whose absmax is
    fp_max have scale RN16(fp_max/fp_max) = 1, so the codes are _float_to_fp of the inputs and the
    dequantized values are _fp_to_float of the codes (reference tables, exhaustive)."""
    from oracle import fp_codec as C
    e, m = FPF[fmt]
    bias, fp_max = C.fp_params(e, m)
    xs = FPD["in/all_fp16"]
    enc = FPD[f"enc/{fmt}"]
    dec = FPD[f"dec/{fmt}"]
    sel = np.abs(xs.astype(np.float32)) <= fp_max
    vals, codes_exp = xs[sel], enc[sel]
    per = 127
    n = (len(vals) + per - 1) // per
    pad = n * per - len(vals)
    vals_p = np.concatenate([vals, np.zeros(pad, np.float16)]).reshape(n, per)
    rows = np.concatenate([np.full((n, 1), fp_max, np.float16), vals_p], axis=1)
    x = to_dev(rows, "float16")
    for flags in FLAG_SETS:
        r = K.quantize_fp(x, e, m, 128, True, 0, want_codes=True, flags=flags)
        assert torch.all(r.scales == 1)
        cb = r.codes.cpu().numpy()
        if 1 + e + m <= 4:
            cb = np.stack([cb & 0xF, cb >> 4], axis=1).reshape(-1)
        cb = cb.reshape(n, 128)[:, 1:].reshape(-1)[: len(vals)]
        assert np.array_equal(cb, codes_exp), (fmt, flags)
        deq = to_np(r.out)[:, 1:].reshape(-1)[: len(vals)]
        assert bits_equal(deq, dec[codes_exp].astype(np.float16)), (fmt, flags)


def _scale_one_rows(vals, bound):
    """Rows of 127 values behind a leading `bound`: with absmax == bound the group scale is exactly 1,
    so t == the value itself and the output is the table entry (sign rules included)."""
    per = 127
    n = (len(vals) + per - 1) // per
    pad = n * per - len(vals)
    vals_p = np.concatenate([vals, np.zeros(pad, np.float16)]).reshape(n, per)
    return np.concatenate([np.full((n, 1), bound, np.float16), vals_p], axis=1), n


@pytest.mark.parametrize("fmt", ["e4m3", "e3m2", "e2m1"])
def test_fp_exhaustive_lut(K, FPD, fmt):
    """The LDS decode-table path (no codes requested) on every finite fp16 in [-fp_max, fp_max],
    +-0 included: dequantized bits == _fp_to_float(_float_to_fp(x)) (reference tables) and == the
    bit-level ALU codec (use_lut=False)."""
    from oracle import fp_codec as C
    e, m = FPF[fmt]
    _, fp_max = C.fp_params(e, m)
    xs = FPD["in/all_fp16"]
    enc, dec = FPD[f"enc/{fmt}"], FPD[f"dec/{fmt}"]
    sel = np.abs(xs.astype(np.float32)) <= fp_max
    vals, codes_exp = xs[sel], enc[sel]
    rows, n = _scale_one_rows(vals, fp_max)
    x = to_dev(rows, "float16")
    r_lut = K.quantize_fp(x, e, m, 128, True, 0)
    r_alu = K.quantize_fp(x, e, m, 128, True, 0, use_lut=False)
    assert torch.all(r_lut.scales == 1)
    deq = to_np(r_lut.out)[:, 1:].reshape(-1)[: len(vals)]
    assert bits_equal(deq, dec[codes_exp].astype(np.float16)), fmt
    assert torch.equal(r_lut.out.view(torch.int16), r_alu.out.view(torch.int16)), fmt
    # asymmetric: zero point != 0, the same table behind (w - z) / s
    a = K.quantize_fp(x, e, m, 128, False, 0)
    b = K.quantize_fp(x, e, m, 128, False, 0, use_lut=False)
    assert torch.equal(a.out.view(torch.int16), b.out.view(torch.int16)), fmt


def test_fp4_grid_exhaustive_lut(K):
    """Grid table path on every fp16 in [-6, 6] at S == 1 (rows with absmax 6) vs the ALU path."""
    xs = np.arange(1 << 16, dtype=np.uint32).astype(np.uint16).view(np.float16)
    vals = xs[np.isfinite(xs) & (np.abs(xs.astype(np.float32)) <= 6.0)]
    rows, _ = _scale_one_rows(vals, 6.0)
    x = to_dev(rows, "float16")
    a = K.fp4_grid(x, 128)
    b = K.fp4_grid(x, 128, use_lut=False)
    assert torch.all(a.scales == 1)
    assert torch.equal(a.out.view(torch.int16), b.out.view(torch.int16))


@pytest.mark.parametrize("hs,hf,tp", [(12, 15, 1), (4, 7, 2), (1, 3, 0), (2, 5, -1)])
def test_fp_approx_exhaustive_lut(K, hs, hf, tp):
    """Approximate table paths on every finite fp16 in [-fp_max, fp_max] at scale 1 vs the ALU path,
    E4M3 and E2M1: single-aligned decode, and the one-pass double-approximate decode (rows shuffled
    so each quad of groups mixes exponents) vs the two-pass reference-order kernel."""
    from oracle import fp_codec as C
    xs = np.arange(1 << 16, dtype=np.uint32).astype(np.uint16).view(np.float16)
    for e, m in ((4, 3), (2, 1)):
        _, fp_max = C.fp_params(e, m)
        vals = xs[np.isfinite(xs) & (np.abs(xs.astype(np.float32)) <= fp_max)]
        rows, _ = _scale_one_rows(vals, fp_max)
        rows = np.concatenate([rows, np.zeros(((-rows.shape[0]) % 4, 128), np.float16)])  # quads of groups
        rng = np.random.default_rng(e * 100 + hs)
        x = to_dev(rows[rng.permutation(rows.shape[0])], "float16")  # mix exponents inside each quad
        for double in (False, True):
            a = K.quantize_fp_approx(x, e, m, 128, 0, hs, hf, tp, double)
            b = K.quantize_fp_approx(x, e, m, 128, 0, hs, hf, tp, double, use_lut=False)
            assert torch.equal(a.out.view(torch.int16), b.out.view(torch.int16)), (e, m, hs, hf, tp, double)
            assert torch.equal(a.scales.view(torch.int16), b.scales.view(torch.int16)), (e, m, hs, hf, tp, double)


@pytest.mark.parametrize("flags", FLAG_SETS)
def test_fp_quantlinear_golden(K, FPD, flags):
    x = to_dev(FPD["in/fp_a"], "float16")
    n = 0
    for key in FPD.files:
        if not key.startswith("ql/"):
            continue
        _, which, fmt, sym, g, qd, kind = key.split("/")
        e, m = FPF[fmt]
        if kind == "error":
            with pytest.raises(RuntimeError):
                K.quantize_fp(x, e, m, int(g), bool(int(sym)), int(qd), flags=flags)
            continue
        if kind != "deq":
            continue
        base = key[:-4]
        r = K.quantize_fp(x, e, m, int(g), bool(int(sym)), int(qd), flags=flags)
        assert bits_equal(to_np(r.out), FPD[key]), key
        assert bits_equal(to_np(r.scales), FPD[base + "/scales"].reshape(-1)), key
        if base + "/zeros" in FPD.files:
            assert bits_equal(to_np(r.zeros), FPD[base + "/zeros"].reshape(-1)), key
        n += 1
    assert n >= 40


def test_fp_quantlinear_python_face(FPD):
    from iron_weight_only_quant_amd import quant_linear as QL
    x = FPD["in/fp_a"]
    for which, fmt in (("fp8", "e4m3"), ("fp6", "e3m2"), ("fp4", "e2m1")):
        key = f"ql/{which}/{fmt}/0/128/0"
        w = to_dev(x, "float16")
        lin = torch.nn.Linear(256, 48, bias=False).to(DEV)
        lin.weight.data = w
        q = QL.QuantLinear.from_linear(lin, weight_format=which, w_group_size=128, symmetric=False)
        assert bits_equal(to_np(w), FPD[key + "/deq"]), which
        assert bits_equal(to_np(q.zeros), FPD[key + "/zeros"]), which
    QL.configure_fp_formats(fp8_exp_bits=5, fp8_mantissa_bits=2)
    try:
        lin = torch.nn.Linear(256, 48, bias=False).half().to(DEV)
        with pytest.raises(RuntimeError):
            QL.QuantLinear.from_linear(lin, weight_format="fp8", w_group_size=128)
    finally:
        QL.configure_fp_formats()


@pytest.mark.parametrize("flags", FLAG_SETS)
def test_fp4_grid_golden(K, FPD, flags):
    from iron_weight_only_quant_amd.fp4_quantize import quantize_fp16_to_fp4_e1m2
    x = to_dev(FPD["in/fp_a"], "float16")
    for g, pt in ((128, False), (32, False), (-1, True), (256, False)):
        r = K.fp4_grid(x, g, pt, flags=flags)
        exp = FPD[f"grid/{g}/{int(pt)}"]
        assert bits_equal(to_np(r.out).reshape(exp.shape), exp, nan_equal=True), (g, pt)
        if flags == 0:
            out = quantize_fp16_to_fp4_e1m2(x, group_size=g, per_tensor=pt)
            assert tuple(out.shape) == exp.shape
            assert bits_equal(to_np(out), exp, nan_equal=True)
            # the reference ignores return_scales (fp4_quantize_cpu.py:47, :72): the same tensor back
            out2 = quantize_fp16_to_fp4_e1m2(x, group_size=g, per_tensor=pt, return_scales=True)
            assert isinstance(out2, torch.Tensor) and bits_equal(to_np(out2), exp, nan_equal=True)


def test_fp_large_sha(K, FPD):
    import hashlib
    x = torch.empty(4096, 4096, dtype=torch.float16, device=DEV)
    K.fill_synthetic(x, 0)
    for which, fmt, sym in (("fp8", "e4m3", True), ("fp8", "e4m3", False), ("fp4", "e2m1", False)):
        e, m = FPF[fmt]
        r = K.quantize_fp(x, e, m, 128, sym, 0)
        assert hashlib.sha256(to_np(r.out).tobytes()).digest() == FPD[f"sha/{which}/{fmt}/{int(sym)}"].tobytes()
    r = K.fp4_grid(x, 128)
    assert hashlib.sha256(to_np(r.out).tobytes()).digest() == FPD["sha/grid/128"].tobytes()


# ----------------------------------------------------------------------------------------------
# fused dequant -> GEMM forward (config 3)
# ----------------------------------------------------------------------------------------------
@pytest.mark.parametrize("M", [1, 7, 16, 128, 300])
@pytest.mark.parametrize("group,sym,bits", [(-2, False, 4), (-2, True, 4), (128, False, 4), (32, True, 4),
                                            (64, False, 3), (544, False, 4)])
def test_w4a16_gemm_vs_fp32_reference(K, M, group, sym, bits):
    """y = x W_deq^T + b with W_deq = the bit-exact fake-quant weight: compared with an fp32 GEMM on the
    same dequantized weight (tolerance: fp16 output rounding + fp32 accumulation-order error)."""
    N, Kd = 384, 4352
    torch.manual_seed(0)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 90)
    r = K.quantize_minmax(w, bits, group, sym, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    # default (decode kernel for M <= 16), the tiled prefill kernel, and every decode variant
    for flags in (0, 1) + tuple(K.gemm_variant_flags(v) for v in abv(*range(1, 18)) if M <= 16):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, bits, group, N, b, flags=flags)
        err = (y.float() - ref).abs()
        assert bool((err <= tol).all()), (flags, float(err.max()))
    # and against the reference forward semantics: F.linear on the dequantized fp16 weight
    y2 = torch.nn.functional.linear(x, r.out, b)
    assert float((y.float() - y2.float()).abs().max()) <= 4 * float(err.max()) + 2e-3


@pytest.mark.parametrize("group,sym", [(128, False), (128, True), (256, False), (64, False), (-2, False)])
def test_gemv_identity_rows_give_w_deq(K, group, sym):
    """Decode GEMV with X = rows of the identity (x[i, k_i] = 1): y[i, n] must be W_deq[n, k_i] BIT
    FOR BIT -- the per-channel kernel's factored scale, the grouped kernel's scale factored per k-step
    (group % 128 == 0: acc += s_g * partial) and the per-weight RN16((q - z) s) forms all keep each
    weight the reference's fp16 value (s (q - z) is exact in fp32)."""
    N, Kd, M = 384, 2048, 8
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 66)
    r = K.quantize_minmax(w, 4, group, sym, 0, want_codes=True)
    ks = [255 * i + 3 for i in range(M)]
    x = torch.zeros(M, Kd, dtype=torch.float16, device=DEV)
    for i, k in enumerate(ks):
        x[i, k] = 1.0
    want = r.out[:, ks].t().contiguous()
    tiled = K.tile_codes(r.codes, N, Kd)
    for v in (0,) + (abv(27, 28) if group != -2 else ()):
        for codes, tl in ((r.codes, False), (tiled, True)):
            y = K.w4a16_gemm(x, codes, r.scales, r.zeros, 4, group, N, tiled=tl, flags=K.gemm_variant_flags(v))
            assert torch.equal(y.view(torch.int16), want.view(torch.int16)), (v, tl)


@pytest.mark.parametrize("group", [128, -2])
@pytest.mark.parametrize("M", [8, 16])
def test_gemv_large_x_image_identity_and_reference(K, group, M):
    """Round 6: M >= 8 on K = 4096 stages the whole X (M x 8 KiB > the 64 KiB ring budget) in LDS when
    the one-tile grid is at most one workgroup per CU (XLDS_BIG): X = rows of the identity still gives
    W_deq bit for bit (row-major and tile layout), random X stays within the fp32-GEMM tolerance, and
    the tile layout is bit-identical to the row-major codes."""
    N, Kd = 512, 4096
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 68)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    tiled = K.tile_codes(r.codes, N, Kd)
    ks = [(257 * i + 9) % Kd for i in range(M)]
    x = torch.zeros(M, Kd, dtype=torch.float16, device=DEV)
    for i, k in enumerate(ks):
        x[i, k] = 1.0
    want = r.out[:, ks].t().contiguous()
    for codes, tl in ((r.codes, False), (tiled, True)):
        y = K.w4a16_gemm(x, codes, r.scales, r.zeros, 4, group, N, tiled=tl)
        assert torch.equal(y.view(torch.int16), want.view(torch.int16)), tl
    xr = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = xr.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (xr.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    y0 = K.w4a16_gemm(xr, r.codes, r.scales, r.zeros, 4, group, N, b)
    y1 = K.w4a16_gemm(xr, tiled, r.scales, r.zeros, 4, group, N, b, tiled=True)
    assert bool(((y0.float() - ref).abs() <= tol).all())
    assert torch.equal(y0.view(torch.int16), y1.view(torch.int16))
    if AB:  # the ring form (X from L2 per k-step, variant 2's kernels) gives the same bits
        y2 = K.w4a16_gemm(xr, tiled, r.scales, r.zeros, 4, group, N, b, tiled=True, flags=K.gemm_variant_flags(13))
        assert bool(((y2.float() - ref).abs() <= tol).all())


@pytest.mark.parametrize("Kd", [4096, 11008])
@pytest.mark.parametrize("group", [128, -2])
@pytest.mark.parametrize("M", [8, 16])
def test_gemv_ksplit_identity_and_reference(K, Kd, group, M):
    """Round 6, the K-split decode (k_w4a16_gemv_ks + k_gemv_ks_reduce: KS workgroups per 64 columns,
    each with its X slice in LDS, fp32 slabs summed in ks order by the reduce): on the q_proj / down_proj
    shapes X = rows of the identity gives W_deq bit for bit and random X stays within the fp32-GEMM
    tolerance, through the default dispatch (row-major and tile layout, bit-identical to each other)
    and, in A/B builds, forced (31) and refused (32)."""
    N = 4096
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 69)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    tiled = K.tile_codes(r.codes, N, Kd)
    ks = [(263 * i + 11) % Kd for i in range(M)]
    x = torch.zeros(M, Kd, dtype=torch.float16, device=DEV)
    for i, k in enumerate(ks):
        x[i, k] = 1.0
    want = r.out[:, ks].t().contiguous()
    xr = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = xr.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (xr.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    for v in (0,) + abv(31, 32):
        fl = K.gemm_variant_flags(v)
        outs = []
        for codes, tl in ((r.codes, False), (tiled, True)):
            y = K.w4a16_gemm(x, codes, r.scales, r.zeros, 4, group, N, tiled=tl, flags=fl)
            assert torch.equal(y.view(torch.int16), want.view(torch.int16)), (v, tl)
            yr = K.w4a16_gemm(xr, codes, r.scales, r.zeros, 4, group, N, b, tiled=tl, flags=fl)
            assert bool(((yr.float() - ref).abs() <= tol).all()), (v, tl, float((yr.float() - ref).abs().max()))
            outs.append(yr)
        assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16)), v


@pytest.mark.skipif(not AB, reason="A/B library only (cross-workgroup K-split decode variants 200-259)")
@pytest.mark.parametrize("Kd,group", [(4096, -2), (11008, 128)])
def test_gemv_cross_workgroup_ksplit(K, Kd, group):
    """Round 6 A/B: the batched decode's cross-workgroup K-split (k_w4a16_gemv_ct<.., KSX>: KS K ranges
    per 4 or 8 column tiles, fp32 slabs, the last arrival finishes the tile) -- X = rows of the identity
    gives W_deq bit for bit, random X within the fp32-GEMM tolerance, three calls in a row on one zeroed
    workspace (the arrival counters are left zero: every call after the first is right too), and the
    workspace's counter region is zero afterwards; grid map per column group (203, 227) and XCD-local
    (243)."""
    N, M = 4096, 16
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 71)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    tiled = K.tile_codes(r.codes, N, Kd)
    ks = [(263 * i + 11) % Kd for i in range(M)]
    x = torch.zeros(M, Kd, dtype=torch.float16, device=DEV)
    for i, k in enumerate(ks):
        x[i, k] = 1.0
    want = r.out[:, ks].t().contiguous()
    xr = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = xr.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (xr.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    for v in (203, 227, 243):
        fl = K.gemm_variant_flags(v)
        zws = torch.zeros(K.gemm_workspace_bytes(M, N, Kd, group, fl), dtype=torch.uint8, device=DEV)
        for codes, tl in ((r.codes, False), (tiled, True)):
            for _ in range(3):
                y = K.w4a16_gemm(x, codes, r.scales, r.zeros, 4, group, N, tiled=tl, flags=fl, zeroed_workspace=zws)
                assert torch.equal(y.view(torch.int16), want.view(torch.int16)), (v, tl)
                yr = K.w4a16_gemm(xr, codes, r.scales, r.zeros, 4, group, N, b, tiled=tl, flags=fl, zeroed_workspace=zws)
                assert bool(((yr.float() - ref).abs() <= tol).all()), (v, tl, float((yr.float() - ref).abs().max()))
        torch.cuda.synchronize()
        assert int(zws[:16384].count_nonzero()) == 0, v


@pytest.mark.skipif(not AB, reason="A/B library only (warp-specialised prefill variants 180-183)")
@pytest.mark.parametrize("M", [256, 300, 1024])
@pytest.mark.parametrize("sym", [False, True])
def test_prefill_warp_specialised(K, M, sym):
    """Round 6 A/B: the warp-specialised prefill (producer waves dequantize into an fp16 B image, consumer
    waves run the MFMA loop; iwq_prefill_ws.hip) -- X = rows of the identity gives W_deq bit for bit
    (per-channel numerics), random X within the fp32-GEMM tolerance, ragged M included, for the
    pipeline depths 180 / 181 and the producer-priority form 182."""
    N, Kd = 512, 4096
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 70)
    r = K.quantize_minmax(w, 4, -2, sym, 0, want_codes=True)
    ks = [(131 * i + 7) % Kd for i in range(M)]
    x = torch.zeros(M, Kd, dtype=torch.float16, device=DEV)
    x[torch.arange(M, device=DEV), torch.tensor(ks, device=DEV)] = 1.0
    want = r.out[:, ks].t().contiguous()
    xr = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = xr.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (xr.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    for v in (180, 181, 182):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, flags=K.gemm_variant_flags(v))
        assert torch.equal(y.view(torch.int16), want.view(torch.int16)), v
        yr = K.w4a16_gemm(xr, r.codes, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(v))
        assert bool(((yr.float() - ref).abs() <= tol).all()), (v, float((yr.float() - ref).abs().max()))


@pytest.mark.parametrize("M", [24, 48, 96])
@pytest.mark.parametrize("group", [128, 64])
def test_mid_m_identity_rows_give_w_deq(K, M, group):
    """The mid-M kernel (17 <= M < 256 without a split workspace): X = rows of the identity gives
    W_deq bit for bit -- with the group scale factored per 128-k step (g128) and per weight (g64),
    and (A/B 56) the per-weight form at g128 within fp32 tolerance of the default."""
    N, Kd = 512, 4096
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 67)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    ks = [(41 * i + 5) % Kd for i in range(M)]
    x = torch.zeros(M, Kd, dtype=torch.float16, device=DEV)
    for i, k in enumerate(ks):
        x[i, k] = 1.0
    want = r.out[:, ks].t().contiguous()
    y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N)
    assert torch.equal(y.view(torch.int16), want.view(torch.int16))
    if AB and group == 128:
        y56 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, flags=K.gemm_variant_flags(56))
        assert torch.equal(y56.view(torch.int16), want.view(torch.int16))
        xr = (torch.randn(M, Kd, device=DEV) * 0.5).half()
        ref = xr.float() @ r.out.float().t()
        tol = 2e-3 * ref.abs() + 1e-3 * (xr.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
        for v in (0, 56):
            yv = K.w4a16_gemm(xr, r.codes, r.scales, r.zeros, 4, group, N, flags=K.gemm_variant_flags(v))
            assert bool(((yv.float() - ref).abs() <= tol).all()), v


@pytest.mark.parametrize("Kd", [256, 1152, 4096])
@pytest.mark.parametrize("M", [1, 16])
def test_gemv_persistent_many_groups(K, Kd, M):
    """Persistent decode GEMV with more column groups than resident workgroups (each workgroup walks
    several groups), k-split waves with unequal step counts (Kd = 1152: 9 steps over 8 waves) and
    waves without any step (Kd = 256): every variant vs an fp32 GEMM on the fake-quant weight."""
    N = 24576
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 77)
    r = K.quantize_minmax(w, 4, 128, False, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    for v in (0,) + abv(14, 15, 16, 17):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, 128, N, b, flags=K.gemm_variant_flags(v))
        err = (y.float() - ref).abs()
        assert bool((err <= tol).all()), (v, float(err.max()))


@pytest.mark.parametrize("group", [-2, 128])
def test_gemv_tiled_layout_identical(K, group):
    """The decode tile layout changes only where the codes are read from: outputs are bit-identical
    to the row-major kernel (same arithmetic, same order), for M = 1, 7, 16."""
    N, Kd = 384, 4352
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 55)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    tiled = K.tile_codes(r.codes, N, Kd)
    assert tiled.numel() == r.codes.numel()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    for m in (1, 7, 16):
        x = (torch.randn(m, Kd, device=DEV) * 0.5).half()
        y0 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b)
        y1 = K.w4a16_gemm(x, tiled, r.scales, r.zeros, 4, group, N, b, tiled=True)
        assert torch.equal(y0.view(torch.int16), y1.view(torch.int16)), m
        if AB and group != -2:  # grouped, scale per weight: parameters per step from global memory (27)
            y2 = K.w4a16_gemm(x, tiled, r.scales, r.zeros, 4, group, N, b, tiled=True, flags=K.gemm_variant_flags(27))
            y3 = K.w4a16_gemm(x, tiled, r.scales, r.zeros, 4, group, N, b, tiled=True, flags=K.gemm_variant_flags(28))
            assert torch.equal(y2.view(torch.int16), y3.view(torch.int16)), m  # vs staged in LDS (28)
    with pytest.raises(Exception):
        K.w4a16_gemm(torch.randn(32, Kd, device=DEV).half(), tiled, r.scales, r.zeros, 4, group, N, tiled=True)
    # tiled A/B variants: same S (k-split) => same summation order as the row-major variant of that
    # number (18-20 have the default's S = 8); out= writes in place
    x = (torch.randn(5, Kd, device=DEV) * 0.5).half()
    y = torch.empty(5, N, dtype=torch.float16, device=DEV)
    for v in abv(1, 2, 4, 5, 7, 8, 9, 10, 12, 13, 18, 19, 20, 21, 22, 23, 24):
        rv = v if v in (2, 4, 5, 7, 8, 9, 10, 12, 13) else (2 if v == 1 else 0)
        y0 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(rv))
        y1 = K.w4a16_gemm(x, tiled, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v),
                          tiled=True, out=y)
        assert y1.data_ptr() == y.data_ptr()
        assert torch.equal(y0.view(torch.int16), y.view(torch.int16)), v
        if v >= 21:  # column-tile kernels on row-major codes: same bits too
            y2 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
            assert torch.equal(y0.view(torch.int16), y2.view(torch.int16)), v
            # M = 16: X (139 KB) exceeds the LDS image budget -> the register-X form of both kernels
            x16 = (torch.randn(16, Kd, device=DEV) * 0.5).half()
            z0 = K.w4a16_gemm(x16, r.codes, r.scales, r.zeros, 4, group, N, b)
            for codes, tl in ((r.codes, False), (tiled, True)):
                z1 = K.w4a16_gemm(x16, codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v),
                                  tiled=tl)
                assert torch.equal(z0.view(torch.int16), z1.view(torch.int16)), (v, tl)
    # a grid wide enough that the default takes the column-tile kernel (N/64 >= 256 -> 4 tiles per
    # wave at M >= 4): same bits as the one-tile kernel with the same k-split (variant 18)
    N2, K2 = 16384, 512
    w2 = torch.empty(N2, K2, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w2, 56)
    r2 = K.quantize_minmax(w2, 4, group, False, 0, want_codes=True)
    t2 = K.tile_codes(r2.codes, N2, K2)
    # long K at M < 4: the default takes the 16-way k-split (variant 13's kernel)
    N3, K3 = 256, 10240
    w3 = torch.empty(N3, K3, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w3, 57)
    r3 = K.quantize_minmax(w3, 4, group, False, 0, want_codes=True)
    t3 = K.tile_codes(r3.codes, N3, K3)
    for m in (1, 3):
        x = (torch.randn(m, K3, device=DEV) * 0.5).half()
        y_rm = K.w4a16_gemm(x, r3.codes, r3.scales, r3.zeros, 4, group, N3)
        for codes, tl in ((r3.codes, False), (t3, True)):
            y = K.w4a16_gemm(x, codes, r3.scales, r3.zeros, 4, group, N3, tiled=tl)
            assert torch.equal(y_rm.view(torch.int16), y.view(torch.int16)), (m, tl)
            if AB:
                ref = K.w4a16_gemm(x, codes, r3.scales, r3.zeros, 4, group, N3, flags=K.gemm_variant_flags(13),
                                   tiled=tl)
                assert torch.equal(ref.view(torch.int16), y.view(torch.int16)), (m, tl)
            want = x.float() @ r3.out.float().t()
            torch.testing.assert_close(y.float(), want, rtol=2e-2, atol=2e-2)
    # M = 2 with X over the LDS budget (K = 16384): two column tiles per wave, same bits as variant 18
    N4, K4 = 8192, 16384
    w4 = torch.empty(N4, K4, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w4, 58)
    r4 = K.quantize_minmax(w4, 4, group, False, 0, want_codes=True)
    del w4
    t4 = K.tile_codes(r4.codes, N4, K4)
    x = (torch.randn(2, K4, device=DEV) * 0.5).half()
    y_rm = K.w4a16_gemm(x, r4.codes, r4.scales, r4.zeros, 4, group, N4)
    torch.testing.assert_close(y_rm.float(), x.float() @ r4.out.float().t(), rtol=2e-2, atol=2e-2)
    for codes, tl in ((r4.codes, False), (t4, True)):
        y = K.w4a16_gemm(x, codes, r4.scales, r4.zeros, 4, group, N4, tiled=tl)
        assert torch.equal(y_rm.view(torch.int16), y.view(torch.int16)), tl
        if AB:
            ref = K.w4a16_gemm(x, codes, r4.scales, r4.zeros, 4, group, N4, flags=K.gemm_variant_flags(18), tiled=tl)
            assert torch.equal(ref.view(torch.int16), y.view(torch.int16)), tl
    del r4, t4
    for m in (1, 4, 9, 16):
        x = (torch.randn(m, K2, device=DEV) * 0.5).half()
        ref = K.w4a16_gemm(x, r2.codes, r2.scales, r2.zeros, 4, group, N2,
                           flags=K.gemm_variant_flags(18 if AB else 0))
        torch.testing.assert_close(ref.float(), x.float() @ r2.out.float().t(), rtol=2e-2, atol=2e-2)
        for codes, tl in ((r2.codes, False), (t2, True)):
            y = K.w4a16_gemm(x, codes, r2.scales, r2.zeros, 4, group, N2, tiled=tl)
            assert torch.equal(ref.view(torch.int16), y.view(torch.int16)), (m, tl)


def test_w4a16_gemm_identity_layout(K):
    """A = I with an asymmetric weight: catches any transposed or permuted output/operand mapping."""
    N, Kd = 128, 128
    w = (torch.arange(N * Kd, device=DEV, dtype=torch.float32).reshape(N, Kd) % 13 - 6).half()
    r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
    x = torch.eye(Kd, device=DEV, dtype=torch.float16)
    y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N)
    assert torch.equal(y, r.out.t().contiguous())
    for m in (1, 5, 16):  # decode kernels: rows of the identity pick weight columns exactly
        for v in (0,) + abv(*range(1, 18), 21, 22, 23, 24):
            y = K.w4a16_gemm(x[:m].contiguous(), r.codes, r.scales, r.zeros, 4, -2, N, flags=K.gemm_variant_flags(v))
            assert torch.equal(y, r.out.t()[:m].contiguous()), (m, v)


def test_quantlinear_fused_forward(K):
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    lin = torch.nn.Linear(512, 256, bias=True).half().to(DEV)
    q = QuantLinear.from_linear(lin, w_bit=4, w_group_size=-2, symmetric=False, fused_forward=True)
    assert q.qweight is not None
    x = torch.randn(3, 5, 512, device=DEV).half()
    y = q(x)
    ref = torch.nn.functional.linear(x, q.weight, q.bias)
    assert y.shape == ref.shape
    torch.testing.assert_close(y, ref, rtol=1e-2, atol=2e-3)


@pytest.mark.parametrize("group", [-2, 128])
def test_quantlinear_fused_forward_nib(K, group):
    """fused_forward=True, nib_prefill=True keeps a NIB-layout copy of the codes (non-persistent,
    dropped on load) and
    reads it at M >= 256: the same bits as the row-major codes; below 256 rows the row-major codes."""
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    lin = torch.nn.Linear(1024, 512, bias=False).half().to(DEV)
    q0 = QuantLinear.from_linear(lin, w_bit=4, w_group_size=group, symmetric=False, fused_forward=True)
    assert q0.qweight_nib is None  # opt-in
    q = QuantLinear.from_linear(lin, w_bit=4, w_group_size=group, symmetric=False, fused_forward=True,
                                nib_prefill=True)
    assert q.qweight_nib is not None and "qweight_nib" not in q.state_dict()
    assert torch.equal(q.qweight_nib, K.nib_codes(q.qweight, 512, 1024))
    z = None if q.zeros is None else q.zeros.view(-1)
    for shape in ((2, 150, 1024), (100, 1024)):
        x = torch.randn(*shape, device=DEV).half()
        ref = K.w4a16_gemm(x, q.qweight, q.scales.view(-1), z, 4, group, 512)
        assert torch.equal(q(x), ref), shape
    q.load_state_dict(q.state_dict())
    assert q.qweight_nib is None


@pytest.mark.parametrize("bits,group,sym", [(4, -2, False), (4, 128, False), (4, 128, True), (3, 64, False),
                                            (2, 32, True), (4, 96, False)])
def test_dequant_packed_bit_exact(K, bits, group, sym):
    """Packed codes -> fp16 W_deq equals the fake-quant weight of the same quantization, bit for bit;
    w4a16_linear (packed-only forward) matches F.linear on it at decode and prefill sizes."""
    N, Kd = 384, 1536
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 91 + bits)
    r = K.quantize_minmax(w, bits, group, sym, 0, want_codes=True)
    deq = K.dequant_packed(r.codes, r.scales, r.zeros, bits, group, N, Kd)
    assert torch.equal(deq.view(torch.int16), r.out.view(torch.int16))
    bias = torch.randn(N, device=DEV).half()
    for m in (1, 9, 600):
        x = torch.randn(m, Kd, device=DEV).half()
        y = K.w4a16_linear(x, r.codes, r.scales, r.zeros, bits, group, N, bias)
        torch.testing.assert_close(y, torch.nn.functional.linear(x, r.out, bias), rtol=1e-2, atol=2e-2)


def test_quantlinear_fused_forward_auto(K, monkeypatch):
    """fused_forward="auto": the packed-weight kernels where kernels.auto_fused_preferred says they
    are faster (tile-layout GEMV up to 16 rows, row-major codes above), F.linear where they are not."""
    from iron_weight_only_quant_amd import quant_linear as QLm
    calls = []
    real = QLm.kernels.w4a16_gemm
    monkeypatch.setattr(QLm.kernels, "w4a16_gemm", lambda *a, **k: calls.append(1) or real(*a, **k))
    lin = torch.nn.Linear(512, 512, bias=True).half().to(DEV)
    q = QLm.QuantLinear.from_linear(lin, w_bit=4, w_group_size=128, symmetric=False, fused_forward="auto")
    assert q.qweight_tiled is not None and q.qweight_tiled.numel() == q.qweight.numel()
    # g128, N = K = 512 (not down-like): fused up to 32 rows (kernels.auto_fused_preferred)
    for shape, fused in (((1, 512), True), ((2, 8, 512), True), ((2, 16, 512), True), ((3, 16, 512), False),
                         ((4, 64, 512), False)):
        calls.clear()
        x = torch.randn(*shape, device=DEV).half()
        y = q(x)
        ref = torch.nn.functional.linear(x, q.weight, q.bias)
        torch.testing.assert_close(y, ref, rtol=1e-2, atol=2e-3)
        assert bool(calls) == fused, shape


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
def test_per_tensor_fast_path(K, dtype):
    """group -1 (per-tensor) on a tensor big enough for many partial-key workgroups, quant_dim 0 and 1,
    sym / asym, with codes: the default path (at 6 MB the two-kernel reduce + apply: the one pass pays
    from 32 MiB), the one pass forced (variant 8; fp16, and bf16 / fp32 without codes) and the
    pair's variants vs the oracle, bit-exact."""
    x = synth(55, (1536, 2048), dtype)
    big = np.float32(-3.25)  # a single outlier decides the scale
    x.reshape(-1)[123457] = O.f32_to_bf16_bits(big).reshape(-1)[0] if dtype == "bfloat16" else big
    xd = to_dev(x, dtype)
    for bits, sym, qd in ((4, False, 0), (8, True, 0), (3, False, 1), (4, True, 1)):
        exp = O.quantlinear_int(x, bits, -1, sym, qd, dtype)
        # + pair variants 1 (non-temporal), 3 (apply walks backwards), 4 / 5 (apply unrolled), 6 (the
        # pair forced), one-pass variants 7 (NV vectors per thread) and 8 (the one pass at any size)
        for flags in FLAG_SETS + [K.gemm_variant_flags(v) for v in (6, 8) + abv(1, 3, 4, 5, 7)]:
            r = K.quantize_minmax(xd, bits, -1, sym, qd, want_codes=True, flags=flags)
            assert bits_equal(to_np(r.out), exp.dequant), (bits, sym, qd, flags)
            assert bits_equal(to_np(r.scales), exp.scales.reshape(-1)), (bits, sym, qd)
            codes = r.codes.cpu().numpy()
            assert np.array_equal(codes.reshape(-1), O.pack_codes(exp.codes, bits).reshape(-1)), (bits, sym, qd, flags)
    # NaN poisons the tensor's scale: every output NaN, flag raised
    y = x.copy()
    y.reshape(-1)[999] = np.nan if dtype != "bfloat16" else 0x7FC0
    r = K.quantize_minmax(to_dev(y, dtype), 4, -1, False, 0)
    assert r.has_nan()


def test_per_tensor_onepass_timeout_retry(K):
    """A one-pass hand-off that gives up (test-only variant 9: every granule sweep gives up at once,
    as it would with workgroups held off the CUs by another stream) ABORTS the launch through the
    consensus word: nan_flag bit 1, and in place NOT ONE byte written (out of place, round 6, a
    workgroup whose sweep completed may go without the consensus; here every sweep gives up, so none
    does).  has_nan() then re-runs the call on the two-kernel form into the same outputs -- out of place
    and IN PLACE (the input is untouched) -- bit-exact vs the oracle.  QuantLinear(w_group_size=-1)
    settles the same way."""
    x = synth(56, (1536, 2048), "float16")
    exp = O.quantlinear_int(x, 4, -1, False, 0, "float16")
    # out of place
    r = K.quantize_minmax(to_dev(x, "float16"), 4, -1, False, 0, want_codes=True, flags=K.gemm_variant_flags(9))
    assert int(r.nan_flag.item()) & 2
    assert not r.has_nan()
    assert r.retried
    assert bits_equal(to_np(r.out), exp.dequant)
    assert bits_equal(to_np(r.scales), exp.scales.reshape(-1))
    assert bits_equal(to_np(r.zeros), exp.zeros.reshape(-1))
    assert np.array_equal(r.codes.cpu().numpy().reshape(-1), O.pack_codes(exp.codes, 4).reshape(-1))
    # in place: the aborted launch leaves the weight (and the poisoned outputs) untouched
    xi = to_dev(x, "float16")
    r = K.quantize_minmax(xi, 4, -1, False, 0, out=xi, want_codes=True, flags=K.gemm_variant_flags(9))
    r.scales.fill_(7.0)
    r.codes.fill_(0xAB)
    torch.cuda.synchronize()
    flag = int(r.nan_flag.item())
    assert flag & 2 and not flag & 4, flag
    assert bits_equal(to_np(xi), x), "aborted one-pass launch wrote into the weight"
    assert bool((r.codes == 0xAB).all()) and bool((r.scales == 7.0).all())
    assert not r.has_nan()
    assert r.retried
    assert bits_equal(to_np(xi), exp.dequant)
    assert bits_equal(to_np(r.scales), exp.scales.reshape(-1))
    assert np.array_equal(r.codes.cpu().numpy().reshape(-1), O.pack_codes(exp.codes, 4).reshape(-1))
    # QuantLinear's in-place per-tensor branch takes the retry too
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    lin = torch.nn.Linear(2048, 1536, bias=False).half().cuda()
    lin.weight.data.copy_(to_dev(x, "float16"))
    orig = K.quantize_minmax
    K.quantize_minmax = lambda *a, **kw: orig(*a, **{**kw, "flags": K.gemm_variant_flags(9)})
    try:
        q = QuantLinear.from_linear(lin, w_bit=4, w_group_size=-1, symmetric=False)
    finally:
        K.quantize_minmax = orig
    assert bits_equal(to_np(q.weight.data), exp.dequant)
    assert bits_equal(to_np(q.scales.view(-1)), exp.scales.reshape(-1))


def test_per_tensor_onepass_timeout_retry_quant_dim1(K):
    """The same abort at quant_dim 1 (the C side takes the one-pass kernel for per-tensor calls at any
    quant_dim: the group is the whole tensor, so the walk does not depend on it): the retry is set
    up there too, out of place and in place, and QuantLinear(quant_dim=1) settles it."""
    x = synth(57, (1536, 2048), "float16")
    exp = O.quantlinear_int(x, 4, -1, False, 1, "float16")
    r = K.quantize_minmax(to_dev(x, "float16"), 4, -1, False, 1, want_codes=True, flags=K.gemm_variant_flags(9))
    assert r.retry is not None
    assert int(r.nan_flag.item()) & 2
    assert not r.has_nan() and r.retried
    assert bits_equal(to_np(r.out), exp.dequant)
    assert bits_equal(to_np(r.scales), exp.scales.reshape(-1))
    assert bits_equal(to_np(r.zeros), exp.zeros.reshape(-1))
    assert np.array_equal(r.codes.cpu().numpy().reshape(-1), O.pack_codes(exp.codes, 4).reshape(-1))
    xi = to_dev(x, "float16")
    r = K.quantize_minmax(xi, 4, -1, False, 1, out=xi, flags=K.gemm_variant_flags(9))
    torch.cuda.synchronize()
    assert bits_equal(to_np(xi), x), "aborted one-pass launch wrote into the weight"
    assert not r.has_nan() and r.retried
    assert bits_equal(to_np(xi), exp.dequant)
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    lin = torch.nn.Linear(2048, 1536, bias=False).half().cuda()
    lin.weight.data.copy_(to_dev(x, "float16"))
    orig = K.quantize_minmax
    K.quantize_minmax = lambda *a, **kw: orig(*a, **{**kw, "flags": K.gemm_variant_flags(9)})
    try:
        q = QuantLinear.from_linear(lin, w_bit=4, w_group_size=-1, symmetric=False, quant_dim=1)
    finally:
        K.quantize_minmax = orig
    assert bits_equal(to_np(q.weight.data), exp.dequant)
    assert bits_equal(to_np(q.scales.view(-1)), exp.scales.reshape(-1))


def _stream_ws(K):
    dev = torch.device("cuda", torch.cuda.current_device())
    return K._tws.bufs.get((dev.index, torch.cuda.current_stream(dev).cuda_stream))


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
def test_per_tensor_workspace_left_zero(K, dtype):
    """Per tensor, eager calls use the stream's cached workspace with IWQ_FLAG_WS_ZEROED (no zeroing
    launch): every path must leave its first half zero -- the one-pass kernel (its last workgroup
    clears the granules, the consensus word and the done counter; variant 8 forces it at these
    sizes), the pair (the default here, variant 6, the bf16 / fp32 codes path: partial keys in the
    second half), the aborted one-pass + retry (variant 9), the universal path (FORCE_GENERIC, a
    ragged numel).  Tensors of different sizes and ranges back to back, each bit-exact vs the oracle
    (a stale granule or consensus word would hand the next launch a wrong range or outcome)."""
    cases = []
    for i, (shape, scale) in enumerate((((1536, 2048), 1.0), ((64, 4096), 300.0), ((4096, 1024), 0.01),
                                        ((7, 9), 2.0), ((2048, 2048), 1.0))):
        x = synth(70 + i, shape, "float32") * np.float32(scale)
        cases.append(x.astype(np.float32) if dtype == "float32" else
                     (O.f32_to_bf16_bits(x) if dtype == "bfloat16" else x.astype(np.float16)))
    runs = 0
    for x in cases:
        xd = to_dev(x, dtype)
        for bits, sym, qd, codes in ((4, False, 0, False), (8, True, 1, False), (4, False, 0, True)):
            exp = O.quantlinear_int(x, bits, -1, sym, qd, dtype)
            for flags in (0, 1, K.gemm_variant_flags(6), K.gemm_variant_flags(8), K.gemm_variant_flags(9)):
                if codes and x.shape[1] % 2:
                    continue
                r = K.quantize_minmax(xd, bits, -1, sym, qd, want_codes=codes, flags=flags)
                assert not r.has_nan()
                assert bits_equal(to_np(r.out), exp.dequant), (x.shape, bits, sym, qd, codes, flags)
                assert bits_equal(to_np(r.scales), exp.scales.reshape(-1)), (x.shape, bits, flags)
                if codes:
                    assert np.array_equal(r.codes.cpu().numpy().reshape(-1),
                                          O.pack_codes(exp.codes, bits).reshape(-1)), (x.shape, bits, flags)
                ws = _stream_ws(K)
                assert ws is not None
                torch.cuda.synchronize()
                half = int(K.L.load().iwq_workspace_bytes(*x.shape, -1, qd)) // 2
                assert int(ws[:half].count_nonzero()) == 0, ("workspace left dirty", x.shape, bits, qd, codes, flags)
                runs += 1
    assert runs >= 70


def test_per_tensor_zeroed_workspace_graph(K):
    """zeroed_workspace= under hipGraph capture (where the per-stream cache is not used): per-tensor
    calls captured on one caller-zeroed workspace (the pair, the one pass forced), and one-pass calls
    on fresh workspaces zeroed by the captured memset, replayed twice on new inputs: bit-exact vs the
    oracle, the zeroed half of the workspace zero after each replay; a workspace too small is
    refused."""
    n = 5
    xs = [synth(80 + i, (1024, 2048), "float16") for i in range(n)]
    dev = [to_dev(x, "float16") for x in xs]
    wsb = int(K.L.load().iwq_workspace_bytes(1024, 2048, -1, 0))
    zw = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        K.quantize_minmax(dev[0], 4, -1, False, 0, zeroed_workspace=zw[:wsb - 16])
    outs = [torch.empty_like(d) for d in dev]
    # calls 0-2 on the zeroed workspace (default = the pair at 4 MB, then the one pass forced twice);
    # calls 3-4 the one pass on captured-memset workspaces
    kws = [dict(zeroed_workspace=zw), dict(zeroed_workspace=zw, flags=K.gemm_variant_flags(8)),
           dict(zeroed_workspace=zw, flags=K.gemm_variant_flags(8)), dict(flags=K.gemm_variant_flags(8)),
           dict(flags=K.gemm_variant_flags(8))]
    res = []
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for d, o, kw in zip(dev, outs, kws):  # warm-up outside the capture (lazy allocations)
            K.quantize_minmax(d, 4, -1, False, 0, out=o, **kw)
        with torch.cuda.graph(g, stream=s):
            for d, o, kw in zip(dev, outs, kws):
                res.append(K.quantize_minmax(d, 4, -1, False, 0, out=o, **kw))
    torch.cuda.current_stream().wait_stream(s)
    for rnd in range(2):
        xs = [synth(90 + n * rnd + i, (1024, 2048), "float16") * np.float16(1 + 5 * i) for i in range(n)]
        for d, x in zip(dev, xs):
            d.copy_(to_dev(x, "float16"))
        g.replay()
        torch.cuda.synchronize()
        assert int(zw[:wsb // 2].count_nonzero()) == 0
        for i, (x, o, r) in enumerate(zip(xs, outs, res)):
            exp = O.quantlinear_int(x, 4, -1, False, 0, "float16")
            assert not (int(r.nan_flag.item()) & 6)
            assert bits_equal(to_np(o), exp.dequant), (rnd, i)
            assert bits_equal(to_np(r.scales), exp.scales.reshape(-1)), (rnd, i)
    del g


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
def test_quant_dim1_register_kernel(K, dtype):
    """quant_dim 1 with groups of 32/64/128/256 rows (the register-resident column kernel; cols not a
    multiple of the 64-column block) vs the oracle, bit-exact incl. codes, scales and zero points."""
    x = synth(61, (512, 328), dtype)
    xd = to_dev(x, dtype)
    for g in (32, 64, 128, 256):
        for bits, sym in ((4, False), (8, True), (3, False)):
            exp = O.quantlinear_int(x, bits, g, sym, 1, dtype)
            for flags in FLAG_SETS + [K.gemm_variant_flags(v) for v in abv(1, 3, 4)]:
                r = K.quantize_minmax(xd, bits, g, sym, 1, want_codes=True, flags=flags)
                assert bits_equal(to_np(r.out), exp.dequant), (g, bits, sym, flags)
                assert bits_equal(to_np(r.scales), exp.scales.reshape(-1)), (g, bits, sym, flags)
                if not sym:
                    assert bits_equal(to_np(r.zeros), exp.zeros.reshape(-1)), (g, bits, flags)
                assert np.array_equal(r.codes.cpu().numpy().reshape(-1),
                                      O.pack_codes(exp.codes, bits).reshape(-1)), (g, bits, sym, flags)


@pytest.mark.parametrize("M", [512, 600, 1024])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("group", [-2, 128, 64])
def test_w4a16_prefill_big_tile(K, M, sym, group):
    """The 256x256 LDS-DMA prefill kernel (per-channel, N % 256 == 0, M >= 512): vs an fp32 GEMM on the
    bit-exact dequantized weight, and against the 128x128 kernel (variant 1)."""
    N, Kd = 512, 4352
    torch.manual_seed(1)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 91)
    r = K.quantize_minmax(w, 4, group, sym, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b)
    err = (y.float() - ref).abs()
    assert bool((err <= tol).all()), float(err.max())
    # variant 2: the round-1 k_w4a16_big (the default is iwq_prefill.hip since round 2)
    y_big = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(2))
    assert bool(((y_big.float() - ref).abs() <= tol).all())
    if group == -2 and AB:
        for v in (24,):  # k-slice-outer: same BK, same accumulation order as k_w4a16_big
            yv = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(v))
            assert torch.equal(yv, y_big), v
        y23 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(23))  # BK=128
        assert bool(((y23.float() - ref).abs() <= tol).all())
    y1 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(1))
    assert float((y.float() - y1.float()).abs().max()) <= 2 * float(err.max()) + 2e-3


def test_w4a16_prefill_big_identity(K):
    """A = I (512x512) through the big-tile kernel: picks W_deq^T exactly (layout / swizzle check)."""
    N, Kd = 512, 512
    w = (torch.arange(N * Kd, device=DEV, dtype=torch.float32).reshape(N, Kd) % 13 - 6).half()
    r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
    x = torch.eye(Kd, device=DEV, dtype=torch.float16)
    y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N)
    assert torch.equal(y, r.out.t().contiguous())


# prefill variants (iwq_prefill.hip) with identical bits within a set: per channel, scale per
# element (exact) or in the epilogue (factored), on 32x32x16 or 16x16x32; grouped: one set per shape.
# The wave layout (60-62: 4 x 2 waves / static priority; 63-64: four waves of 128 x 128) changes
# neither the k order nor the accumulation order, so those join the 32x32x16 sets.
# 150 / 151 / 154-157: 74 on the 16x16x32 MFMA (iwq_prefill16.hip; per channel and group % 64 == 0)
B32_SETS_PC = ((40, 44, 46, 61, 64), (41, 42, 43, 45, 60, 62, 63, 65, 68, 70, 73, 74, 76, 78, 79, 80, 97, 98), (47,),
               (48,), (150, 151, 154, 155, 156, 157, 162, 164, 170, 171))
B32_SETS_G = ((40, 41, 42, 43, 45, 60, 62, 63, 65, 68, 70, 74, 76, 78, 79, 80, 98), (47,), (150, 151, 154, 155, 156, 157, 162, 164, 170, 171))
B32_ALL = tuple(v for vs in B32_SETS_PC for v in vs)


def nib_layout(codes, N, K):
    """Row-major codes -> the NIB layout of prefill variants 66/67 (tools/ab_gemm.py)."""
    c = codes.view(N, K // 8, 4)
    lo, hi = c & 0xF, c >> 4
    out = torch.stack([lo[..., 0] | (lo[..., 1] << 4), lo[..., 2] | (lo[..., 3] << 4),
                       hi[..., 0] | (hi[..., 1] << 4), hi[..., 2] | (hi[..., 3] << 4)], dim=-1)
    return out.reshape(N, K // 2).contiguous()


# NIB-layout variants: same k order and accumulation order as their row-major twins
B32_NIB = {66: 45, 67: 46, 69: 45, 71: 45, 75: 45, 77: 45, 81: 45, 99: 45, 152: 150, 153: 151, 163: 162, 165: 164, 168: 170, 169: 170, 172: 171}


@pytest.mark.parametrize("M", [300, 512, 1024])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("group", [-2, 128, 64])
def test_w4a16_prefill_default(K, M, sym, group):
    """The product prefill path (default dispatch, row-major and NIB codes, with and without the split-K
    workspace) vs an fp32 GEMM on the bit-exact dequantized weight; both code layouts give the same
    bits wherever they take the same kernel."""
    N, Kd = 512, 4352
    torch.manual_seed(2)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 93)
    r = K.quantize_minmax(w, 4, group, sym, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    nib = K.nib_codes(r.codes, N, Kd)
    y0 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b)
    assert bool(((y0.float() - ref).abs() <= tol).all()), float((y0.float() - ref).abs().max())
    assert torch.equal(y0, K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, group, N, b, nib=True))
    # without a workspace (iwq_w4a16_gemm): the unsplit kernels, row-major and NIB, same bits
    L = K.L
    lib = L.load()
    ys = []
    for cd, fl in ((r.codes, 0), (nib, L.IWQ_FLAG_NIB_CODES)):
        y1 = torch.empty(M, N, dtype=torch.float16, device=DEV)
        st = lib.iwq_w4a16_gemm(L.ptr(x), M, Kd, Kd, L.ptr(cd), L.ptr(r.scales), L.ptr(r.zeros), 4, group, N,
                                L.ptr(b), L.ptr(y1), N, fl, L.stream_handle(x.device))
        assert st == 0, st
        assert bool(((y1.float() - ref).abs() <= tol).all())
        ys.append(y1)
    if M >= 512:  # below, a row-major call without the split's workspace takes the mid-M kernel
        assert torch.equal(ys[0], ys[1])


@needs_ab
@pytest.mark.parametrize("M", [300, 512, 1024])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("group", [-2, 128, 64])
def test_w4a16_prefill_b32(K, M, sym, group):
    """The 32x32x16 prefill kernel (iwq_prefill.hip, variants 40-44) vs an fp32 GEMM on the bit-exact
    dequantized weight; variants that differ only in scheduling give identical bits."""
    N, Kd = 512, 4352
    torch.manual_seed(2)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 93)
    r = K.quantize_minmax(w, 4, group, sym, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    ys = {}
    for v in B32_ALL:
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        err = (y.float() - ref).abs()
        assert bool((err <= tol).all()), (v, float(err.max()))
        ys[v] = y
    for vs in (B32_SETS_PC if group == -2 else B32_SETS_G):
        for v in vs[1:]:
            assert torch.equal(ys[v], ys[vs[0]]), (vs[0], v)
    nib = nib_layout(r.codes, N, Kd)
    for v, twin in B32_NIB.items():
        if group != -2 and v in (67, 71, 77, 81, 99):
            continue  # grouped: one exact kernel, variant 66
        y = K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, ys[twin if group == -2 or v in (152, 153, 163, 165, 168, 169, 172) else 45]), (v, twin)  # grouped: 75 = 45


def test_nib_codes_layout(K):
    """iwq_nib_codes (one HIP pass, in place or not) == the torch restatement of the NIB layout, and
    decoding it back with the nibble permutation (0,2,4,6,1,3,5,7) returns the row-major codes."""
    torch.manual_seed(11)
    for N, Kd in ((256, 4096), (48, 96), (11008, 4096)):
        codes = torch.randint(0, 256, (N, Kd // 2), dtype=torch.uint8, device=DEV)
        ref = nib_layout(codes, N, Kd)
        got = K.nib_codes(codes, N, Kd)
        assert torch.equal(got, ref), (N, Kd)
        perm = (0, 2, 4, 6, 1, 3, 5, 7)
        g32 = got.view(torch.int32).view(N, Kd // 8).cpu().numpy().view("uint32")
        nib = np.stack([(g32 >> (4 * p)) & 0xF for p in range(8)], axis=-1)
        back = np.empty_like(nib)
        back[..., list(perm)] = nib
        c = codes.cpu().numpy().reshape(N, Kd // 2)
        rm = np.stack([c & 0xF, c >> 4], axis=-1).reshape(N, Kd // 8, 8)
        assert np.array_equal(back, rm)
        inplace = codes.clone()
        K.nib_codes(inplace, N, Kd, out=inplace)
        assert torch.equal(inplace, ref)


@pytest.mark.parametrize("M", [256, 300, 1024, 4096])
@pytest.mark.parametrize("group", [-2, 128, 64])
def test_w4a16_nib_default(K, M, group):
    """iwq_w4a16_gemm with IWQ_FLAG_NIB_CODES (74's NIB twin, split-K or not by the same rule)
    returns the default row-major path's bits; below 256 rows the NIB layout is refused."""
    N, Kd = (2048, 4096) if M == 4096 else (512, 4352)
    torch.manual_seed(12)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 95)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    nib = K.nib_codes(r.codes, N, Kd)
    y0 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b)
    y1 = K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, group, N, b, nib=True)
    assert torch.equal(y0, y1)
    if AB:  # without a workspace the NIB path runs unsplit: 74 vs 75, 151 vs 153 on the same shapes
        y74 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(74))
        y75 = K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(75))
        assert torch.equal(y74, y75)
        y151 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(151))
        y153 = K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(153))
        assert torch.equal(y151, y153)
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    assert bool(((y1.float() - ref).abs() <= tol).all())
    with pytest.raises(ValueError):
        K.w4a16_gemm(x[:255], nib, r.scales, r.zeros, 4, group, N, b, nib=True)
    if K.packed_fused_preferred(M, N, Kd, group):  # else w4a16_linear dequantizes once for hipBLASLt
        yl = K.w4a16_linear(x, r.codes, r.scales, r.zeros, 4, group, N, b, nib_codes=nib)
        assert torch.equal(yl, y0)


@pytest.mark.parametrize("M,N,Kd", [(256, 4096, 4096), (512, 512, 4608), (2304, 768, 2304)])
@pytest.mark.parametrize("group,sym", [(128, False), (64, True), (256, False), (192, False)])
def test_w4a16_group_major_params(K, M, N, Kd, group, sym):
    """IWQ_FLAG_GROUP_MAJOR: the prefill kernel reading group-major copies of the parameters returns the
    bits of the reference-order call on the same kernel, row-major and NIB codes; where it does not
    apply (split-K wanted, M < 256, per channel, variants) the C-ABI refuses it and w4a16_gemm keeps the
    reference-order parameters."""
    if Kd % group:
        pytest.skip("group must divide K")
    torch.manual_seed(21)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 97)
    r = K.quantize_minmax(w, 4, group, sym, 0, want_codes=True)
    sgm, zgm = K.group_major_params(r.scales, r.zeros, N, Kd, group)
    gpr = Kd // group
    assert torch.equal(sgm.view(gpr, N), r.scales.view(N, gpr).t())
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    nib = K.nib_codes(r.codes, N, Kd)
    L = K.L
    lib = L.load()

    def raw(cd, sc, zr, fl, m=M):
        y = torch.empty(m, N, dtype=torch.float16, device=DEV)
        st = lib.iwq_w4a16_gemm(L.ptr(x), m, Kd, Kd, L.ptr(cd), L.ptr(sc), L.ptr(zr), 4, group, N, L.ptr(b),
                                L.ptr(y), N, fl, L.stream_handle(x.device))
        return st, y
    # unsplit prefill kernel, reference order (NIB flag: the prefill kernel at any M >= 256) vs group-major
    st0, y0 = raw(nib, r.scales, r.zeros, L.IWQ_FLAG_NIB_CODES)
    st1, y1 = raw(nib, sgm, zgm, L.IWQ_FLAG_NIB_CODES | L.IWQ_FLAG_GROUP_MAJOR)
    st2, y2 = raw(r.codes, sgm, zgm, L.IWQ_FLAG_GROUP_MAJOR)
    assert (st0, st1, st2) == (0, 0, 0)
    assert torch.equal(y0, y1) and torch.equal(y0, y2)
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    assert bool(((y1.float() - ref).abs() <= tol).all())
    # the Python face: group-major where gm_prefill_applies, else the reference order -- same bits either way
    yk = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, scales_gm=sgm, zeros_gm=zgm)
    yd = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b)
    assert torch.equal(yk, yd)
    if K.gm_prefill_applies(M, N, Kd, group):
        assert torch.equal(yk, y2)
    # refusals
    assert raw(r.codes, sgm, zgm, L.IWQ_FLAG_GROUP_MAJOR, m=255)[0] == L.IWQ_ERR_ARG
    assert raw(r.codes, sgm, zgm, L.IWQ_FLAG_GROUP_MAJOR | L.IWQ_FLAG_FORCE_GENERIC)[0] == L.IWQ_ERR_ARG
    st, y150 = raw(r.codes, sgm, zgm, L.IWQ_FLAG_GROUP_MAJOR | K.gemm_variant_flags(150))
    if AB:  # the A/B library takes the grouped 16x16x32 variants on group-major parameters (gmNNN arms)
        assert st == 0 and torch.equal(y150, y2)
    else:
        assert st == L.IWQ_ERR_ARG


def test_w4a16_group_major_refuses_per_channel(K):
    N, Kd, M = 512, 1024, 512
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 98)
    r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    y = torch.empty(M, N, dtype=torch.float16, device=DEV)
    L = K.L
    st = L.load().iwq_w4a16_gemm(L.ptr(x), M, Kd, Kd, L.ptr(r.codes), L.ptr(r.scales), L.ptr(r.zeros), 4, -2, N,
                                 None, L.ptr(y), N, L.IWQ_FLAG_GROUP_MAJOR, L.stream_handle(x.device))
    assert st == L.IWQ_ERR_ARG
    with pytest.raises(ValueError):
        K.group_major_params(r.scales, r.zeros, N, Kd, -2)


@pytest.mark.parametrize("group", [128, -2])
def test_quantlinear_group_major_params(K, group):
    """fused_forward=True on grouped weights keeps group-major parameter copies (non-persistent, dropped
    on load); the forward reads them at prefill sizes: the same bits as the reference-order call."""
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    lin = torch.nn.Linear(1024, 512, bias=True).half().to(DEV)
    q = QuantLinear.from_linear(lin, w_bit=4, w_group_size=group, symmetric=False, fused_forward=True)
    if group == -2:
        assert q.scales_gm is None and q.zeros_gm is None
        return
    assert q.scales_gm is not None and "scales_gm" not in q.state_dict()
    assert torch.equal(q.scales_gm.view(1024 // group, 512), q.scales.view(512, -1).t())
    z = q.zeros.view(-1)
    for shape in ((2, 300, 1024), (100, 1024), (1024, 1024)):
        x = torch.randn(*shape, device=DEV).half()
        ref = K.w4a16_gemm(x, q.qweight, q.scales.view(-1), z, 4, group, 512, q.bias)
        assert torch.equal(q(x), ref), shape
    q.load_state_dict(q.state_dict())
    assert q.scales_gm is None and q.zeros_gm is None


@pytest.mark.parametrize("M", [256, 384])
@pytest.mark.parametrize("group", [-2, 128])
def test_w4a16_nib_default_wide_unsplit(K, M, group):
    """Wide weights (Llama-2-70B gate/up: N = 28672, K = 8192) at 256 <= M < 512: the split model
    picks ONE range (224 tiles), and the row-major default must then take the unsplit prefill
    kernel like the NIB path does (not the mid-M kernel): same bits, within tolerance of fp32."""
    N, Kd = 28672, 8192
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 96)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    del w
    torch.manual_seed(13)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    nib = K.nib_codes(r.codes, N, Kd)
    y0 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N)
    y1 = K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, group, N, nib=True)
    assert torch.equal(y0, y1)
    ref = x.float() @ r.out.float().t()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    assert bool(((y0.float() - ref).abs() <= tol).all())


@pytest.mark.parametrize("M", [64, 512])
def test_w4a16_split_misaligned_y(K, M):
    """A y that is only 2-B aligned cannot take the split reduces' 8-B stores: the C-ABI then runs
    the unsplit kernels instead (the workspace is dropped), and the result stays correct."""
    N, Kd = 512, 4352
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 97)
    r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
    torch.manual_seed(14)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    buf = torch.full((M * N + 1,), float("nan"), dtype=torch.float16, device=DEV)
    y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, out=buf[1:])
    assert y.data_ptr() % 8 == 2
    assert torch.isnan(buf[0])
    ref = x.float() @ r.out.float().t()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    assert bool(((y.float() - ref).abs() <= tol).all())


@pytest.mark.parametrize("M", [200, 256, 300, 512, 1024])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("group", [-2, 128])
def test_w4a16_prefill_splitk(K, M, sym, group):
    """Split-K prefill (iwq_w4a16_gemm_ws: fp32 partial tiles summed in range order by a second
    kernel): within the fp16 tolerance of an fp32 GEMM on the bit-exact dequantized weight for the
    default split and forced 2/4/8/15 ranges (15 > K-steps / 2 clamps), deterministic, and A = I
    still picks W_deq^T exactly (every partial but one is an exact 0)."""
    N, Kd = 512, 4352
    torch.manual_seed(3)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 94)
    r = K.quantize_minmax(w, 4, group, sym, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    ys = {}
    for v in (0,) + abv(82, 84, 88, 95, 96):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        err = (y.float() - ref).abs()
        assert bool((err <= tol).all()), (v, float(err.max()))
        y2 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, y2), v
        ys[v] = y
    # partials from the hand-ordered kernel (default) and the first split kernel (96): same k order,
    # same reduce -> same bits (below M = 256 this small weight takes the mid-M kernel by default)
    if M >= 256 and AB:
        assert torch.equal(ys[0], ys[96])
    xi = torch.eye(Kd, device=DEV, dtype=torch.float16)[:M].contiguous()
    for v in (0,) + abv(84, 95):
        y = K.w4a16_gemm(xi, r.codes, r.scales, r.zeros, 4, group, N, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, r.out[:, :M].t().contiguous()), v


@pytest.mark.parametrize("M", [17, 64, 100, 128, 200])
@pytest.mark.parametrize("group", [-2, 128])
def test_w4a16_short_tile_split(K, M, group):
    """Short-tile split prefill (k_w4a16_b32s: 128- / 64-row tiles, variants 110-145 force the tile
    and the K ranges): within the fp16 tolerance of an fp32 GEMM, deterministic, and A = I picks
    W_deq^T exactly."""
    N, Kd = 512, 4352
    torch.manual_seed(7)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 98)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    for v in (0,) + abv(110, 112, 117, 130, 132, 140):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        err = (y.float() - ref).abs()
        assert bool((err <= tol).all()), (v, float(err.max()))
        y2 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, y2), v
    xi = torch.eye(Kd, device=DEV, dtype=torch.float16)[:M].contiguous()
    for v in (0,) + abv(112, 132):
        y = K.w4a16_gemm(xi, r.codes, r.scales, r.zeros, 4, group, N, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, r.out[:, :M].t().contiguous()), v


def test_w4a16_midm_split_default(K):
    """16 < M < 256 on a gate_proj-shaped weight: the default takes the split the plan prefers
    (round 5, N >= 8192: 128-row tiles -- M = 128: 4 K ranges, M = 200: 2 K ranges) -- same bits as
    forcing that plan, within tolerance of fp32."""
    if torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("the modelled split count is for 256 CUs")
    N, Kd, M = 11008, 4096, 128
    torch.manual_seed(6)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 97)
    r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    ref = x.float() @ r.out.float().t()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    y0 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N)
    assert bool(((y0.float() - ref).abs() <= tol).all())
    x2 = (torch.randn(200, Kd, device=DEV) * 0.5).half()
    z0 = K.w4a16_gemm(x2, r.codes, r.scales, r.zeros, 4, -2, N)
    torch.testing.assert_close(z0.float(), x2.float() @ r.out.float().t(), rtol=2e-2, atol=2e-2)
    if AB:
        y4 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, flags=K.gemm_variant_flags(112))
        assert torch.equal(y0, y4)
        z4 = K.w4a16_gemm(x2, r.codes, r.scales, r.zeros, 4, -2, N, flags=K.gemm_variant_flags(110))
        assert torch.equal(z0, z4)


def test_w4a16_splitk_workspace_rule(K):
    """iwq_w4a16_gemm_workspace_bytes: the split the time model picks (iwq_prefill.hip
    prefill_splitk_count, 256 CUs), sized tiles x ranges x 256 KiB; none where the prefill kernel
    does not run (N % 256), where splitting does not pay, or (16 < M < 256) where the mid-M kernel
    is modelled faster (prefill_split_preferred)."""
    lib = K.L.load()
    if torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("expected split counts are for 256 CUs")
    tile = 65536 * 4
    assert lib.iwq_w4a16_gemm_workspace_bytes(128, 4096, 4096, -2) == 0  # mid-M kernel modelled faster
    short = 2 * 8192 * 4  # one 64-row partial tile (prefill_short_split)
    assert lib.iwq_w4a16_gemm_workspace_bytes(64, 4096, 4096, -2) == 0  # mid-M kernel
    assert lib.iwq_w4a16_gemm_workspace_bytes(64, 11008, 4096, -2) == 43 * 5 * short
    assert lib.iwq_w4a16_gemm_workspace_bytes(64, 4096, 11008, -2) == 16 * 12 * short
    # 64 < M <= 128 on wide weights: 128-row tiles (twice the partial bytes), S = min(256 / tiles, nk / 16, 8)
    assert lib.iwq_w4a16_gemm_workspace_bytes(128, 11008, 4096, -2) == 43 * 4 * 2 * short
    assert lib.iwq_w4a16_gemm_workspace_bytes(128, 28672, 8192, 128) == 112 * 2 * 2 * short
    assert lib.iwq_w4a16_gemm_workspace_bytes(96, 8192, 28672, -2) == 32 * 8 * 2 * short
    assert lib.iwq_w4a16_gemm_workspace_bytes(96, 4096, 11008, -2) == 32 * 8 * short  # N = 4096: 64-row
    assert lib.iwq_w4a16_gemm_workspace_bytes(192, 8192, 28672, 128) == 64 * 4 * 2 * short  # <= 128 tiles
    assert lib.iwq_w4a16_gemm_workspace_bytes(200, 4096, 11008, -2) == 64 * 4 * short  # short: 4 x 16 tiles
    assert lib.iwq_w4a16_gemm_workspace_bytes(200, 11008, 4096, -2) == 86 * 2 * 2 * short  # wide: 128-row tiles
    assert lib.iwq_w4a16_gemm_workspace_bytes(16, 11008, 4096, -2) == 0  # decode GEMV
    assert lib.iwq_w4a16_gemm_workspace_bytes(256, 4096, 4096, -2) == 16 * 8 * tile
    assert lib.iwq_w4a16_gemm_workspace_bytes(512, 4096, 4096, -2) == 32 * 5 * tile
    assert lib.iwq_w4a16_gemm_workspace_bytes(512, 11008, 4096, 128) == 86 * 2 * tile
    assert lib.iwq_w4a16_gemm_workspace_bytes(1024, 11008, 4096, -2) == 0  # 172 tiles: no gain
    assert lib.iwq_w4a16_gemm_workspace_bytes(1024, 4096, 11008, -2) == 64 * 4 * tile
    assert lib.iwq_w4a16_gemm_workspace_bytes(8192, 4096, 4096, -2) == 0  # 512 tiles
    assert lib.iwq_w4a16_gemm_workspace_bytes(512, 4224, 4096, -2) == 0  # N % 256 != 0: no prefill kernel


@pytest.mark.parametrize("group", [-2, 128])
def test_w4a16_prefill_b32_identity(K, group):
    """A = I through the 32x32x16 prefill kernel picks W_deq^T exactly for every variant (operand k
    order, LDS swizzles, C layout; factored scale: s * (q - z) is exact in fp32)."""
    N, Kd = 768, 512
    w = (torch.arange(N * Kd, device=DEV, dtype=torch.float32).reshape(N, Kd) % 13 - 6).half()
    w[:, 128:256] *= 0.25  # a different scale per group along k
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    x = torch.eye(Kd, device=DEV, dtype=torch.float16)
    for v in (0,) + abv(*B32_ALL):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, r.out.t().contiguous()), v


@pytest.mark.parametrize("Kd", [128, 256, 384])
def test_w4a16_prefill_short_k(K, Kd):
    """2, 4, 6 K-steps (the C-ABI takes K % 128 == 0) through the hand-ordered kernels (prologue,
    peeled last step, the 2- / 3-stage rings' wrap): identical bits to variant 45 (NIB twins on NIB
    codes)."""
    N, M = 512, 300
    torch.manual_seed(5)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 96)
    r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    y0 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, b)
    assert bool(((y0.float() - ref).abs() <= tol).all())
    if not AB:
        return
    y45 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(45))
    assert bool(((y45.float() - ref).abs() <= tol).all())
    for v in (70, 74, 76, 78, 79, 80):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, y45), v
    for v in (110, 112, 130, 132, 150, 151):  # short-tile splits: 1-3 K-steps per range; 16x16x32 forms
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(v))
        assert bool(((y.float() - ref).abs() <= tol).all()), v
    nib = nib_layout(r.codes, N, Kd)
    for v in (71, 75, 77, 81):
        y = K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, y45), v
    y150 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(150))
    for v, cd in ((151, r.codes), (152, nib), (153, nib), (162, r.codes), (163, nib), (164, r.codes), (165, nib), (168, nib), (169, nib), (170, r.codes), (171, r.codes), (172, nib)):  # 16x16x32 forms: one set of bits
        y = K.w4a16_gemm(x, cd, r.scales, r.zeros, 4, -2, N, b, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, y150), v


@needs_ab
@pytest.mark.parametrize("M", [2560, 2600])
@pytest.mark.parametrize("group", [-2, 128])
def test_w4a16_prefill_persistent_many_tiles(K, M, group):
    """The persistent prefill (k_w4a16_b16p, 171 / NIB 172) with more tiles than CUs (320 / 352
    tiles: workgroups walk two, the DMA stream crossing tile boundaries; a partial last row tile at
    M = 2600): the bits of the one-tile-per-workgroup forms (162 / 151), within fp32 tolerance."""
    N, Kd = 8192, 512
    torch.manual_seed(21)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 99)
    r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    nib = nib_layout(r.codes, N, Kd)
    y162 = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(162))
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    assert bool(((y162.float() - ref).abs() <= tol).all())
    for v, cd in ((171, r.codes), (172, nib), (151, r.codes)):
        y = K.w4a16_gemm(x, cd, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        assert torch.equal(y, y162), v


MID_VARIANTS = (50, 51, 52, 53, 54, 55)  # k_w4a16_mid: (MT row tiles, CT column tiles) shapes


@pytest.mark.parametrize("M", [17, 40, 64, 100, 257])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("group", [-2, 128, 32])
def test_w4a16_mid(K, M, sym, group):
    """The mid-M weight-streaming kernel (iwq_prefill.hip k_w4a16_mid, variants 50-55; row tiles past
    M) vs an fp32 GEMM on the bit-exact dequantized weight."""
    N, Kd = 256, 2304
    torch.manual_seed(3)
    w = torch.empty(N, Kd, dtype=torch.float16, device=DEV)
    K.fill_synthetic(w, 95)
    r = K.quantize_minmax(w, 4, group, sym, 0, want_codes=True)
    x = (torch.randn(M, Kd, device=DEV) * 0.5).half()
    b = (torch.randn(N, device=DEV) * 0.1).half()
    ref = x.float() @ r.out.float().t() + b.float()
    tol = 2e-3 * ref.abs() + 1e-3 * (x.float().abs() @ r.out.float().abs().t()).max() / Kd ** 0.5 + 1e-3
    for v in abv(*MID_VARIANTS) + (0,):
        y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, b, flags=K.gemm_variant_flags(v))
        err = (y.float() - ref).abs()
        assert bool((err <= tol).all()), (v, float(err.max()))


def test_w4a16_mid_identity(K):
    """A = I (rows 0..M-1 of the identity) through every mid-M variant picks W_deq^T rows exactly."""
    N, Kd = 256, 512
    w = (torch.arange(N * Kd, device=DEV, dtype=torch.float32).reshape(N, Kd) % 13 - 6).half()
    for group in (-2, 128):
        r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
        for M in (48, 130):
            x = torch.eye(Kd, device=DEV, dtype=torch.float16)[:M].contiguous()
            for v in (0,) + abv(*MID_VARIANTS):
                y = K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, flags=K.gemm_variant_flags(v))
                assert torch.equal(y, r.out.t()[:M].contiguous()), (group, M, v)

"""Parity at the sizes that are timed and named in BASELINE.json's configs (bit-exact unless noted):

* configs[1]: the bench's whole-model batched launch (all 224 Llama-2-7B Linear weights, exactly
  bench.make_weights' synthetic set, ONE k_group launch) gives every tensor the single-call bits,
  and the tensors whose inputs match tests/golden/int_large.json give the reference's SHA-256s;
* configs[3]: the four Llama-2-70B Linear shapes against SHA-256s of the reference's own outputs
  (tests/golden/int_large_70b.json, made by tests/golden/make_golden.py), and one rank's 8-way
  shard.plan_shards bin quantized in place through BatchPlan exactly as bench.py --model llama2-70b;
* configs[2]: the per-channel (and g128) fused dequant+GEMM forward at its PPL batch M = 8192
  (4 x 2048) on the Llama-2-7B shapes, within the fp16 output tolerance of an fp32 GEMM on the
  dequantized weight whose bits are pinned to the reference's SHA-256.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import iwq_oracle as O

from .golden_util import GOLD, sha

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def K():
    from iron_weight_only_quant_amd import kernels
    return kernels


def _np(t):
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:  # the bit patterns, as the golden generator hashes them
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def _cases(fname):
    return json.load(open(os.path.join(GOLD, fname)))["cases"]


def _check_case(K, x, c):
    """One golden case (int_large*.json) on the single-tensor C-ABI path."""
    if c["kind"] == "qf":
        g = c["q_group_size"]
        r = K.quantize_minmax(x, c["n_bits"], g if g > 0 else -2, not c["zero_point"], 0)
        assert not r.has_nan()
        assert sha(_np(r.out)) == c["sha_deq"], c
    else:
        r = K.quantize_minmax(x, c["w_bit"], c["w_group_size"], c["symmetric"], 0)
        assert sha(_np(r.out)) == c["sha_deq"], c
        assert sha(_np(r.scales).reshape(-1, 1)) == c["sha_scales"], c
        if c["sha_zeros"] is not None:
            assert sha(_np(r.zeros).reshape(-1, 1)) == c["sha_zeros"], c


def _golden_by_seed(fname):
    out = {}
    for c in _cases(fname):
        out.setdefault(c["seed"], []).append(c)
    return out


def _bench_config_case(cases):
    return [c for c in cases if c["kind"] == "ql" and c["w_bit"] == 4 and not c["symmetric"]
            and c["w_group_size"] == 128][0]


def test_bench_batched_7b_every_tensor_matches_single_and_reference(K):
    """configs[1] at full size: bench.py's exact workload (shard.model_linear_shapes("llama2-7b"),
    seeds 0..223 = bench.make_weights at N = 1) in ONE batched launch, out of place, INT4 g128 asym;
    plus layer 0's gate / down regenerated with int_large.json's seeds 1 / 2 as two extra entries
    of the same launch.  Every tensor's dequantized weight, scales and zeros equal its own
    quantize_minmax call; the seed-0/1/2 tensors equal the reference's SHA-256s."""
    from iron_weight_only_quant_amd import shard
    shapes = shard.model_linear_shapes("llama2-7b")
    seeds = list(range(len(shapes))) + [1, 2]
    shp = [s for _, s in shapes] + [(11008, 4096), (4096, 11008)]
    ws = []
    for seed, s in zip(seeds, shp):
        t = torch.empty(s, dtype=torch.float16, device=DEV)
        K.fill_synthetic(t, seed)
        ws.append(t)
    plan = K.BatchPlan(ws, 4, 128, False)
    assert len(plan.launches) == 1  # ONE launch for the whole model
    plan.run()
    torch.cuda.synchronize()
    assert plan.nan_flag.item() == 0
    for i, w in enumerate(ws):
        r = K.quantize_minmax(w, 4, 128, False, 0)
        assert torch.equal(plan.outs[i].view(torch.int16), r.out.view(torch.int16)), i
        assert torch.equal(plan.scales[i].view(torch.int16), r.scales.view(torch.int16)), i
        assert torch.equal(plan.zeros[i].view(torch.int16), r.zeros.view(torch.int16)), i
        del r
    gold = _golden_by_seed("int_large.json")
    for i, seed in ((0, 0), (len(shapes), 1), (len(shapes) + 1, 2)):
        inp = [c for c in gold[seed] if c["kind"] == "input"][0]
        assert tuple(inp["shape"]) == tuple(ws[i].shape)
        assert sha(_np(ws[i])) == inp["sha_input"]
        c = _bench_config_case(gold[seed])
        assert sha(_np(plan.outs[i])) == c["sha_deq"], (i, seed)
        assert sha(_np(plan.scales[i]).reshape(-1, 1)) == c["sha_scales"], (i, seed)
        assert sha(_np(plan.zeros[i]).reshape(-1, 1)) == c["sha_zeros"], (i, seed)


@pytest.mark.parametrize("name", ["q_proj", "k_proj", "gate_proj", "down_proj"])
def test_llama70b_shapes_vs_reference_sha(K, name):
    """configs[3] shapes on the single-tensor path: SHA-256 equal to the reference's own outputs."""
    cases = [c for c in _cases("int_large_70b.json") if c["name"] == name]
    inp = cases[0]
    x = torch.empty(tuple(inp["shape"]), dtype=torch.float16, device=DEV)
    K.fill_synthetic(x, inp["seed"])
    assert sha(_np(x)) == inp["sha_input"]
    for c in cases[1:]:
        _check_case(K, x, c)


def test_llama70b_rank_bin_in_place(K):
    """bench.py --model llama2-70b --gpus 8, rank 0's bin (shard.plan_shards(70B, 8)[0]: ~70 weights,
    ~17 GB) quantized IN PLACE in one batched launch with packed codes (as --gather keeps them).
    The first weight of each shape in the bin is regenerated with the 70B golden seed of that shape
    and must give the reference's SHA-256s; every weight equals its own single call, codes too."""
    from iron_weight_only_quant_amd import shard
    shapes = shard.model_linear_shapes("llama2-70b")
    bin0 = shard.plan_shards(shapes, 8)[0]
    gold = {tuple(c["shape"]): c for c in _cases("int_large_70b.json") if c["kind"] == "input"}
    golden_cases = _cases("int_large_70b.json")
    seeds, pinned = [], {}
    for i in bin0:
        s = shapes[i][1]
        if s in gold and s not in pinned:
            pinned[s] = len(seeds)
            seeds.append(gold[s]["seed"])
        else:
            seeds.append(100_000 + i)
    assert len(pinned) >= 3, pinned  # the bin holds (almost) every 70B shape
    ws = []
    for i, seed in zip(bin0, seeds):
        t = torch.empty(shapes[i][1], dtype=torch.float16, device=DEV)
        K.fill_synthetic(t, seed)
        ws.append(t)
    plan = K.BatchPlan(ws, 4, 128, False, outs=ws, want_codes=True)
    plan.run()
    torch.cuda.synchronize()
    assert plan.nan_flag.item() == 0
    for k, (i, seed) in enumerate(zip(bin0, seeds)):
        x = torch.empty(shapes[i][1], dtype=torch.float16, device=DEV)
        K.fill_synthetic(x, seed)
        r = K.quantize_minmax(x, 4, 128, False, 0, out=x, want_codes=True)
        assert torch.equal(ws[k].view(torch.int16), x.view(torch.int16)), k
        assert torch.equal(plan.scales[k].view(torch.int16), r.scales.view(torch.int16)), k
        assert torch.equal(plan.zeros[k].view(torch.int16), r.zeros.view(torch.int16)), k
        assert torch.equal(plan.codes[k], r.codes), k
        del x, r
    for s, k in pinned.items():
        c = [c for c in golden_cases if tuple(c["shape"]) == s and c["kind"] == "ql" and c["w_bit"] == 4
             and not c["symmetric"] and c["w_group_size"] == 128][0]
        assert sha(_np(ws[k])) == c["sha_deq"], s
        assert sha(_np(plan.scales[k]).reshape(-1, 1)) == c["sha_scales"], s
        assert sha(_np(plan.zeros[k]).reshape(-1, 1)) == c["sha_zeros"], s


@pytest.mark.parametrize("name", ["q_proj", "gate_proj", "down_proj"])
@pytest.mark.parametrize("group", [-2, 128])
def test_config3_fused_forward_m8192(K, name, group):
    """configs[2]: QuantLinear(fused_forward=True) -- the packed-code MFMA prefill kernel -- at the
    PPL batch M = 4 x 2048 = 8192 on the Llama-2-7B shape, per channel and g128.  The dequantized
    weight the kernel reads is pinned to the reference (SHA-256 of QuantLinear.from_linear's output
    on the same input); the GEMM is compared with an fp32 GEMM on that weight.
    Tolerance: |y - ref| <= 2e-3 |ref| + 1e-3 max|x||W| / sqrt(K) + 1e-3 (fp16 output rounding plus
    fp32 accumulation-order differences over K = 4096 / 11008)."""
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    gold = [c for c in _cases("int_large.json") if c["name"] == name]
    inp = gold[0]
    N, Kd = inp["shape"]
    lin = torch.nn.Linear(Kd, N, bias=False, dtype=torch.float16, device=DEV)
    K.fill_synthetic(lin.weight.data, inp["seed"])
    q = QuantLinear.from_linear(lin, w_bit=4, w_group_size=group, symmetric=False, fused_forward=True)
    c = [c for c in gold if c["kind"] == "ql" and c["w_bit"] == 4 and not c["symmetric"]
         and c["w_group_size"] == group][0]
    assert sha(_np(q.weight.data)) == c["sha_deq"]
    assert sha(_np(q.scales)) == c["sha_scales"]
    torch.manual_seed(21)
    x = (torch.randn(4, 2048, Kd, device=DEV) * 0.5).half()
    y = q(x)
    assert y.shape == (4, 2048, N)
    y2 = y.reshape(-1, N)
    x2 = x.reshape(-1, Kd).float()
    W = q.weight.data.float()
    worst = 0.0
    for r0 in range(0, 8192, 2048):  # fp32 reference in slices (memory)
        ref = x2[r0:r0 + 2048] @ W.t()
        bound = (x2[r0:r0 + 2048].abs() @ W.abs().t()).max() / Kd ** 0.5
        tol = 2e-3 * ref.abs() + 1e-3 * bound + 1e-3
        err = (y2[r0:r0 + 2048].float() - ref).abs()
        assert bool((err <= tol).all()), (name, group, r0, float((err - tol).max()))
        worst = max(worst, float((err / tol).max()))
    # and the reference forward itself (F.linear on the dequantized weight) agrees to the same bound
    yl = torch.nn.functional.linear(x, q.weight)
    assert float(((yl.float() - y.float()).abs()).max()) < 0.05, float(((yl.float() - y.float()).abs()).max())
    assert worst <= 1.0


@pytest.mark.parametrize("name", ["q_proj", "gate_proj", "down_proj"])
def test_per_tensor_one_pass_full_size(K, name):
    """Per-tensor (-1) on the single-call path at the Llama-2-7B shapes: the one-pass kernel (the
    whole weight held in registers, per-workgroup keys exchanged inside the launch) equals the
    reference's SHA-256s (tests/golden/int_large_pt.json: pseudo_quantize_tensor(per_tensor=True)
    and QuantLinear w_group_size=-1) and the two-kernel pair (variant 6), in place and out of place,
    with packed codes; the exchange's timeout bit (nan_flag & 2) never fires."""
    cases = [c for c in _cases("int_large_pt.json") if c["name"] == name]
    inp = cases[0]
    x = torch.empty(tuple(inp["shape"]), dtype=torch.float16, device=DEV)
    K.fill_synthetic(x, inp["seed"])
    assert sha(_np(x)) == inp["sha_input"]
    for c in cases[1:]:
        if c["kind"] == "qf_pt":
            r = K.quantize_minmax(x, c["n_bits"], -1, not c["zero_point"], 0)
            assert int(r.nan_flag.item()) == 0
            assert sha(_np(r.out)) == c["sha_deq"], c
        else:
            r = K.quantize_minmax(x, c["w_bit"], -1, c["symmetric"], 0, want_codes=True)
            assert int(r.nan_flag.item()) == 0
            assert sha(_np(r.out)) == c["sha_deq"], c
            assert sha(_np(r.scales).reshape(-1, 1)) == c["sha_scales"], c
            if c["sha_zeros"] is not None:
                assert sha(_np(r.zeros).reshape(-1, 1)) == c["sha_zeros"], c
            r6 = K.quantize_minmax(x, c["w_bit"], -1, c["symmetric"], 0, want_codes=True,
                                   flags=K.gemm_variant_flags(6))
            assert torch.equal(r6.out.view(torch.int16), r.out.view(torch.int16))
            assert torch.equal(r6.codes, r.codes)
            y = x.clone()
            ri = K.quantize_minmax(y, c["w_bit"], -1, c["symmetric"], 0, out=y)
            assert torch.equal(y.view(torch.int16), r.out.view(torch.int16))
            assert int(ri.nan_flag.item()) == 0


@pytest.mark.parametrize("case", [("bfloat16", "q_proj"), ("bfloat16", "gate_proj"), ("bfloat16", "down_proj"),
                                  ("float32", "q_proj")])
def test_per_tensor_one_pass_dtypes_full_size(K, case):
    """Round 5: per tensor on bf16 / fp32 weights takes the one-pass kernel too (keys in two dwords for
    fp32; the literal op chain on the register-held vectors): equal to the reference's SHA-256s
    (tests/golden/int_large_pt_dt.json: pseudo_quantize_tensor(per_tensor=True) and QuantLinear
    w_group_size=-1 on bf16 / fp32 weights), to the two-kernel pair (variant 6), and in place."""
    dtype, name = case
    td = getattr(torch, dtype)
    cases = [c for c in _cases("int_large_pt_dt.json") if c["name"] == name and c["dtype"] == dtype]
    inp = cases[0]
    x = torch.empty(tuple(inp["shape"]), dtype=td, device=DEV)
    K.fill_synthetic(x, inp["seed"])
    bits_of = (lambda t: t.view(torch.int16)) if td != torch.float32 else (lambda t: t.view(torch.int32))
    assert sha(_np(x)) == inp["sha_input"]
    for c in cases[1:]:
        if c["kind"] == "qf_pt":
            r = K.quantize_minmax(x, c["n_bits"], -1, not c["zero_point"], 0)
            assert int(r.nan_flag.item()) == 0
            assert sha(_np(r.out)) == c["sha_deq"], c
        else:
            r = K.quantize_minmax(x, c["w_bit"], -1, c["symmetric"], 0)
            assert int(r.nan_flag.item()) == 0
            assert sha(_np(r.out)) == c["sha_deq"], c
            assert sha(_np(r.scales).reshape(-1, 1)) == c["sha_scales"], c
            if c["sha_zeros"] is not None:
                assert sha(_np(r.zeros).reshape(-1, 1)) == c["sha_zeros"], c
            r6 = K.quantize_minmax(x, c["w_bit"], -1, c["symmetric"], 0, flags=K.gemm_variant_flags(6))
            assert torch.equal(bits_of(r6.out), bits_of(r.out))
            y = x.clone()
            ri = K.quantize_minmax(y, c["w_bit"], -1, c["symmetric"], 0, out=y)
            assert torch.equal(bits_of(y), bits_of(r.out))
            assert int(ri.nan_flag.item()) == 0
            # the one-pass hand-off aborted on purpose (test-only variant 9): the retry on the pair
            ra = K.quantize_minmax(x, c["w_bit"], -1, c["symmetric"], 0, flags=K.gemm_variant_flags(9))
            assert int(ra.nan_flag.item()) & 2
            assert not ra.has_nan() and ra.retried
            assert torch.equal(bits_of(ra.out), bits_of(r.out))


@pytest.mark.parametrize("shape", [(1, 8), (3, 40), (48, 256), (1000, 1000), (2048, 3000)])
@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_per_tensor_one_pass_ragged_dtypes(K, shape, dtype):
    """Small / ragged per-tensor sizes on bf16 / fp32 weights (one workgroup, partial chunks, the
    buffer range check at a 32-B vector for fp32): equal to the oracle and the pair, sym and asym."""
    from oracle.synth import synth as _synth
    x_np = _synth(91 + shape[0], shape, dtype)
    x = torch.empty(shape, dtype=getattr(torch, dtype), device=DEV)
    K.fill_synthetic(x, 91 + shape[0])
    # 4 / 8 bits: the Markstein fast path; 12 bits: bf16 leaves it (integers above 2^8), fp32 keeps it
    for bits, sym in ((4, False), (4, True), (8, False), (8, True), (12, False)):
        ref = O.quantlinear_int(x_np, w_bit=bits, w_group_size=-1, symmetric=sym, dtype=dtype)
        r = K.quantize_minmax(x, bits, -1, sym, 0)
        got = _np(r.out)
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(ref.dequant).view(np.uint8)), (shape, bits, sym)
        r6 = K.quantize_minmax(x, bits, -1, sym, 0, flags=K.gemm_variant_flags(6))
        assert np.array_equal(_np(r6.out).view(np.uint8), got.view(np.uint8))
        r8 = K.quantize_minmax(x, bits, -1, sym, 0, flags=K.gemm_variant_flags(8))  # the one pass forced
        assert np.array_equal(_np(r8.out).view(np.uint8), got.view(np.uint8))
        assert int(r.nan_flag.item()) == 0 and int(r8.nan_flag.item()) == 0
    # a constant huge tensor (range clamped to 1e-5: max|w| / s ~ 1e36 > 2^100) takes the literal
    # chain: same bits as the oracle
    big = np.full(shape, 1e30, dtype=np.float32)
    big_np = big if dtype == "float32" else O.f32_to_bf16_bits(big)
    ref = O.quantlinear_int(big_np, w_bit=4, w_group_size=-1, symmetric=False, dtype=dtype)
    xb = torch.from_numpy(np.ascontiguousarray(big_np).view(np.int32 if dtype == "float32" else np.int16))
    xb = xb.to(DEV).view(getattr(torch, dtype))
    for fl in (0, K.gemm_variant_flags(8)):
        rb = K.quantize_minmax(xb, 4, -1, False, 0, flags=fl)
        assert np.array_equal(_np(rb.out).view(np.uint8), np.ascontiguousarray(ref.dequant).view(np.uint8))
    # non-finite values take the literal chain (the fast path's preconditions fail): NaN poisons all
    y = x.clone()
    y.view(-1)[len(y.view(-1)) // 2] = float("nan")
    assert K.quantize_minmax(y, 4, -1, False, 0).has_nan()
    assert K.quantize_minmax(y, 4, -1, False, 0, flags=K.gemm_variant_flags(8)).has_nan()


@pytest.mark.parametrize("shape", [(1, 8), (3, 40), (48, 256), (1000, 1000), (2048, 3000)])
@pytest.mark.parametrize("sym", [False, True])
def test_per_tensor_one_pass_ragged(K, shape, sym):
    """Small / ragged per-tensor sizes (one workgroup, partial chunks, a last chunk's out-of-range
    buffer loads): the default (the pair below 32 MiB), the one pass forced (variant 8) and the pair
    forced (6) equal to the oracle."""
    from oracle.synth import synth as _synth
    x_np = _synth(77 + shape[0], shape, "float16")
    x = torch.from_numpy(x_np).to(DEV)
    ref = O.quantlinear_int(x_np, w_bit=4, w_group_size=-1, symmetric=sym)
    r = K.quantize_minmax(x, 4, -1, sym, 0, want_codes=shape[1] % 2 == 0)
    assert np.array_equal(_np(r.out).view(np.uint16), ref.dequant.view(np.uint16)), shape
    assert np.array_equal(_np(r.scales).view(np.uint16), ref.scales.reshape(-1).view(np.uint16))
    r6 = K.quantize_minmax(x, 4, -1, sym, 0, flags=K.gemm_variant_flags(6))
    assert torch.equal(r6.out.view(torch.int16), r.out.view(torch.int16))
    r8 = K.quantize_minmax(x, 4, -1, sym, 0, want_codes=shape[1] % 2 == 0, flags=K.gemm_variant_flags(8))
    assert torch.equal(r8.out.view(torch.int16), r.out.view(torch.int16))
    if r.codes is not None:
        assert torch.equal(r8.codes, r.codes)
    assert int(r.nan_flag.item()) == 0 and int(r8.nan_flag.item()) == 0

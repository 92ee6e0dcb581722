"""GPU: FP packed codes -> fp16 weights (iwq_dequant_fp_packed, config 5's "unpack") and the E2M1
codes of the fp4_quantize_cpu grid (iwq_fp4_grid_packed, its "pack").  Bit-exact against the fake-
quant outputs of the same quantization and, code by code, against the CPU restatement of
_fp_to_float (oracle/fp_codec.py, quant_linear.py:213-235) times the scale in fp16."""
import numpy as np
import pytest
import torch

from oracle import fp_codec as FC
from oracle.synth import synth

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def K():
    from iron_weight_only_quant_amd import kernels
    return kernels


def weights(rows, cols, seed):
    w = torch.from_numpy(synth(seed, (rows, cols), "float16")).to(DEV)
    return w


FORMATS = [(2, 1), (1, 2), (3, 2), (2, 3), (4, 3), (3, 4)]
GOLD_FORMATS = [(2, 1), (3, 2), (4, 3)]  # the formats the reference's own fixtures pin (test_fp_golden)


@pytest.mark.parametrize("em", GOLD_FORMATS)
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("group", [32, 128, -2, -1])
def test_unpack_matches_fake_quant(K, em, sym, group):
    """quantize_fp(want_codes) -> (codes, scales, zeros, out_deq); dequant_fp_packed(codes) == out_deq
    bit for bit (the QuantLinear FP branches' dequantized weight, quant_linear.py:773-777)."""
    E, M = em
    rows, cols = 96, 512
    w = weights(rows, cols, 11 + E * 7 + M)
    r = K.quantize_fp(w, E, M, group, sym, 0, want_codes=True)
    y = K.dequant_fp_packed(r.codes, r.scales, r.zeros, E, M, group, rows, cols)
    assert torch.equal(y.view(torch.int16), r.out.view(torch.int16)), (em, sym, group)


def _expected(codes_2d, scales, zeros, E, M):
    """fp16(fp16(_fp_to_float(code)) * s) (+ z), per row scale/zero (numpy float16 arithmetic = ATen's:
    fp32 op, one rounding to fp16)."""
    bias, _ = FC.fp_params(E, M)
    dec = FC.fp_to_float(codes_2d, E, M, bias).astype(np.float16)
    # each op in fp32, then one rounding to fp16 (ATen's fp16 arithmetic, spelled out): products of
    # large codes and 1e3 scales overflow fp16 to +-inf, which the kernels must give too
    with np.errstate(over="ignore"):
        out = (dec.astype(np.float32) * scales[:, None].astype(np.float32)).astype(np.float16)
        if zeros is not None:
            out = (out.astype(np.float32) + zeros[:, None].astype(np.float32)).astype(np.float16)
    return out


@pytest.mark.parametrize("em", FORMATS)
@pytest.mark.parametrize("sym", [True, False])
def test_unpack_every_code(K, em, sym):
    """Every code of the format under 64 per-row scales (subnormal to 1e3) and zero points: the
    CDNA4 conversions (E2M1, E4M3 incl. the reference's +-480 at 0x7F / 0xFF) and the table path."""
    E, M = em
    nbits = 1 + E + M
    ncode = 1 << nbits
    rows = 64
    cols = max(8, ncode)
    rng = np.random.default_rng(E * 10 + M)
    codes = np.tile(np.arange(cols) % ncode, (rows, 1)).astype(np.uint8)
    scales = np.concatenate([
        np.array([1.0, 2.0 ** -14, 2.0 ** -20, 2.0 ** -24, 1000.0, 0.5, 3.0, 65504.0 / 480.0], np.float32),
        rng.uniform(1e-4, 2.0, rows - 8).astype(np.float32)]).astype(np.float16)
    zeros = None if sym else rng.uniform(-0.5, 0.5, rows).astype(np.float16)
    exp = _expected(codes, scales, zeros, E, M)
    if nbits <= 4:
        packed = (codes[:, 0::2] | (codes[:, 1::2] << 4)).astype(np.uint8)
    else:
        packed = codes
    cd = torch.from_numpy(np.ascontiguousarray(packed).reshape(-1)).to(DEV)
    sc = torch.from_numpy(scales).to(DEV)
    zr = None if zeros is None else torch.from_numpy(zeros).to(DEV)
    y = K.dequant_fp_packed(cd, sc, zr, E, M, -2, rows, cols).cpu().numpy()
    assert np.array_equal(y.view(np.uint16), exp.view(np.uint16)), (
        em, np.argwhere(y.view(np.uint16) != exp.view(np.uint16))[:8])


@pytest.mark.parametrize("group,per_tensor", [(128, False), (32, False), (0, False), (128, True)])
def test_grid_pack_unpack(K, group, per_tensor):
    """fp4_grid(want_codes=True): same output as the table path, and its E2M1 codes unpack to it."""
    rows, cols = 64, 1024
    w = weights(rows, cols, 5)
    a = K.fp4_grid(w, group, per_tensor)
    b = K.fp4_grid(w, group, per_tensor, want_codes=True)
    assert torch.equal(a.out.view(torch.int16), b.out.view(torch.int16))
    assert torch.equal(a.scales.view(torch.int16), b.scales.view(torch.int16))
    g = -1 if per_tensor else (group if group > 0 else -2)
    y = K.dequant_fp_packed(b.codes, b.scales, None, 2, 1, g, rows, cols)
    assert torch.equal(y.view(torch.int16), b.out.view(torch.int16))
    # on the CPU: out == RN16(q * S) with q the E2M1 value of each code (fp4_quantize_cpu.py:72)
    codes = b.codes.cpu().numpy()
    nib = np.stack([codes & 0xF, codes >> 4], axis=-1).reshape(rows, cols)
    q = FC.fp_to_float(nib, 2, 1, 1).astype(np.float16)
    S = b.scales.cpu().numpy()
    if per_tensor:
        s_el = np.full((rows, cols), S[0], np.float16)
    elif group > 0:
        s_el = S[(np.arange(rows * cols) // group).reshape(rows, cols)]
    else:
        s_el = np.repeat(S[:, None], cols, axis=1)
    exp = (q * s_el).astype(np.float16)
    assert np.array_equal(exp.view(np.uint16), b.out.cpu().numpy().view(np.uint16))


def _specials(rows, cols, seed):
    """synthetic weights with an all-zero group, a +-inf group, a NaN group and a group of -0 / tiny
    values: the table kernels' non-table (exact ALU) path and the sign-of-zero codes"""
    w = weights(rows, cols, seed)
    w[0, :128] = 0.0
    w[1, 5] = float("inf")
    w[2, 130] = float("-inf")
    w[3, 7] = float("nan")
    w[4, :128] = -0.0
    w[4, 3] = 1e-6
    w[5, 256:384] = torch.linspace(-1e-3, 1e-3, 128, device=DEV).half()
    return w


@pytest.mark.parametrize("em", FORMATS)
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("group", [32, 128])
def test_codes_table_path_equals_codec(K, em, sym, group):
    """quantize_fp(want_codes): the table path's codes (round 6: carried by the table entries where
    E + 2M <= 10 -- every format here but E3M4 -- else re-encoded from the decoded values) == the
    bit-level codec's codes, outputs and scales identical too."""
    E, M = em
    w = _specials(64, 1024, 3 + E * 5 + M)
    a = K.quantize_fp(w, E, M, group, sym, 0, want_codes=True, use_lut=False)
    b = K.quantize_fp(w, E, M, group, sym, 0, want_codes=True, use_lut=True)
    assert torch.equal(a.codes, b.codes), (em, sym, group)
    assert torch.equal(a.out.view(torch.int16), b.out.view(torch.int16))
    assert torch.equal(a.scales.view(torch.int16), b.scales.view(torch.int16))


@pytest.mark.parametrize("group,per_tensor", [(128, False), (32, False), (0, False), (128, True)])
def test_grid_codes_table_path_equals_codec(K, group, per_tensor):
    w = _specials(64, 1024, 9)
    w[1, 5] = 1.0  # the grid flags inf groups as NaN everywhere; keep its finite groups comparable
    a = K.fp4_grid(w, group, per_tensor, use_lut=False, want_codes=True)
    b = K.fp4_grid(w, group, per_tensor, use_lut=True, want_codes=True)
    assert torch.equal(a.codes, b.codes), (group, per_tensor)
    assert torch.equal(a.out.view(torch.int16), b.out.view(torch.int16))


def test_unpack_errors(K):
    cd = torch.zeros(64 * 64 // 2, dtype=torch.uint8, device=DEV)
    sc = torch.ones(64, dtype=torch.float16, device=DEV)
    with pytest.raises(ValueError):
        K.dequant_fp_packed(cd[:-1], sc, None, 2, 1, -2, 64, 64)
    with pytest.raises(ValueError):
        K.dequant_fp_packed(cd, sc[:-1], None, 2, 1, -2, 64, 64)
    cd8 = torch.zeros(64 * 64, dtype=torch.uint8, device=DEV)
    with pytest.raises(RuntimeError):  # E5M2: fp_max 114688 overflows fp16 (quant_linear.py:852)
        K.dequant_fp_packed(cd8, sc, None, 5, 2, -2, 64, 64)


def _ab_built():
    try:
        from iron_weight_only_quant_amd import _lib
        return _lib.ab_built()
    except OSError:
        return False


@pytest.mark.skipif(not _ab_built(), reason="A/B kernel variants: IWQ_AB=1 library")
@pytest.mark.parametrize("em", FORMATS)
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("group", [32, 128])
def test_embedded_codes_equal_reencoded(K, em, sym, group):
    """Round 6: the table path with the codes embedded in the table entries and the entries read into
    register halves (variant 0) == the round-5 form (variant 7: v_perm-joined reads, codes re-encoded
    from the decoded values), codes / outputs / scales / zeros bit for bit, on specials and on a
    grid-stride-sized tensor."""
    E, M = em
    for w in (_specials(64, 1024, 5 + E * 3 + M), weights(2048, 4096, 17 + E)):
        a = K.quantize_fp(w, E, M, group, sym, 0, want_codes=True, flags=7 << 16)
        b = K.quantize_fp(w, E, M, group, sym, 0, want_codes=True)
        c = K.quantize_fp(w, E, M, group, sym, 0)
        assert torch.equal(a.codes, b.codes), (em, sym, group)
        for x in (b, c):
            assert torch.equal(a.out.view(torch.int16), x.out.view(torch.int16)), (em, sym, group)
            assert torch.equal(a.scales.view(torch.int16), x.scales.view(torch.int16))
            if not sym:
                assert torch.equal(a.zeros.view(torch.int16), x.zeros.view(torch.int16))

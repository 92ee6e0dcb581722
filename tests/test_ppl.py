"""PPL harness (reference main.py:42-140 arithmetic) — CPU arithmetic checks + GPU plumbing run.

The GPU test is the config-1 plumbing check (BASELINE config 1: OPT-125M, w_bits 8, group -2)
on a RANDOM-INIT OPT-125M-shaped model with synthetic tokens: no weights or datasets can be
fetched here, so absolute PPLs are meaningless; what is checked is that quantize_model's
replaced layers are bit-identical to the oracle and that the evaluator runs end to end.
"""
import math
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from iron_weight_only_quant_amd.ppl import SequentialPPLEvaluator

transformers = pytest.importorskip("transformers")


def _tiny_opt(seed=0):
    torch.manual_seed(seed)
    cfg = transformers.OPTConfig(vocab_size=97, hidden_size=32, num_hidden_layers=2, ffn_dim=64,
                                 num_attention_heads=4, max_position_embeddings=64, word_embed_proj_dim=32)
    return transformers.OPTForCausalLM(cfg).eval()


def _manual_ppl(model, tokens, seqlen, nchunks):
    nll, cnt = 0.0, 0
    with torch.no_grad():
        for i in range(nchunks):
            x = tokens[:, i * seqlen:(i + 1) * seqlen]
            logits = model(x).logits[:, :-1].float()
            lp = torch.log_softmax(logits, -1).gather(-1, x[:, 1:, None])
            nll += float(-lp.sum())
            cnt += seqlen - 1
    return math.exp(nll / cnt), cnt


def test_ppl_arithmetic_matches_token_level_nll():
    m = _tiny_opt()
    g = torch.Generator().manual_seed(3)
    tokens = torch.randint(0, 97, (1, 7 * 16 + 5), generator=g)
    ev = SequentialPPLEvaluator(m, device="cpu", seqlen=16, tokens=tokens)
    ppl, ntok, nch = ev.calculate_ppl("wikitext")
    assert nch == 7 and ntok == 7 * 15           # 2 batches: 4 + 3 chunks, trailing 5 tokens dropped
    ref, cnt = _manual_ppl(m, tokens, 16, 7)
    assert cnt == ntok
    assert abs(ppl - ref) / ref < 1e-5


def test_ppl_max_chunks_and_short_stream():
    m = _tiny_opt()
    tokens = torch.randint(0, 97, (1, 10 * 16))
    ev = SequentialPPLEvaluator(m, device="cpu", seqlen=16, tokens=tokens)
    ppl, ntok, nch = ev.calculate_ppl("wikitext", max_chunks=3)
    assert nch == 3 and ntok == 45
    ref, _ = _manual_ppl(m, tokens, 16, 3)
    assert abs(ppl - ref) / ref < 1e-5
    short = SequentialPPLEvaluator(m, device="cpu", seqlen=16, tokens=tokens[:, :15])
    with pytest.raises(ValueError):
        short.calculate_ppl("wikitext")


def test_ppl_seqlen_defaults_and_missing_dataset(tmp_path):
    m = _tiny_opt()
    assert SequentialPPLEvaluator(m, device="cpu").seqlen == 64       # config.max_position_embeddings
    m.seqlen = 32
    assert SequentialPPLEvaluator(m, device="cpu").seqlen == 32       # model.seqlen wins (main.py:50-56)
    ev = SequentialPPLEvaluator(m, device="cpu", dataset_dir=str(tmp_path))
    with pytest.raises(FileNotFoundError):
        ev.calculate_ppl("wikitext")


GOLD_DIR = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["wikitext2", "ptb", "c4", "ptb_new", "c4_new"])
def test_loaders_match_reference_get_loaders(name):
    """ppl.load_local_tokens == the token ids the reference's own gptq/datautils.get_loaders returned
    on the committed tiny datasets + tokenizer (tests/golden/make_golden_ppl.py): the joins, the
    split choice, the c4 random windows (random.seed(0), 256 x seqlen) and the c4_new truncation."""
    import os
    from iron_weight_only_quant_amd.ppl import load_local_tokens
    gold = np.load(os.path.join(GOLD_DIR, "ppl_tokens.npz"))
    seqlen = int(gold["seqlen"])
    fix = os.path.join(GOLD_DIR, "ppl_fixture")
    ids = load_local_tokens(name, os.path.join(fix, "tokenizer"), seqlen, dataset_dir=os.path.join(fix, "datasets"))
    assert ids.dim() == 2 and ids.shape[0] == 1
    assert np.array_equal(ids.numpy().astype(np.int64), gold[name]), name


def test_evaluator_dataset_map_and_hf_device_map():
    """The evaluator's names map like main.py:45-49 (wikitext -> wikitext2, ptb -> get_ptb, c4 ->
    get_c4), and an accelerate-dispatched model (hf_device_map) is fed on its embedding's device and
    never moved (main.py:89-98) -- here 'cpu' while the evaluator's own device names a GPU."""
    import os
    gold = np.load(os.path.join(GOLD_DIR, "ppl_tokens.npz"))
    seqlen = int(gold["seqlen"])
    fix = os.path.join(GOLD_DIR, "ppl_fixture")
    m = _tiny_opt()
    tok_dir = os.path.join(fix, "tokenizer")
    m.hf_device_map = {"model.decoder.embed_tokens": "cpu", "model.embed_tokens": "cpu", "lm_head": "cpu"}
    moved = []
    m.to = lambda *a, **k: moved.append(a) or m  # a dispatched model must not be moved
    ev = SequentialPPLEvaluator(m, model_path=tok_dir, device="cuda:7", seqlen=seqlen,
                                dataset_dir=os.path.join(fix, "datasets"))
    assert ev.input_device() == (torch.device("cpu"), True)
    vocab = 97
    for name, key in (("wikitext", "wikitext2"), ("ptb", "ptb"), ("c4", "c4")):
        toks = ev._load_tokens(name)
        assert np.array_equal(toks.numpy(), gold[key]), name
        ev.test_cache[key] = toks % vocab  # the tiny model's vocabulary
        ppl, ntok, nch = ev.calculate_ppl(name, max_chunks=2)
        assert nch == 2 and ntok == 2 * (seqlen - 1) and math.isfinite(ppl)
    assert not moved
    del m.hf_device_map["model.embed_tokens"]  # falls back to the map's first device
    assert ev.input_device() == (torch.device("cpu"), True)


@pytest.mark.gpu
@pytest.mark.parametrize("w_bit,group", [(8, -2), (4, 128)])
def test_ppl_delta_random_opt125m(w_bit, group):
    import copy
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    from oracle.iwq_oracle import quantlinear_int

    torch.manual_seed(0)
    base = transformers.OPTForCausalLM(transformers.OPTConfig()).half().cuda().eval()
    tokens = torch.randint(0, base.config.vocab_size, (1, 5 * 256), generator=torch.Generator().manual_seed(1))
    ppl0, ntok, nch = SequentialPPLEvaluator(base, device="cuda", seqlen=256, tokens=tokens).calculate_ppl("wikitext")
    assert nch == 5 and ntok == 5 * 255 and math.isfinite(ppl0)

    model = copy.deepcopy(base)
    orig = {n: mod.weight.detach().cpu().numpy().copy() for n, mod in model.named_modules()
            if isinstance(mod, torch.nn.Linear) and "lm_head" not in n}
    quantize_model(model, SimpleNamespace(w_bit=w_bit, a_bit=16, w_group_size=group, w_symmetric=False,
                                          w_format="int", quant_dim=0), verbose=False)
    nq = 0
    for n, mod in model.named_modules():
        if n in orig:
            assert isinstance(mod, QuantLinear), n
            want = quantlinear_int(orig[n], w_bit, group, False, 0, "float16").dequant
            got = mod.weight.detach().cpu().numpy()
            assert np.array_equal(got.view(np.uint16), want.view(np.uint16)), n
            nq += 1
    assert nq == 72                                                  # 12 layers x (q,k,v,out,fc1,fc2)
    ppl1, _, _ = SequentialPPLEvaluator(model, device="cuda", seqlen=256, tokens=tokens).calculate_ppl("wikitext")
    assert math.isfinite(ppl1)
    # random-init weights: logits are near-uniform, so RTN shifts PPL only slightly
    assert abs(ppl1 - ppl0) / ppl0 < (0.01 if w_bit == 8 else 0.1)

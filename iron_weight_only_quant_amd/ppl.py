"""Perplexity harness for the PPL-delta half of the metric (BASELINE config 1).

Same evaluation arithmetic as the reference's SequentialPPLEvaluator (main.py:42-140): the test
token stream is cut into nsamples = len // seqlen chunks, batched 4 at a time, and
    ppl = exp( sum(loss_b * (seqlen - 1) * bs_b) / sum((seqlen - 1) * bs_b) )
with the HF causal-LM loss of each batch.  Token sources: the reference's local dataset layout
(`datasets.load_from_disk(LOCAL_PPL_DATASET_DIR/<name>)`, gptq/datautils.py:14-29) tokenized with
the model's local tokenizer, or an explicit token tensor (synthetic runs).  Nothing is fetched from
the network: a missing dataset / tokenizer raises FileNotFoundError.
"""
import math
import os
from pathlib import Path

import torch

DATASET_MAP = {"wikitext": "wikitext2", "ptb": "ptb", "c4": "c4"}


def load_local_tokens(dataset_name, model_path, seqlen, dataset_dir=None):
    """Test tokens of wikitext2 / ptb / c4 from a local `datasets` directory (no download)."""
    root = Path(dataset_dir or os.getenv("LOCAL_PPL_DATASET_DIR", ""))
    key = DATASET_MAP.get(dataset_name.lower(), dataset_name)
    local = {"wikitext2": "wikitext", "ptb": "ptb", "c4": "c4"}.get(key, key)
    path = root / local
    if not root or not path.exists():
        raise FileNotFoundError(f"local PPL dataset '{local}' not found under '{root}' (set LOCAL_PPL_DATASET_DIR)")
    from datasets import load_from_disk
    from transformers import AutoTokenizer
    ds = load_from_disk(str(path))
    tok = AutoTokenizer.from_pretrained(model_path, use_fast=False, local_files_only=True)
    if key == "wikitext2":
        text = "\n\n".join(ds["test"]["text"])                       # gptq/datautils.py:45-50
        ids = tok(text, return_tensors="pt").input_ids
    elif key == "ptb":
        split = ds["validation"] if "validation" in ds else ds["valid"]
        ids = tok(" ".join(split[:1100]["text"]), return_tensors="pt").input_ids
        ids = ids[:, : 256 * seqlen]
    else:
        split = ds["validation"]
        ids = tok(" ".join(split[:1100]["text"]), return_tensors="pt").input_ids
        ids = ids[:, : 256 * seqlen]
    return ids.long()


class SequentialPPLEvaluator:
    """main.py:42-140 semantics; `tokens` may be passed directly (shape [1, T])."""

    def __init__(self, model, model_path=None, device="cuda", seqlen=None, tokens=None, dataset_dir=None):
        self.model = model
        self.model_path = model_path
        self.device = device
        if seqlen is not None:
            self.seqlen = int(seqlen)
        elif getattr(model, "seqlen", None):
            self.seqlen = int(model.seqlen)
        elif getattr(model.config, "max_position_embeddings", None):
            self.seqlen = int(model.config.max_position_embeddings)
        else:
            self.seqlen = 2048
        self.dataset_dir = dataset_dir
        self.test_cache = {}
        if tokens is not None:
            t = tokens if tokens.dim() == 2 else tokens.unsqueeze(0)
            self.test_cache["__tokens__"] = t.long()

    def _load_tokens(self, dataset_name):
        if "__tokens__" in self.test_cache:
            return self.test_cache["__tokens__"]
        key = DATASET_MAP.get(dataset_name.lower(), dataset_name)
        if key not in self.test_cache:
            self.test_cache[key] = load_local_tokens(dataset_name, self.model_path, self.seqlen, self.dataset_dir)
        return self.test_cache[key]

    @torch.no_grad()
    def calculate_ppl(self, dataset_name="wikitext", max_chunks=None, batch_size=4):
        tokens = self._load_tokens(dataset_name)
        nsamples = tokens.shape[1] // self.seqlen
        if nsamples == 0:
            raise ValueError(f"Dataset {dataset_name} is shorter than the model sequence length ({self.seqlen}).")
        if max_chunks is not None and max_chunks > 0:
            nsamples = min(nsamples, max_chunks)
        dev = torch.device(self.device)
        model = self.model
        model.eval()
        total_nll, total_tokens = 0.0, 0
        for start in range(0, nsamples, batch_size):
            end = min(start + batch_size, nsamples)
            batch = torch.cat([tokens[:, i * self.seqlen:(i + 1) * self.seqlen] for i in range(start, end)], dim=0)
            batch = batch.to(dev, non_blocking=True)
            out = model(batch, labels=batch)
            eff = max(batch.size(1) - 1, 1)
            total_nll += out.loss.item() * (eff * batch.size(0))
            total_tokens += eff * batch.size(0)
        if total_tokens == 0:
            return float("inf"), 0, nsamples
        return math.exp(total_nll / total_tokens), total_tokens, nsamples

"""Perplexity harness for the PPL-delta half of the metric (BASELINE config 1).

Same evaluation arithmetic as the reference's SequentialPPLEvaluator (main.py:42-140): the test
token stream is cut into nsamples = len // seqlen chunks, batched 4 at a time, and
    ppl = exp( sum(loss_b * (seqlen - 1) * bs_b) / sum((seqlen - 1) * bs_b) )
with the HF causal-LM loss of each batch.  An accelerate-dispatched model (hf_device_map) gets its
batches on the embedding's device and is not moved (main.py:89-98).

Token sources restate the reference's test-set loaders (gptq/datautils.py), reading the same local
`datasets` layout (`load_from_disk(LOCAL_PPL_DATASET_DIR/<wikitext|ptb|c4>)`, datautils.py:14-36)
and tokenizing with the model's local tokenizer (AutoTokenizer, use_fast=False):
    wikitext2  "\\n\\n".join(test["text"])                                 (get_wikitext2, :39-62)
    ptb        "\\n\\n".join(validation (or valid)["sentence"])           (get_ptb, :64-87)
    c4         random.seed(0); 256 random seqlen windows of validation
               documents with >= seqlen tokens, concatenated             (get_c4, :89-137)
    ptb_new    " ".join(test["sentence"])                                (get_ptb_new, :139-162)
    c4_new     " ".join(validation[:1100]["text"])[:, :256 * seqlen]      (get_c4_new, :164-203)
The evaluator maps "wikitext" / "ptb" / "c4" to the first three (main.py:45-49, datautils.py:205-217).
Pinned by tests/golden/ppl_tokens.npz (token ids the reference's own get_loaders produced on the
committed tiny datasets + tokenizer, tests/golden/make_golden_ppl.py).  Nothing is fetched from the
network: where the reference would download (missing local split), this raises FileNotFoundError.
"""
import math
import os
import random
from pathlib import Path

import torch

DATASET_MAP = {"wikitext": "wikitext2", "ptb": "ptb", "c4": "c4"}


def _local_dataset(root, name):
    """datautils.py:17-24: load_from_disk(root/name) if that directory exists (else None)."""
    path = Path(root) / name
    if not path.exists():
        return None
    from datasets import load_from_disk
    return load_from_disk(str(path))


def _split(dataset, split):
    """datautils.py:27-36."""
    if dataset is None:
        return None
    from datasets import DatasetDict
    if isinstance(dataset, (DatasetDict, dict)):
        return dataset.get(split)
    return getattr(dataset, split, None)


def _missing(name, root):
    return FileNotFoundError(f"local PPL dataset '{name}' (with the splits the reference reads) not found under "
                             f"'{root}'; the reference would download it -- set LOCAL_PPL_DATASET_DIR")


def _tokenizer(model_path):
    from transformers import AutoTokenizer
    return AutoTokenizer.from_pretrained(model_path, use_fast=False, local_files_only=True)


def load_local_tokens(dataset_name, model_path, seqlen, dataset_dir=None):
    """Test token ids [1, T] of the reference's loader for `dataset_name` (a get_loaders name:
    "wikitext2", "ptb", "c4", "ptb_new", "c4_new"; or the evaluator's "wikitext")."""
    root = dataset_dir or os.getenv("LOCAL_PPL_DATASET_DIR", "")
    if not root:
        raise FileNotFoundError("no local PPL dataset directory (set LOCAL_PPL_DATASET_DIR)")
    key = DATASET_MAP.get(dataset_name.lower(), dataset_name)
    if "wikitext2" in key:                                                   # datautils.py:208
        ds = _local_dataset(root, "wikitext")
        test = _split(ds, "test")
        if _split(ds, "train") is None or test is None:
            raise _missing("wikitext", root)
        return _tokenizer(model_path)("\n\n".join(test["text"]), return_tensors="pt").input_ids
    if "ptb" in key:
        ds = _local_dataset(root, "ptb")
        if "new" in key:                                                     # get_ptb_new
            test = _split(ds, "test")
            if _split(ds, "train") is None or test is None:
                raise _missing("ptb", root)
            return _tokenizer(model_path)(" ".join(test["sentence"]), return_tensors="pt").input_ids
        val = _split(ds, "validation") or _split(ds, "valid")                # get_ptb (:67)
        if _split(ds, "train") is None or val is None:
            raise _missing("ptb", root)
        return _tokenizer(model_path)("\n\n".join(val["sentence"]), return_tensors="pt").input_ids
    if "c4" in key:
        ds = _local_dataset(root, "c4")
        val = _split(ds, "validation")
        tok = _tokenizer(model_path)
        if "new" in key:                                                     # get_c4_new (:195-196)
            if _split(ds, "train") is None or val is None:
                raise _missing("c4", root)
            ids = tok(" ".join(val[:1100]["text"]), return_tensors="pt").input_ids
            return ids[:, :(256 * seqlen)]
        if val is None:                                                      # get_c4 (:93, :120-131)
            raise _missing("c4", root)
        rng = random.Random(0)  # the reference reseeds the global `random` with 0 before the windows
        windows = []
        for _ in range(256):
            while True:
                i = rng.randint(0, len(val) - 1)
                tmp = tok(val[i]["text"], return_tensors="pt")
                if tmp.input_ids.shape[1] >= seqlen:
                    break
            i = rng.randint(0, tmp.input_ids.shape[1] - seqlen - 1)
            windows.append(tmp.input_ids[:, i:i + seqlen])
        return torch.hstack(windows)
    raise ValueError(f"unknown PPL dataset '{dataset_name}' (get_loaders knows wikitext2 / ptb / c4)")


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
            t = load_local_tokens(key, self.model_path, self.seqlen, self.dataset_dir)
            self.test_cache[key] = (t if t.dim() == 2 else t.unsqueeze(0)).long()
        return self.test_cache[key]

    def input_device(self):
        """main.py:89-98: an accelerate-dispatched model takes its input on the embedding's device
        (or the first device of its map) and is left where it is; otherwise self.device."""
        hf_map = getattr(self.model, "hf_device_map", None)
        if hf_map is not None:
            d = hf_map.get("model.embed_tokens", None)
            if d is None:
                d = next(iter(hf_map.values()))
            if isinstance(d, int):
                d = f"cuda:{d}"
            return torch.device(d), True
        return torch.device(self.device), False

    @torch.no_grad()
    def calculate_ppl(self, dataset_name="wikitext", max_chunks=None, batch_size=4):
        tokens = self._load_tokens(dataset_name)
        nsamples = tokens.shape[1] // self.seqlen
        if nsamples == 0:
            raise ValueError(f"Dataset {dataset_name} is shorter than the model sequence length ({self.seqlen}).")
        if max_chunks is not None and max_chunks > 0:
            nsamples = min(nsamples, max_chunks)
        dev, dispatched = self.input_device()
        model = self.model if dispatched else self.model.to(dev)
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

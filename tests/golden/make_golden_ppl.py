"""Golden token ids for the PPL harness's test-set loaders, FROM THE REFERENCE ITSELF.

Run only in the build container (it imports /root/reference/gptq/datautils.py, which does not exist
on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ppl.py

1. Writes tiny deterministic stand-ins of the reference's local dataset layout
   (datasets.save_to_disk, gptq/datautils.py:14-36) to tests/golden/ppl_fixture/datasets/:
     wikitext  train/test          'text'      (wikitext-2-raw-like: headings, paragraphs, blanks)
     ptb       train/validation/test 'sentence'
     c4        train/validation    'text'      (documents of varying length, some shorter than seqlen)
   The text is synthetic (no corpus is available offline); what is pinned is the LOADERS' logic --
   joins, splits, truncation, the seeded random windows of get_c4 -- not the data.
2. Trains a small byte-level BPE tokenizer on that text (tokenizers, offline) and saves it as a
   transformers tokenizer directory (tests/golden/ppl_fixture/tokenizer).
3. Points LOCAL_PPL_DATASET_DIR at (1), imports the reference's gptq/datautils.get_loaders and saves
   the test token ids it returns for wikitext2 / ptb / c4 / ptb_new / c4_new to
   tests/golden/ppl_tokens.npz (with the seqlen used).
"""
import os
import random
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "ppl_fixture")
DS = os.path.join(FIX, "datasets")
TOK = os.path.join(FIX, "tokenizer")
SEQLEN = 64

WORDS = ("the of and to in a is was for on that with as by at from his an were are which this be or has had "
         "it not but first new one two year city game film river station album season team war band series "
         "north south league music school church county party village house church records published song "
         "during after between world national american british early later government several known "
         "including however although became released").split()


def sentence(rng, lo=4, hi=28):
    w = [rng.choice(WORDS) for _ in range(rng.randint(lo, hi))]
    w[0] = w[0].capitalize()
    if rng.random() < 0.3:
        w.insert(rng.randint(1, len(w)), str(rng.randint(1800, 2020)))
    if rng.random() < 0.2:
        w.insert(rng.randint(1, len(w)), ",")
    return " ".join(w) + " ."


def wikitext_lines(rng, n):
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.35:
            out.append("")
        elif r < 0.45:
            out.append(f" = {' '.join(rng.choice(WORDS).capitalize() for _ in range(rng.randint(1, 4)))} = \n")
        else:
            out.append(" " + " ".join(sentence(rng) for _ in range(rng.randint(1, 5))) + " \n")
    return out


def build_datasets():
    from datasets import Dataset, DatasetDict
    rng = random.Random(20250101)
    if os.path.exists(DS):
        shutil.rmtree(DS)
    wiki = DatasetDict(train=Dataset.from_dict({"text": wikitext_lines(rng, 400)}),
                       test=Dataset.from_dict({"text": wikitext_lines(rng, 160)}))
    ptb = DatasetDict(**{s: Dataset.from_dict({"sentence": [sentence(rng, 3, 20).lower()[:-2] for _ in range(n)]})
                         for s, n in (("train", 600), ("validation", 200), ("test", 220))})
    docs = lambda n: [" ".join(sentence(rng) for _ in range(rng.randint(1, 14))) for _ in range(n)]  # noqa: E731
    c4 = DatasetDict(train=Dataset.from_dict({"text": docs(80)}), validation=Dataset.from_dict({"text": docs(120)}))
    wiki.save_to_disk(os.path.join(DS, "wikitext"))
    ptb.save_to_disk(os.path.join(DS, "ptb"))
    c4.save_to_disk(os.path.join(DS, "c4"))
    return wiki, ptb, c4


def build_tokenizer(corpus):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors, trainers
    from transformers import PreTrainedTokenizerFast
    tk = Tokenizer(models.BPE(unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=400, special_tokens=["<unk>", "<s>", "</s>"], show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(corpus, trainer=trainer)
    tk.post_processor = processors.TemplateProcessing(single="<s> $A", special_tokens=[("<s>", tk.token_to_id("<s>"))])
    t = PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="<unk>", bos_token="<s>", eos_token="</s>")
    if os.path.exists(TOK):
        shutil.rmtree(TOK)
    t.save_pretrained(TOK)


def main():
    wiki, ptb, c4 = build_datasets()
    corpus = list(wiki["train"]["text"]) + list(ptb["train"]["sentence"]) + list(c4["train"]["text"])
    build_tokenizer(corpus)
    os.environ["LOCAL_PPL_DATASET_DIR"] = DS  # read at import time (datautils.py:14)
    sys.dont_write_bytecode = True
    sys.path.insert(0, "/root/reference/gptq")
    import datautils  # noqa: E402  (reference: gptq/datautils.py)
    out = {"seqlen": np.array(SEQLEN)}
    for name in ("wikitext2", "ptb", "c4", "ptb_new", "c4_new"):
        _, test = datautils.get_loaders(name, nsamples=1, seed=0, seqlen=SEQLEN, model=TOK)
        ids = getattr(test, "input_ids", test)
        out[name] = ids.numpy().astype(np.int64)
        print(name, out[name].shape, flush=True)
    np.savez_compressed(os.path.join(HERE, "ppl_tokens.npz"), **out)


if __name__ == "__main__":
    main()

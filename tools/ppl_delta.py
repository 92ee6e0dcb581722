"""PPL delta of weight-only RTN quantization (BASELINE metric, second half; config 1 plumbing).

    python tools/ppl_delta.py --model_path /path/to/local/hf/model --dataset wikitext --w_bits 4 8 \
        --w_group_size 128            # real run: local weights + LOCAL_PPL_DATASET_DIR
    python tools/ppl_delta.py --random opt-125m --synthetic_tokens 65536 --w_bits 8 --w_group_size -2
                                      # weights-free plumbing run (random init, synthetic tokens)

Mirrors main.py's run_ppl loop (main.py:378-424): for each w_bit, build the fp16 model, quantize
it with quantize_model (here: ONE batched gfx950 launch for all Linear layers), evaluate with the
SequentialPPLEvaluator arithmetic; the fp16 PPL is measured once first.  Prints one JSON line per
w_bit with ppl_fp16, ppl_quant, ppl_delta and the quantization wall time.  A random-init model
gives meaningless absolute PPLs; it exercises the plumbing and reports the delta honestly as such.
"""
import argparse
import copy
import json
import os
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_model(args):
    from transformers import AutoModelForCausalLM, OPTConfig, OPTForCausalLM, LlamaConfig, LlamaForCausalLM
    if args.model_path:
        if args.device_map:  # utils.py:43-44: accelerate placement over the visible GPUs (e.g. a 70B)
            return AutoModelForCausalLM.from_pretrained(args.model_path, torch_dtype=torch.float16,
                                                        local_files_only=True, device_map=args.device_map)
        m = AutoModelForCausalLM.from_pretrained(args.model_path, torch_dtype=torch.float16, local_files_only=True)
        return m.cuda()
    torch.manual_seed(args.seed)
    if args.random == "opt-125m":
        cfg = OPTConfig()  # facebook/opt-125m shapes (transformers defaults)
        m = OPTForCausalLM(cfg)
    elif args.random == "llama-tiny":
        cfg = LlamaConfig(hidden_size=512, intermediate_size=1408, num_hidden_layers=4, num_attention_heads=8,
                          num_key_value_heads=8, vocab_size=32000, max_position_embeddings=2048)
        m = LlamaForCausalLM(cfg)
    else:
        raise SystemExit("--model_path or --random {opt-125m,llama-tiny} required")
    return m.half().cuda()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model_path", default=None)
    ap.add_argument("--random", default=None, choices=[None, "opt-125m", "llama-tiny"])
    ap.add_argument("--dataset", default="wikitext")
    ap.add_argument("--local_dataset_dir", default=None)
    ap.add_argument("--synthetic_tokens", type=int, default=0)
    ap.add_argument("--ppl_seqlen", type=int, default=2048)
    ap.add_argument("--max_chunks", type=int, default=0)
    ap.add_argument("--w_bits", type=int, nargs="+", default=[4])
    ap.add_argument("--w_group_size", type=int, default=128)
    ap.add_argument("--w_symmetric", action="store_true")
    ap.add_argument("--w_format", default="int")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device_map", default=None,
                    help='e.g. "balanced" (the reference\'s placement, utils.py:43): the evaluator then feeds '
                         'batches to the embedding\'s device (main.py:89-98)')
    ap.add_argument("--fused_forward", default="false", choices=["false", "auto", "true"],
                    help="QuantLinear forward on the packed codes (MI355X addition; false = the reference's F.linear)")
    args = ap.parse_args()

    from iron_weight_only_quant_amd.ppl import SequentialPPLEvaluator
    from iron_weight_only_quant_amd.quant_wrapper import quantize_model

    base = build_model(args)
    tokens = None
    if args.synthetic_tokens:
        g = torch.Generator().manual_seed(args.seed + 1)
        tokens = torch.randint(0, base.config.vocab_size, (1, args.synthetic_tokens), generator=g)
    seqlen = min(args.ppl_seqlen, getattr(base.config, "max_position_embeddings", args.ppl_seqlen))
    ev = SequentialPPLEvaluator(base, args.model_path, "cuda", seqlen=seqlen, tokens=tokens,
                                dataset_dir=args.local_dataset_dir)
    ppl_fp16, ntok, nch = ev.calculate_ppl(args.dataset, max_chunks=args.max_chunks or None)
    fused = {"false": False, "auto": "auto", "true": True}[args.fused_forward]
    for wb in args.w_bits:
        # main.py:285-375 builds a fresh fp16 model per w_bit; a dispatched model is rebuilt the same way
        model = build_model(args) if args.device_map else copy.deepcopy(base)
        qargs = SimpleNamespace(w_bit=wb, a_bit=16, w_group_size=args.w_group_size, w_symmetric=args.w_symmetric,
                                w_format=args.w_format, quant_dim=0, fused_forward=fused)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        quantize_model(model, qargs, verbose=False)
        torch.cuda.synchronize()
        tq = time.perf_counter() - t0
        ev_q = SequentialPPLEvaluator(model, args.model_path, "cuda", seqlen=seqlen, tokens=tokens,
                                      dataset_dir=args.local_dataset_dir)
        ppl_q, _, _ = ev_q.calculate_ppl(args.dataset, max_chunks=args.max_chunks or None)
        print(json.dumps({"model": args.model_path or f"random:{args.random}", "dataset":
                          ("synthetic" if tokens is not None else args.dataset), "seqlen": seqlen,
                          "num_tokens": ntok, "num_chunks": nch, "w_bit": wb, "w_group_size": args.w_group_size,
                          "w_symmetric": args.w_symmetric, "w_format": args.w_format, "ppl_fp16": ppl_fp16,
                          "ppl_quant": ppl_q, "ppl_delta": ppl_q - ppl_fp16, "quantize_s": round(tq, 4)}),
              flush=True)
        del model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Generate the golden fixtures for the INT min-max path FROM THE REFERENCE ITSELF.

Run only in the survey/build container (it imports /root/reference, which does
not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Produces (committed, data only):
  tests/golden/int_small.npz   full inputs + reference outputs for small shapes, all modes
  tests/golden/int_edge.npz    edge-row tensors (constant, zero, subnormal, one-sided, ties, +-0, ...)
  tests/golden/int_large.json  SHA-256 of reference outputs at Llama-2-7B shapes over oracle/synth inputs
  tests/golden/int_large_70b.json  the same at the four Llama-2-70B Linear shapes (configs[3])
                                   (`--only 70b` regenerates just this file)
  tests/golden/int_large_pt.json   per-tensor (-1) at the 7B shapes (`--only pt`)
  tests/golden/int_large_pt_dt.json  per-tensor (-1) on bf16 (7B shapes) and fp32 (4096^2) (`--only pt_dt`)
  tests/golden/int_batched.json    quantize_model's batched group modes on a 4-tensor set, fp16 and
                                   bf16, SHA-256 of every layer's outputs (`--only batched`)

Reference entry points exercised:
  quant_funcs.pseudo_quantize_tensor                  (quant_funcs.py:4-46)
  quant_linear.QuantLinear.from_linear(...).weight/.scales/.zeros   (quant_linear.py:974-1033, :885-956)
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

import quant_funcs  # noqa: E402  (reference)
import quant_linear  # noqa: E402  (reference)

from oracle.synth import synth  # noqa: E402

TD = {"float16": torch.float16, "bfloat16": torch.bfloat16, "float32": torch.float32}


def to_np(t):
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def from_np(a, dtype):
    if dtype == "bfloat16":
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16)
    return torch.from_numpy(np.ascontiguousarray(a))


def ref_qf(x_np, dtype, **kw):
    t = from_np(x_np, dtype).clone()
    try:
        out = quant_funcs.pseudo_quantize_tensor(t, **kw)
    except AssertionError:
        return None
    return to_np(out)


def ref_ql(w_np, dtype, **kw):
    w = from_np(w_np, dtype).clone()
    lin = torch.nn.Linear(w.shape[1], w.shape[0], bias=False)
    lin.weight.data = w
    ql = quant_linear.QuantLinear.from_linear(lin, **kw)
    z = ql.zeros
    return to_np(ql.weight.data), to_np(ql.scales), (None if z is None else to_np(z)), bool(ql.quantized)


def small_cases():
    torch.manual_seed(0)
    d = {}
    shapes = {"a": (48, 256), "b": (24, 384)}
    for tag, shp in shapes.items():
        for dtype in ("float16", "bfloat16", "float32"):
            if tag != "a" and dtype != "float16":
                continue
            x = synth(100 + len(tag) + shp[0], shp, dtype)
            d[f"in/{tag}/{dtype}"] = x
            bits_list = (2, 3, 4, 8) if dtype == "float16" else (4,)
            for bits in bits_list:
                for zp in (True, False):
                    for g, pt in ((32, False), (128, False), (-1, False), (-1, True), (64, False)):
                        if dtype != "float16" and g == 64:
                            continue
                        out = ref_qf(x, dtype, n_bits=bits, zero_point=zp, q_group_size=g, per_tensor=pt)
                        key = f"qf/{tag}/{dtype}/{bits}/{int(zp)}/{g}/{int(pt)}"
                        d[key] = out if out is not None else np.zeros(0, np.uint8)
                for sym in (False, True):
                    for qd in (0, 1):
                        groups = (32, 128, -1, -2) if qd == 0 else (8, 24, -1, -2)
                        for g in groups:
                            if qd == 0 and shp[1] % max(g, 1) != 0:
                                continue
                            if qd == 1 and g > 0 and shp[0] % g != 0:
                                continue
                            deq, s, z, qz = ref_ql(x, dtype, w_bit=bits, w_group_size=g, symmetric=sym, quant_dim=qd)
                            key = f"ql/{tag}/{dtype}/{bits}/{int(sym)}/{g}/{qd}"
                            d[key + "/deq"] = deq
                            d[key + "/scales"] = s
                            if z is not None:
                                d[key + "/zeros"] = z
    return d


def edge_rows():
    """[R,128] fp16 rows that exercise every quirk listed in SURVEY.md §7 'Hard parts'."""
    rng = np.random.default_rng(7)
    rows = []
    rows.append(np.full(128, 0.5, np.float32))                          # constant -> range clamps to 1e-5
    rows.append(np.zeros(128, np.float32))                              # all zero
    rows.append(np.full(128, -0.0, np.float32))                         # all -0
    r = rng.standard_normal(128).astype(np.float32) * 0.02
    r[::7] = 0.0
    rows.append(np.abs(r))                                              # one-sided >= 0, min == 0 -> zeros = -0.0
    rows.append(-np.abs(rng.standard_normal(128).astype(np.float32)))   # one-sided negative
    rows.append((rng.integers(1, 1024, 128) * 2.0 ** -24).astype(np.float32))   # fp16 subnormals
    rows.append(np.linspace(-1, 1, 128).astype(np.float32))             # many exact ties after /s
    rows.append((rng.integers(-8, 8, 128) * 0.5).astype(np.float32))   # half-integers -> ties
    big = rng.standard_normal(128).astype(np.float32)
    big[3] = 30000.0
    big[77] = -30000.0
    rows.append(big)                                                    # huge but finite range
    t = rng.standard_normal(128).astype(np.float32)
    t[5] = 1000.0
    rows.append(t)                                                      # single outlier
    rows.append(np.array([1e-5, 2e-5] * 64, np.float32))                # tiny range
    rows.append(np.array([6e-5, -6e-5] * 64, np.float32))               # around fp16 min normal
    m = rng.standard_normal(128).astype(np.float32)
    m[10] = 0.0
    m[11] = -0.0
    rows.append(np.abs(m))                                              # mixed +-0 as min (sign ambiguity)
    rows.append(np.full(128, 65504.0, np.float32))                      # constant at fp16 max
    rows.append(np.array([-65504.0, 65504.0] * 64, np.float32))        # asym max-min overflows to inf -> NaN output
    return np.stack(rows).astype(np.float16)


def edge_cases():
    d = {}
    e = edge_rows()
    d["in/edge"] = e
    finite_rows = np.arange(e.shape[0] - 1)          # last row overflows max-min -> inf -> NaN output
    d["in/edge_finite_rows"] = finite_rows
    ef = e[finite_rows]
    for bits in (2, 3, 4, 8):
        for zp in (True, False):
            out = ref_qf(ef, "float16", n_bits=bits, zero_point=zp, q_group_size=128)
            d[f"qf/edge/{bits}/{int(zp)}"] = out if out is not None else np.zeros(0, np.uint8)
            out = ref_qf(e, "float16", n_bits=bits, zero_point=zp, q_group_size=128)
            d[f"qf/edge_all/{bits}/{int(zp)}"] = out if out is not None else np.zeros(0, np.uint8)
            deq, s, z, _ = ref_ql(e, "float16", w_bit=bits, w_group_size=128, symmetric=not zp)
            d[f"ql/edge_all/{bits}/{int(not zp)}/deq"] = deq
            d[f"ql/edge_all/{bits}/{int(not zp)}/scales"] = s
            if z is not None:
                d[f"ql/edge_all/{bits}/{int(not zp)}/zeros"] = z
    # inf / nan inputs
    inf_t = synth(55, (4, 128), "float16")
    inf_t[1, 9] = np.inf
    inf_t[2, 17] = np.nan
    d["in/nonfinite"] = inf_t
    for zp in (True, False):
        out = ref_qf(inf_t, "float16", n_bits=4, zero_point=zp, q_group_size=128)
        d[f"qf/nonfinite/{int(zp)}"] = out if out is not None else np.zeros(0, np.uint8)
        deq, s, z, _ = ref_ql(inf_t, "float16", w_bit=4, w_group_size=128, symmetric=not zp)
        d[f"ql/nonfinite/{int(not zp)}/deq"] = deq
        d[f"ql/nonfinite/{int(not zp)}/scales"] = s
        if z is not None:
            d[f"ql/nonfinite/{int(not zp)}/zeros"] = z
    return d


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


LARGE = [("q_proj", (4096, 4096), 0), ("gate_proj", (11008, 4096), 1), ("down_proj", (4096, 11008), 2)]


def large_cases():
    res = {"generator": "oracle/synth.py (seed, shape) fp16", "cases": []}
    for name, shp, seed in LARGE:
        x = synth(seed, shp, "float16")
        res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "input", "sha_input": sha(x)})
        for bits, zp, g in ((4, True, 128), (4, False, 128), (8, True, 128), (4, True, -1)):
            out = ref_qf(x, "float16", n_bits=bits, zero_point=zp, q_group_size=g)
            res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "qf", "n_bits": bits,
                                 "zero_point": zp, "q_group_size": g, "sha_deq": sha(out)})
        for bits, sym, g in ((4, False, 128), (4, True, 128), (4, False, -2), (4, True, -2), (8, False, -2)):
            deq, s, z, _ = ref_ql(x, "float16", w_bit=bits, w_group_size=g, symmetric=sym)
            res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "ql", "w_bit": bits,
                                 "symmetric": sym, "w_group_size": g, "sha_deq": sha(deq), "sha_scales": sha(s),
                                 "sha_zeros": None if z is None else sha(z)})
        print("large", name, flush=True)
    return res


LARGE_70B = [("q_proj", (8192, 8192), 10), ("k_proj", (1024, 8192), 11), ("gate_proj", (28672, 8192), 12),
             ("down_proj", (8192, 28672), 13)]


def large70b_cases():
    """Llama-2-70B shapes (BASELINE configs[3], 4-bit g=128): the config's own case on both reference
    entry points, plus per-row and per-channel (down_proj's 28672-element rows exceed the GPU's
    register-resident row kernel, so they cover the universal path at full size)."""
    res = {"generator": "oracle/synth.py (seed, shape) fp16", "cases": []}
    for name, shp, seed in LARGE_70B:
        x = synth(seed, shp, "float16")
        res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "input", "sha_input": sha(x)})
        for bits, zp, g in ((4, True, 128), (4, True, -1)):
            out = ref_qf(x, "float16", n_bits=bits, zero_point=zp, q_group_size=g)
            res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "qf", "n_bits": bits,
                                 "zero_point": zp, "q_group_size": g, "sha_deq": sha(out)})
            del out
        for bits, sym, g in ((4, False, 128), (4, True, 128), (4, False, -2)):
            deq, s, z, _ = ref_ql(x, "float16", w_bit=bits, w_group_size=g, symmetric=sym)
            res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "ql", "w_bit": bits,
                                 "symmetric": sym, "w_group_size": g, "sha_deq": sha(deq), "sha_scales": sha(s),
                                 "sha_zeros": None if z is None else sha(z)})
            del deq, s, z
        print("large70b", name, flush=True)
    return res


def large_pt_cases():
    """Per-tensor (-1) at the Llama-2-7B shapes on both reference entry points (round 3: the one-pass
    per-tensor kernel holds a whole weight in registers)."""
    res = {"generator": "oracle/synth.py (seed, shape) fp16", "cases": []}
    for name, shp, seed in LARGE:
        x = synth(seed, shp, "float16")
        res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "input", "sha_input": sha(x)})
        for bits, zp in ((4, True), (8, False)):
            out = ref_qf(x, "float16", n_bits=bits, zero_point=zp, q_group_size=-1, per_tensor=True)
            res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "qf_pt", "n_bits": bits,
                                 "zero_point": zp, "sha_deq": sha(out)})
        for bits, sym in ((4, False), (4, True), (8, False)):
            deq, s, z, _ = ref_ql(x, "float16", w_bit=bits, w_group_size=-1, symmetric=sym)
            res["cases"].append({"name": name, "shape": list(shp), "seed": seed, "kind": "ql", "w_bit": bits,
                                 "symmetric": sym, "w_group_size": -1, "sha_deq": sha(deq), "sha_scales": sha(s),
                                 "sha_zeros": None if z is None else sha(z)})
        print("large_pt", name, flush=True)
    return res


def large_pt_dt_cases():
    """Per-tensor (-1) on bf16 and fp32 weights (round 5: the one-pass kernel also holds bf16 / fp32
    weights in registers, keys in two dwords for fp32): bf16 at the three Llama-2-7B shapes, fp32 at
    4096 x 4096 (the larger fp32 shapes exceed the register capacity and take the two-kernel pair)."""
    res = {"generator": "oracle/synth.py (seed, shape, dtype)", "cases": []}
    for dtype, names in (("bfloat16", ("q_proj", "gate_proj", "down_proj")), ("float32", ("q_proj",))):
        for name, shp, seed in LARGE:
            if name not in names:
                continue
            x = synth(seed, shp, dtype)
            base = {"dtype": dtype, "name": name, "shape": list(shp), "seed": seed}
            res["cases"].append({**base, "kind": "input", "sha_input": sha(x)})
            for bits, zp in ((4, True), (8, False)):
                out = ref_qf(x, dtype, n_bits=bits, zero_point=zp, q_group_size=-1, per_tensor=True)
                res["cases"].append({**base, "kind": "qf_pt", "n_bits": bits, "zero_point": zp, "sha_deq": sha(out)})
            for bits, sym in ((4, False), (4, True)):
                deq, s, z, _ = ref_ql(x, dtype, w_bit=bits, w_group_size=-1, symmetric=sym)
                res["cases"].append({**base, "kind": "ql", "w_bit": bits, "symmetric": sym, "w_group_size": -1,
                                     "sha_deq": sha(deq), "sha_scales": sha(s),
                                     "sha_zeros": None if z is None else sha(z)})
            print("large_pt_dt", dtype, name, flush=True)
    return res


# quantize_model's batched launches in every non-headline group mode (per-channel, per-tensor,
# quant_dim 1, long and non-power-of-two groups) on multi-tensor sets, fp16 AND bf16 (round 4:
# the batched bf16 modes were compared with the per-layer path only)
BATCHED_SPECS = {"a": (384, 3072), "b": (256, 1536), "c": (128, 2304), "d": (512, 1536)}
BATCHED_MODES = ((-2, 0), (-1, 0), (128, 1), (-2, 1), (64, 1), (768, 0), (96, 0))
BATCHED_BITS = ((4, False), (8, False), (3, True))


def batched_inputs(dtype):
    """{name: [out, in] array}: oracle/synth inputs (seeds 300..), row 3 of "b" constant 0.5."""
    out = {}
    for i, (n, shp) in enumerate(sorted(BATCHED_SPECS.items())):
        x = synth(300 + i, shp, dtype)
        if n == "b":  # a constant row (range 0 -> clamp 1e-5); bf16 arrays hold the bit patterns
            x[3] = {"bfloat16": np.uint16(0x3F00), "float16": np.float16(0.5)}[dtype]
        out[n] = x
    return out


def batched_cases():
    res = {"generator": "oracle/synth.py (300 + sorted index, shape), row 3 of 'b' = 0.5", "specs": BATCHED_SPECS,
           "cases": []}
    for dtype in ("float16", "bfloat16"):
        ins = batched_inputs(dtype)
        for n, x in ins.items():
            res["cases"].append({"dtype": dtype, "name": n, "kind": "input", "sha_input": sha(x)})
        for g, qd in BATCHED_MODES:
            for bits, sym in BATCHED_BITS:
                for n, x in ins.items():
                    deq, s, z, _ = ref_ql(x, dtype, w_bit=bits, w_group_size=g, symmetric=sym, quant_dim=qd)
                    res["cases"].append({"dtype": dtype, "name": n, "kind": "ql", "w_bit": bits, "symmetric": sym,
                                         "w_group_size": g, "quant_dim": qd, "sha_deq": sha(deq),
                                         "sha_scales": sha(s), "sha_zeros": None if z is None else sha(z)})
        print("batched", dtype, flush=True)
    return res


if __name__ == "__main__":
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "batched":
        with open(os.path.join(HERE, "int_batched.json"), "w") as f:
            json.dump(batched_cases(), f, indent=1)
        print("batched done", flush=True)
        sys.exit(0)
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "pt_dt":
        with open(os.path.join(HERE, "int_large_pt_dt.json"), "w") as f:
            json.dump(large_pt_dt_cases(), f, indent=1)
        print("large_pt_dt done", flush=True)
        sys.exit(0)
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "pt":
        with open(os.path.join(HERE, "int_large_pt.json"), "w") as f:
            json.dump(large_pt_cases(), f, indent=1)
        print("large_pt done", flush=True)
        sys.exit(0)
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "70b":
        with open(os.path.join(HERE, "int_large_70b.json"), "w") as f:
            json.dump(large70b_cases(), f, indent=1)
        print("large70b done", flush=True)
        sys.exit(0)
    np.savez_compressed(os.path.join(HERE, "int_small.npz"), **small_cases())
    print("small done", flush=True)
    np.savez_compressed(os.path.join(HERE, "int_edge.npz"), **edge_cases())
    print("edge done", flush=True)
    with open(os.path.join(HERE, "int_large.json"), "w") as f:
        json.dump(large_cases(), f, indent=1)
    print("large done", flush=True)
    with open(os.path.join(HERE, "int_large_70b.json"), "w") as f:
        json.dump(large70b_cases(), f, indent=1)
    print("large70b done", flush=True)
    with open(os.path.join(HERE, "int_large_pt.json"), "w") as f:
        json.dump(large_pt_cases(), f, indent=1)
    print("large_pt done", flush=True)

"""Where the out-of-place outputs of the whole-model launch live, A/B (the out-of-place penalty that
depends on placement): the 224 Llama-2-7B weights quantized INT4 g128 by one batched launch into
  default        torch.empty_like per weight (what BatchPlan allocates)
  inplace        copies of the weights, quantized onto themselves
  arena@D        one flat buffer, weight i's output at a running offset + D bytes (a uniform shift)
  arena+S        one flat buffer, weight i's output at a running offset + i * S bytes (a skew per weight)
  rev            torch.empty_like per weight, allocated in reverse order
For each arm and each variant in --variants (0 = the product kernel; 100-102 copy probes and 118 the
kernel's walk without arithmetic; other numbers are A/B-library forms, IWQ_AB=1) the HIP-event time
of a launch, best of 3 x 10 launches after a 1 s clock ramp; arms interleaved over --rounds.
`ceiling/fresh`: the nt copy probe on two freshly allocated buffers that are not the plan's (a
single [n / 4096, 4096] entry each), the box's own copy rate independent of where the plan's
tensors were placed."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


# copy probes and arithmetic-free skeletons (iwq_minmax.hip launch_variant): not quantizers
NON_QUANTIZING = set(range(100, 128)) | {133, 134, 135, 139, 140, 146, 147, 153, 154, 160, 163}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--shifts", default="0,256,1024,4096,16384,65536,262144,1048576")
    ap.add_argument("--skews", default="4096")
    ap.add_argument("--variants", default="0,100,118")
    ap.add_argument("--no-rev", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--pmc", action="store_true",
                    help="for a rocprofv3 --pmc run: one round, no ramp or check, and a separator launch "
                         "(iwq_fill_synthetic on 16 elements) before every arm x variant, so that "
                         "tools/pmc_arms.py can cut the per-dispatch counters by arm")
    a = ap.parse_args()
    import bench
    from iron_weight_only_quant_amd import kernels
    weights, names, _ = bench.make_weights("llama2-7b", 0, 1)
    numel = sum(w.numel() for w in weights)
    alg = numel * 4 + numel // 128 * 4
    variants = [int(v) for v in a.variants.split(",")]
    arms = {"default": None, "inplace": weights}
    shifts = [int(x) for x in a.shifts.split(",") if x != ""]
    skews = [int(x) for x in a.skews.split(",") if x != ""]
    keep = []
    if shifts:
        total = sum(w.numel() * 2 for w in weights) + max(shifts) + 4096
        buf = torch.empty(total, dtype=torch.uint8, device="cuda")
        keep.append(buf)
        for d in shifts:
            outs, off = [], d
            for w in weights:
                nb = w.numel() * 2
                outs.append(buf[off:off + nb].view(torch.float16).view(w.shape))
                off += nb
            arms[f"arena@{d}"] = outs
    for sk in skews:
        total = sum(w.numel() * 2 for w in weights) + sk * len(weights) + 4096
        buf = torch.empty(total, dtype=torch.uint8, device="cuda")
        keep.append(buf)
        outs, off = [], 0
        for w in weights:
            nb = w.numel() * 2
            outs.append(buf[off:off + nb].view(torch.float16).view(w.shape))
            off += (nb + sk + 255) // 256 * 256
        arms[f"arena+{sk}"] = outs
    if not a.no_rev:
        arms["rev"] = list(reversed([torch.empty_like(w) for w in reversed(weights)]))
    clones = [w.clone() for w in weights]  # in place on copies: the other arms' inputs stay untouched
    plans = {k: (kernels.BatchPlan(clones, 4, 128, False, outs=clones) if k == "inplace"
                 else kernels.BatchPlan(weights, 4, 128, False, outs=v)) for k, v in arms.items()}
    # the box's own copy rate on buffers that are not the plan's
    rows = numel // 4096
    src = torch.empty(rows, 4096, dtype=torch.float16, device="cuda")
    kernels.fill_synthetic(src, 12345)
    fresh = kernels.BatchPlan([src], 4, 128, False)
    st = torch.cuda.current_stream()
    # every quantizing variant must give the product kernel's bits on every weight
    p0 = plans["default"]
    p0.run(st, variant=0)
    torch.cuda.synchronize()
    ref = [o.clone() for o in p0.outs]
    for v in ([] if a.pmc else variants):
        if v == 0 or v in NON_QUANTIZING:
            continue
        for o in p0.outs:
            o.zero_()
        p0.run(st, variant=v)
        torch.cuda.synchronize()
        bad = sum(not torch.equal(o.view(torch.int16), r.view(torch.int16)) for o, r in zip(p0.outs, ref))
        assert p0.nan_flag.item() == 0
        print(json.dumps({"check": v, "weights_differing": int(bad)}), flush=True)
        assert bad == 0, f"variant {v} differs from the product kernel on {bad} weights"
    del ref
    if not a.pmc:
        bench.clock_ramp(plans["default"], 1.0)
    sep = torch.empty(16, dtype=torch.float16, device="cuda")
    fh = open(a.out, "a") if a.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if fh:
            fh.write(line + "\n")
            fh.flush()

    def best_ms(plan, v):
        best = None
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(10):
                plan.run(st, variant=v)
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            best = ms if best is None else min(best, ms)
        return best

    for rnd in range(1 if a.pmc else a.rounds):
        if a.pmc:
            kernels.fill_synthetic(sep, 0)
        ms = best_ms(fresh, 100)
        emit({"round": rnd, "arm": "ceiling/fresh", "variant": 100, "ms": round(ms, 4),
              "GBps": round(numel * 4 / (ms * 1e-3) / 1e9, 1)})
        for k, plan in plans.items():
            for v in variants:
                if a.pmc:
                    kernels.fill_synthetic(sep, 0)
                ms = best_ms(plan, v)
                b = numel * 4 if v in NON_QUANTIZING else alg
                emit({"round": rnd, "arm": k, "variant": v, "ms": round(ms, 4),
                      "GBps": round(b / (ms * 1e-3) / 1e9, 1), "frac": round(b / (ms * 1e-3) / 8e12, 4)})


if __name__ == "__main__":
    main()

"""Interleaved A/B timing of prefill GEMM variants (iwq_w4a16_gemm flags variant) against the
reference forward F.linear(x, W_deq) (hipBLASLt fp16): every round times each arm once (R calls
back to back, HIP events), arms in rotating order, median over rounds (cdna_hip_programming.md
§5.4 rule 24: same process, interleaved, after a clock ramp).  One JSON line per (shape, arm)."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"q_proj": (4096, 4096), "gate_proj": (11008, 4096), "down_proj": (4096, 11008),
          "70b_q": (8192, 8192), "70b_gate": (28672, 8192), "70b_down": (8192, 28672)}


def nib_layout(codes, N, K):
    """Row-major packed codes -> the NIB layout of prefill variants 66/67 (nibble p of each code dword
    holds k = (0, 2, 4, 6, 1, 3, 5, 7)[p]); A/B and tests only."""
    c = codes.view(N, K // 8, 4)
    lo, hi = c & 0xF, c >> 4
    out = torch.stack([lo[..., 0] | (lo[..., 1] << 4), lo[..., 2] | (lo[..., 3] << 4),
                       hi[..., 0] | (hi[..., 1] << 4), hi[..., 2] | (hi[..., 3] << 4)], dim=-1)
    return out.reshape(N, K // 2).contiguous()


NIB_VARIANTS = (66, 67, 69, 71, 75, 77, 81, 99, 152, 153, 163, 165, 168, 169, 172)
GM_VARIANTS = (158, 159, 160)  # grouped parameters held group-major


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--group", type=int, default=-2)
    ap.add_argument("--variants", default="0,45,47")
    ap.add_argument("--shapes", default="q_proj,gate_proj,down_proj")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--warm-seconds", type=float, default=2.0)
    ap.add_argument("--lib", default=None, help="load this library build instead (A/B of two builds)")
    ap.add_argument("--tag", default=None)
    ap.add_argument("--scales", default="data", choices=("data", "pow2", "ones"),
                    help="DIAGNOSTIC: replace the scales by 2^round(log2 s) or 1 (low-entropy B operand; "
                         "hipblaslt then runs on the matching dequantized weight)")
    a = ap.parse_args()
    if a.lib:
        from iron_weight_only_quant_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    from iron_weight_only_quant_amd import kernels
    xw = torch.randn(8192, 4096, device="cuda").half()
    ww = torch.randn(4096, 4096, device="cuda").half()
    t_end = time.time() + a.warm_seconds
    while time.time() < t_end:
        for _ in range(20):
            torch.nn.functional.linear(xw, ww)
        torch.cuda.synchronize()
    del xw, ww
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        w = torch.empty(N, K, dtype=torch.float16, device="cuda")
        kernels.fill_synthetic(w, 7)
        r = kernels.quantize_minmax(w, 4, a.group, False, 0, want_codes=True)
        if a.scales != "data":
            s = r.scales.float()
            s = torch.ones_like(s) if a.scales == "ones" else torch.exp2(torch.round(torch.log2(s)))
            r.scales.copy_(s.half())
            kernels.dequant_packed(r.codes, r.scales, r.zeros, 4, a.group, N, K, out=r.out)
        x = (torch.randn(a.m, K, device="cuda") * 0.5).half()
        y = torch.empty(a.m, N, dtype=torch.float16, device="cuda")
        arms = {"hipblaslt": lambda: torch.nn.functional.linear(x, r.out)}
        nib = nib_layout(r.codes, N, K)
        toks = a.variants.split(",")
        if "nib" in toks:  # the product NIB path: iwq_nib_codes + IWQ_FLAG_NIB_CODES, default dispatch
            toks.remove("nib")
            nc = kernels.nib_codes(r.codes, N, K)
            arms["nib"] = lambda nc=nc: kernels.w4a16_gemm(x, nc, r.scales, r.zeros, 4, a.group, N, out=y, nib=True)
        if "gm" in toks or "nibgm" in toks:  # group-major parameter copies (IWQ_FLAG_GROUP_MAJOR), grouped only
            sgm, zgm = kernels.group_major_params(r.scales, r.zeros, N, K, a.group)
            if "gm" in toks:
                toks.remove("gm")
                arms["gm"] = lambda sgm=sgm, zgm=zgm: kernels.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, a.group, N,
                                                                         out=y, scales_gm=sgm, zeros_gm=zgm)
            if "nibgm" in toks:
                toks.remove("nibgm")
                ncg = kernels.nib_codes(r.codes, N, K)
                arms["nibgm"] = lambda sgm=sgm, zgm=zgm, ncg=ncg: kernels.w4a16_gemm(
                    x, ncg, r.scales, r.zeros, 4, a.group, N, out=y, nib=True, scales_gm=sgm, zeros_gm=zgm)
        for t in [t for t in toks if t.startswith("gm")]:  # gmNNN: A/B variant NNN on group-major parameters
            toks.remove(t)
            v = int(t[2:])
            sgm, zgm = kernels.group_major_params(r.scales, r.zeros, N, K, a.group)
            cd = nib if v in NIB_VARIANTS else r.codes
            fl = kernels.gemm_variant_flags(v) | kernels.L.IWQ_FLAG_GROUP_MAJOR
            arms[t] = (lambda fl=fl, cd=cd, sgm=sgm, zgm=zgm: kernels.w4a16_gemm(x, cd, sgm, zgm, 4, a.group, N,
                                                                                  flags=fl, out=y))
        for v in [int(t) for t in toks]:
            fl = kernels.gemm_variant_flags(v)
            cd = nib if v in NIB_VARIANTS else r.codes
            sc, zr = r.scales, r.zeros
            if v in GM_VARIANTS:  # group-major parameters, [gpr, N]
                gpr = sc.numel() // N
                sc = sc.reshape(N, gpr).t().contiguous().reshape(r.scales.shape)
                zr = None if zr is None else zr.reshape(N, gpr).t().contiguous().reshape(r.zeros.shape)
            arms[f"v{v}"] = (lambda fl=fl, cd=cd, sc=sc, zr=zr: kernels.w4a16_gemm(x, cd, sc, zr, 4, a.group, N,
                                                                                   flags=fl, out=y))
        for f in arms.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in arms}
        st = torch.cuda.current_stream()
        keys = list(arms)
        for rd in range(a.rounds):
            order = keys[rd % len(keys):] + keys[:rd % len(keys)]
            for k in order:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.reps):
                    arms[k]()
                e1.record(st)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.reps)
        flops = 2.0 * a.m * N * K
        for k in keys:
            ts = sorted(times[k])
            med = ts[len(ts) // 2]
            print(json.dumps({"shape": name, "M": a.m, "N": N, "K": K, "group": a.group, "arm": k, "tag": a.tag,
                              "ms": round(med, 4), "ms_min": round(ts[0], 4), "tflops": round(flops / med / 1e9, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()

"""ISA lint for the hand-ordered prefill kernels (iwq_prefill.hip: k_w4a16_b32w / b32v / b32s / w4h / w4b).

Those kernels issue their LDS reads and writes as inline asm and count the lgkmcnt waits by hand,
which the compiler cannot see: a register an asm ds_read fills is only valid once a wait has retired
that read.  This tool compiles iwq_prefill.hip for gfx950 to assembly (the build's flags) and walks
every such kernel in program order, modelling the LDS queue: ds_read_b128 / ds_write_b128 enter it,
`s_waitcnt lgkmcnt(n)` retires all but the n newest.  Any instruction that touches a VGPR of a
still-pending read is reported (a use before the data landed, or an overwrite racing it).
Straight-line model: branches are ignored, which is exact for these kernels' loop bodies (one basic
block each) and conservative at block boundaries.

Second check (--store-hazard, every csrc/*.hip): a buffer_store_dwordx3/x4 whose data VGPRs the very
next instruction overwrites.  ROCm 7.2's LLVM inserts no wait state there when the store carries an
SGPR soffset, and gfx950 then stores the overwritten value (seen as scattered garbage dwords in the
per-tensor one-pass kernel's output before it moved to global stores).

usage: python tools/check_lds_waits.py [--asm file.s] [--store-hazard]   (exit 1 on any finding)"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "iron_weight_only_quant_amd", "csrc")
KERNELS = re.compile(r"^(_ZN3iwq12_GLOBAL__N_1\d+k_w4a16_(?:b32w|b32v|b32s|w4h|w4b|h2v)\w*):", re.M)


def compile_asm(out):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "--offload-device-only", "-S", os.path.join(CSRC, "iwq_prefill.hip"), "-I", CSRC, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)


def vregs(text):
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        regs.update(range(int(a), int(b) + 1))
    regs.update(int(x) for x in re.findall(r"\bv(\d+)\b", text))
    return regs


def check_kernel(lines):
    pending = []  # (kind, vgpr set) in issue order
    findings = []
    for n, raw in enumerate(lines):
        t = raw.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op == "s_waitcnt" and "lgkmcnt" in t:
            keep = int(re.search(r"lgkmcnt\((\d+)\)", t).group(1))
            pending = pending[len(pending) - keep:] if keep else []
            continue
        if op.startswith("ds_read"):
            dst = t.split(None, 1)[1].split(",")[0]
            hit = [p for p in pending if p[1] & vregs(t.split(",", 1)[1])]
            if hit:
                findings.append((n, t))
            pending.append(("r", vregs(dst)))
            continue
        if op.startswith("ds_write"):
            hit = [p for p in pending if p[0] == "r" and p[1] & vregs(t)]
            if hit:
                findings.append((n, t))
            pending.append(("w", set()))
            continue
        used = vregs(t)
        if any(p[0] == "r" and p[1] & used for p in pending):
            findings.append((n, t))
    return findings


def check_store_hazard(lines):
    """(line, store, next) for each >8-byte buffer store whose data registers the next instruction writes."""
    insts = [(n, r.strip()) for n, r in enumerate(lines)
             if r.strip() and not r.strip().startswith((";", ".")) and not r.strip().endswith(":")]
    out = []
    for (n, t), (_, nxt) in zip(insts, insts[1:]):
        if not re.match(r"buffer_store_dwordx[34]\b", t):
            continue
        data = vregs(t.split(None, 1)[1].split(",")[0])
        parts = nxt.split(None, 1)
        if len(parts) == 2 and not parts[0].startswith(("s_", "buffer_store", "global_store", "ds_write")):
            if vregs(parts[1].split(",")[0]) & data:
                out.append((n, t, nxt))
    return out


def store_hazard_all():
    bad = 0
    with tempfile.TemporaryDirectory() as d:
        for f in sorted(os.listdir(CSRC)):
            if not f.endswith(".hip"):
                continue
            out = os.path.join(d, f + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                            "-ffp-contract=off", "--offload-device-only", "-S", os.path.join(CSRC, f),
                            "-I", CSRC, "-o", out], check=True, capture_output=True)
            found = check_store_hazard(open(out).read().split("\n"))
            bad += len(found)
            print(f"{f}: {len(found)} store-data hazard(s)" + "".join(f"\n    line {n}: {t}  ->  {x}" for n, t, x in found[:5]))
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", help="existing gfx950 assembly of iwq_prefill.hip")
    ap.add_argument("--store-hazard", action="store_true", help="also scan every csrc/*.hip for the buffer-store data hazard")
    a = ap.parse_args()
    if a.asm:
        text = open(a.asm).read()
    else:
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "iwq_prefill.s")
            compile_asm(out)
            text = open(out).read()
    names = KERNELS.findall(text)
    bad = 0
    for name in names:
        i = text.index(name + ":")
        j = text.index(".Lfunc_end", i)
        f = check_kernel(text[i:j].split("\n"))
        bad += len(f)
        print(f"{name}: {len(f)} finding(s)" + "".join(f"\n    line {n}: {t}" for n, t in f[:5]))
    print(f"{len(names)} kernels checked, {bad} finding(s)")
    if a.store_hazard:
        bad += store_hazard_all()
    return 1 if bad or not names else 0


if __name__ == "__main__":
    sys.exit(main())

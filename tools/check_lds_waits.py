"""ISA lint for the hand-ordered prefill kernels (iwq_prefill.hip: k_w4a16_b32w / b32v / b32s / w4h / w4b;
iwq_prefill16.hip: k_w4a16_b16w, k_w4a16_b16q).

Those kernels issue their LDS reads and writes as inline asm and count the lgkmcnt waits by hand,
which the compiler cannot see: a register an asm ds_read fills is only valid once a wait has retired
that read.  This tool compiles iwq_prefill.hip for gfx950 to assembly (the build's flags) and walks
every such kernel in program order, modelling the LDS queue: ds_read_b128 / ds_write_b128 enter it,
`s_waitcnt lgkmcnt(n)` retires all but the n newest.  Any instruction that touches a VGPR of a
still-pending read is reported (a use before the data landed, or an overwrite racing it).
Control flow: the kernel is cut into basic blocks (labels, s_branch / s_cbranch_*), and the queue at
a block's entry is the merge of its predecessors' exit queues aligned from the newest entry (what
`lgkmcnt(n)` keeps), iterated to a fixed point -- exact for straight-line loop bodies and for the
wave-uniform branches around the staggered barriers of k_w4a16_b16w.

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
KERNELS = re.compile(r"^(_ZN3iwq12_GLOBAL__N_1\d+k_w4a16_(?:b32w|b32v|b32s|w4h|w4b|h2v|b16w|b16q|b16r|b16p)\w*):", re.M)
SOURCES = ("iwq_prefill.hip", "iwq_prefill16.hip")


def compile_asm(out, src="iwq_prefill.hip"):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-DIWQ_AB=1", "--offload-device-only", "-S", os.path.join(CSRC, src), "-I", CSRC, "-o", out]  # every variant
    subprocess.run(cmd, check=True, capture_output=True)


def vregs(text):
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        regs.update(range(int(a), int(b) + 1))
    regs.update(int(x) for x in re.findall(r"\bv(\d+)\b", text))
    return regs


def _step(pending, t, n, findings):
    """One instruction: updated queue; appends (n, t) to findings on a hazard."""
    op = t.split()[0]
    if op == "s_waitcnt" and "lgkmcnt" in t:
        keep = int(re.search(r"lgkmcnt\((\d+)\)", t).group(1))
        return pending[len(pending) - keep:] if keep else []
    if op.startswith("ds_read"):
        dst = t.split(None, 1)[1].split(",")[0]
        if any(p[1] & vregs(t.split(",", 1)[1]) for p in pending):
            findings.append((n, t))
        return pending + [("r", vregs(dst))]
    if op.startswith("ds_write"):
        if any(p[0] == "r" and p[1] & vregs(t) for p in pending):
            findings.append((n, t))
        return pending + [("w", set())]
    used = vregs(t)
    if any(p[0] == "r" and p[1] & used for p in pending):
        findings.append((n, t))
    return pending


def _merge(a, b):
    """Queues aligned from the newest entry; an entry is a read if either is, registers united."""
    if a is None:
        return b
    la, lb = len(a), len(b)
    out = []
    for i in range(max(la, lb), 0, -1):
        ea = a[la - i] if i <= la else None
        eb = b[lb - i] if i <= lb else None
        if ea is None or eb is None:
            out.append(ea or eb)
        else:
            out.append(("r" if "r" in (ea[0], eb[0]) else "w", ea[1] | eb[1]))
    return out


def check_kernel(lines):
    # basic blocks: (first line, [(n, instruction)], successor labels, falls through)
    blocks, cur, label_of = [], None, {}
    for n, raw in enumerate(lines):
        t = raw.strip()
        if not t or t.startswith(";") or (t.startswith(".") and not t.endswith(":")):
            continue
        if t.endswith(":"):
            if cur is not None:
                blocks.append(cur)
            cur = {"label": t[:-1], "ins": [], "succ": [], "fall": True}
            label_of[t[:-1]] = len(blocks)
            continue
        if cur is None:
            cur = {"label": None, "ins": [], "succ": [], "fall": True}
        cur["ins"].append((n, t))
        op = t.split()[0]
        if op == "s_branch" or op.startswith("s_cbranch") or op == "s_endpgm":
            if op != "s_endpgm":
                cur["succ"].append(t.split()[-1])
            cur["fall"] = op.startswith("s_cbranch")
            blocks.append(cur)
            cur = {"label": None, "ins": [], "succ": [], "fall": True}
    if cur is not None:
        blocks.append(cur)
    index = {b["label"]: i for i, b in enumerate(blocks) if b["label"]}
    succs = []
    for i, b in enumerate(blocks):
        s = [index[x] for x in b["succ"] if x in index]
        if b["fall"] and i + 1 < len(blocks):
            s.append(i + 1)
        succs.append(s)
    entry = [None] * len(blocks)
    entry[0] = []
    work = [0]
    findings = set()
    while work:
        i = work.pop()
        q = entry[i]
        f = []
        for n, t in blocks[i]["ins"]:
            q = _step(q, t, n, f)
        findings.update(f)
        for j in succs[i]:
            m = _merge(entry[j], q)
            if m != entry[j]:
                entry[j] = m
                work.append(j)
    return sorted(findings)


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
                            "-ffp-contract=off", "-DIWQ_AB=1", "--offload-device-only", "-S", os.path.join(CSRC, f),
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
        text = ""
        with tempfile.TemporaryDirectory() as d:
            for src in SOURCES:
                out = os.path.join(d, src + ".s")
                compile_asm(out, src)
                text += open(out).read()
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

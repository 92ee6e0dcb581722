"""In-tree build of the HIP library (hipcc, gfx950).  No torch JIT cache: the .so travels with the repo."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(OUT_DIR, "libiwq.so")
# IWQ_AB=1: the A/B library (every kernel variant kept for timing and its bit-identity tests,
# csrc/iwq_common.cuh), built beside the product one from its own objects; _lib.py loads it when
# IWQ_AB=1 is set in the environment.
AB_OUT_DIR = os.path.join(OUT_DIR, "ab")
LIB_AB = os.path.join(OUT_DIR, "libiwq_ab.so")


def ab_requested():
    return os.environ.get("IWQ_AB", "0") == "1"
SOURCES = ["iwq_minmax.hip", "iwq_batched.hip", "iwq_fp.hip", "iwq_bfp.hip", "iwq_gemm.hip", "iwq_prefill.hip", "iwq_synth.hip",
           "iwq_fpunpack.hip", "iwq_codes.hip", "iwq_prefill16.hip", "iwq_fpdt.hip", "iwq_prefill_ws.hip"]
DEPS = SOURCES + ["iwq_minmax.cuh", "iwq_common.cuh", "iwq_seg.cuh", "iwq_fp.cuh", "iwq_fp_tables.h", "iwq_prefill.h",
                  "iwq_fp_tables_dt.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# Numerics: no FMA contraction, IEEE fp32 division, denormals preserved.
# --offload-compress: the gfx950 code objects are stored compressed in the .so (35 -> ~9 MiB; the HIP
# runtime inflates them once at load), which keeps every push of the tree to a GPU box small.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall",
         "-Wno-unused-function", "--offload-compress"]


def library_path(ab=None):
    return LIB_AB if (ab_requested() if ab is None else ab) else LIB


def _stale(ab=False):
    lib = LIB_AB if ab else LIB
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(HERE, "..", "include", "iwq.h")]
    if any(os.path.getmtime(d) > t for d in deps if os.path.exists(d)):
        return True
    # a source edited while a build was running is older than the library that build linked, but
    # newer than the object compiled from its previous text: compare objects with their sources too
    out_dir = AB_OUT_DIR if ab else OUT_DIR
    headers = [os.path.join(CSRC, d) for d in DEPS if d not in SOURCES] + [os.path.join(HERE, "..", "include", "iwq.h")]
    newest_header = max(os.path.getmtime(h) for h in headers if os.path.exists(h))
    for src in SOURCES:
        obj = os.path.join(out_dir, os.path.splitext(src)[0] + ".o")
        if os.path.exists(obj) and (os.path.getmtime(obj) < os.path.getmtime(os.path.join(CSRC, src))
                                    or os.path.getmtime(obj) < newest_header):
            return True
    return False


def build_library(force=False, verbose=True, ab=None):
    """Compile each translation unit in parallel (-fgpu-rdc not needed: no cross-TU device calls),
    then link the shared library (ab: the A/B library, default from IWQ_AB)."""
    ab = ab_requested() if ab is None else ab
    lib = LIB_AB if ab else LIB
    if not force and not _stale(ab):
        return lib
    from concurrent.futures import ThreadPoolExecutor
    out_dir = AB_OUT_DIR if ab else OUT_DIR
    os.makedirs(out_dir, exist_ok=True)
    objs = [os.path.join(out_dir, os.path.splitext(s)[0] + ".o") for s in SOURCES]
    compile_flags = [f for f in FLAGS if f != "-shared"] + (["-DIWQ_AB=1"] if ab else [])

    def cc(src_obj):
        src, obj = src_obj
        cmd = [HIPCC] + compile_flags + ["-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print("[iwq build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd=CSRC)

    # recompile only objects older than their source or any shared header
    headers = [os.path.join(CSRC, d) for d in DEPS if d not in SOURCES] + [os.path.join(HERE, "..", "include", "iwq.h")]
    newest_header = max(os.path.getmtime(h) for h in headers if os.path.exists(h))

    def obj_stale(src_obj):
        src, obj = src_obj
        return (force or not os.path.exists(obj) or os.path.getmtime(obj) < newest_header
                or os.path.getmtime(obj) < os.path.getmtime(os.path.join(CSRC, src)))
    todo = [so for so in zip(SOURCES, objs) if obj_stale(so)]
    with ThreadPoolExecutor(max_workers=max(1, min(len(todo), os.cpu_count() or 1))) as ex:
        list(ex.map(cc, todo))
    tmp = lib + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print("[iwq build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    import sys
    build_library(force="--force" in sys.argv, ab=True if "--ab" in sys.argv else None)

"""In-tree build of the HIP library (hipcc, gfx950).  No torch JIT cache: the .so travels with the repo."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(OUT_DIR, "libiwq.so")
SOURCES = ["iwq_minmax.hip", "iwq_synth.hip"]
DEPS = SOURCES + ["iwq_common.cuh"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# Numerics: no FMA contraction, IEEE fp32 division, denormals preserved.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall",
         "-Wno-unused-function"]


def library_path():
    return LIB


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(HERE, "..", "include", "iwq.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_library(force=False, verbose=True):
    if not force and not _stale():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print("[iwq build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, LIB)
    return LIB

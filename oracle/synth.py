"""Counter-based synthetic weight generator (test/bench infrastructure, NOT product code).

The same generator is implemented in HIP (`iwq_fill_synthetic` in
iron_weight_only_quant_amd/csrc/iwq_synth.hip) so the GPU box can regenerate the
exact inputs that the golden fixtures were computed on, without torch RNG and
without the reference.  Every step is integer arithmetic or a single correctly
rounded IEEE operation, so numpy and the GPU produce identical bits:

    state = seed * 0xD2B74407B1CE6E93 + index          (mod 2^64)
    h     = splitmix64(state)
    S     = sum of the four 16-bit fields of h          (Irwin-Hall(4), ~N(0,1) after centring)
    x     = f32(S - 131070) * f32(0.02 / 37837.23)      (one f32 multiply, RNE)
    x     = x * 8  if (u0 ^ u3) & 0x3FF == 0            (1/1024 outliers, exact power of two)
    w     = RNE_to_dtype(x)

i.e. Llama-like weights w ~ N(0, 0.02^2) with a sparse x8 outlier tail
(SURVEY.md §8d "Synthetic inputs").
"""
import numpy as np

MASK64 = (1 << 64) - 1
SEED_MUL = np.uint64(0xD2B74407B1CE6E93)
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
MIX1 = np.uint64(0xBF58476D1CE4E5B9)
MIX2 = np.uint64(0x94D049BB133111EB)
SCALE = np.float32(0.02 / 37837.23)


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + GOLDEN
        z = (z ^ (z >> np.uint64(30))) * MIX1
        z = (z ^ (z >> np.uint64(27))) * MIX2
        return z ^ (z >> np.uint64(31))


def synth_f32(seed, start, count):
    """f32 values (before the final rounding to the storage dtype) for flat indices [start, start+count)."""
    idx = np.arange(start, start + count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        state = np.uint64(seed) * SEED_MUL + idx
    h = _splitmix64(state)
    u0 = (h & np.uint64(0xFFFF)).astype(np.int64)
    u1 = ((h >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64)
    u2 = ((h >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)
    u3 = ((h >> np.uint64(48)) & np.uint64(0xFFFF)).astype(np.int64)
    s = (u0 + u1 + u2 + u3 - 131070).astype(np.float32)  # exact: |s| < 2^18
    x = s * SCALE
    outlier = ((u0 ^ u3) & 0x3FF) == 0
    x = np.where(outlier, x * np.float32(8.0), x).astype(np.float32)
    return x


def synth(seed, shape, dtype="float16"):
    """Synthetic tensor of `shape` (row-major flat index) as numpy array.

    dtype: "float16" | "float32" | "bfloat16" (bfloat16 returned as uint16 bit patterns)."""
    n = int(np.prod(shape))
    out = np.empty(n, dtype=np.float32)
    chunk = 1 << 24
    for s in range(0, n, chunk):
        c = min(chunk, n - s)
        out[s:s + c] = synth_f32(seed, s, c)
    if dtype == "float16":
        return out.astype(np.float16).reshape(shape)
    if dtype == "float32":
        return out.reshape(shape)
    if dtype == "bfloat16":
        from .iwq_oracle import f32_to_bf16_bits
        return f32_to_bf16_bits(out).reshape(shape)
    raise ValueError(dtype)

"""Helpers for loading the committed golden fixtures (data only; no reference code)."""
import hashlib
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_small():
    return np.load(os.path.join(GOLD, "int_small.npz"))


def load_edge():
    return np.load(os.path.join(GOLD, "int_edge.npz"))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def raw_bits(a):
    a = np.ascontiguousarray(a)
    if a.dtype in (np.float16, np.int16, np.uint16):
        return a.view(np.uint16)
    if a.dtype in (np.float32, np.int32, np.uint32):
        return a.view(np.uint32)
    raise TypeError(a.dtype)


def bits_equal(a, b, nan_equal=False):
    """Bit-exact equality of two 16/32-bit float arrays (NaNs equal to any NaN if nan_equal)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    ra, rb = raw_bits(a), raw_bits(b)
    if nan_equal:
        fa = a.astype(np.float32) if a.dtype != np.uint16 else None
        fb = b.astype(np.float32) if b.dtype != np.uint16 else None
        if fa is not None:
            na, nb = np.isnan(fa), np.isnan(fb)
            if not np.array_equal(na, nb):
                return False
            return bool(np.array_equal(ra[~na], rb[~nb]))
    return bool(np.array_equal(ra, rb))

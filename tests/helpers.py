"""Shared helpers for the tests: exact big-integer references and slot maps."""
import numpy as np


def to_int(limbs):
    a = np.ascontiguousarray(limbs, dtype=np.uint64)
    return int.from_bytes(a.tobytes(), "little")


def from_int(v, nlimbs):
    if v < 0:
        v += 1 << (64 * nlimbs)
    return np.frombuffer(v.to_bytes(8 * nlimbs, "little"), dtype=np.uint64).copy()


def revbin(x, bits):
    out = 0
    for _ in range(bits):
        out = (out << 1) | (x & 1)
        x >>= 1
    return out


def log2(v):
    d = 0
    while (1 << d) < v:
        d += 1
    return d


def chunks(x, count, bits1):
    """FFT_split_bits (mul_fft.c:115): the bits1-bit pieces of integer x."""
    mask = (1 << bits1) - 1
    return [(x >> (j * bits1)) & mask for j in range(count)]


def valid_shape(depth, w, n1, n2):
    n = 1 << depth
    if (n * w) % 64:
        return False
    bits1 = (n * w - depth) // 2
    j1 = (64 * n1 - 1) // bits1 + 1
    j2 = (64 * n2 - 1) // bits1 + 1
    return j1 + j2 - 1 <= 2 * n


def max_limbs(depth, w):
    """largest balanced n1 = n2 that fits the length-2^(depth+1) convolution"""
    n = 1 << depth
    bits1 = (n * w - depth) // 2
    lo, hi = 1, (2 * n * bits1) // 64 + 2
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if valid_shape(depth, w, mid, mid):
            lo = mid
        else:
            hi = mid - 1
    return lo

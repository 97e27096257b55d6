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


def valid_shape6(depth, w, n1, n2):
    """new_mpn_mul6 (mul_fft.c:3573): bits1 = (N - depth - 1)/2, room for 4n coefficients"""
    n = 1 << depth
    if (n * w) % 64:
        return False
    bits1 = (n * w - depth - 1) // 2
    j1 = (64 * n1 - 1) // bits1 + 1
    j2 = (64 * n2 - 1) // bits1 + 1
    return j1 + j2 - 1 <= 4 * n


def max_limbs6(depth, w):
    """largest balanced n1 = n2 that fits the length-2^(depth+2) sqrt2 convolution"""
    n = 1 << depth
    bits1 = (n * w - depth - 1) // 2
    lo, hi = 1, (4 * n * bits1) // 64 + 2
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if valid_shape6(depth, w, mid, mid):
            lo = mid
        else:
            hi = mid - 1
    return lo


def shapes6(rng, count):
    """new_mpn_mul6 shapes: odd w (sqrt2 twiddles) and even w, full, truncated past 2n,
    below 2n (second half unused) and unbalanced"""
    out = []
    for depth, w in ((6, 1), (6, 3), (7, 1), (8, 1), (8, 2), (9, 1), (10, 1), (11, 1), (8, 5), (6, 4), (12, 1)):
        if ((1 << depth) * w) % 64:
            continue
        mx = max_limbs6(depth, w)
        out.append((depth, w, mx, mx))
        out.append((depth, w, max(1, (3 * mx) // 4), max(1, (3 * mx) // 4)))
        for _ in range(count):
            n1 = rng.randint(1, 2 * mx - 1)
            n2 = rng.randint(1, max(1, 2 * mx - n1))
            if valid_shape6(depth, w, n1, n2):
                out.append((depth, w, n1, n2))
    return out

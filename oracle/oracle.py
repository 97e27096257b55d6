"""TEST INFRASTRUCTURE ONLY -- ctypes view of oracle/liboracle.so.

The oracle is the CPU restatement of wbhart/mpir-fft's new_mpn_mul path
(oracle/mpfft_oracle.c, citing /root/reference/mul_fft.c line by line).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it,
and only as the checker or the timed CPU baseline -- never as product code.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPFFT_ORACLE_LIB: another build of the same source (make -C oracle asan: AddressSanitizer +
# UBSan, scripts/asan_cpu.sh)
_LIB = os.environ.get("MPFFT_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
_lib = None

_u64p = ctypes.POINTER(ctypes.c_uint64)
_L = ctypes.c_long
_UL = ctypes.c_ulong


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        h = ctypes.CDLL(_LIB)
        sig = {
            "orc_new_mpn_mul": [_u64p, _u64p, _L, _u64p, _L, _UL, _UL],
            "orc_params": [_L, _L, _UL, _UL, ctypes.POINTER(ctypes.c_long)],
            "orc_new_mpn_mul6": [_u64p, _u64p, _L, _u64p, _L, _UL, _UL],
            "orc_params6": [_L, _L, _UL, _UL, ctypes.POINTER(ctypes.c_long)],
            "orc_normmod": [_u64p, _L],
            "orc_mul_2expmod": [_u64p, _u64p, _L, ctypes.c_uint],
            "orc_div_2expmod": [_u64p, _u64p, _L, ctypes.c_uint],
            "orc_mul_2exp": [_u64p, _u64p, _L, _UL],
            "orc_lshB_sumdiffmod": [_u64p, _u64p, _u64p, _u64p, _L, _L, _L],
            "orc_sumdiff_rshBmod": [_u64p, _u64p, _u64p, _u64p, _L, _L, _L],
            "orc_mulmod_2expp1": [_u64p, _u64p, _u64p, ctypes.c_int, _L],
            "orc_transform": [ctypes.c_int, _u64p, _L, _UL, _L, _L],
            "orc_split": [_u64p, _L, _u64p, _L, _UL, _L],
            "orc_combine": [_u64p, _u64p, _L, _UL, _L, _L],
            "orc_gmp_mul": [_u64p, _u64p, _L, _u64p, _L],
            "orc_fill_random": [_u64p, _L, ctypes.c_uint64],
        }
        for name, args in sig.items():
            f = getattr(h, name)
            f.argtypes = args
            f.restype = None
        h.orc_mulmod_2expp1.restype = ctypes.c_uint64
        h.orc_split.restype = ctypes.c_long
        _lib = h
    return _lib


def _p(a):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u64p)


def params(n1, n2, depth, w):
    """(n, l, sqrt, j1, j2, trunc, bits1) exactly as new_mpn_mul (mul_fft.c:3193-3203)."""
    out = (ctypes.c_long * 7)()
    lib().orc_params(n1, n2, depth, w, out)
    return tuple(out)


def new_mpn_mul(i1, i2, depth, w):
    i1 = np.ascontiguousarray(i1, dtype=np.uint64)
    i2 = np.ascontiguousarray(i2, dtype=np.uint64)
    r = np.zeros(len(i1) + len(i2), dtype=np.uint64)
    lib().orc_new_mpn_mul(_p(r), _p(i1), len(i1), _p(i2), len(i2), depth, w)
    return r


def params6(n1, n2, depth, w):
    """(n, l, sqrt, j1, j2, trunc, bits1) exactly as new_mpn_mul6 (mul_fft.c:3575-3603)."""
    out = (ctypes.c_long * 7)()
    lib().orc_params6(n1, n2, depth, w, out)
    return tuple(out)


def new_mpn_mul6(i1, i2, depth, w):
    """sqrt2 front end (mul_fft.c:3573-3668): length-4n convolution mod 2^(2^depth w) + 1."""
    i1 = np.ascontiguousarray(i1, dtype=np.uint64)
    i2 = np.ascontiguousarray(i2, dtype=np.uint64)
    r = np.zeros(len(i1) + len(i2), dtype=np.uint64)
    lib().orc_new_mpn_mul6(_p(r), _p(i1), len(i1), _p(i2), len(i2), depth, w)
    return r


def gmp_mul(a, b):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    r = np.zeros(len(a) + len(b), dtype=np.uint64)
    lib().orc_gmp_mul(_p(r), _p(a), len(a), _p(b), len(b))
    return r


def fill_random(count, seed):
    buf = np.empty(count, dtype=np.uint64)
    lib().orc_fill_random(_p(buf), count, seed)
    return buf


def normmod(t, l):
    t = np.array(t, dtype=np.uint64)
    lib().orc_normmod(_p(t), l)
    return t


def mul_2expmod(a, l, d):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    t = np.zeros(l + 1, dtype=np.uint64)
    lib().orc_mul_2expmod(_p(t), _p(a), l, d)
    return t


def div_2expmod(a, l, d):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    t = np.zeros(l + 1, dtype=np.uint64)
    lib().orc_div_2expmod(_p(t), _p(a), l, d)
    return t


def mul_2exp(a, l, e):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    t = np.zeros(l + 1, dtype=np.uint64)
    lib().orc_mul_2exp(_p(t), _p(a), l, e)
    return t


def lshB_sumdiffmod(a, b, l, x, y):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    t = np.zeros(l + 1, dtype=np.uint64)
    u = np.zeros(l + 1, dtype=np.uint64)
    lib().orc_lshB_sumdiffmod(_p(t), _p(u), _p(a), _p(b), l, x, y)
    return t, u


def sumdiff_rshBmod(a, b, l, x, y):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    t = np.zeros(l + 1, dtype=np.uint64)
    u = np.zeros(l + 1, dtype=np.uint64)
    lib().orc_sumdiff_rshBmod(_p(t), _p(u), _p(a), _p(b), l, x, y)
    return t, u


def mulmod_2expp1(a, b, flag, l):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    r = np.zeros(l, dtype=np.uint64)
    top = lib().orc_mulmod_2expp1(_p(r), _p(a), _p(b), flag, l)
    return r, int(top)


FFT, IFFT, FFT_TRUNC, IFFT_TRUNC, FFT_MFA_TRUNC, IFFT_MFA_TRUNC = range(6)


def transform(kind, flat, n, w, n1=0, trunc=0):
    """flat: (2n, l+1) uint64, modified copy returned."""
    flat = np.array(flat, dtype=np.uint64, order="C")
    lib().orc_transform(kind, _p(flat), n, w, n1, trunc)
    return flat


def split(src, count, bits, l):
    src = np.ascontiguousarray(src, dtype=np.uint64)
    flat = np.zeros((count, l + 1), dtype=np.uint64)
    lib().orc_split(_p(flat), count, _p(src), len(src), bits, l)
    return flat


def combine(flat, length, bits, l, total):
    flat = np.ascontiguousarray(flat, dtype=np.uint64)
    r = np.zeros(total, dtype=np.uint64)
    lib().orc_combine(_p(r), _p(flat), length, bits, l, total)
    return r


# ---- exact big-integer helpers (the reference tests' mpz conversions) ----

def to_int(limbs, signed_top=False):
    """mpn_to_mpz (mul_fft.c:3677): little-endian limbs; optional signed top limb."""
    a = np.ascontiguousarray(limbs, dtype=np.uint64)
    v = int.from_bytes(a.tobytes(), "little")
    if signed_top and len(a) and int(a[-1]) >> 63:
        v -= 1 << (64 * len(a))
    return v


def from_int(v, nlimbs):
    if v < 0:
        v += 1 << (64 * nlimbs)
    return np.frombuffer(v.to_bytes(8 * nlimbs, "little"), dtype=np.uint64).copy()

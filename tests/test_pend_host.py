"""Host-side check of the closed form k_rpass uses for DIF pending exponents carried across
passes (rkernels.hpp rp_pend_pos / rp_pend, PassArgs::pcarry / ccarry).

In-place DIF (FFT_radix2 / FFT_radix2_twiddle, mul_fft.c:786, :1397) with deferred
multiplications: a level-lev butterfly on (i, i + h) leaves the top with the top's pending
exponent and the bottom with the top's plus the twiddle rho 2^lev (i mod h).  The kernels use
    E(p) after levels [lo, hi) = sum over lev in [lo, hi) with bit (lbM - lev - 1) of p set of
                                 rho 2^lev (p mod 2^(lbM - hi))   (mod 2N)
for any lo (the levels an earlier pass left pending) -- this test simulates the butterflies
and compares, and also against the per-pass group formula the kernel used before (rp_tw).
"""
import random


def pend_pos(rho, lbm, lo, hi, p, n2):
    xm = p & ((1 << (lbm - hi)) - 1)
    e = 0
    for lev in range(lo, hi):
        if (p >> (lbm - lev - 1)) & 1:
            e = (e + (rho << lev) * xm) % n2
    return e


def simulate(rho, lbm, lo, hi, n2):
    m = 1 << lbm
    e = [0] * m
    for lev in range(lo, hi):
        h = m >> (lev + 1)
        for i in range(m):
            if not i & h:
                e[i + h] = (e[i] + rho * (1 << lev) * (i % h)) % n2
    return e


def group_formula(rho, lbm, lvl0, logg, pos0, pstep, done, s, n2):
    """rp_pend as k_rpass computed it within one pass (no carried levels)."""
    e = 0
    for j in range(done):
        if (s >> (logg - 1 - j)) & 1:
            x = s & ~(((1 << (done - 1 - j)) - 1) << (logg - done))
            jb, level = logg - 1 - j, lvl0 + j
            h = 1 << (lbm - level - 1)
            unit = rho << level
            e = (e + (pos0 & (h - 1)) * unit + (x & ((1 << jb) - 1)) * pstep * unit) % n2
    return e


def test_pending_closed_form():
    rng = random.Random(5)
    for _ in range(120):
        lbm = rng.randint(2, 9)
        n = rng.choice([64, 128, 256]) * 1024
        rho = (2 * n) >> lbm
        logg = rng.randint(1, min(3, lbm))
        lvl0 = rng.randint(0, lbm - logg)
        lo = rng.randint(0, lvl0)
        for done in range(logg + 1):
            want = simulate(rho, lbm, lo, lvl0 + done, 2 * n)
            assert [pend_pos(rho, lbm, lo, lvl0 + done, p, 2 * n) for p in range(1 << lbm)] == want
            if lo == lvl0:
                lobits = lbm - lvl0 - logg
                for grp in range(1 << (lbm - logg)):
                    pos0 = ((grp >> lobits) << (lbm - lvl0)) | (grp & ((1 << lobits) - 1))
                    for s in range(1 << logg):
                        got = group_formula(rho, lbm, lvl0, logg, pos0, 1 << lobits, done, s, 2 * n)
                        assert got == want[pos0 + s * (1 << lobits)]

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


def test_general_rotation_two_reads():
    """rp_get_rot (rkernels.hpp): 2^e y mod 2^N + 1 for y in the register pair form (128-bit words
    w_q plus a small signed overflow h_q at 2^128) from two aligned pair reads: e = ea + d,
    z = 2^ea y (pairwise, signs folded), pair pp of 2^d z = lo(z_pp) + hi(z_pp-1) with
    lo = (w << d) mod 2^128, hi = floor(z / 2^(128 - d)), and pair 0 subtracting hi of the top
    pair (2^N == -1, negated after the floor).  Exact big-integer check of that decomposition."""
    rng = random.Random(11)
    for hp in (2, 3, 8, 16):
        n = 128 * hp
        p = (1 << n) + 1
        for _ in range(200):
            w = [rng.getrandbits(128) for _ in range(hp)]
            h = [rng.randint(-3, 3) for _ in range(hp)]
            v = sum((w[q] + h[q] * (1 << 128)) << (128 * q) for q in range(hp)) % p
            e = rng.randrange(2 * n)
            d, ea = e & 127, e - (e & 127)

            def pair(pp):   # rp_get_al: pair pp of 2^ea y as a signed value
                sg = ea >= n
                src = pp - (((ea - n) if sg else ea) >> 7)
                wr = src < 0
                src += hp if wr else 0
                z = w[src] + h[src] * (1 << 128)
                return -z if wr != sg else z

            out = []
            for pp in range(hp):
                a = pair(pp)
                if d == 0:
                    out.append(a)
                    continue
                b = pair(pp - 1 if pp else hp - 1)
                lo = ((a % (1 << 128)) << d) % (1 << 128)
                hi = b >> (128 - d)
                out.append(lo + (hi if pp else -hi))
            assert sum(out[q] << (128 * q) for q in range(hp)) % p == v * pow(2, e, p) % p

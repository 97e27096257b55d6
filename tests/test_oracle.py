"""CPU tests pinning the oracle (oracle/mpfft_oracle.c) to the reference's own
test semantics (/root/reference/mul_fft.c:3777-5608):

  primitives  vs exact big-integer restatements of ref_norm / ref_mul_2expmod /
              ref_div_2expmod / ref_lshB_sumdiffmod / ref_sumdiff_rshBmod
              (mul_fft.c:3699-3760) over reduced versions of the parameter grids
              of test_norm :3777, test_mul_2expmod :3825, test_div_2expmod :3973,
              test_lshB_sumdiffmod :4030, test_sumdiff_rshBmod :4109
  transforms  round trips test_fft_ifft :4276, test_fft_truncate :5031,
              test_fft_ifft_truncate :4472, test_fft_ifft_mfa_truncate :4938 and the
              SURVEY 8a/a3 slot-map spec of FFT_radix2_mfa_truncate
  new_mpn_mul vs the exact product (Python int, GMP mpn_mul -- the reference's
              integration oracle, mul_fft.c:5542) over random/adversarial shapes
"""
import random

import numpy as np
import pytest

from helpers import chunks, from_int, log2, max_limbs, revbin, to_int, valid_shape


def signed_val(limbs):
    """mpn_to_mpz (mul_fft.c:3677): (l+1) limbs, signed top limb."""
    v = to_int(limbs)
    n = len(limbs)
    if int(limbs[-1]) >> 63:
        v -= 1 << (64 * n)
    return v


def rand_n(rng, l):
    """rand_n (mul_fft.c:3770): l random limbs, top limb in [-9, 9]."""
    a = np.array([rng.getrandbits(64) for _ in range(l)] + [0], dtype=np.uint64)
    top = rng.randrange(10) * (-1 if rng.randrange(2) else 1)
    a[l] = np.uint64(top & (2**64 - 1))
    return a


def grid(rng, max_i, count):
    """(n, w) pairs of the reference grids: n = i/k, w = j*k, n*w % 64 == 0."""
    out = []
    for i in range(64, max_i, 64):
        for j in range(1, 10):
            for k in (1, 2, 4, 8, 16, 32, 64):
                n, w = i // k, j * k
                if n >= 1 and (n * w) % 64 == 0:
                    out.append((n, w))
    rng.shuffle(out)
    return out[:count]


def test_normmod(oracle):
    rng = random.Random(1)
    for n, w in grid(rng, 32 * 64, 120):
        l = n * w // 64
        p = (1 << (n * w)) + 1
        a = np.array([rng.getrandbits(64) for _ in range(l + 1)], dtype=np.uint64)
        got = oracle.normmod(a, l)
        assert to_int(got) == signed_val(a) % p


def test_normmod_edges(oracle):
    for l in (1, 2, 5):
        p = (1 << (64 * l)) + 1
        for v in (0, 1, p - 1, p - 2, (1 << (64 * l)) - 1):
            for top in (-2, -1, 0, 1, 2):
                a = from_int(v % (1 << (64 * l)), l + 1)
                a[l] = np.uint64(top & (2**64 - 1))
                got = oracle.normmod(a, l)
                want = (v % (1 << (64 * l)) + top * (1 << (64 * l))) % p
                assert to_int(got) == want
                assert int(got[l]) in (0, 1)


def test_mul_div_2expmod(oracle):
    rng = random.Random(2)
    for n, w in grid(rng, 64 * 64, 60):
        l = n * w // 64
        p = (1 << (n * w)) + 1
        for d in rng.sample(range(64), 6):
            a = rand_n(rng, l)
            m = oracle.mul_2expmod(a, l, d)
            assert signed_val(m) % p == (signed_val(a) << d) % p
            q = oracle.div_2expmod(a, l, d)
            assert (signed_val(q) << d) % p == signed_val(a) % p


def test_mul_2exp_any_exponent(oracle):
    rng = random.Random(3)
    for l in (1, 2, 3, 8):
        N = 64 * l
        p = (1 << N) + 1
        for _ in range(40):
            a = rand_n(rng, l)
            e = rng.randrange(2 * N)
            got = oracle.mul_2exp(a, l, e)
            assert signed_val(got) % p == (signed_val(a) * pow(2, e, p)) % p


def test_lshB_sumdiffmod(oracle):
    rng = random.Random(4)
    for n, w in grid(rng, 20 * 64, 40):
        l = n * w // 64
        p = (1 << (n * w)) + 1
        for _ in range(min(l, 6)):
            x, y = rng.randrange(l + 1), rng.randrange(l + 1)
            a, b = rand_n(rng, l), rand_n(rng, l)
            t, u = oracle.lshB_sumdiffmod(a, b, l, x, y)
            A, B = signed_val(a), signed_val(b)
            assert signed_val(t) % p == ((A + B) << (64 * x)) % p
            assert signed_val(u) % p == ((A - B) << (64 * y)) % p


def test_sumdiff_rshBmod(oracle):
    rng = random.Random(5)
    for n, w in grid(rng, 20 * 64, 40):
        l = n * w // 64
        p = (1 << (n * w)) + 1
        for _ in range(min(l, 6)):
            x, y = rng.randrange(l), rng.randrange(l)
            a, b = rand_n(rng, l), rand_n(rng, l)
            t, u = oracle.sumdiff_rshBmod(a, b, l, x, y)
            ia = pow(1 << (64 * x), -1, p)
            ib = pow(1 << (64 * y), -1, p)
            A, B = signed_val(a) * ia, signed_val(b) * ib
            assert signed_val(t) % p == (A + B) % p
            assert signed_val(u) % p == (A - B) % p


def test_mulmod_2expp1(oracle):
    rng = random.Random(6)
    for l in (1, 2, 4, 16, 33):
        N = 64 * l
        p = (1 << N) + 1
        vals = [0, 1, p - 2, p - 1, rng.getrandbits(N), rng.getrandbits(N)]
        for A in vals:
            for B in vals:
                a = from_int(A, l + 1)
                b = from_int(B, l + 1)
                flag = int(a[l]) + 2 * int(b[l])
                r, top = oracle.mulmod_2expp1(a[:l], b[:l], flag, l)
                assert to_int(r) + (top << N) == A * B % p


def _norm_all(flat, l):
    return np.stack([np.asarray(__import__("oracle").normmod(row, l)) for row in flat])


def test_fft_ifft_roundtrip(oracle):
    """test_fft_ifft (mul_fft.c:4276): IFFT(FFT(x)) = 2n x."""
    rng = random.Random(7)
    for depth, w in ((4, 4), (6, 1), (7, 2)):
        n = 1 << depth
        l = n * w // 64
        p = (1 << (n * w)) + 1
        x = np.stack([rand_n(rng, l) for _ in range(2 * n)])
        x = _norm_all(x, l)
        y = oracle.transform(oracle.IFFT, oracle.transform(oracle.FFT, x, n, w), n, w)
        for i in range(2 * n):
            assert signed_val(y[i]) % p == (2 * n * to_int(x[i])) % p


def test_fft_truncate_matches_full(oracle):
    """test_fft_truncate (mul_fft.c:5031): truncated FFT == full FFT on outputs < trunc."""
    rng = random.Random(8)
    depth, w = 6, 1
    n = 1 << depth
    l = n * w // 64
    p = (1 << (n * w)) + 1
    for _ in range(12):
        trunc = ((rng.randrange(2 * n) + 1 + 7) // 8) * 8
        x = np.stack([rand_n(rng, l) if i < trunc else np.zeros(l + 1, np.uint64) for i in range(2 * n)])
        x = _norm_all(x, l)
        full = oracle.transform(oracle.FFT, x, n, w)
        tr = oracle.transform(oracle.FFT_TRUNC, x, n, w, 0, trunc)
        for i in range(trunc):
            assert signed_val(full[i]) % p == signed_val(tr[i]) % p


def test_fft_ifft_truncate_roundtrip(oracle):
    """test_fft_ifft_truncate (mul_fft.c:4472)."""
    rng = random.Random(9)
    depth, w = 6, 2
    n = 1 << depth
    l = n * w // 64
    p = (1 << (n * w)) + 1
    for _ in range(12):
        trunc = ((rng.randrange(2 * n) + 1 + 7) // 8) * 8
        x = np.stack([rand_n(rng, l) if i < trunc else np.zeros(l + 1, np.uint64) for i in range(2 * n)])
        x = _norm_all(x, l)
        y = oracle.transform(oracle.IFFT_TRUNC, oracle.transform(oracle.FFT_TRUNC, x, n, w, 0, trunc), n, w, 0, trunc)
        for i in range(trunc):
            assert signed_val(y[i]) % p == (2 * n * to_int(x[i])) % p


@pytest.mark.parametrize("depth,w", [(6, 1), (8, 1), (9, 2)])
def test_mfa_truncate_roundtrip(oracle, depth, w):
    """test_fft_ifft_mfa_truncate (mul_fft.c:4938): random trunc multiple of 2*sqrt."""
    rng = random.Random(10 + depth)
    n = 1 << depth
    sq = 1 << (depth // 2)
    l = n * w // 64
    p = (1 << (n * w)) + 1
    for _ in range(4):
        trunc = (rng.randrange(n // sq) + 1) * sq * 2
        x = _norm_all(np.stack([rand_n(rng, l) for _ in range(2 * n)]), l)
        f = oracle.transform(oracle.FFT_MFA_TRUNC, x, n, w, sq, trunc)
        f = _norm_all(f, l)
        y = oracle.transform(oracle.IFFT_MFA_TRUNC, f, n, w, sq, trunc)
        for j in range(trunc):
            assert signed_val(y[j]) % p == (2 * n * to_int(x[j])) % p


@pytest.mark.parametrize("depth,w", [(6, 1), (7, 2), (8, 1)])
def test_mfa_slot_map(oracle, depth, w):
    """slot r*NC + c == X_{r + NR c} for computed rows r = revbin(s), s < trunc/NC."""
    rng = random.Random(20 + depth)
    n = 1 << depth
    NC = 1 << (depth // 2)
    NR = 2 * n // NC
    N = n * w
    l = N // 64
    p = (1 << N) + 1
    trunc = 2 * NC * max(1, rng.randrange(n // NC) + 1)
    xs = [rng.getrandbits(N - 2) if j < trunc else 0 for j in range(2 * n)]
    flat = np.stack([from_int(v, l + 1) for v in xs])
    f = oracle.transform(oracle.FFT_MFA_TRUNC, flat, n, w, NC, trunc)
    for s in range(trunc // NC):
        r = revbin(s, log2(NR))
        for c in range(NC):
            k = r + NR * c
            want = sum(xj * pow(2, (w * j * k) % (2 * N), p) for j, xj in enumerate(xs) if xj) % p
            assert to_int(f[r * NC + c]) == want


def _shapes(rng, count):
    base = [(2, 16), (3, 8), (4, 4), (5, 2), (6, 1), (6, 3), (7, 1), (8, 2), (9, 1), (10, 3), (11, 1),
            (8, 64), (9, 5), (12, 1), (6, 16), (7, 9)]
    out = []
    for depth, w in base:
        if ((1 << depth) * w) % 64:
            continue
        mx = max_limbs(depth, w)
        out.append((depth, w, mx, mx))
        for _ in range(count):
            n1 = rng.randint(1, 2 * mx - 1)
            n2 = rng.randint(1, 2 * mx - n1) if 2 * mx - n1 >= 1 else 1
            if valid_shape(depth, w, n1, n2):
                out.append((depth, w, n1, n2))
    return out


def test_new_mpn_mul_random(oracle):
    rng = random.Random(11)
    for depth, w, n1, n2 in _shapes(rng, 4):
        a = oracle.fill_random(n1, rng.getrandbits(64))
        b = oracle.fill_random(n2, rng.getrandbits(64))
        r = oracle.new_mpn_mul(a, b, depth, w)
        assert to_int(r) == to_int(a) * to_int(b), (depth, w, n1, n2)


def test_new_mpn_mul_adversarial(oracle):
    """all-ones limbs (max carries), single bits, unbalanced, a coefficient hitting 2^N."""
    for depth, w in ((6, 1), (8, 2), (10, 1)):
        mx = max_limbs(depth, w)
        ones = np.full(mx, 2**64 - 1, dtype=np.uint64)
        cases = [(ones, ones), (ones[:1], ones), (np.eye(1, mx, mx - 1, dtype=np.uint64)[0], ones)]
        one_bit = np.zeros(mx, np.uint64)
        one_bit[0] = 1
        cases.append((one_bit, ones))
        cases.append((np.zeros(mx, np.uint64), ones))
        for a, b in cases:
            if not valid_shape(depth, w, len(a), len(b)):
                continue
            r = oracle.new_mpn_mul(a, b, depth, w)
            assert to_int(r) == to_int(a) * to_int(b)


def test_gmp_checker_agrees(oracle):
    rng = random.Random(12)
    for n1, n2 in ((1, 1), (17, 5), (300, 301), (2000, 100)):
        a = oracle.fill_random(n1, rng.getrandbits(64))
        b = oracle.fill_random(n2, rng.getrandbits(64))
        assert to_int(oracle.gmp_mul(a, b)) == to_int(a) * to_int(b)


def test_split_combine_roundtrip(oracle):
    rng = random.Random(13)
    for bits1, l in ((29, 1), (100, 2), (1018, 32), (8186, 256)):
        n1 = rng.randint(1, 50)
        a = oracle.fill_random(n1, rng.getrandbits(64))
        cnt = (64 * n1 - 1) // bits1 + 1
        flat = oracle.split(a, cnt, bits1, l)
        assert [to_int(r) for r in flat] == chunks(to_int(a), cnt, bits1)
        back = oracle.combine(flat, cnt, bits1, l, n1)
        assert (back == a).all()


def test_oracle_golden_vectors(oracle):
    """The committed golden products (exact: Python int / GMP) reproduce through the oracle."""
    import hashlib
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "products.json")) as f:
        cases = json.load(f)
    for c in cases:
        if c["n1"] + c["n2"] > 1_000_000:
            continue          # the 10^9-bit digests are checked on the GPU box (test_gpu_parity)
        a = oracle.fill_random(c["n1"], int(c["seed1"], 16))
        b = oracle.fill_random(c["n2"], int(c["seed2"], 16))
        r = oracle.new_mpn_mul(a, b, c["depth"], c["w"])
        assert hashlib.sha256(r.tobytes()).hexdigest() == c["sha256"], c["name"]
        if "product_hex" in c:
            assert format(to_int(r), "x") == c["product_hex"]


def test_new_mpn_mul6_random(oracle):
    """sqrt2 front end (mul_fft.c:3573): the oracle's length-4n transforms give the exact
    product (the reference's own check, test_mul4 :5559, compares with mpn_mul)"""
    from helpers import shapes6
    rng = random.Random(21)
    for depth, w, n1, n2 in shapes6(rng, 3):
        a = oracle.fill_random(n1, rng.getrandbits(64))
        b = oracle.fill_random(n2, rng.getrandbits(64))
        r = oracle.new_mpn_mul6(a, b, depth, w)
        assert to_int(r) == to_int(a) * to_int(b), (depth, w, n1, n2)


def test_new_mpn_mul6_test_mul4_shape(oracle):
    """test_mul4 (mul_fft.c:5559-5608): depth 14, w 1, n1 = n2 = 3/4 of 2n bits1 bits"""
    depth, w = 14, 1
    n = 1 << depth
    bits1 = (n * w - (depth + 1)) // 2
    int_limbs = 2 * n * bits1 // 64
    n1 = n2 = (3 * int_limbs) // 4
    a = oracle.fill_random(n1, 0x1001)
    b = oracle.fill_random(n2, 0x2002)
    r = oracle.new_mpn_mul6(a, b, depth, w)
    assert (r == oracle.gmp_mul(a, b)).all()


def test_new_mpn_mul6_adversarial(oracle):
    from helpers import max_limbs6
    for depth, w in ((6, 1), (7, 1), (8, 2)):
        mx = max_limbs6(depth, w)
        ones = np.full(mx, 2**64 - 1, dtype=np.uint64)
        one_bit = np.zeros(mx, np.uint64)
        one_bit[mx - 1] = 1 << 63
        for a, b in ((ones, ones), (ones[:1], ones), (one_bit, ones), (np.zeros(mx, np.uint64), ones)):
            r = oracle.new_mpn_mul6(a, b, depth, w)
            assert to_int(r) == to_int(a) * to_int(b), (depth, w, len(a), len(b))

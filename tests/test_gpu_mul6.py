"""GPU parity of the sqrt2 front end new_mpn_mul6 (mul_fft.c:3573-3668).

The HIP path (k_s2op top level around two length-2n MFA multiplies, through the C ABI)
against the exact product (GMP mpn_mul, the reference's own check in test_mul4,
mul_fft.c:5559-5608) and the oracle's restatement (oracle/mpfft_oracle.c
orc_new_mpn_mul6).  Bit-exact is the only bar.  Covers odd w (sqrt2 twiddles) and even
w, trunc in (2n, 4n] (both halves live), trunc <= 2n (second half unused), unbalanced
operands, all-ones limbs, every coefficient-kernel family (wave l <= 256, generic
512, register-resident 1024-4096) and test_mul4's own shape (depth 14, w 1).
"""
import random

import numpy as np
import pytest

from helpers import max_limbs6, shapes6, to_int, valid_shape6

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def test_mul6_random_vs_oracle(mp, oracle, torch_dev):
    rng = random.Random(31)
    bad = []
    for depth, w, n1, n2 in shapes6(rng, 2):
        a = mp.fill_random(n1, rng.getrandbits(64))
        b = mp.fill_random(n2, rng.getrandbits(64))
        r = mp.mul6(a, b, depth, w)
        if not (r == oracle.gmp_mul(a, b)).all():
            bad.append((depth, w, n1, n2))
        elif n1 + n2 < 20000 and not (r == oracle.new_mpn_mul6(a, b, depth, w)).all():
            bad.append(("oracle", depth, w, n1, n2))
    assert not bad, bad


# (depth, w): coefficient sizes l = 384 / 512 (generic kernels), 1024 / 2048 / 4096
# (register-resident passes, nested negacyclic pointwise at 2048 / 4096), odd w at l = 384 / 512
BIG6 = [(6, 512), (7, 512), (6, 1024), (7, 1024), (6, 2048), (7, 2048), (6, 4096), (9, 64), (9, 128),
        (12, 8), (11, 16), (13, 4), (13, 3)]


@pytest.mark.parametrize("depth,w", BIG6)
def test_mul6_big_coefficients(mp, oracle, torch_dev, depth, w):
    if ((1 << depth) * w) % 64 or (1 << depth) * w // 64 > 4096:
        pytest.skip("unsupported shape")
    mx = max_limbs6(depth, w)
    for n1, n2 in ((mx, mx), ((3 * mx) // 4, (3 * mx) // 4), (mx // 3, mx + mx // 2)):
        if not valid_shape6(depth, w, n1, n2):
            continue
        a = mp.fill_random(n1, 0x61 + n1)
        b = mp.fill_random(n2, 0x62 + n2)
        assert (mp.mul6(a, b, depth, w) == oracle.gmp_mul(a, b)).all(), (depth, w, n1, n2)


@pytest.mark.parametrize("depth,w", [(10, 1), (11, 3), (12, 1), (8, 5)])
def test_mul6_odd_w_all_ones(mp, oracle, torch_dev, depth, w):
    """all-ones limbs: maximal coefficients through the sqrt2 twiddles"""
    mx = max_limbs6(depth, w)
    ones = np.full(mx, 2**64 - 1, dtype=np.uint64)
    for a, b in ((ones, ones), (ones[: mx // 5 + 1], ones)):
        assert (mp.mul6(a, b, depth, w) == oracle.gmp_mul(a, b)).all()


def test_mul6_odd_w_l512(mp, oracle, torch_dev):
    """depth 15, w 1: l = 512 with sqrt2 twiddles, trunc just past 2n"""
    depth, w = 15, 1
    n = 1 << depth
    bits1 = (n * w - (depth + 1)) // 2
    n1 = n2 = (2 * n * bits1 // 64) * 9 // 16
    assert valid_shape6(depth, w, n1, n2)
    a = mp.fill_random(n1, 0x15)
    b = mp.fill_random(n2, 0x16)
    assert (mp.mul6(a, b, depth, w) == oracle.gmp_mul(a, b)).all()


def test_mul6_test_mul4_shape(mp, oracle, torch_dev):
    """test_mul4 (mul_fft.c:5559-5608): depth 14, w 1, n1 = n2 = 3/4 of 2n bits1 bits,
    checked like the reference does, against mpn_mul"""
    depth, w = 14, 1
    n = 1 << depth
    bits1 = (n * w - (depth + 1)) // 2
    int_limbs = 2 * n * bits1 // 64
    n1 = n2 = (3 * int_limbs) // 4
    a = mp.fill_random(n1, 0x1001)
    b = mp.fill_random(n2, 0x2002)
    r = np.zeros(n1 + n2, dtype=np.uint64)
    mp.new_mpn_mul6(r, a, n1, b, n2, depth, w)
    assert (r == oracle.gmp_mul(a, b)).all()


def test_mul6_device_entry(mp, oracle, torch_dev):
    """mpfft_mul6_device on HBM-resident operands equals the host entry"""
    import torch
    depth, w, n1, n2 = 11, 1, 5000, 3000
    assert valid_shape6(depth, w, n1, n2)
    a = mp.fill_random(n1, 5)
    b = mp.fill_random(n2, 6)
    da = torch.from_numpy(a.view(np.int64)).to(torch_dev)
    db = torch.from_numpy(b.view(np.int64)).to(torch_dev)
    dr = torch.zeros(n1 + n2, dtype=torch.int64, device=torch_dev)
    ws = mp.alloc_workspace6(n1, n2, depth, w, device=torch_dev)
    mp.mul6_device(dr, da, n1, db, n2, depth, w, ws)
    torch.cuda.synchronize()
    r = dr.cpu().numpy().view(np.uint64)
    assert (r == oracle.gmp_mul(a, b)).all()
    assert to_int(r) == to_int(a) * to_int(b)


def test_mul6_rejects_bad_parameters(mp, torch_dev):
    with pytest.raises(mp.MpfftError):
        mp.mul6(np.ones(10**6, np.uint64), np.ones(10**6, np.uint64), 6, 1)   # does not fit 4n
    with pytest.raises(mp.MpfftError):
        mp.mul6(np.ones(4, np.uint64), np.ones(4, np.uint64), 5, 1)           # 64 does not divide N

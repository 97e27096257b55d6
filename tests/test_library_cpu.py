"""CPU-only checks of the product library (no compute: this container has no GPU).

- libmpfft.so loads and exports every function include/mpfft.h declares
- parameter derivation equals the reference's (mul_fft.c:3193-3203, via the oracle)
- invalid calls are rejected with a reason instead of the reference's segfault
- with no GPU the compute entry points fail loudly (no CPU fallback exists)
- the synthetic-input PRNG is the oracle's stream
"""
import os
import random
import re

import numpy as np
import pytest

from helpers import valid_shape

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "mpfft.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:void|int|long|size_t|const char \*)\s*\*?\s*(\w+)\s*\(", src, flags=re.M)))


def test_exports_every_declared_symbol(mp):
    names = declared_functions()
    assert "new_mpn_mul" in names and "mpfft_mul_device" in names
    lib = mp.lib()
    for n in names:
        assert hasattr(lib, n), n
    assert lib.mpfft_version() >= 1


def test_plan_matches_reference_parameters(mp, oracle):
    rng = random.Random(3)
    checked = 0
    for _ in range(400):
        depth = rng.randint(2, 17)
        w = rng.choice([1, 2, 3, 4, 5, 8, 16, 64])
        n1, n2 = rng.randint(1, 5000), rng.randint(1, 5000)
        ok = ((1 << depth) * w) % 64 == 0 and valid_shape(depth, w, n1, n2) and (1 << depth) * w // 64 <= 4096
        rc = mp.check_params(n1, n2, depth, w)
        assert (rc == 0) == ok, (depth, w, n1, n2, rc)
        if ok:
            P = mp.plan_info(n1, n2, depth, w)
            n, l, sq, j1, j2, trunc, bits1 = oracle.params(n1, n2, depth, w)
            # the MFA split is internal: at l = 2048 make_plan doubles the columns in truncation
            # case b, and in case a at depth 13-15; at l = 4096 in case b (mpfft.hip make_plan)
            # (case a only where the doubled column count's rounding adds at most 1/64 to trunc)
            alt_tr = -(-(j1 + j2 - 1) // (4 * sq)) * 4 * sq
            alt = (l == 2048 and (trunc > n or (13 <= depth <= 15 and alt_tr <= trunc + trunc // 64))) or \
                  (l == 4096 and trunc > n)
            assert (P["n"], P["l"], P["NC"], P["j1"], P["j2"], P["trunc"], P["bits1"]) == \
                (n, l, 2 * sq if alt else sq, j1, j2, alt_tr if alt else trunc, bits1)
            assert P["NR"] * P["NC"] == 2 * n
            checked += 1
    assert checked > 50


def test_invalid_parameters_rejected(mp):
    assert mp.check_params(10, 10, 5, 3) == 1          # n*w % 64
    assert mp.check_params(0, 10, 8, 1) == 1
    assert mp.check_params(10, 10, 1, 64) == 1         # depth < 2
    assert mp.check_params(10**6, 10**6, 6, 1) == 2    # does not fit
    assert mp.check_params(10, 10, 14, 64) == 3        # l > 4096
    with pytest.raises(mp.MpfftError):
        mp.plan_info(10, 10, 5, 3)


def test_compute_fails_loudly_without_gpu(mp):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    a = np.ones(4, np.uint64)
    with pytest.raises(mp.MpfftError):
        mp.mul(a, a, 6, 1)


def test_prng_matches_oracle(mp, oracle):
    for seed in (0x1001, 0x2002, 7):
        assert (mp.fill_random(1000, seed) == oracle.fill_random(1000, seed)).all()


def test_chooser_picks_valid_parameters(mp):
    """mpfft_choose (the reference leaves (depth, w) to the caller,
    mul_fft.c:3190-3191): every pick is a valid, supported plan that holds the product,
    across 1e3- to 1e10-bit operands, balanced and unbalanced."""
    sizes = [1, 2, 16, 100, 1000, 16384, 10**5, 261952, 10**6, 15625000, 20312500, 156250000]
    for n1 in sizes:
        for n2 in (n1, max(1, n1 // 7), 3):
            d, w = mp.choose(n1, n2)
            assert w & (w - 1) == 0 and ((1 << d) * w) % 64 == 0
            assert mp.check_params(n1, n2, d, w) == 0, (n1, n2, d, w)
    with pytest.raises(mp.MpfftError):
        mp.choose(10**12, 10**12)                       # beyond 4096-limb coefficients at depth 24


def test_plan6_matches_reference_parameters(mp, oracle):
    """new_mpn_mul6's derived parameters (mul_fft.c:3575-3603) equal the oracle's"""
    from helpers import valid_shape6
    rng = random.Random(4)
    checked = 0
    for _ in range(400):
        depth = rng.randint(2, 17)
        w = rng.choice([1, 2, 3, 4, 5, 8, 16, 64])
        n1, n2 = rng.randint(1, 9000), rng.randint(1, 9000)
        ok = ((1 << depth) * w) % 64 == 0 and valid_shape6(depth, w, n1, n2) and (1 << depth) * w // 64 <= 4096
        rc = mp.check_params6(n1, n2, depth, w)
        assert (rc == 0) == ok, (depth, w, n1, n2, rc)
        if ok:
            P = mp.plan_info6(n1, n2, depth, w)
            n, l, sq, j1, j2, trunc, bits1 = oracle.params6(n1, n2, depth, w)
            assert (P["n"], P["l"], P["NC"], P["j1"], P["j2"], P["trunc"], P["bits1"]) == \
                (n, l, sq, j1, j2, trunc, bits1)
            assert mp.workspace_bytes6(n1, n2, depth, w) > mp.workspace_bytes(1, 1, depth, w)
            checked += 1
    assert checked > 50
    with pytest.raises(mp.MpfftError):
        mp.mul6(np.ones(4, np.uint64), np.ones(4, np.uint64), 6, 1)   # no GPU here: fails loudly


def test_pwss_pair_order_is_a_permutation():
    """k_pwss FUSE=1 (pkernels.hpp) deals slot pairs to workgroups b and b + 8 (one XCD):
    slot(b) = 2 (8 (j >> 1) + (b & 7)) + (j & 1), j = b >> 3, identity on the last nb % 16
    blocks.  It must be a permutation of the slots with both slots of a pair on one XCD."""
    def slot(b, nb):
        main = nb - nb % 16
        if b >= main:
            return b
        x, j = b & 7, b >> 3
        return 2 * (((j >> 1) << 3) + x) + (j & 1)
    for nb in (2, 16, 18, 64, 130, 39680, 30720, 4098):
        s = [slot(b, nb) for b in range(nb)]
        assert sorted(s) == list(range(nb)), nb
        where = {v: b for b, v in enumerate(s)}
        for p in range(0, nb - nb % 16, 2):
            assert where[p] % 8 == where[p + 1] % 8, (nb, p)


def test_fold_plans_on_bench_configs(mp):
    """C2, C3, C4 (truncated, l = 2048 / 4096) run without a scaling pass -- the
    2^-(depth+1) in the last inverse row pass, the reduced-form combine (fold.hpp); C1 (l = 256,
    wave kernels) and the sqrt2 front end keep k_rscale / k_wscale + k_combine1"""
    for depth, w, n in ((15, 4, 15625000), (15, 4, 20312500), (17, 2, 156250000)):
        k = mp.stage_kernels(n, n, depth, w)
        assert "k_combine_red" in k["combine"] and "folded" in k["scale"], k
    k = mp.stage_kernels(261952, 261952, 11, 8)
    assert "k_combine_red" not in k["combine"] and "folded" not in k["scale"]

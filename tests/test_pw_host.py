"""CPU test: the nested negacyclic pointwise arithmetic of k_pwss (pkernels.hpp) --
rotated add in Z/(2^N'+1), inner product, canonical residue and the sqrt 2 weight step
(pw_sqrt2) -- compiled for the host and checked against GMP (tests/pw_host/pw_host_test.cpp),
for every inner size the library instantiates (M = 10, 18, 20 limbs).  Reference algorithm: FFT_mulmod_2expp1
(/root/reference/mul_fft.c:2998-3117), whose test oracle is mpn_mulmod_2expp1 (:4224)."""
import os
import subprocess

import pytest

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pw_host", "pw_host_test")


def test_pointwise_inner_arithmetic_vs_gmp():
    if not os.path.exists(EXE):
        pytest.skip("tests/pw_host/pw_host_test not built (run __graft_entry__.build())")
    p = subprocess.run([EXE], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and p.stdout.strip().endswith("OK"), p.stdout + p.stderr


def _fwd_rotations(M, LK):
    """E mod N' of every thread at every forward level, computed exactly as pw_slot_product and
    pw_level do (pkernels.hpp): P_t starts at the negacyclic weight, bottom threads add tw"""
    K, NP = 1 << LK, 64 * M
    N2 = 2 * NP
    W2 = N2 >> LK
    P = [((t * W2) >> 1) + (NP // 4 if (W2 & 1) and (t & 1) else 0) for t in range(K)]
    levels = []
    for j in range(LK):
        h = K >> (j + 1)
        E = [((P[t ^ h] + N2 - P[t]) % N2) % NP for t in range(K)]
        levels.append(E)
        P = [P[t] if not (t & h) else (P[t] + ((t & ~h) & (h - 1)) * (1 << j) * W2) % N2 for t in range(K)]
    return levels


import pytest  # noqa: E402


@pytest.mark.parametrize("M,LK", [(10, 8), (18, 8), (20, 9)])
def test_forward_level_rotations_fixed(M, LK):
    """the compile-time rotations of k_pwss's first forward levels (pw_transform): level 0 is
    exactly N'/2 for every thread; levels 1 .. LK - 7 are wave-uniform odd multiples of
    N' / 2^(j+1) (the kernel's scalar switch has exactly those 2^j cases)"""
    NP = 64 * M
    levels = _fwd_rotations(M, LK)
    assert set(levels[0]) == {NP // 2}
    for j in range(1, LK - 6):
        E = levels[j]
        for w in range(len(E) // 64):
            assert len(set(E[64 * w: 64 * w + 64])) == 1, (j, w)
        unit = NP >> (j + 1)
        assert all(e % unit == 0 and (e // unit) % 2 == 1 for e in E), j
    if LK - 6 < LK:   # the next level is not wave-uniform (the kernel keeps the general form there)
        E = levels[LK - 6]
        assert any(len(set(E[64 * w: 64 * w + 64])) > 1 for w in range(len(E) // 64))

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

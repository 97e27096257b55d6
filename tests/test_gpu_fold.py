"""GPU tests of the folded scaling + reduced-form combine (csrc/fold.hpp).

On the truncated register-pass plans (C2, C3, C4 among them) new_mpn_mul has no scaling pass:
2^-(depth+1) rides in the last inverse row pass's un-twiddle, the truncated inverse's deferred
doubling is a one-bit shift of those rows' windows, and the combine reads the passes' reduced
form (limbs, +-1 carry masks, carry limb) with one wrap correction per coefficient (k_cmeta ->
k_combine_red).  Reference: the scaling loop mul_fft.c:3256-3260 and FFT_combine_bits
:3261-3262 / :207-267; the reference's own TODO:53-59.

- the combine stage alone (MPFFT_STAGE_FOLD_COMBINE) on hand-made reduced-form coefficients:
  random ones and patterns whose carries ripple through every limb, into and out of the carry
  limb, and values at and next to multiples of p = 2^N + 1 (the wrap corrections +-1), in doubled
  and plain rows, against sum_k ((2^s_k V_k) mod p) 2^(k bits1) in exact integers;
- whole products on fold plans against GMP, including all-ones operands (maximal carries).
"""
import random

import numpy as np
import pytest

from test_gpu_parity import _reduced_pattern

pytestmark = pytest.mark.gpu
MAX = (1 << 64) - 1

# l = 1024 / 2048 / 4096, truncation case a (Tr <= NR / 2) and case b, the l = 2048 doubled-column split
FOLD_SHAPES = [(8, 256, 40000, 40000), (8, 512, 40000, 40000), (8, 512, 140000, 140000), (8, 512, 100000, 30000),
               (9, 256, 120000, 200000), (7, 1024, 80000, 70000), (7, 2048, 150000, 120000), (5, 4096, 20000, 19000)]


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _int(a):
    return int.from_bytes(np.ascontiguousarray(a, dtype=np.uint64).tobytes(), "little")


def _folds(mp, n1, n2, depth, w):
    return "k_combine_red" in mp.stage_kernels(n1, n2, depth, w)["combine"]


def _dbl_rows(P):
    """rows whose top-level doubling the truncated inverse defers (mpfft.hip plan_dbl)"""
    T, NR = P["trunc"] // P["NC"], P["NR"]
    if T == NR:
        return 0, 0
    return (0, T) if T <= NR // 2 else (T - NR // 2, NR // 2)


def _wrap_pattern(kind, l, N, rng):
    """reduced forms of values at and next to m p (m = -2 .. 2), some with carries: the wrap
    corrections of k_cmeta's slow path (Xlo < Xhi, Xlo - Xhi >= p) and c = 0, 1, 2^N"""
    p = (1 << N) + 1
    m = rng.randint(-2, 2)
    v = m * p + rng.choice([0, 1, -1, 2, -2])
    top = v >> N
    low = v - (top << N)
    limbs = [(low >> (64 * i)) & MAX for i in range(l)]
    pos, neg = set(), set()
    if kind % 2:   # the same value with carries: one unit of limb i moved into limb i - 1's carry
        i = rng.randrange(1, l)
        if limbs[i]:
            limbs[i] -= 1
            pos.add(i - 1)
        else:          # limb i = 2^64 - 1 instead of 0, a borrow out of it (limb l - 1: out of 2^N)
            limbs[i] = MAX
            pos.add(i - 1)
            neg.add(i)
    return limbs, pos, neg, top


@pytest.mark.parametrize("depth,w,n1,n2", FOLD_SHAPES)
def test_fold_combine_stage(mp, torch_dev, depth, w, n1, n2):
    import torch
    assert _folds(mp, n1, n2, depth, w)
    P = mp.plan_info(n1, n2, depth, w)
    l, N, bits1 = P["l"], P["n"] * w, P["bits1"]
    p = (1 << N) + 1
    L = P["j1"] + P["j2"] - 1
    lay = mp.workspace_layout(n1, n2, depth, w)
    ws = mp.alloc_workspace(n1, n2, depth, w, torch_dev)
    ws.fill_(0)
    digA, topA, _, _ = mp.workspace_views(ws, n1, n2, depth, w)
    cbw = lay["cbw"]
    lo, hi = _dbl_rows(P)
    rng = random.Random(depth * 131 + w + n1)
    dig = np.zeros((L, l), np.uint64)
    top = np.zeros(L, np.int32)
    cbm = np.zeros((L, cbw), np.uint64)
    want = 0
    for k in range(L):
        r = k % 16
        if r < 8:
            limbs, pos, neg, t = _reduced_pattern(r if r != 7 else 9, l, rng)
        elif r < 12:
            limbs, pos, neg, t = _wrap_pattern(r, l, N, rng)
        else:   # random reduced form: dense carries both ways, small top
            limbs = [rng.getrandbits(64) for _ in range(l)]
            pos = {i for i in range(l) if rng.random() < 0.3}
            neg = {i for i in range(l) if rng.random() < 0.3} - pos
            t = rng.randint(-2, 2)
        dig[k] = np.array(limbs, dtype=np.uint64)
        top[k] = t
        cp = np.zeros(l + 1, np.uint64)   # the carries as numbers: limb i + 1 of cp / cn = carry out of limb i
        cn = np.zeros(l + 1, np.uint64)
        for i in pos:
            cbm[k, 2 * (i // 64)] |= np.uint64(1 << (i % 64))
            cp[i + 1] = 1
        for i in neg:
            cbm[k, 2 * (i // 64) + 1] |= np.uint64(1 << (i % 64))
            cn[i + 1] = 1
        v = _int(dig[k]) + t * (1 << N) + _int(cp) - _int(cn)
        s = 1 if lo <= k // P["NC"] < hi else 0
        want += ((v << s) % p) << (k * bits1)
    total = n1 + n2
    want &= (1 << (64 * total)) - 1
    digA[:L] = torch.from_numpy(dig.view(np.int64)).to(torch_dev)
    topA[:L] = torch.from_numpy(top).to(torch_dev)
    u8 = ws.view(torch.uint8)
    u8[lay["cbA"]: lay["cbA"] + L * cbw * 8] = torch.from_numpy(cbm.view(np.uint8).reshape(-1)).to(torch_dev)
    d_r = torch.full((total,), -1, dtype=torch.int64, device=torch_dev)
    z = torch.zeros(1, dtype=torch.int64, device=torch_dev)
    mp.stage(mp.STAGE_FOLD_COMBINE, z, z, d_r, n1, n2, depth, w, ws)
    torch.cuda.synchronize()
    got = d_r.cpu().numpy().view(np.uint64)
    wl = np.frombuffer(want.to_bytes(8 * total, "little"), dtype=np.uint64)
    bad = np.nonzero(got != wl)[0]
    assert len(bad) == 0, f"{len(bad)} of {total} limbs wrong, first at {bad[:8]} (limb / bits1 = {bad[:8] * 64 // bits1})"


@pytest.mark.parametrize("depth,w,n1,n2", FOLD_SHAPES)
def test_fold_products(mp, oracle, depth, w, n1, n2):
    """whole products on fold plans: random, all-ones (maximal carries everywhere), one-sided"""
    assert _folds(mp, n1, n2, depth, w)
    rng = random.Random(depth + w + n2)
    ones1 = np.full(n1, MAX, dtype=np.uint64)
    ones2 = np.full(n2, MAX, dtype=np.uint64)
    bit = np.zeros(n1, np.uint64)
    bit[n1 // 3] = 1 << 63
    cases = [(mp.fill_random(n1, rng.getrandbits(64)), mp.fill_random(n2, rng.getrandbits(64))),
             (ones1, ones2), (ones1, mp.fill_random(n2, 5)), (bit, ones2), (np.zeros(n1, np.uint64), ones2)]
    for a, b in cases:
        got = mp.mul(a, b, depth, w)
        assert (got == oracle.gmp_mul(a, b)).all()

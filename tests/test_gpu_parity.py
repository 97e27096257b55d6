"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the
exact product.  Bit-exact is the only bar (integer work).

Covers: every stage against exact big-integer math (tests/gpu_stages.py), the
reference-shaped new_mpn_mul over random and adversarial shapes (cf. the
reference's integration tests test_mul4/test_mul5, mul_fft.c:5507-5608), the
committed golden vectors, error behaviour, and the benchmark configs.
"""
import json
import os
import random

import numpy as np
import pytest

from helpers import max_limbs, to_int, valid_shape

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


STAGE_SHAPES = [(6, 1, 3, 2), (6, 1, 1, 1), (7, 1, 5, 4), (7, 3, 13, 2), (8, 2, 30, 25), (8, 4, 60, 50),
                (9, 1, 30, 31), (10, 3, 300, 200), (11, 1, 1000, 1000), (5, 2, 2, 1), (4, 4, 1, 1),
                (3, 8, 1, 1), (2, 16, 1, 1)]
# coefficient sizes l = 128 ... 4096 limbs: the int8-MFMA pointwise (k_pwm, k_pwm2)
MFMA_SHAPES = [(9, 16, 2000, 1500), (8, 64, 3000, 2000), (7, 256, 4000, 3000), (6, 1024, 6000, 5000),
               (5, 4096, 8000, 8000), (6, 4096, 20000, 20000)]
# l = 2048 / 4096 with enough levels for the register-resident passes (k_rpass): 3-level
# column / row passes, the twiddle-on-load first row pass, the general-multiplier last
# inverse row pass, the fused split; truncation case a (T <= n) and b (T > n)
BIG_SHAPES = [(8, 512, 40000, 40000), (8, 512, 140000, 140000), (8, 512, 100000, 30000),
              (7, 2048, 150000, 120000), (9, 256, 120000, 200000),
              (7, 1024, 80000, 70000), (5, 4096, 20000, 19000)]   # l = 2048 case b: the doubled-column split


@pytest.mark.parametrize("depth,w,n1,n2", STAGE_SHAPES + MFMA_SHAPES + BIG_SHAPES)
def test_stages_exact(mp, oracle, torch_dev, depth, w, n1, n2):
    from gpu_stages import run_stages
    if not valid_shape(depth, w, n1, n2):
        pytest.skip("shape does not fit")
    a = mp.fill_random(n1, 1000 + depth * 7 + n1)
    b = mp.fill_random(n2, 2000 + w * 3 + n2)
    fails = run_stages(mp, depth, w, a, b, dev=torch_dev, mul=oracle.gmp_mul)
    assert not fails, "\n".join(fails[:5])


def _random_shapes(seed, per):
    rng = random.Random(seed)
    out = []
    for depth in range(2, 14):
        for w in (1, 2, 3, 4, 5, 8, 16, 32, 64):
            if ((1 << depth) * w) % 64 or (1 << depth) * w // 64 > 4096:
                continue
            mx = max_limbs(depth, w)
            if mx > 200000:
                continue
            out.append((depth, w, mx, mx))
            for _ in range(per):
                n1 = rng.randint(1, 2 * mx - 1)
                n2 = rng.randint(1, max(1, 2 * mx - n1))
                if valid_shape(depth, w, n1, n2):
                    out.append((depth, w, n1, n2))
    return out


def test_new_mpn_mul_random_sweep(mp, oracle):
    rng = random.Random(77)
    shapes = _random_shapes(5, 2)
    assert len(shapes) > 100
    for depth, w, n1, n2 in shapes:
        a = mp.fill_random(n1, rng.getrandbits(64))
        b = mp.fill_random(n2, rng.getrandbits(64))
        r = np.zeros(n1 + n2, dtype=np.uint64)
        mp.new_mpn_mul(r, a, n1, b, n2, depth, w)
        want = oracle.gmp_mul(a, b)
        assert (r == want).all(), (depth, w, n1, n2)


def test_adversarial_inputs(mp, oracle):
    """all-ones (max carries), single bits, zeros, unbalanced, max size; values that
    make transform coefficients hit 2^N (the pointwise c-flag, mul_fft.c:3250)."""
    for depth, w in ((6, 1), (8, 2), (10, 1), (11, 8), (9, 64)):
        mx = max_limbs(depth, w)
        ones = np.full(mx, 2**64 - 1, dtype=np.uint64)
        zero = np.zeros(mx, np.uint64)
        bit = zero.copy()
        bit[mx // 2] = 1 << 63
        top1 = zero.copy()
        top1[-1] = 1
        alt = np.full(mx, 0xAAAAAAAAAAAAAAAA, np.uint64)
        cases = [(ones, ones), (ones[:1], ones), (bit, ones), (zero, ones), (top1, top1), (alt, ones),
                 (ones[: mx // 3], ones), (np.ones(1, np.uint64), ones)]
        for a, b in cases:
            if not valid_shape(depth, w, len(a), len(b)):
                continue
            got = mp.mul(a, b, depth, w)
            assert (got == oracle.gmp_mul(a, b)).all(), (depth, w, len(a), len(b))


def _pattern(kind, l, N, rng):
    """canonical residues (limbs, top) that stress the pointwise kernels"""
    if kind == 1:
        return 0, 1                                          # 2^N == -1
    v = {0: rng.getrandbits(N), 2: (1 << N) - 1, 3: 0, 4: 1,
         5: int.from_bytes(b"\x80" * (8 * l), "little"), 6: int.from_bytes(b"\x7f" * (8 * l), "little"),
         7: (1 << N) - 1 - rng.getrandbits(64)}[kind]
    return v, 0


PW_CASES = [(k, d, w) for k in ("mfma", "mfma1", "valu")
            for d, w in ((11, 1), (9, 16), (8, 64), (7, 256), (6, 1024), (5, 4096), (6, 4096))] + \
           [("pwss", 6, 1024), ("pwss", 5, 4096), ("pwss", 6, 4096), ("auto", 5, 4096), ("auto", 6, 4096)]


@pytest.mark.parametrize("kind,depth,w", PW_CASES)
def test_pointwise_direct(mp, torch_dev, kind, depth, w):
    """The pointwise stage alone on hand-placed canonical inputs (every pair of the
    special values 0, 1, 2^N - 1, 2^N, 0x80.. and 0x7f.. bytes, random), for every
    kernel family MPFFT_POINTWISE selects: the int8-MFMA kernels (mfma: k_pwm2 when
    l % 256 == 0; mfma1: k_pwm), the VALU schoolbook (valu: k_pw) and the nested
    negacyclic k_pwss (pwss: l = 1024, 2048, 4096 -- the default from l = 2048 on,
    "auto").  The kernel that ran is checked through mpfft_stage_kernels."""
    import torch
    from gpu_stages import _cbs, _val_reduced
    mx = max_limbs(depth, w)
    n1 = n2 = mx
    P = mp.plan_info(n1, n2, depth, w)
    l, T, N = P["l"], P["trunc"], P["n"] * w
    p = (1 << N) + 1
    rng = random.Random(depth * 1000 + w)
    ws = mp.alloc_workspace(n1, n2, depth, w, torch_dev)
    ws.fill_(0)
    digA, topA, digB, topB = mp.workspace_views(ws, n1, n2, depth, w)
    want = []
    host = {k: (np.zeros((T, l), np.uint64), np.zeros(T, np.int32)) for k in "AB"}
    for sl in range(T):
        va, ta = _pattern(sl % 8, l, N, rng)
        vb, tb = _pattern((sl // 8) % 8, l, N, rng)
        for k, v, t in (("A", va, ta), ("B", vb, tb)):
            host[k][0][sl] = np.frombuffer(v.to_bytes(8 * l, "little"), dtype=np.uint64)
            host[k][1][sl] = t
        want.append((va + ta * (1 << N)) * (vb + tb * (1 << N)) % p)
    for k, dig, top in (("A", digA, topA), ("B", digB, topB)):
        dig[:T] = torch.from_numpy(host[k][0].view(np.int64)).to(torch_dev)
        top[:T] = torch.from_numpy(host[k][1]).to(torch_dev)
    da = torch.zeros(n1, dtype=torch.int64, device=torch_dev)
    db = torch.zeros(n2, dtype=torch.int64, device=torch_dev)
    dr = torch.zeros(n1 + n2, dtype=torch.int64, device=torch_dev)
    old = os.environ.get("MPFFT_POINTWISE")
    if kind == "auto":
        os.environ.pop("MPFFT_POINTWISE", None)
    else:
        os.environ["MPFFT_POINTWISE"] = kind
    try:
        ran = mp.stage_kernels(n1, n2, depth, w)["pointwise"].split(" ")[0].split("<")[0]
        mfma1 = "k_pwm" if l % 128 == 0 else "k_pw"
        expect = {"pwss": "k_pwss", "auto": "k_pwss", "valu": "k_pw", "mfma1": mfma1,
                  "mfma": "k_pwm2" if l % 256 == 0 else mfma1}[kind]
        assert ran == expect, (kind, l, ran)
        mp.stage(mp.STAGE_POINTWISE, da, db, dr, n1, n2, depth, w, ws)
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("MPFFT_POINTWISE", None)
        else:
            os.environ["MPFFT_POINTWISE"] = old
    dig = digA.cpu().numpy().view(np.uint64)
    top = topA.cpu().numpy().astype(np.int64)
    cb = _cbs(mp, ws, n1, n2, depth, w, 0)
    bad = [sl for sl in range(T) if _val_reduced(dig, top, cb, sl, N) % p != want[sl]]
    assert not bad, f"{len(bad)} of {T} slots wrong, first {bad[:8]}"


def test_coefficient_equal_2N(mp, oracle):
    """Operands whose transform has coefficients == 2^N == -1 mod p exercise the
    top-limb-1 path of the pointwise product.  x_j = 2^bits1-1 pieces with the
    all-ones operand hit it at small N; check many (depth, w) combinations."""
    for depth, w in ((6, 1), (6, 2), (7, 1), (8, 1)):
        mx = max_limbs(depth, w)
        for fill in (0x8000000000000000, 0xFFFFFFFFFFFFFFFF, 1):
            a = np.full(mx, fill, np.uint64)
            for n1 in (1, 2, mx):
                got = mp.mul(a[:n1], a, depth, w)
                assert (got == oracle.gmp_mul(a[:n1], a)).all()


def test_golden_vectors(mp):
    path = os.path.join(GOLDEN, "products.json")
    if not os.path.exists(path):
        pytest.skip("no golden vectors")
    with open(path) as f:
        cases = json.load(f)
    import hashlib
    for c in cases:
        a = mp.fill_random(c["n1"], int(c["seed1"], 16))
        b = mp.fill_random(c["n2"], int(c["seed2"], 16))
        got = mp.mul(a, b, c["depth"], c["w"])
        if "product_hex" in c:
            assert format(to_int(got), "x") == c["product_hex"], c["name"]
        assert hashlib.sha256(got.tobytes()).hexdigest() == c["sha256"], c["name"]


def test_errors_fail_loudly(mp):
    a = np.ones(10, np.uint64)
    with pytest.raises(mp.MpfftError):
        mp.mul(a, a, 5, 3)            # n*w not a multiple of 64
    big = np.ones(100000, np.uint64)
    with pytest.raises(mp.MpfftError):
        mp.mul(big, big, 6, 1)        # product does not fit
    with pytest.raises(mp.MpfftError):
        mp.mul(a, a, 1, 64)           # depth < 2


def test_device_api_and_workspace_reuse(mp, oracle, torch_dev):
    import torch
    depth, w = 11, 8
    for n1, n2 in ((261952, 261952), (1000, 250000), (5, 7)):
        a = mp.fill_random(n1, 11)
        b = mp.fill_random(n2, 12)
        da = torch.from_numpy(a.view(np.int64)).to(torch_dev)
        db = torch.from_numpy(b.view(np.int64)).to(torch_dev)
        dr = torch.zeros(n1 + n2, dtype=torch.int64, device=torch_dev)
        ws = mp.alloc_workspace(261952, 261952, depth, w, torch_dev)   # larger workspace is fine
        ws.fill_(0x77)
        for _ in range(2):                                            # reuse without re-zeroing
            mp.mul_device(dr, da, n1, db, n2, depth, w, ws)
        torch.cuda.synchronize()
        assert (dr.cpu().numpy().view(np.uint64) == oracle.gmp_mul(a, b)).all()


@pytest.mark.parametrize("cfg", ["C0", "C1"])
def test_bench_configs_exact_vs_oracle(mp, oracle, cfg):
    """C0/C1 at full size against the CPU restatement of the reference (bit-exact)."""
    depth, w, nl = {"C0": (11, 1, 16384), "C1": (11, 8, 261952)}[cfg]
    a = mp.fill_random(nl, 0x1001)
    b = mp.fill_random(nl, 0x2002)
    got = mp.mul(a, b, depth, w)
    assert (got == oracle.new_mpn_mul(a, b, depth, w)).all()


@pytest.mark.slow
def test_c2_c3_exact_vs_gmp(mp, oracle):
    """C2 (10^9-bit) and C3 (1.3x10^9-bit, odd trunc) against GMP mpn_mul."""
    for depth, w, nl in ((15, 4, 15625000), (15, 4, 20312500)):
        a = mp.fill_random(nl, 0x1001)
        b = mp.fill_random(nl, 0x2002)
        got = mp.mul(a, b, depth, w)
        assert (got == oracle.gmp_mul(a, b)).all()


def test_nested_pointwise_full_products(mp, oracle):
    """Whole products through k_pwss at l = 1024, 2048 (the C2 shape: fused pair + last
    row level) and 4096 (fused pair), against GMP mpn_mul."""
    old = os.environ.get("MPFFT_POINTWISE")
    os.environ["MPFFT_POINTWISE"] = "pwss"
    try:
        for depth, w, nl in ((6, 1024, 32760), (7, 1024, 131064), (15, 4, 15625000), (6, 4096, 131064)):
            ran = mp.stage_kernels(nl, nl, depth, w)["pointwise"]
            assert ran.startswith("k_pwss<"), ran
            a = mp.fill_random(nl, 0x3003 + depth)
            b = mp.fill_random(nl - 17, 0x4004 + w)
            assert (mp.mul(a, b, depth, w) == oracle.gmp_mul(a, b)).all(), (depth, w, ran)
    finally:
        if old is None:
            os.environ.pop("MPFFT_POINTWISE", None)
        else:
            os.environ["MPFFT_POINTWISE"] = old


def test_pointwise_norm_spill_branch(mp, oracle):
    """k_pwss's rare pw_norm branch (a lane whose low word would under/overflow keeps its top,
    ~2^-32 per lane, so random inputs never reach it) and the readers' T_q != -1 path behind it,
    on every lane of every exchange: libmpfft_pwspill.so is the shipped build with pwss.hip
    compiled -DPW_NORM_SPILL_ALL=1 (csrc/Makefile `pwspill`, built by build()).  Whole products
    through its C ABI at l = 1024 (k_pwss forced), 2048 (C2's fused quad) and 4096 against GMP
    (ADVICE r5)."""
    import ctypes
    path = os.path.join(os.path.dirname(mp.LIB_PATH), "libmpfft_pwspill.so")
    assert os.path.exists(path), "build() builds libmpfft_pwspill.so"
    v = ctypes.CDLL(path)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    v.mpfft_mul_ex.argtypes = [u64p, u64p, ctypes.c_long, u64p, ctypes.c_long, ctypes.c_ulong, ctypes.c_ulong]
    v.mpfft_mul_ex.restype = ctypes.c_int
    p = lambda x: x.ctypes.data_as(u64p)
    old = os.environ.get("MPFFT_POINTWISE")
    os.environ["MPFFT_POINTWISE"] = "pwss"
    try:
        for depth, w, n1, n2 in ((6, 1024, 32760, 32000), (15, 4, 15625000, 15625000), (7, 2048, 150000, 120000),
                                 (6, 4096, 131064, 100000)):
            assert mp.stage_kernels(n1, n2, depth, w)["pointwise"].startswith("k_pwss<")
            a = mp.fill_random(n1, 0x5005 + depth)
            b = mp.fill_random(n2, 0x6006 + w)
            r = np.zeros(n1 + n2, dtype=np.uint64)
            assert v.mpfft_mul_ex(p(r), p(a), n1, p(b), n2, depth, w) == 0
            assert (r == oracle.gmp_mul(a, b)).all(), (depth, w, n1, n2)
            o1, o2 = np.full(n1, 2**64 - 1, dtype=np.uint64), np.full(n2, 2**64 - 1, dtype=np.uint64)
            assert v.mpfft_mul_ex(p(r), p(o1), n1, p(o2), n2, depth, w) == 0
            assert (r == oracle.gmp_mul(o1, o2)).all(), ("all ones", depth, w, n1, n2)
    finally:
        if old is None:
            os.environ.pop("MPFFT_POINTWISE", None)
        else:
            os.environ["MPFFT_POINTWISE"] = old


@pytest.mark.parametrize("depth,w,nl", [(13, 32, 9800000), (11, 128, 2600000), (7, 2048, 150000)])
def test_fill_fold_l4096_case_b(mp, oracle, depth, w, nl):
    """The truncated inverse's FILL step folded into the last DIT pass of a block IFFT
    (k_rpass DIR 1, mode bit 2: a second, rotated store of the same registers) at l = 4096,
    truncation case b (T > n), with C4's proportions: the top-level block of NR/2 rows runs
    two or three DIT passes and FILL covers rows [t - h, h).  Guards against the failure that
    only the full-size C4 digest caught mid round 3 (gpurun_out/pytest_fill1.log: C4 digest
    a775e4... instead of 36ca70...): a FILL store built from registers the first store had
    already changed.  Checked against a mutant build with that defect (scripts/mutant_fill.sh:
    rp_store adding the pair-overflow carry into the registers in place): this test fails on
    it and passes on the shipped library (profiles/r04/mutant_fill.log)."""
    P = mp.plan_info(nl, nl, depth, w)
    assert P["l"] == 4096 and 2 * P["n"] >= P["trunc"] > P["n"], P   # case b
    assert "k_rpass" in mp.stage_kernels(nl, nl, depth, w)["inv_columns"]
    a = mp.fill_random(nl, 0x7007 + depth)
    b = mp.fill_random(nl - 3, 0x8008 + w)
    assert (mp.mul(a, b, depth, w) == oracle.gmp_mul(a, b)).all()


@pytest.mark.parametrize("depth,w,nl,caseb", [(12, 32, 2200000, True), (13, 16, 4500000, True),
                                              (14, 8, 9000000, True), (13, 16, 3000000, False),
                                              (16, 2, 30000000, False), (12, 32, 1500000, False),
                                              (5, 4096, 20000, True), (6, 2048, 40000, True),
                                              (7, 1024, 80000, True)])
def test_mfa_split_l2048(mp, oracle, depth, w, nl, caseb):
    """The plan's MFA split at l = 2048 (make_plan): truncation case b, and case a at depth 13-15
    (round 6), take twice the reference's columns (mul_fft.c:3195) with four-level forward
    k_rpass passes (7 row or column levels -> 4 + 3); case a elsewhere keeps the reference split;
    whole products against GMP."""
    P = mp.plan_info(nl, nl, depth, w)
    assert P["l"] == 2048 and (P["trunc"] > P["n"]) == caseb, P
    alt = caseb or 13 <= depth <= 15
    assert P["NC"] == 1 << (depth // 2 + (1 if alt else 0)), P
    a = mp.fill_random(nl, 0x9009 + depth)
    b = mp.fill_random(nl - 5, 0xA00A + w)
    assert (mp.mul(a, b, depth, w) == oracle.gmp_mul(a, b)).all()


@pytest.mark.parametrize("depth,w,n1,n2", [(16, 4, 3000000, 2999991), (17, 2, 1500000, 1400000)])
def test_quad_fused_rows(mp, oracle, depth, w, n1, n2):
    """The row DIF's last two levels inside the pointwise (k_pwss FUSE 2: slot quads, the h = 2
    level's twiddle 2^(N/2) as a piece rotation on load) where that saves a row pass (l = 4096,
    8 row levels: 3 + 3 instead of 3 + 3 + 2, C4's shape); whole products against GMP."""
    assert "quad + last two row levels" in mp.stage_kernels(n1, n2, depth, w)["pointwise"]
    a = mp.fill_random(n1, 0xB00B + depth)
    b = mp.fill_random(n2, 0xC00C + w)
    assert (mp.mul(a, b, depth, w) == oracle.gmp_mul(a, b)).all()


@pytest.mark.parametrize("kind", ["mfma", "mfma1", "valu"])
def test_l4096_products_every_pointwise_kind(mp, oracle, kind):
    """Whole products at l = 4096 with every MPFFT_POINTWISE family.  Those kinds need the
    canonical store in the last forward row pass, which k_rpass declines, so that pass falls
    back to k_bpass -- which fits only two levels in LDS at l = 4096.  With lbC = 6 (depth 13)
    the row split is 3 + 3: before the cap (Exec::fit) the last pass asked for k_bpass<3> and
    the launch failed.  depth 17 (C4's shape, 3 + 3 + 2) beside it."""
    old = os.environ.get("MPFFT_POINTWISE")
    os.environ["MPFFT_POINTWISE"] = kind
    try:
        # + l = 2048 in truncation case b (the doubled-column split, four-level row passes: the
        # canonical last row pass again falls back to k_bpass at its own level cap)
        for depth, w, n1, n2 in ((13, 32, 1000000, 999983), (17, 2, 1500000, 1400000), (12, 32, 2200000, 2100000)):
            a = mp.fill_random(n1, 0x5005 + depth)
            b = mp.fill_random(n2, 0x6006 + w)
            assert (mp.mul(a, b, depth, w) == oracle.gmp_mul(a, b)).all(), (kind, depth, w)
    finally:
        if old is None:
            os.environ.pop("MPFFT_POINTWISE", None)
        else:
            os.environ["MPFFT_POINTWISE"] = old


def test_mul_auto_exact_across_sizes(mp, oracle):
    """mpn_mul-style entry with the chooser's (depth, w): exact products from 1e3- to
    1e9-bit operands (balanced and unbalanced) against GMP mpn_mul."""
    rng = random.Random(91)
    for n in (16, 157, 1000, 4096, 31250, 10**5, 10**6, 15625000):
        for n2 in (n, max(1, n // 5)):
            a = mp.fill_random(n, rng.getrandbits(64))
            b = mp.fill_random(n2, rng.getrandbits(64))
            got = mp.mul_auto(a, b)
            assert (got == oracle.gmp_mul(a, b)).all(), (n, n2, mp.choose(n, n2))


def _reduced_pattern(kind, l, rng):
    """(limbs, pos-carry limb set, neg-carry limb set, top) of a reduced-form residue built to
    make the canonicalisation's carry chains long: through every limb, across the segment
    boundaries of the multi-wave sweep, into and out of the carry limb."""
    MAX = (1 << 64) - 1
    if kind == 0:
        return [MAX] * l, set(range(l)), set(), 0            # +1 into every limb: one chain through all
    if kind == 1:
        return [0] * l, set(), set(range(l)), 0              # -1 into every limb: borrows through all
    if kind == 2:
        return [MAX] * l, set(range(l)), set(), 1
    if kind == 3:
        return [0] * l, set(), set(range(l)), -1
    if kind == 4:                                            # chains starting just below each segment boundary
        limbs = [rng.getrandbits(64) for _ in range(l)]
        pos = set()
        for k in range(1, 8):
            b = k * l // 8
            for m in range(b - 3, b + 3):
                limbs[m] = MAX
            pos.add(b - 4)
        return limbs, pos, set(), 0
    if kind == 5:
        limbs = [0] * l
        neg = set()
        for k in range(1, 8):
            b = k * l // 8
            neg.add(b - 4)
        limbs[l - 1] = 0
        return limbs, set(), neg, 2
    if kind == 6:
        return [MAX] * l, set(), set(), 0                    # 2^N - 1
    if kind == 7:
        return [0] * l, set(), set(), 1                      # 2^N
    if kind == 8:
        return [0] * l, {l - 1}, set(), 0                    # the top limb's carry: 2^N
    limbs = [rng.getrandbits(64) for _ in range(l)]
    ms = rng.sample(range(l), 40)
    return limbs, set(ms[:20]), set(ms[20:]), rng.randint(-2, 2)


@pytest.mark.parametrize("depth,w,nl", [(9, 128, 30000), (8, 512, 100000), (7, 2048, 150000)])
def test_scale_canonicalisation_adversarial(mp, torch_dev, depth, w, nl):
    """The scaling stage (x 2^-(depth+1), canonical store: k_rscale's multi-wave carry sweep at
    l = 1024, 2048, 4096) on hand-made reduced-form residues whose carries ripple through every
    limb, across the sweep's segment boundaries and through the carry limb, against exact
    big-integer arithmetic (mpn_normmod_2expp1 / mpn_div_2expmod_2expp1 semantics,
    mul_fft.c:272, :494, :3256-3260)."""
    import torch
    from gpu_stages import _cbs, _val
    P = mp.plan_info(nl, nl, depth, w)
    l, T, N = P["l"], P["trunc"], P["n"] * w
    p = (1 << N) + 1
    lay = mp.workspace_layout(nl, nl, depth, w)
    ws = mp.alloc_workspace(nl, nl, depth, w, torch_dev)
    ws.fill_(0)
    digA, topA, _, _ = mp.workspace_views(ws, nl, nl, depth, w)
    cbw = lay["cbw"]
    rng = random.Random(depth * 31 + w)
    dig = np.zeros((T, l), np.uint64)
    top = np.zeros(T, np.int32)
    cbm = np.zeros((T, cbw), np.uint64)
    want = []
    for sl in range(T):
        limbs, pos, neg, t = _reduced_pattern(sl % 10, l, rng)
        dig[sl] = np.array(limbs, dtype=np.uint64)
        top[sl] = t
        v = sum(x << (64 * m) for m, x in enumerate(limbs)) + t * (1 << N)
        for m in pos:
            cbm[sl, 2 * (m // 64)] |= np.uint64(1 << (m % 64))
            v += 1 << (64 * (m + 1))
        for m in neg:
            cbm[sl, 2 * (m // 64) + 1] |= np.uint64(1 << (m % 64))
            v -= 1 << (64 * (m + 1))
        want.append(v * pow(2, 2 * N - depth - 1, p) % p)
    digA[:T] = torch.from_numpy(dig.view(np.int64)).to(torch_dev)
    topA[:T] = torch.from_numpy(top).to(torch_dev)
    u8 = ws.view(torch.uint8)
    u8[lay["cbA"]: lay["cbA"] + T * cbw * 8] = torch.from_numpy(cbm.view(np.uint8).reshape(-1)).to(torch_dev)
    z = torch.zeros(1, dtype=torch.int64, device=torch_dev)
    mp.stage(mp.STAGE_SCALE, z, z, z, nl, nl, depth, w, ws)
    torch.cuda.synchronize()
    gd = digA.cpu().numpy().view(np.uint64)
    gt = topA.cpu().numpy().astype(np.int64)
    gc = _cbs(mp, ws, nl, nl, depth, w, 0)
    bad = []
    for sl in range(T):
        v = _val(gd, gt, sl, N)
        canon = not gc[sl].any() and (gt[sl] == 0 or (gt[sl] == 1 and not gd[sl].any()))
        if not canon or v != want[sl]:
            bad.append(sl)
    assert not bad, f"{len(bad)} of {T} slots wrong or not canonical, first {bad[:8]}"

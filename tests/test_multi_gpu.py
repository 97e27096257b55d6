"""GPU tests of the one-process multi-GPU entries mpfft_mul_multi / mpfft_mul_multi_device
(csrc/multi.hip) and the new_mpn_mul device policy (mpfft_set_devices).  On the one-GPU box
every rank is placed on device 0: the ranks' stages, the two exchanges (same-device copies
instead of xGMI peer DMA -- the copy plan, offsets and event ordering are the same), the
per-stripe halo, the striped combine and the device-side stripe carry scan run exactly as on
eight GPUs.  C4 (BASELINE configs[4], 10^10 bits) at world 8 and 2 is checked against its
committed GMP digest.  The cross-device peer path itself (hipMemcpyPeerAsync between distinct
GPUs) has not run on separate GPUs from these tests."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("depth,w,n1,n2", [(13, 32, 1000000, 999000), (15, 4, 2000000, 1900000),
                                          (11, 8, 261952, 261952), (10, 1, 2000, 1800)])
def test_mul_multi_one_device(mp, oracle, world, depth, w, n1, n2):
    """l = 4096 (8 columns per rank at world 8), l = 2048 (the C2/C3 size, fused row level),
    C1's shape (l = 256) and a small l = 16 case, every world size, against GMP; the second
    call reuses the cached buffers."""
    P = mp.plan_info(n1, n2, depth, w)
    if P["NC"] % world:
        pytest.skip("world does not divide NC")
    a = mp.fill_random(n1, 0x11 + depth + world)
    b = mp.fill_random(n2, 0x22 + w)
    want = oracle.gmp_mul(a, b)
    for _ in range(2):
        assert (mp.mul_multi(a, b, depth, w, [0] * world) == want).all()


@pytest.mark.parametrize("world,rep", [(2, "0"), (4, "1"), (8, "1")])
@pytest.mark.parametrize("depth,w,n1,n2", [(13, 32, 1000000, 999000), (15, 4, 2000000, 1900000), (10, 1, 2000, 1800)])
def test_mul_multi_column_policy_forced(mp, oracle, monkeypatch, world, rep, depth, w, n1, n2):
    """the forward-column policy forced against its default (MPFFT_REPLICATE_COLUMNS): world 2
    with exchange #1 over the peers, worlds 4 and 8 with every column block on every rank"""
    monkeypatch.setenv("MPFFT_REPLICATE_COLUMNS", rep)
    a = mp.fill_random(n1, 0x31 + depth + world)
    b = mp.fill_random(n2, 0x42 + w)
    assert (mp.mul_multi(a, b, depth, w, [0] * world) == oracle.gmp_mul(a, b)).all()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("depth,w,n", [(13, 32, 1000000), (15, 4, 2000000), (10, 1, 2000)])
def test_mul_multi_all_ones(mp, oracle, world, depth, w, n):
    """all-ones operands: the product's upper half is all-ones limbs, so carries cross stripe
    and rank boundaries and k_stripe_carry decides them"""
    a = np.full(n, (1 << 64) - 1, dtype=np.uint64)
    assert (mp.mul_multi(a, a, depth, w, [0] * world) == oracle.gmp_mul(a, a)).all()


@pytest.mark.parametrize("world", [1, 2, 8])
@pytest.mark.parametrize("depth,w,n1,n2", [(13, 32, 1000000, 999000), (15, 4, 2000000, 1900000)])
def test_mul_multi_device_entry(mp, oracle, world, depth, w, n1, n2):
    """mpfft_mul_multi_device: packed operand slices already on the devices (mpfft_shard_pack),
    stripes back on the devices, ordered on the callers' torch streams; twice (the second call
    queued behind the first on the same streams)"""
    import torch
    dev = torch.device("cuda:0")
    a = mp.fill_random(n1, 0x51 + world)
    b = mp.fill_random(n2, 0x62 + world)
    part = mp.shard_partition(n1, n2, depth, w, world)
    src1 = [torch.from_numpy(mp.shard_pack(a, n1, n2, depth, w, world, g).view(np.int64)).to(dev) for g in range(world)]
    src2 = [torch.from_numpy(mp.shard_pack(b, n1, n2, depth, w, world, g).view(np.int64)).to(dev) for g in range(world)]
    outs = [torch.empty(part["Tr"] * part["SL"], dtype=torch.int64, device=dev) for _ in range(world)]
    st = torch.cuda.Stream(dev)
    want = oracle.gmp_mul(a, b)
    for _ in range(2):
        with torch.cuda.stream(st):
            for o in outs:
                o.fill_(-1)
            mp.mul_multi_device(n1, n2, depth, w, [0] * world, src1, src2, outs, streams=[st] * world)
        st.synchronize()
        got = mp.assemble_stripes(part, world, [o.cpu().numpy().view(np.uint64) for o in outs])
        assert (got == want).all()
    mp.mul_multi_device(n1, n2, depth, w, [0] * world, src1, src2, outs)   # streams=None: synchronous
    got = mp.assemble_stripes(part, world, [o.cpu().numpy().view(np.uint64) for o in outs])
    assert (got == want).all()


@pytest.mark.parametrize("world", [2, 8])
def test_mul_multi_device_back_to_back_rank_streams(mp, oracle, world):
    """Two device-resident calls queued back to back on separate per-rank streams with no host
    synchronisation between them, each call with its own operands and stripes: the second call's
    first writes into a rank's arrays must wait for the first call's pulls from them on the other
    ranks' streams (the event graph is checked on the CPU in test_multi_schedule.py).
    Both products exact."""
    import torch
    dev = torch.device("cuda:0")
    depth, w, n1, n2 = 15, 4, 2000000, 1900000
    part = mp.shard_partition(n1, n2, depth, w, world)
    sts = [torch.cuda.Stream(dev) for _ in range(world)]
    calls = []
    for k in range(2):
        a = mp.fill_random(n1, 0x700 + 16 * k + world)
        b = mp.fill_random(n2, 0x800 + 16 * k + world)
        src1 = [torch.from_numpy(mp.shard_pack(a, n1, n2, depth, w, world, g).view(np.int64)).to(dev)
                for g in range(world)]
        src2 = [torch.from_numpy(mp.shard_pack(b, n1, n2, depth, w, world, g).view(np.int64)).to(dev)
                for g in range(world)]
        outs = [torch.full((part["Tr"] * part["SL"],), -1, dtype=torch.int64, device=dev) for _ in range(world)]
        calls.append((oracle.gmp_mul(a, b), src1, src2, outs))
    torch.cuda.synchronize()
    for want, src1, src2, outs in calls:
        mp.mul_multi_device(n1, n2, depth, w, [0] * world, src1, src2, outs, streams=sts)
    for s in sts:
        s.synchronize()
    for want, src1, src2, outs in calls:
        got = mp.assemble_stripes(part, world, [o.cpu().numpy().view(np.uint64) for o in outs])
        assert (got == want).all()


def test_mul_multi_c4_world2_digest(mp):
    """C4 over two ranks on device 0 with the default (replicated) forward columns, against the
    GMP digest"""
    with open(os.path.join(HERE, "golden", "products.json")) as f:
        case = {c["name"]: c for c in json.load(f)}["C4"]
    n1, n2, depth, w = case["n1"], case["n2"], case["depth"], case["w"]
    a = mp.fill_random(n1, int(case["seed1"], 16))
    b = mp.fill_random(n2, int(case["seed2"], 16))
    r = mp.mul_multi(a, b, depth, w, [0] * 2)
    del a, b
    assert hashlib.sha256(r.tobytes()).hexdigest() == case["sha256"]
    mp.multi_release()


def test_mul_multi_c4_world8_digest(mp):
    """C4 split 8 ways exactly as on an 8-GPU node (the plan's columns and live rows dealt evenly
    over 8 ranks, seven-peer exchanges, per-stripe halo, stripe carry scan) with all ranks on
    device 0, against the GMP digest."""
    with open(os.path.join(HERE, "golden", "products.json")) as f:
        case = {c["name"]: c for c in json.load(f)}["C4"]
    n1, n2, depth, w = case["n1"], case["n2"], case["depth"], case["w"]
    part = mp.shard_partition(n1, n2, depth, w, 8)
    P = mp.plan_info(n1, n2, depth, w)
    rc = [part["rows"][d + 1] - part["rows"][d] for d in range(8)]
    assert part["C"] == P["NC"] // 8 and part["Tr"] == P["trunc"] // P["NC"] and max(rc) - min(rc) <= 1
    a = mp.fill_random(n1, int(case["seed1"], 16))
    b = mp.fill_random(n2, int(case["seed2"], 16))
    r = mp.mul_multi(a, b, depth, w, [0] * 8)
    del a, b
    assert hashlib.sha256(r.tobytes()).hexdigest() == case["sha256"]
    mp.multi_release()


def test_new_mpn_mul_device_policy(mp, oracle):
    """mpfft_set_devices: new_mpn_mul shards products with coefficients of >= min_l limbs over
    the listed devices (here four ranks on device 0) and runs smaller ones on one device;
    both exact.  Turned off again afterwards."""
    try:
        mp.set_devices([0, 0, 0, 0], min_l=1024)
        for depth, w, n1, n2 in ((13, 32, 800000, 700000), (9, 2, 120, 97)):
            a = mp.fill_random(n1, 0x33 + depth)
            b = mp.fill_random(n2, 0x44 + depth)
            assert (mp.mul(a, b, depth, w) == oracle.gmp_mul(a, b)).all()
            assert mp.lib().mpfft_last_ngpus() == (4 if depth == 13 else 1)
    finally:
        mp.set_devices([])
        mp.multi_release()


def test_mul_multi_rejects_bad_worlds(mp):
    a = mp.fill_random(1000, 1)
    with pytest.raises(mp.MpfftError):
        mp.mul_multi(a, a, 10, 1, [0, 0, 0])          # not a power of two
    with pytest.raises(mp.MpfftError):
        mp.mul_multi(a, a, 10, 1, [0] * 64)           # more ranks than columns
    with pytest.raises(mp.MpfftError):
        mp.mul_multi(a, a, 10, 1, [0, 99])            # no such device

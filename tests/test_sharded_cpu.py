"""Multi-rank (gloo, CPU) tests of the column-sharded multiply
(mpir-fft_amd/sharded.py): partitioning, the three all-to-all exchanges, the
halo all-gather and the cross-rank carry scan, with every stage computed
exactly (tests/mock_backend.py) on the same buffer layouts as the GPU.
The assembled product must equal the exact product.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, depth, w, n1, n2, seed, q, replicate=False):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mpfft_loader
        mp = mpfft_loader.load()
        from mpir_fft_amd.sharded import ShardPlan, ShardedMul, TorchComm
        from mock_backend import MockBackend
        plan = ShardPlan(mp, n1, n2, depth, w, world)
        rng = random.Random(seed)
        a = mp.fill_random(n1, rng.getrandbits(64))
        b = mp.fill_random(n2, rng.getrandbits(64))
        job = ShardedMul(plan, rank, MockBackend(plan), TorchComm(), sliced=not replicate, replicate=replicate)
        if replicate:   # replicated forward columns: the whole operands on every rank
            sa, sb = a, b
        else:
            sa, sb = plan.slice_operand(a, rank), plan.slice_operand(b, rank)   # this rank's column slices
        m0, limbs = job.run(torch.from_numpy(sa.view(np.int64)), torch.from_numpy(sb.view(np.int64)))
        # gather the distributed product on every rank
        sizes = [plan.M[d + 1] - plan.M[d] for d in range(world)]
        pad = torch.zeros(max(sizes), dtype=torch.int64)
        pad[: limbs.numel()] = limbs
        bufs = [torch.zeros(max(sizes), dtype=torch.int64) for _ in range(world)]
        dist.all_gather(bufs, pad)
        if rank == 0:
            prod = np.concatenate([bufs[d][: sizes[d]].numpy() for d in range(world)]).view(np.uint64)
            got = int.from_bytes(prod.tobytes(), "little")
            want = int.from_bytes(a.tobytes(), "little") * int.from_bytes(b.tobytes(), "little")
            q.put(("ok" if got == want else "mismatch", plan.rows, plan.M))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("error", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def _run(world, depth, w, n1, n2, seed=1, replicate=False):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, w, n1, n2, seed, q, replicate))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    res = q.get(timeout=5)
    assert res[0] == "ok", res


@pytest.mark.parametrize("world,depth,w,n1,n2", [
    (2, 6, 2, 7, 6),       # NC 8, T/NC = 4 rows: full truncation variety at tiny size
    (2, 7, 1, 5, 4),       # trunc < 2n (van der Hoeven case a)
    (4, 8, 1, 100, 90),    # 4 ranks, truncated
    (2, 8, 2, 50, 3),      # unbalanced operands
    (1, 7, 1, 5, 4),       # one rank: row arrays alias the column arrays, exchanges move nothing
    (8, 8, 1, 100, 90),    # 8 ranks (C4's world): 2 columns and one live row per rank
    (8, 10, 1, 2000, 1800),  # 8 ranks, 4 columns and 2 rows each; the halo reaches into rank d-1
])
def test_sharded_gloo_exact(world, depth, w, n1, n2):
    _run(world, depth, w, n1, n2)


@pytest.mark.parametrize("world,depth,w,n1,n2", [
    (2, 6, 2, 7, 6),       # world 2 (the replicated policy's world), full truncation variety
    (2, 8, 2, 50, 3),      # unbalanced operands
    (4, 8, 1, 100, 90),    # forced at 4 ranks (MPFFT_REPLICATE_COLUMNS=1)
])
def test_sharded_gloo_replicated_columns(world, depth, w, n1, n2):
    """every rank computes every column block from the whole operands and keeps its rows:
    exchange #1 played locally (ShardedMul.replicate)"""
    _run(world, depth, w, n1, n2, seed=3, replicate=True)


def test_replicate_policy(mp, monkeypatch):
    from mpir_fft_amd.sharded import ShardedMul
    monkeypatch.delenv("MPFFT_REPLICATE_COLUMNS", raising=False)
    assert [ShardedMul.replicates(W) for W in (1, 2, 4, 8)] == [False, True, False, False]
    monkeypatch.setenv("MPFFT_REPLICATE_COLUMNS", "0")
    assert not ShardedMul.replicates(2)
    monkeypatch.setenv("MPFFT_REPLICATE_COLUMNS", "1")
    assert ShardedMul.replicates(8) and not ShardedMul.replicates(1)


def test_shard_plan_partition(mp):
    import importlib
    sh = importlib.import_module("mpir_fft_amd.sharded")
    p = sh.ShardPlan(mp, 156250000, 156250000, 17, 2, 8)        # C4 over 8 GPUs
    P = mp.plan_info(156250000, 156250000, 17, 2)               # (whatever split the library plans)
    assert p.C == P["NC"] // 8 and p.rows[-1] == p.Tr == P["trunc"] // P["NC"]
    assert max(p.rcount(d) for d in range(8)) - min(p.rcount(d) for d in range(8)) <= 1
    assert p.M[0] == 0 and p.M[-1] == p.total and sorted(p.M) == p.M
    with pytest.raises(ValueError):
        sh.ShardPlan(mp, 100, 90, 8, 1, 3)                      # world must be a power of two


def _py_partition(mp, n1, n2, depth, w, world):
    """SURVEY 8e's partition restated in Python (independent of csrc/multi.hip)."""
    import math
    P = mp.plan_info(n1, n2, depth, w)
    NC, T, bits1 = P["NC"], P["trunc"], P["bits1"]
    N = P["n"] * w
    Tr, total = T // NC, n1 + n2
    C = NC // world
    rows = [(d * Tr) // world for d in range(world + 1)]
    M = [0] + [min(total, (rows[d] * NC * bits1) // 64) for d in range(1, world)] + [total]
    H = math.ceil((N + 128) / bits1) + 1
    return rows, M, C, (C * bits1 + 63) // 64 + 2, H


@pytest.mark.parametrize("world,depth,w,n1,n2", [
    (8, 17, 2, 156250000, 156250000), (4, 17, 2, 156250000, 156250000), (2, 17, 2, 156250000, 156250000),
    (8, 15, 4, 20312500, 20312500), (8, 13, 32, 1000000, 1000000), (4, 8, 1, 100, 90), (2, 6, 2, 7, 6),
    (8, 10, 1, 2000, 1800), (1, 7, 1, 5, 4)])
def test_c_partition_matches_restatement(mp, world, depth, w, n1, n2):
    """mpfft_shard_partition (the C planner both sharded drivers use) against the partition
    restated in Python: rows per rank, product limb ranges, columns, slice chunk, halo."""
    rows, M, C, chunk, H = _py_partition(mp, n1, n2, depth, w, world)
    c = mp.shard_partition(n1, n2, depth, w, world)
    assert (c["rows"], c["M"], c["C"], c["chunk"], c["H"]) == (rows, M, C, chunk, H)


@pytest.mark.parametrize("world,depth,w,n1,n2", [(8, 13, 32, 1000000, 1000000), (4, 8, 1, 100, 90),
                                                 (8, 10, 1, 2000, 1800), (2, 6, 2, 7, 6), (1, 7, 1, 5, 4)])
def test_c_exchange_plans_move_every_slot_once(mp, world, depth, w, n1, n2):
    """mpfft_shard_exchange_plan on CPU: apply each exchange's copies to labelled arrays and
    check the result slot by slot against the layouts' definitions (include/mpfft.h):
    #1 moves every live (position, column) of both operands from its column owner to its row
    owner, #2 moves the product back, #3 the limbs again; nothing written twice."""
    P = mp.plan_info(n1, n2, depth, w)
    part = mp.shard_partition(n1, n2, depth, w, world)
    NC, NR, C, rows, Tr = P["NC"], P["NR"], part["C"], part["rows"], part["Tr"]
    l, cbw = P["l"], 2 * ((P["l"] + 63) // 64)
    width = (l, cbw, 1)

    def label(pos, c, f, e):   # a unique id per (position, column, field, element)
        return ((pos * NC + c) * 3 + f) * (l + 1) + e

    for which, ops, fields in ((1, (0, 1), (0, 1, 2)), (2, (0,), (0, 1, 2)), (3, (0,), (0,))):
        col = {(d, op, f): np.full(NR * C * width[f], -1, dtype=np.int64) for d in range(world)
               for op in (0, 1) for f in range(3)}
        row = {(d, op, f): np.full((rows[d + 1] - rows[d]) * NC * width[f], -1, dtype=np.int64)
               for d in range(world) for op in (0, 1) for f in range(3)}
        src_is_col = which != 2
        for d in range(world):   # fill the sending layout with labels
            for op in ops:
                for f in fields:
                    wd = width[f]
                    if src_is_col:
                        for pos in range(Tr):
                            for cl in range(C):
                                s = pos * C + cl
                                col[(d, op, f)][s * wd:(s + 1) * wd] = [label(pos, d * C + cl, f, e) for e in range(wd)]
                    else:
                        rc = rows[d + 1] - rows[d]
                        for pl in range(rc):
                            for c in range(NC):
                                s = (c // C) * rc * C + pl * C + c % C
                                row[(d, op, f)][s * wd:(s + 1) * wd] = [label(rows[d] + pl, c, f, e) for e in range(wd)]
        written = {}
        for cp in mp.shard_exchange_plan(n1, n2, depth, w, world, which):
            assert cp["op"] in ops and cp["field"] in fields
            src = (col if cp["src_layout"] == 0 else row)[(cp["src"], cp["op"], cp["field"])]
            dst = (col if cp["dst_layout"] == 0 else row)[(cp["dst"], cp["op"], cp["field"])]
            key = (cp["dst"], cp["dst_layout"], cp["op"], cp["field"])
            rng = set(range(cp["dst_off"], cp["dst_off"] + cp["count"]))
            assert not (written.setdefault(key, set()) & rng), "element written twice"
            written[key] |= rng
            dst[cp["dst_off"]: cp["dst_off"] + cp["count"]] = src[cp["src_off"]: cp["src_off"] + cp["count"]]
        for d in range(world):   # the receiving layout must hold every live slot's own labels
            for op in ops:
                for f in fields:
                    wd = width[f]
                    if src_is_col:
                        rc = rows[d + 1] - rows[d]
                        for pl in range(rc):
                            for c in range(NC):
                                s = (c // C) * rc * C + pl * C + c % C
                                want = [label(rows[d] + pl, c, f, e) for e in range(wd)]
                                assert list(row[(d, op, f)][s * wd:(s + 1) * wd]) == want, (which, d, pl, c, f)
                    else:
                        for pos in range(Tr):
                            for cl in range(C):
                                s = pos * C + cl
                                want = [label(pos, d * C + cl, f, e) for e in range(wd)]
                                assert list(col[(d, op, f)][s * wd:(s + 1) * wd]) == want, (which, d, pos, cl, f)

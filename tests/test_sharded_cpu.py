"""Multi-rank (gloo, CPU) tests of the column-sharded multiply
(mpir-fft_amd/sharded.py): partitioning, the two exchanges, the per-stripe halo,
the striped combine and the stripe carry scan, with every stage computed exactly
(tests/mock_backend.py) on the same buffer layouts as the GPU; and the overlapped
exchange orderings under a deferred-completion transport (tests/deferred_comm.py),
with mutants of the ordering that it must catch.  The assembled product must equal
the exact product.
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


# textual mutants of sharded.py (ShardedMul.run) that the deferred transport must catch: an
# exchange waited for only after a stage that reads its receive buffers
MUTANTS = {
    # exchange #2 waited after the inverse columns (they read the column arrays it fills)
    "wait2_after_inv_columns": (
        '        self.comm.wait(pend2)          # exchange #2 complete before the inverse columns\n'
        '        mark("exchange2")\n'
        '        be.stage("inv_columns", sh, i1, i2)\n',
        '        mark("exchange2")\n'
        '        be.stage("inv_columns", sh, i1, i2)\n'
        '        self.comm.wait(pend2)\n'),
    # exchange #1 waited after the row phase (its stages read the row arrays it fills)
    "wait1_after_fwd_rows": (
        '            self.comm.wait(pend1)          # exchange #1 complete before the row passes\n',
        '            self._late = pend1\n'),
}


def _sharded_module(mutant):
    """mpir_fft_amd.sharded, or a copy of it with one of MUTANTS applied"""
    import importlib
    import types
    mod = importlib.import_module("mpir_fft_amd.sharded")
    if not mutant:
        return mod
    old, new = MUTANTS[mutant]
    src = open(mod.__file__).read()
    assert src.count(old) == 1, f"mutant {mutant}: pattern not found once in sharded.py"
    src = src.replace(old, new)
    if mutant == "wait1_after_fwd_rows":   # the late wait goes after the whole chunked row phase
        pat = '            mark("inv_rows")\n            sh = sh_inv\n'
        assert src.count(pat) == 1
        src = src.replace(pat, pat + '            self.comm.wait(self._late)\n')
    m = types.ModuleType("sharded_mutant")
    m.__file__ = mod.__file__
    exec(compile(src, mod.__file__, "exec"), m.__dict__)
    return m


def _worker(rank, world, port, depth, w, n1, n2, seed, q, replicate=False, comm="gloo", ones=False, mutant=None):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mpfft_loader
        mp = mpfft_loader.load()
        sh = _sharded_module(mutant)
        from mock_backend import MockBackend
        from deferred_comm import DeferredComm
        plan = sh.ShardPlan(mp, n1, n2, depth, w, world)
        rng = random.Random(seed)
        if ones:   # all-ones operands: long runs of all-ones product limbs, carries across stripes
            a = np.full(n1, (1 << 64) - 1, dtype=np.uint64)
            b = np.full(n2, (1 << 64) - 1, dtype=np.uint64)
        else:
            a = mp.fill_random(n1, rng.getrandbits(64))
            b = mp.fill_random(n2, rng.getrandbits(64))
        tc = sh.TorchComm()
        cm = DeferredComm(tc) if comm == "deferred" else tc
        job = sh.ShardedMul(plan, rank, MockBackend(plan), cm, sliced=not replicate, replicate=replicate)
        if replicate:   # replicated forward columns: the whole operands on every rank
            sa, sb = a, b
        else:
            sa, sb = plan.slice_operand(a, rank), plan.slice_operand(b, rank)   # this rank's column slices
        try:
            limbs = job.run(torch.from_numpy(sa.view(np.int64)), torch.from_numpy(sb.view(np.int64)))
        except Exception as e:
            import traceback
            q.put(("raised", type(e).__name__, str(e), traceback.format_exc()[-1500:]))
            return
        # gather the striped product on every rank
        bufs = [torch.zeros_like(limbs) for _ in range(world)]
        dist.all_gather(bufs, limbs)
        if rank == 0:
            prod = plan.assemble([x.numpy().view(np.uint64) for x in bufs])
            got = int.from_bytes(prod.tobytes(), "little")
            want = int.from_bytes(a.tobytes(), "little") * int.from_bytes(b.tobytes(), "little")
            asy = getattr(cm, "issued", None)
            q.put(("ok" if got == want else "mismatch", plan.rows, asy))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("error", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def _run(world, depth, w, n1, n2, seed=1, replicate=False, comm="gloo", ones=False, mutant=None):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, w, n1, n2, seed, q, replicate, comm, ones,
                                               mutant))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60 if res[0] == "ok" else 5)
        if p.is_alive():   # a rank left waiting for a peer that raised
            p.kill()
    return res


@pytest.mark.parametrize("world,depth,w,n1,n2", [
    (2, 6, 2, 7, 6),       # NC 8, T/NC = 4 rows: full truncation variety at tiny size
    (2, 7, 1, 5, 4),       # trunc < 2n (van der Hoeven case a)
    (4, 8, 1, 100, 90),    # 4 ranks, truncated; C = 4 columns < H: a halo spans stripes
    (2, 8, 2, 50, 3),      # unbalanced operands
    (1, 7, 1, 5, 4),       # one rank: row arrays alias the column arrays, the halo is local
    (8, 8, 1, 100, 90),    # 8 ranks (C4's world): 2 columns and one live row per rank
    (8, 10, 1, 2000, 1800),  # 8 ranks, 4 columns and 2 rows each; H = C
])
def test_sharded_gloo_exact(world, depth, w, n1, n2):
    res = _run(world, depth, w, n1, n2)
    assert res[0] == "ok", res


@pytest.mark.parametrize("world,depth,w,n", [(2, 8, 2, 60), (4, 10, 1, 1000), (8, 10, 1, 1000)])
def test_sharded_gloo_all_ones(world, depth, w, n):
    """all-ones operands: the product's upper half is all-ones limbs, so carries run across
    stripe (and rank) boundaries and the stripe carry scan decides every one"""
    res = _run(world, depth, w, n, n, ones=True)
    assert res[0] == "ok", res


# deferred-completion transport (tests/deferred_comm.py) through both overlapped paths: exchange
# #1 per operand beside operand 2's column passes, and the four-chunk row phase with each
# chunk's exchange #2 in flight
@pytest.mark.parametrize("world,depth,w,n1,n2", [(2, 8, 2, 50, 40), (4, 10, 1, 1000, 900), (8, 10, 1, 2000, 1800)])
def test_sharded_deferred_transport(world, depth, w, n1, n2):
    res = _run(world, depth, w, n1, n2, seed=7, comm="deferred")
    assert res[0] == "ok", res
    # 2 exchange-#1 batches + 4 row-chunk exchange-#2 batches went through the deferred path
    assert res[2] == 6, res


@pytest.mark.parametrize("mutant", sorted(MUTANTS))
def test_deferred_transport_catches_misordered_wait(mutant):
    """a run() that waits for an exchange only after a stage reading its receive buffers must
    fail under the deferred transport (wrong product or a raised error), where the immediate
    gloo transport would pass it"""
    res = _run(4, 10, 1, 1000, 900, seed=7, comm="deferred", mutant=mutant)
    assert res[0] in ("mismatch", "raised"), res


@pytest.mark.parametrize("world,depth,w,n1,n2", [
    (2, 6, 2, 7, 6),       # world 2 (the replicated policy's world), full truncation variety
    (2, 8, 2, 50, 3),      # unbalanced operands
    (4, 8, 1, 100, 90),    # forced at 4 ranks (MPFFT_REPLICATE_COLUMNS=1)
])
def test_sharded_gloo_replicated_columns(world, depth, w, n1, n2):
    """every rank computes every column block from the whole operands and keeps its rows:
    exchange #1 played locally (ShardedMul.replicate)"""
    res = _run(world, depth, w, n1, n2, seed=3, replicate=True)
    assert res[0] == "ok", res


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
    assert p.S == 8 * p.Tr and len(p.ms) == p.S + 1
    assert p.ms[0] == 0 and p.ms[-1] == p.total and sorted(p.ms) == p.ms
    assert max(p.ms[s + 1] - p.ms[s] for s in range(p.S)) <= p.SL
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
    H = math.ceil((N + 128) / bits1) + 1
    S = world * Tr
    ms = [min(total, (s * C * bits1) // 64) for s in range(S)] + [total]
    SL = ((C + 1) * bits1) // 64 + 2
    return rows, C, (C * bits1 + 63) // 64 + 2, H, S, ms, SL


@pytest.mark.parametrize("world,depth,w,n1,n2", [
    (8, 17, 2, 156250000, 156250000), (4, 17, 2, 156250000, 156250000), (2, 17, 2, 156250000, 156250000),
    (8, 15, 4, 20312500, 20312500), (8, 13, 32, 1000000, 1000000), (4, 8, 1, 100, 90), (2, 6, 2, 7, 6),
    (8, 10, 1, 2000, 1800), (1, 7, 1, 5, 4)])
def test_c_partition_matches_restatement(mp, world, depth, w, n1, n2):
    """mpfft_shard_partition / mpfft_shard_stripes (the C planner both sharded drivers use)
    against the partition restated in Python: rows per rank, columns, slice chunk, halo, the
    stripes' product limb ranges and stride; every stripe's limbs fit its stride."""
    rows, C, chunk, H, S, ms, SL = _py_partition(mp, n1, n2, depth, w, world)
    c = mp.shard_partition(n1, n2, depth, w, world)
    assert (c["rows"], c["C"], c["chunk"], c["H"], c["S"], c["ms"], c["SL"]) == (rows, C, chunk, H, S, ms, SL)
    assert all(ms[s + 1] - ms[s] <= SL for s in range(S))


@pytest.mark.parametrize("world,depth,w,n1,n2", [(8, 13, 32, 1000000, 1000000), (4, 8, 1, 100, 90),
                                                 (8, 10, 1, 2000, 1800), (2, 6, 2, 7, 6), (1, 7, 1, 5, 4),
                                                 (8, 8, 1, 100, 90)])
def test_c_halo_plan(mp, world, depth, w, n1, n2):
    """mpfft_shard_halo_plan applied to labelled column layouts: every rank's halo slot
    j H + i holds coefficient (j world + g) C - H + i (for those >= 0), nothing written twice,
    sources read inside their column layout"""
    P = mp.plan_info(n1, n2, depth, w)
    part = mp.shard_partition(n1, n2, depth, w, world)
    C, H, Tr, l = part["C"], part["H"], part["Tr"], P["l"]
    col = {d: np.array([((pos * world + d) * C + cl) for pos in range(P["NR"]) for cl in range(C)]) for d in range(world)}
    halo = {d: np.full(Tr * H, -1) for d in range(world)}
    for c in mp.shard_halo_plan(n1, n2, depth, w, world):
        assert c["field"] == 0 and c["src_layout"] == 0 and c["dst_layout"] == mp.LAYOUT_HALO
        assert c["src_off"] % l == 0 and c["dst_off"] % l == 0 and c["count"] % l == 0
        so, do, n = c["src_off"] // l, c["dst_off"] // l, c["count"] // l
        assert so + n <= Tr * C, "a halo source past the live rows"
        assert (halo[c["dst"]][do: do + n] == -1).all(), "halo slot written twice"
        halo[c["dst"]][do: do + n] = col[c["src"]][so: so + n]
    for g in range(world):
        for j in range(Tr):
            k0 = (j * world + g) * C - H
            want = [k0 + i if k0 + i >= 0 else -1 for i in range(H)]
            assert list(halo[g][j * H: (j + 1) * H]) == want, (g, j)


@pytest.mark.parametrize("world,depth,w,n1,n2", [(8, 13, 32, 1000000, 1000000), (4, 8, 1, 100, 90),
                                                 (8, 10, 1, 2000, 1800), (2, 6, 2, 7, 6), (1, 7, 1, 5, 4)])
def test_c_exchange_plans_move_every_slot_once(mp, world, depth, w, n1, n2):
    """mpfft_shard_exchange_plan on CPU: apply each exchange's copies to labelled arrays and
    check the result slot by slot against the layouts' definitions (include/mpfft.h):
    #1 moves every live (position, column) of both operands from its column owner to its row
    owner, #2 moves the product back; nothing written twice."""
    P = mp.plan_info(n1, n2, depth, w)
    part = mp.shard_partition(n1, n2, depth, w, world)
    NC, NR, C, rows, Tr = P["NC"], P["NR"], part["C"], part["rows"], part["Tr"]
    l, cbw = P["l"], 2 * ((P["l"] + 63) // 64)
    width = (l, cbw, 1)

    def label(pos, c, f, e):   # a unique id per (position, column, field, element)
        return ((pos * NC + c) * 3 + f) * (l + 1) + e

    for which, ops, fields in ((1, (0, 1), (0, 1, 2)), (2, (0,), (0, 1, 2))):
        col = {(d, op, f): np.full(NR * C * width[f], -1, dtype=np.int64) for d in range(world)
               for op in (0, 1) for f in range(3)}
        row = {(d, op, f): np.full((rows[d + 1] - rows[d]) * NC * width[f], -1, dtype=np.int64)
               for d in range(world) for op in (0, 1) for f in range(3)}
        src_is_col = which == 1
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

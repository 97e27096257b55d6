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


def _worker(rank, world, port, depth, w, n1, n2, seed, q):
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
        job = ShardedMul(plan, rank, MockBackend(plan), TorchComm())
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


def _run(world, depth, w, n1, n2, seed=1):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, w, n1, n2, seed, q)) for r in range(world)]
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
])
def test_sharded_gloo_exact(world, depth, w, n1, n2):
    _run(world, depth, w, n1, n2)


def test_shard_plan_partition(mp):
    import importlib
    sh = importlib.import_module("mpir_fft_amd.sharded")
    p = sh.ShardPlan(mp, 156250000, 156250000, 17, 2, 8)        # C4 over 8 GPUs
    assert p.C == 32 and p.rows[-1] == p.Tr == 598
    assert all(p.rcount(d) in (74, 75) for d in range(8))
    assert p.M[0] == 0 and p.M[-1] == p.total and sorted(p.M) == p.M
    with pytest.raises(ValueError):
        sh.ShardPlan(mp, 100, 90, 8, 1, 3)                      # world must be a power of two

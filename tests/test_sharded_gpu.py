"""GPU tests of the column-sharded multiply through the mpfft_shard_* C ABI.
world 1 runs in-process; world 2 runs two ranks on the same MI355X with the
exchanges host-staged through gloo (RCCL needs one GPU per rank; the 8-GPU
RCCL run is the driver's)."""
import os
import random
import socket

import numpy as np
import pytest


pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _exact(a, b, limbs):
    got = int.from_bytes(np.asarray(limbs).view(np.uint64).tobytes(), "little")
    return got == int.from_bytes(a.tobytes(), "little") * int.from_bytes(b.tobytes(), "little")


@pytest.mark.parametrize("depth,w,n1,n2", [(6, 2, 7, 6), (8, 1, 100, 90), (11, 8, 261952, 261952),
                                          (11, 1, 16384, 16384), (10, 3, 1000, 17),
                                          (15, 4, 2000000, 1900000), (13, 32, 1000000, 1000000)])
def test_sharded_world1(mp, oracle, depth, w, n1, n2):
    """World 1 through the sharded code path (column slices, local exchanges) at l = 32 ... 4096:
    (15, 4) is a C2/C3-shaped l = 2048 case, (13, 32) an l = 4096 case with 8 row levels.
    Two runs of the same job: the fused-pointwise array swap must leave the row arrays views
    of the column arrays, and the second product exact too."""
    import torch
    from mpir_fft_amd.sharded import ShardPlan, ShardedMul, GpuBackend, _SoloComm
    dev = torch.device("cuda:0")
    plan = ShardPlan(mp, n1, n2, depth, w, 1)
    a = mp.fill_random(n1, 5 + depth)
    b = mp.fill_random(n2, 6 + w)
    job = ShardedMul(plan, 0, GpuBackend(mp, plan, dev), _SoloComm())
    sa, sb = plan.slice_operand(a, 0), plan.slice_operand(b, 0)
    da, db = torch.from_numpy(sa.view(np.int64)).to(dev), torch.from_numpy(sb.view(np.int64)).to(dev)
    want = oracle.gmp_mul(a, b)
    for run in range(2):
        limbs = job.run(da, db)
        torch.cuda.synchronize()
        got = plan.assemble([limbs.cpu().numpy().view(np.uint64)])
        assert (got == want).all(), run
        for k in range(2):   # world 1: every row array is a view of its column array
            assert job.row[k]["dig"].data_ptr() == job.col[k]["dig"].data_ptr()


def test_sharded_world1_c4_digest(mp):
    """BASELINE configs[4] (10^10-bit, depth 17, w 2, l = 4096) through the column-sharded
    code path at world 1 -- operand column slices, the fused-split loaders at l = 4096, the
    local exchanges, the halo and the striped combine -- against the committed GMP digest of C4."""
    import hashlib
    import json
    import torch
    from mpir_fft_amd.sharded import ShardPlan, ShardedMul, GpuBackend, _SoloComm
    with open(os.path.join(HERE, "golden", "products.json")) as f:
        want = {c["name"]: c for c in json.load(f)}["C4"]
    depth, w, nl = want["depth"], want["w"], want["n1"]
    dev = torch.device("cuda:0")
    plan = ShardPlan(mp, nl, nl, depth, w, 1)
    a = mp.fill_random(nl, int(want["seed1"], 16))
    sa = torch.from_numpy(plan.slice_operand(a, 0).view(np.int64)).to(dev)
    del a
    b = mp.fill_random(nl, int(want["seed2"], 16))
    sb = torch.from_numpy(plan.slice_operand(b, 0).view(np.int64)).to(dev)
    del b
    job = ShardedMul(plan, 0, GpuBackend(mp, plan, dev), _SoloComm())
    for run in range(2):   # the second run on swapped (still aliased) arrays
        limbs = job.run(sa, sb)
        torch.cuda.synchronize()
        got = plan.assemble([limbs.cpu().numpy().view(np.uint64)])
        assert len(got) == 2 * nl
        assert hashlib.sha256(got.tobytes()).hexdigest() == want["sha256"], run
        del got
    del job, sa, sb, limbs
    torch.cuda.empty_cache()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, depth, w, n1, n2, q, replicate=False):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mpfft_loader
        mp = mpfft_loader.load()
        from mpir_fft_amd.sharded import ShardPlan, ShardedMul, GpuBackend, TorchComm
        dev = torch.device("cuda:0")
        plan = ShardPlan(mp, n1, n2, depth, w, world)
        a = mp.fill_random(n1, 0x1001)
        b = mp.fill_random(n2, 0x2002)
        job = ShardedMul(plan, rank, GpuBackend(mp, plan, dev), TorchComm(host_staging=True),
                         sliced=not replicate, replicate=replicate)
        if replicate:   # replicated forward columns: the whole operands on every rank
            sa, sb = a, b
        else:
            sa, sb = plan.slice_operand(a, rank), plan.slice_operand(b, rank)   # this rank's column slices
        limbs = job.run(torch.from_numpy(sa.view(np.int64)).to(dev), torch.from_numpy(sb.view(np.int64)).to(dev))
        limbs = limbs.cpu()
        bufs = [torch.zeros_like(limbs) for _ in range(world)]
        dist.all_gather(bufs, limbs)
        if rank == 0:
            import oracle as O
            prod = plan.assemble([x.numpy().view(np.uint64) for x in bufs])
            q.put("ok" if (prod == O.gmp_mul(a, b)).all() else "mismatch")
    except Exception as e:  # pragma: no cover
        q.put("error " + repr(e))
        raise
    finally:
        dist.destroy_process_group()


# ranks sharing one GPU, exchanges host-staged through gloo: C1's shape (l = 256), a small
# unbalanced case, a depth-15 w-4 case (l = 2048, the C2/C3 coefficient size) and a depth-13
# w-32 case (l = 4096, the C4 coefficient size, 8 row levels) at 2 ranks; the l = 4096 case
# at 4 and 8 ranks too (C4's world: 8 columns and 2 live rows per rank, seven-peer batches)
@pytest.mark.parametrize("world,depth,w,n1,n2", [(2, 11, 8, 261952, 261952), (2, 9, 2, 2000, 1500),
                                                 (2, 15, 4, 2000000, 2000000), (2, 13, 32, 1000000, 1000000),
                                                 (4, 13, 32, 1000000, 1000000), (8, 13, 32, 1000000, 1000000),
                                                 (8, 15, 4, 2000000, 1900000)])
def test_sharded_ranks_one_gpu(world, depth, w, n1, n2):
    _ranks_one_gpu(world, depth, w, n1, n2)


# replicated forward columns (bench.py's policy at world 2): every column block computed from
# the whole operands on each rank, exchange #1 local; l = 2048 and l = 4096, and 4 ranks forced
@pytest.mark.parametrize("world,depth,w,n1,n2", [(2, 15, 4, 2000000, 2000000), (2, 13, 32, 1000000, 1000000),
                                                 (2, 9, 2, 2000, 1500), (4, 13, 32, 1000000, 1000000)])
def test_sharded_ranks_one_gpu_replicated(world, depth, w, n1, n2):
    _ranks_one_gpu(world, depth, w, n1, n2, replicate=True)


def _ranks_one_gpu(world, depth, w, n1, n2, replicate=False):
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, w, n1, n2, q, replicate))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert q.get(timeout=5) == "ok"

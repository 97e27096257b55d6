"""GPU tests of the column-sharded multiply through the mpfft_shard_* C ABI.
world 1 runs in-process; world 2 runs two ranks on the same MI355X with the
exchanges host-staged through gloo (RCCL needs one GPU per rank; the 8-GPU
RCCL run is the driver's)."""
import os
import random
import socket

import numpy as np
import pytest

from helpers import max_limbs

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _exact(a, b, limbs):
    got = int.from_bytes(np.asarray(limbs).view(np.uint64).tobytes(), "little")
    return got == int.from_bytes(a.tobytes(), "little") * int.from_bytes(b.tobytes(), "little")


@pytest.mark.parametrize("depth,w,n1,n2", [(6, 2, 7, 6), (8, 1, 100, 90), (11, 8, 261952, 261952),
                                          (11, 1, 16384, 16384), (10, 3, 1000, 17)])
def test_sharded_world1(mp, depth, w, n1, n2):
    import torch
    from mpir_fft_amd.sharded import ShardPlan, ShardedMul, GpuBackend, _SoloComm
    dev = torch.device("cuda:0")
    plan = ShardPlan(mp, n1, n2, depth, w, 1)
    a = mp.fill_random(n1, 5 + depth)
    b = mp.fill_random(n2, 6 + w)
    job = ShardedMul(plan, 0, GpuBackend(mp, plan, dev), _SoloComm())
    sa, sb = plan.slice_operand(a, 0), plan.slice_operand(b, 0)
    m0, limbs = job.run(torch.from_numpy(sa.view(np.int64)).to(dev), torch.from_numpy(sb.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    assert m0 == 0 and _exact(a, b, limbs.cpu().numpy())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, depth, w, n1, n2, q):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
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
        job = ShardedMul(plan, rank, GpuBackend(mp, plan, dev), TorchComm(host_staging=True))
        sa, sb = plan.slice_operand(a, rank), plan.slice_operand(b, rank)   # this rank's column slices
        m0, limbs = job.run(torch.from_numpy(sa.view(np.int64)).to(dev), torch.from_numpy(sb.view(np.int64)).to(dev))
        limbs = limbs.cpu()
        sizes = [plan.M[d + 1] - plan.M[d] for d in range(world)]
        pad = torch.zeros(max(sizes), dtype=torch.int64)
        pad[: limbs.numel()] = limbs
        bufs = [torch.zeros(max(sizes), dtype=torch.int64) for _ in range(world)]
        dist.all_gather(bufs, pad)
        if rank == 0:
            prod = np.concatenate([bufs[d][: sizes[d]].numpy() for d in range(world)])
            q.put("ok" if _exact(a, b, prod) else "mismatch")
    except Exception as e:  # pragma: no cover
        q.put("error " + repr(e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,depth,w,n1,n2", [(2, 11, 8, 261952, 261952), (2, 9, 2, 2000, 1500)])
def test_sharded_two_ranks_one_gpu(world, depth, w, n1, n2):
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, w, n1, n2, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert q.get(timeout=5) == "ok"

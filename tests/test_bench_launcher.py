"""CPU test of bench.py's multi-GPU launcher: `bench.py --gpus N` without a
torch.distributed environment starts N rank processes itself (torch.distributed.run,
127.0.0.1 rendezvous) before anything touches a GPU; --dry-run makes each rank join a
gloo group instead of running the multiply, so the driver-facing n_gpus is checked here."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_spawns_n_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == n and d["ranks_seen"] == n

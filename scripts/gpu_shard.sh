#!/bin/bash
# Sharded path on one GPU: its GPU tests and the stage tests, then world-1 sharded C4 (GMP digest
# checked) beside the single-GPU C4 multiply.  usage: scripts/gpu_shard.sh <tag>
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "sharded or stages_exact or mul6" > gpurun_out/pytest_$T.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --mode sharded --config C4 --steps 2 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4s_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for c in c4s c4; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_${c}_$T.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), d.get('exact'), {k: (round(x,3) if isinstance(x,float) else x) for k,x in (d.get('stages_ms') or {}).items()})" 2>/dev/null; done
tail -c 1500 gpurun_out/bench_c4s_$T.log
exit $rc

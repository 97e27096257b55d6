#!/bin/bash
# Quick loop: C3 bench (+ e2e), C4 bench, then a -k selection of the GPU suite.
# usage: scripts/gpu_quick.sh <tag> "<pytest -k expression>"
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-q} && \
timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --e2e-reps 2 > gpurun_out/bench_$T.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$2" > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for f in gpurun_out/bench_$T.log gpurun_out/bench_c4_$T.log; do python3 -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()}, (d.get('e2e_host') or {}).get('ms'))" 2>/dev/null; done
exit $rc

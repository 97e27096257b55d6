#!/bin/bash
# GPU suite, then the C3 bench with and without an env knob (A/B): usage gpu_ab.sh VAR=value
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_a.log 2>&1 && \
env $1 timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_b.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
for v in a b; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" ; done
exit $rc

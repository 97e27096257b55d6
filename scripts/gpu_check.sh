#!/bin/bash
# Round-3 loop: C3 bench (exact vs the GMP digest), C3 kernel stats, then the GPU suite.
# usage: scripts/gpu_check.sh <tag> [pytest -k expression]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 300 python3 -u bench.py --steps 10 --cpu-reps 1 --cpu-warmup 0 --e2e-reps 1 > gpurun_out/bench_$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$T -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/ks_$T.log 2>&1 && \
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${2:+-k "$2"} > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -c 1500 gpurun_out/bench_$T.log; echo; tail -4 gpurun_out/pytest_$T.log
python3 scripts/kstats.py gpurun_out/ks_$T 2>/dev/null
exit $rc

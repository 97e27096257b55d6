#!/bin/bash
# Round-5 start: the GPU suite and the default bench line at HEAD on a fresh box.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5a} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_default_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log; tail -c 1500 gpurun_out/bench_default_$T.log; exit $rc

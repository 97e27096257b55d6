#!/bin/bash
# Round validation on one MI355X: GPU parity suite, the driver's default bench line,
# and a rocprofv3 kernel-stats pass of the same C3 bench (stops at the first failure).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_default.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c3 -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/p_c3.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench_default.log; exit $rc

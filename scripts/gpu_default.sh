#!/bin/bash
# The driver's round-end sequence on one GPU: smoke(), then the default bench line (C3, CPU
# baseline, e2e), then its rocprofv3 kernel statistics.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 && \
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default_$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$T -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/ks_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/smoke_$T.log; tail -c 3000 gpurun_out/bench_default_$T.log
python3 scripts/kstats.py gpurun_out/ks_$T 2>/dev/null | head -12
exit $rc

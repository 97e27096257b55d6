#!/bin/bash
# Where the world-1 sharded C4 multiply spends its time (kernel stats), and the combine block size V = 16.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c4s -o c4s -- python3 bench.py --mode sharded --config C4 --steps 1 --warmup 1 --no-check > gpurun_out/p_c4s.log 2>&1 && \
MPFFT_CB_V=16 timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_cbv16.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/p_c4s.log | cut -c1-300; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_cbv16.log').read().strip().splitlines()[-1]); print('cbv16', round(d['ms_per_step'],3), d['exact'], round(d['stages_ms']['combine'],3))"
head -25 gpurun_out/p_c4s/c4s_kernel_stats.csv | cut -d, -f1-5; exit $rc

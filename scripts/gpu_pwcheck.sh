#!/bin/bash
# Pointwise change check: direct + whole-product parity, stage timing on C3/C4, both benches.
# usage: scripts/gpu_pwcheck.sh <tag>
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-pc} && L=gpurun_out/pwc_$T.log && : > $L && \
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pointwise_direct or nested_pointwise_full or coefficient_equal" >> $L 2>&1 && \
for cfg in C3 C4; do timeout -k 10 120 python3 -u scripts/pw_time.py $cfg 5 >> $L 2>&1 || exit 1; done && \
timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_$T.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "passed|failed|pointwise k_|FAILED|Error" $L | tail -20
for f in gpurun_out/bench_$T.log gpurun_out/bench_c4_$T.log; do python3 -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null; done
exit $rc

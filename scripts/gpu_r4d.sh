#!/bin/bash
# round 4, call D: the pass-shaped HBM ceiling (tests/microbench/pass_bw) and column batching
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 tests/microbench/pass_bw > gpurun_out/r4d_pass_bw.log 2>&1 || exit $?
cat gpurun_out/r4d_pass_bw.log
for b in 0 12 6 24; do
  MPFFT_LIB=diag MPFFT_COL_BATCH=$b timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline \
    --e2e-reps 0 --no-twin > gpurun_out/r4d_colb_$b.log 2>&1 || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r4d_colb_$b.log') if l.startswith('{')][-1])
print('batch $b', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})"
done

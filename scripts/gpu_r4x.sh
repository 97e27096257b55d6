#!/bin/bash
# round 4, call X: C3 with the quad-fused pointwise -- shipped vs late operand-B load at l = 2048
# (libmpfft_lb.so) vs + four quad inputs in flight (libmpfft_q4lb.so); digests checked
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in main lb q4lb main lb q4lb; do
  if [ $v = main ]; then unset MPFFT_LIB; else export MPFFT_LIB=libmpfft_$v.so; fi
  timeout -k 10 300 python3 bench.py --config C3 --steps 10 --warmup 2 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/x3_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/x3_$v.log') if x.startswith('{')][-1]); print('C3 $v', round(d['ms_per_step'],3), d.get('exact'), 'pointwise', round(d['stages_ms']['pointwise'],3))"
done

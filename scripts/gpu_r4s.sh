#!/bin/bash
# round 4, call S: operand B loaded after A's transform also at l = 2048 (libmpfft_lateb.so)
# vs the shipped build (B up front at l = 2048), C3 and C2; parity of the variant at l = 2048
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MPFFT_LIB=libmpfft_lateb.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "nested or mfa_split or c2_c3 or pointwise_direct" > gpurun_out/pytest_lateb.log 2>&1 || { tail -30 gpurun_out/pytest_lateb.log; exit 1; }
tail -1 gpurun_out/pytest_lateb.log
for c in C3 C2; do
for v in main lateb main lateb; do
  if [ $v = main ]; then unset MPFFT_LIB; else export MPFFT_LIB=libmpfft_$v.so; fi
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/lateb_${c}_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/lateb_${c}_$v.log') if x.startswith('{')][-1]); print('$c $v', round(d['ms_per_step'],3), d.get('exact'), 'pointwise', round(d['stages_ms']['pointwise'],3))"
done
done

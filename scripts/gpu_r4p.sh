#!/bin/bash
# round 4, call P: tight k_pwss variants at C4 -- libmpfft_tight.so (two WGs per CU) vs
# libmpfft_tightz.so (+ the inner product's limbs through LDS), parity of tightz at l = 4096
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MPFFT_LIB=libmpfft_tightz.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "4096 or nested or fill_fold" > gpurun_out/pytest_tightz.log 2>&1 || { tail -40 gpurun_out/pytest_tightz.log; exit 1; }
tail -2 gpurun_out/pytest_tightz.log
for v in tight tightz tight tightz; do
  export MPFFT_LIB=libmpfft_$v.so
  timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/tightz_C4_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/tightz_C4_$v.log') if x.startswith('{')][-1]); print('C4 $v', round(d['ms_per_step'],2), d.get('exact'), 'pointwise', round(d['stages_ms']['pointwise'],2))"
done

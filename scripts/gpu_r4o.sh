#!/bin/bash
# round 4, call O: the tight k_pwss (K = 512 in 80 KiB of LDS, two workgroups per CU;
# libmpfft_tight.so, -DPW_TIGHT9=1) -- parity at l = 4096, then C4 A/B against the shipped one
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MPFFT_LIB=libmpfft_tight.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "4096 or nested or fill_fold" > gpurun_out/pytest_tight.log 2>&1 || { tail -40 gpurun_out/pytest_tight.log; exit 1; }
tail -2 gpurun_out/pytest_tight.log
for v in main tight main tight; do
  if [ $v = main ]; then unset MPFFT_LIB; else export MPFFT_LIB=libmpfft_tight.so; fi
  timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/tight_C4_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/tight_C4_$v.log') if x.startswith('{')][-1]); print('C4 $v', round(d['ms_per_step'],2), d.get('exact'), 'pointwise', round(d['stages_ms']['pointwise'],2))"
done

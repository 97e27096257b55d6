#!/bin/bash
# round 4, call R: tight k_pwss at C4 -- operand B loaded after A's transform (shipped build),
# + the product's limbs through LDS (libmpfft_zs.so), against HEAD a66a3cd (libmpfft_base.so:
# both operands loaded up front); parity of both new builds at l = 4096
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for L in "" libmpfft_zs.so; do
  MPFFT_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "4096 or nested or fill_fold" > gpurun_out/pytest_late_$L.log 2>&1 || { tail -30 gpurun_out/pytest_late_$L.log; exit 1; }
  tail -1 gpurun_out/pytest_late_$L.log
done
for v in main zs base main zs base; do
  if [ $v = main ]; then unset MPFFT_LIB; else export MPFFT_LIB=libmpfft_$v.so; fi
  timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/late_C4_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/late_C4_$v.log') if x.startswith('{')][-1]); print('C4 $v', round(d['ms_per_step'],2), d.get('exact'), 'pointwise', round(d['stages_ms']['pointwise'],2))"
done

#!/bin/bash
# round 4, call V: quad-fused rows with the inputs fetched two at a time -- parity (quad test,
# C4 digest through the C ABI), C4 A/B against MPFFT_NO_FUSE2 (diag library)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_c_abi.py -m gpu -x -q --timeout 300 --timeout-method thread -k "quad or c4 or north_star" > gpurun_out/pytest_quad2.log 2>&1 || { tail -30 gpurun_out/pytest_quad2.log; exit 1; }
tail -1 gpurun_out/pytest_quad2.log
for v in quad none quad none; do
  if [ $v = none ]; then export MPFFT_NO_FUSE2=1; else unset MPFFT_NO_FUSE2; fi
  MPFFT_LIB=diag timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/quad2_C4_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/quad2_C4_$v.log') if x.startswith('{')][-1]); print('C4 $v', round(d['ms_per_step'],2), d.get('exact'), {k: round(x,2) for k,x in d['stages_ms'].items()})"
done

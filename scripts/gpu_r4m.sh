#!/bin/bash
# round 4, call M: k_combine1 with per-wave window bookkeeping and batched window loads --
# parity, then A/B against the per-limb form (diag library, MPFFT_COMB_LIMB=1) and batch sizes
# (libmpfft_cb2 / _cb8: COMB_CB limbs per batch; the shipped one 4) at C3 and C4
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_multi_gpu.py tests/test_sharded_gpu.py tests/test_c_abi.py -m gpu > gpurun_out/pytest_comb.log 2>&1 || { tail -30 gpurun_out/pytest_comb.log; exit 1; }
tail -2 gpurun_out/pytest_comb.log
for c in C3 C4; do
  for v in cb4 limb cb2 cb8; do
    unset MPFFT_COMB_LIMB; L=diag
    [ $v = limb ] && export MPFFT_COMB_LIMB=1
    [ $v = cb2 ] && L=libmpfft_cb2.so
    [ $v = cb8 ] && L=libmpfft_cb8.so
    MPFFT_LIB=$L timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-twin > gpurun_out/comb_${c}_$v.log 2>&1 || exit 1
    python3 -c "
import json,sys
for line in open('gpurun_out/comb_${c}_$v.log'):
    if line.startswith('{'):
        d=json.loads(line); print('$c $v', round(d['ms_per_step'],3), d.get('exact'), 'combine', round(d['stages_ms']['combine'],3))"
  done
done

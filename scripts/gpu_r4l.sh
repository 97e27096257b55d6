#!/bin/bash
# round 4, call L: the l = 2048 split rule -- parity (new split tests, stage tests, C2/C3 vs
# GMP, sharded one-GPU cases) and the ref / alt sweep over truncation ratios
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_multi_gpu.py tests/test_sharded_gpu.py -m gpu > gpurun_out/pytest_split.log 2>&1 || { tail -30 gpurun_out/pytest_split.log; exit 1; }
tail -3 gpurun_out/pytest_split.log
for s in ref alt; do
  MPFFT_LIB=diag MPFFT_SPLIT=$s timeout -k 10 300 python3 scripts/split_sweep.py > gpurun_out/split_sweep_$s.log 2>&1 || exit 1
done
paste -d' ' gpurun_out/split_sweep_ref.log gpurun_out/split_sweep_alt.log | cut -c1-400

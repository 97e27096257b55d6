#!/bin/bash
# round 4, call J: four-level forward passes at l = 2048 with the 256 x 256 split (libmpfft_fwd4.so):
# exactness through that library, then A/B against the shipped one
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MPFFT_LIB=libmpfft_fwd4.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread \
  -k "stages_exact or c2_c3 or nested or random_sweep" > gpurun_out/r4j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4j_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_libab.sh fwd4 libmpfft_fwd4.so "C3 C2"

#!/bin/bash
# round 4, call I: the MFA split chosen by pass cost (C4: 512 x 512): exactness, then A/B vs HEAD
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py tests/test_multi_gpu.py tests/test_c_abi.py -m gpu -x -q --timeout 400 --timeout-method thread \
  -k "stages_exact or fill_fold or l4096 or c2_c3 or sharded or mul_multi or c4_north or nested or c_caller" > gpurun_out/r4i_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4i_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_libab.sh split libmpfft_base.so "C4 C3"

#!/bin/bash
# round 4, call G: split loads four slots at a time (k_rpass MODE 2): exactness, then A/B vs HEAD
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mul6.py tests/test_sharded_gpu.py tests/test_multi_gpu.py tests/test_c_abi.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "stages_exact or fill_fold or l4096 or c2_c3 or mul6 or sharded_world1 or mul_multi_one or random_sweep or nested or c4_north" > gpurun_out/r4g_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4g_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_libab.sh spl libmpfft_base.so "C3 C2 C4"

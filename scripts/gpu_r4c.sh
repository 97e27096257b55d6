#!/bin/bash
# round 4, call C: limb loads issued behind the mask loads (rp_codes_load): exactness, then A/B vs HEAD
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "stages_exact or fill_fold or l4096 or scale_canon or c4_north or mul6 or sharded_world1" > gpurun_out/r4c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4c_pytest.log; [ $rc -ne 0 ] && exit $rc
sed -i 's/MPFFT_LIB=$LIBB/MPFFT_LIB=$LIBB/' scripts/gpu_libab.sh
# a = HEAD (libmpfft_base.so), b = this tree: swap roles via the variable
bash scripts/gpu_libab.sh codes libmpfft_base.so "C3 C2 C4"

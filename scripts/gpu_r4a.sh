#!/bin/bash
# round 4, call A: new tests on the shipped library, the FILL mutant, the fwd1k A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "fill_fold or l4096_products or sharded or stages_exact or chooser or multi or c_caller" > gpurun_out/r4a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4a_pytest.log
[ $rc -ne 0 ] && exit $rc
MPFFT_LIB=$PWD/mpir-fft_amd/libmpfft_mutfill.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -v \
  --timeout 200 --timeout-method thread -k "fill_fold" > gpurun_out/r4a_mutant.log 2>&1
rc=$?; echo "mutant pytest rc=$rc (1 = the test caught the defect)"; tail -5 gpurun_out/r4a_mutant.log
[ $rc -ne 1 ] && exit 3
bash scripts/gpu_libab.sh fwd1k mpir-fft_amd/libmpfft_fwd1k.so "C3 C2 C4"

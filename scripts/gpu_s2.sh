#!/bin/bash
# sqrt2 top level at l = 2048 on four limbs per thread (512 threads) vs k_s2op<2> (MPFFT_S2_U2,
# diagnostic build): the mul6 GPU tests, then the mul6 timings under each.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mul6" > gpurun_out/pytest_$T.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/time_mul6.py gpurun_out/mul6_$T.json > gpurun_out/mul6_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_S2_U2=1 timeout -k 10 300 python3 -u scripts/time_mul6.py gpurun_out/mul6b_$T.json > gpurun_out/mul6b_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pytest_$T.log; head -1 gpurun_out/mul6_$T.log | cut -c1-400; head -1 gpurun_out/mul6b_$T.log | cut -c1-400
exit $rc

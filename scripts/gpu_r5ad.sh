#!/bin/bash
# Round 5, call AD: pointwise phase stamps (diag build) of one C3 and one C4 multiply.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5ad} && \
MPFFT_LIB=diag MPFFT_PW_STAMPS=1 timeout -k 10 200 python3 -u bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin > gpurun_out/pw_stamps_c3_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_PW_STAMPS=1 timeout -k 10 200 python3 -u bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin > gpurun_out/pw_stamps_c4_$T.log 2>&1
rc=$?; grep -h stamps gpurun_out/pw_stamps_c3_$T.log | head -4; grep -h stamps gpurun_out/pw_stamps_c4_$T.log | head -4; exit $rc

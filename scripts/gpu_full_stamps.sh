#!/bin/bash
# gpu_full.sh, then the per-pass phase stamps of one C3 multiply (diagnostic build).
cd $GRAFT_REPO_ROOT && T=${1:-x} && bash scripts/gpu_full.sh $T && \
MPFFT_LIB=diag MPFFT_RP_STAMPS=1 timeout -k 10 200 python3 -u bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/rp_stamps_$T.log 2>&1
rc=$?; grep rp_stamps gpurun_out/rp_stamps_$T.log | head -24; exit $rc

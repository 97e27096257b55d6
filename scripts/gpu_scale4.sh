#!/bin/bash
# C4 k_rscale with 1024-thread workgroups (MPFFT_SCALE_NT=1024, diagnostic build) vs the default
# 512, digest-checked; then the PMC records for C3 and C4.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
MPFFT_LIB=diag MPFFT_SCALE_NT=1024 timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "scale_canon" > gpurun_out/pytest_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_SCALE_NT=1024 timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4b_$T.log 2>&1 && \
bash scripts/gpu_pmc_all.sh C3 C4 > gpurun_out/pmc_all_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pytest_$T.log
for c in c4 c4b; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_${c}_$T.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" 2>/dev/null; done
exit $rc

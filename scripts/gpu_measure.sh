#!/bin/bash
# Measurements beside the headline: mul6 vs new_mpn_mul timings, single-GPU C4, and the
# k_pwss phase stamps at C3 (diagnostic build path, MPFFT_PW_STAMPS).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python3 -u scripts/time_mul6.py gpurun_out/mul6_timing.json > gpurun_out/mul6_timing.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_single.log 2>&1 && \
MPFFT_PW_STAMPS=1 timeout -k 10 200 python3 -u bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pw_stamps.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/mul6_timing.log | tail -5; tail -1 gpurun_out/bench_c4_single.log | cut -c1-600; grep pw_stamps gpurun_out/pw_stamps.log | head -3; exit $rc

#!/bin/bash
# Forward-pass change check: the stage / C-ABI GPU tests, then C4 (digest-checked) and C3 benches
# with stage times, each beside an A/B through the diagnostic build (MPFFT_LIB=diag):
# C4 with two-level passes at l = 4096 (MPFFT_RPLOGG=2), C3 without carried pending exponents.
# usage: scripts/gpu_c4.sh <tag> [pytest -k expression]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${2:-stages_exact or c_abi or nested_pointwise or scale_canon or c2_c3 or bench_configs}" > gpurun_out/pytest_$T.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_RPLOGG=2 timeout -k 10 400 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4b_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_NO_CARRY=1 timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3b_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for c in c4 c4b c3 c3b; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_${c}_$T.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" 2>/dev/null; done
exit $rc

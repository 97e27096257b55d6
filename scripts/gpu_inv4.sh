#!/bin/bash
# Four-level inverse passes at l = 2048: the stage / multiply GPU tests that reach them, then the
# C3 bench beside the three-level build (MPFFT_RPLOGG_INV=3, diagnostic build) and kernel stats.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stages_exact or c2_c3 or bench_configs or nested_pointwise or mul6 or sharded_world1" > gpurun_out/pytest_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_RPLOGG_INV=3 timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3b_$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$T -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/ks_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pytest_$T.log
for c in c3 c3b; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_${c}_$T.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" 2>/dev/null; done
python3 scripts/kstats.py gpurun_out/ks_$T 2>/dev/null | head -24
exit $rc

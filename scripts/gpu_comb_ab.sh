#!/bin/bash
# k_combine1 per-wave windows vs per-lane windows (MPFFT_COMB_LANE, diagnostic build): the
# multiply tests that reach the combine, C3 / C4 benches under each.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "random_sweep or adversarial or golden or c2_c3 or bench_configs or sharded_world1 or c4_north" > gpurun_out/pytest_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_COMB_LANE=1 timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3b_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1 && \
MPFFT_LIB=diag MPFFT_COMB_LANE=1 timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4b_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pytest_$T.log
for c in c3 c3b c4 c4b; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_${c}_$T.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" 2>/dev/null; done
exit $rc

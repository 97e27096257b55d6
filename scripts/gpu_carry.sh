#!/bin/bash
# A/B of the pending-exponent hand-overs between forward passes (MPFFT_CARRY_MASK, diagnostic
# build): C3 and C4 benches (digest-checked) for masks 6 (default), 7, 2, 0.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3_$T.log 2>&1 && \
for m in 7 2 0; do MPFFT_LIB=diag MPFFT_CARRY_MASK=$m timeout -k 10 200 python3 -u bench.py --config C3 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c3m${m}_$T.log 2>&1 || exit 1; done && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1 && \
for m in 7 2 0; do MPFFT_LIB=diag MPFFT_CARRY_MASK=$m timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4m${m}_$T.log 2>&1 || exit 1; done
rc=$?; echo "rc=$rc"
for c in c3 c3m7 c3m2 c3m0 c4 c4m7 c4m2 c4m0; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_${c}_$T.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call N: k_combine1 with consecutive limbs per thread (one coefficient walk per wave,
# 16-B pair loads, two funnel shifts per limb): whole GPU suite, then C3 / C4 / C2 benches with
# the new form and (diag build, MPFFT_COMB_CT=0) the per-limb form, interleaved.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5n} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_ct$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_COMB_CT=0 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_old$r.log 2>&1 && \
  timeout -k 10 300 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c2_ct$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_COMB_CT=0 timeout -k 10 300 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c2_old$r.log 2>&1 && \
  timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ab_${T}_c4_ct$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_COMB_CT=0 timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ab_${T}_c4_old$r.log 2>&1 || exit 1
done
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), s.get('combine'), s.get('scale'))" 2>/dev/null; done
exit $rc

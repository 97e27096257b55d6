#!/bin/bash
# Round 5, call P: k_combine1 consecutive form: per-lane 16-B pair loads (default) vs coalesced
# wave loads handed out through LDS (diag MPFFT_COMB_XP), 256 / 512 threads.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5p} && \
MPFFT_LIB=diag MPFFT_COMB_XP=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stages_exact or sweep or adversarial" --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -1 gpurun_out/pytest_$T.log && \
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 40 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_ct$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_COMB_XP=1 timeout -k 10 300 python3 -u bench.py --steps 40 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_xp$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_COMB_XP=1 MPFFT_COMB_NT=512 timeout -k 10 300 python3 -u bench.py --steps 40 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_xp512_$r.log 2>&1 && \
  timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ab_${T}_c4_ct$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_COMB_XP=1 timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ab_${T}_c4_xp$r.log 2>&1 || exit 1
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), s.get('combine'), s.get('scale'))" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call Q: k_combine1 consecutive form by default (coalesced wave loads handed out through
# LDS, 512-thread blocks): whole GPU suite, C1 / C2 / C3 / C4 benches, C3 against NT = 256.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5q} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -1 gpurun_out/pytest_$T.log && \
timeout -k 10 200 python3 -u bench.py --config C1 --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c1.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c2.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 40 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_COMB_NT=256 timeout -k 10 300 python3 -u bench.py --steps 40 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_nt256_$r.log 2>&1 || exit 1
done && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ab_${T}_c4.log 2>&1
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), s.get('combine'), s.get('scale'))" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call X: operand B loaded after A's transform at l = 2048 too (PW_LATE_B_ALL=1; lb: B's
# fixed levels 0 only, lb2: 0-1), against the shipped early load; C3 and C2.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5x} && \
for r in 1 2; do
  for v in base lb lb2; do
    if [ $v = base ]; then L=""; else L="$PWD/mpir-fft_amd/libmpfft_$v.so"; fi
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_${v}_$r.log 2>&1 && \
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c2_${v}_$r.log 2>&1 || exit 1
  done
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), 'pw', round(s.get('pointwise'),3))" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call AI: timing probe of the pointwise load phase at C3 (products wrong by design):
# operand B's quad loads skipped (nob), and also A's with one input in flight (nobq).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5ai} && \
for r in 1 2; do
  for v in base nob nobq; do
    if [ $v = base ]; then L=""; else L="$PWD/mpir-fft_amd/libmpfft_$v.so"; fi
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 --no-check > gpurun_out/ab_${T}_c3_${v}_$r.log 2>&1 || exit 1
  done
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), 'pw', round(s.get('pointwise'),3))" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call U: operand B's forward transform with fewer compile-time-rotation levels at l = 4096
# (its register peak: A's transformed limbs stay live) -- PW_FIXB = 2 (shipped), 1, 0; C4 pointwise.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5u} && \
for r in 1 2; do
  for v in base fixb1 fixb0; do
    if [ $v = base ]; then L=""; else L="$PWD/mpir-fft_amd/libmpfft_$v.so"; fi
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ab_${T}_c4_${v}_$r.log 2>&1 || exit 1
  done
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), 'pw', round(s.get('pointwise'),3))" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call AJ: C4 pointwise partner-word prefetch distance (PW_PD_TIGHT 16 shipped, 8, 12) now
# that the kernel has no scratch.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5aj} && \
for r in 1 2; do
  for v in base pdt8 pdt12; do
    if [ $v = base ]; then L=""; else L="$PWD/mpir-fft_amd/libmpfft_$v.so"; fi
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c4_${v}_$r.log 2>&1 || exit 1
  done
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), 'pw', round(s.get('pointwise'),3))" 2>/dev/null; done
exit $rc

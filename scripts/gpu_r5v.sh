#!/bin/bash
# Round 5, call V: the late operand-B quad loader with one input in flight (PW_LATE_INFL=1: the C4
# kernel without scratch) against two (shipped); C4 pointwise, parity of the variant's l = 4096 paths.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5v} && V=$PWD/mpir-fft_amd/libmpfft_infl1.so && \
MPFFT_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "4096 or quad or pointwise" --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -1 gpurun_out/pytest_$T.log && \
for r in 1 2; do
  for v in base infl1; do
    if [ $v = base ]; then L=""; else L=$V; fi
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ab_${T}_c4_${v}_$r.log 2>&1 || exit 1
  done
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), 'pw', round(s.get('pointwise'),3))" 2>/dev/null; done
exit $rc

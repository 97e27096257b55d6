#!/bin/bash
# Round 5, call AH: rp_rot_all (the general rotation after the inverse row DIT) with four rotated
# pair reads per fence (RP_ROT_INFL=4, variant rot4) against one: C3 / C4 inverse rows.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5ah} && \
MPFFT_LIB=$PWD/mpir-fft_amd/libmpfft_rot4.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stages or sweep or 4096" --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -1 gpurun_out/pytest_$T.log && \
for r in 1 2 3; do
  for v in base rot4; do
    if [ $v = base ]; then L=""; else L="$PWD/mpir-fft_amd/libmpfft_$v.so"; fi
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_${v}_$r.log 2>&1 || exit 1
  done
done && \
for v in base rot4; do
  if [ $v = base ]; then L=""; else L="$PWD/mpir-fft_amd/libmpfft_$v.so"; fi
  MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c4_${v}.log 2>&1 || exit 1
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), 'inv_rows', round(s.get('inv_rows'),3))" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call Z: the fused split's source loads batched (RP_SPLIT_BATCH slots in flight, clamped
# loads): the whole GPU suite with the shipped 4, then C3 / C4 / C2 with batches 1 / 4 / 8.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5z} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -1 gpurun_out/pytest_$T.log && \
for r in 1 2; do
  for v in base sb1 sb8; do
    if [ $v = base ]; then L=""; else L="$PWD/mpir-fft_amd/libmpfft_$v.so"; fi
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_${v}_$r.log 2>&1 && \
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c2_${v}_$r.log 2>&1 && \
    MPFFT_LIB=$L timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c4_${v}_$r.log 2>&1 || exit 1
  done
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), 'fwd_columns', round(s.get('fwd_columns'),3))" 2>/dev/null; done
exit $rc

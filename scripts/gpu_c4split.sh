#!/bin/bash
# Round 6: C4 (l = 4096) with twice the reference's columns (diag knob MPFFT_SPLIT=alt4) vs the reference split,
# re-measured after the live-group launches; exactness by the bench's golden digest.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && D=$GRAFT_REPO_ROOT/mpir-fft_amd/libmpfft_diag.so
rc=0
for rep in 1 2; do
  for sp in ref alt4; do
    MPFFT_LIB=$D MPFFT_SPLIT=$sp timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline \
      --e2e-reps 0 --no-twin > gpurun_out/c4s_${sp}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
echo "rc=$rc"
for f in gpurun_out/c4s_*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items() if k in ('fwd_columns','fwd_rows','pointwise','inv_rows','inv_columns','combine')})" 2>/dev/null || tail -n 3 $f; done
exit $rc

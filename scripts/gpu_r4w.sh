#!/bin/bash
# round 4, call W: C3 (256 x 256 split, four-level row passes 4 + 4) vs the last two row levels
# in k_pwss (6 row levels: 3 + 3), MPFFT_FORCE_FUSE2 in the diag library; exactness by digest
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in base quad base quad; do
  if [ $v = quad ]; then export MPFFT_FORCE_FUSE2=1; else unset MPFFT_FORCE_FUSE2; fi
  MPFFT_LIB=diag timeout -k 10 300 python3 bench.py --config C3 --steps 10 --warmup 2 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/q3_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/q3_$v.log') if x.startswith('{')][-1]); print('C3 $v', round(d['ms_per_step'],3), d.get('exact'), {k: round(x,3) for k,x in d['stages_ms'].items()})"
done

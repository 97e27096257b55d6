#!/bin/bash
# round 4, call U: the row DIF's last two levels fused into k_pwss (slot quads) at l = 4096 --
# whole GPU suite, then C4 A/B against the pair-less plan (MPFFT_NO_FUSE2, diag library)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_quad.log 2>&1 || { tail -40 gpurun_out/pytest_quad.log; exit 1; }
tail -2 gpurun_out/pytest_quad.log
for v in quad none quad none; do
  if [ $v = none ]; then export MPFFT_NO_FUSE2=1; else unset MPFFT_NO_FUSE2; fi
  MPFFT_LIB=diag timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/quad_C4_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/quad_C4_$v.log') if x.startswith('{')][-1]); print('C4 $v', round(d['ms_per_step'],2), d.get('exact'), {k: round(x,2) for k,x in d['stages_ms'].items()})"
done

#!/bin/bash
# round 4, call Q: the tight k_pwss as the default -- whole GPU suite, C4 A/B against the
# round-3 form (libmpfft_wide.so, -DPW_TIGHT9=0), C4 PMC passes and kernel statistics
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_tightdef.log 2>&1 || { tail -40 gpurun_out/pytest_tightdef.log; exit 1; }
tail -2 gpurun_out/pytest_tightdef.log
for v in main wide main wide; do
  if [ $v = main ]; then unset MPFFT_LIB; else export MPFFT_LIB=libmpfft_wide.so; fi
  timeout -k 10 300 python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/tw_C4_$v.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/tw_C4_$v.log') if x.startswith('{')][-1]); print('C4 $v', round(d['ms_per_step'],2), d.get('exact'), {k: round(x,2) for k,x in d['stages_ms'].items()})"
done
unset MPFFT_LIB
bash scripts/gpu_pmc_all.sh C4

#!/bin/bash
# A/B of an experiment build against the shipped library: the bench of each config, alternating
# a / b twice.  usage: scripts/gpu_libab.sh <tag> <variant .so path> "<configs>"   (e.g. "C3 C4")
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-ab} && LIBB=$2 && CFGS=${3:-C3}
rc=0
for c in $CFGS; do
  st=10; [ "$c" = C4 ] && st=3
  for rep in 1 2; do
    timeout -k 10 300 python3 -u bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline --e2e-reps 0 \
      > gpurun_out/ab_${T}_${c}_a$rep.log 2>&1 || { rc=$?; break 2; }
    MPFFT_LIB=$LIBB timeout -k 10 300 python3 -u bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline \
      --e2e-reps 0 > gpurun_out/ab_${T}_${c}_b$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null || tail -3 $f; done
exit $rc

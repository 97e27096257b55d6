#!/bin/bash
# Round 5, call AK: the MFA split at C2 (truncation case a) with the current kernels: the reference
# 128 x 512 (shipped) against 256 x 256 with the quad fusion (diag MPFFT_SPLIT=alt).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5ak} && \
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c2_base_$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_SPLIT=alt timeout -k 10 300 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c2_alt_$r.log 2>&1 || exit 1
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), {k: round(v,3) for k,v in s.items()})" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 5, call AG: the MFA split at C3 with the current kernels: 256 x 256 (shipped) against the
# reference 128 x 512 (diag MPFFT_SPLIT=ref).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5ag} && \
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_base_$r.log 2>&1 && \
  MPFFT_LIB=diag MPFFT_SPLIT=ref timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/ab_${T}_c3_ref_$r.log 2>&1 || exit 1
done
rc=$?; echo "rc=$rc"
for f in gpurun_out/ab_${T}_*.log; do python3 -c "import json; d=json.loads([x for x in open('$f') if x.startswith('{')][-1]); s=d.get('stages_ms') or {}; print('$f', round(d['ms_per_step'],3), d.get('exact'), {k: round(v,3) for k,v in s.items()})" 2>/dev/null; done
exit $rc

#!/bin/bash
# Round 6: C3 / C2 split and levels-per-pass choices re-measured after the live-group launches (libmpfft_diag.so
# knobs MPFFT_SPLIT=ref, MPFFT_RPLOGG=3): default 256 x 256 4+4 vs the reference 128 x 512 split vs 3-level passes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && D=$GRAFT_REPO_ROOT/mpir-fft_amd/libmpfft_diag.so
rc=0
run() {   # tag cfg env...
  local tag=$1 cfg=$2; shift 2
  env "$@" MPFFT_LIB=$D timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/rs_$tag.log 2>&1
}
for rep in 1 2; do
  run c3_def_$rep C3 X=0 || { rc=$?; break; }
  run c3_ref_$rep C3 MPFFT_SPLIT=ref || { rc=$?; break; }
  run c3_l3_$rep C3 MPFFT_RPLOGG=3 || { rc=$?; break; }
  run c3_refl3_$rep C3 MPFFT_SPLIT=ref MPFFT_RPLOGG=3 || { rc=$?; break; }
done
[ $rc = 0 ] && { run c2_def C2 X=0 && run c2_alt C2 MPFFT_SPLIT=alt && run c4_def C4 X=0 && run c4_l2 C4 MPFFT_RPLOGG=2 || rc=$?; }
echo "rc=$rc"
for f in gpurun_out/rs_*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items() if k in ('fwd_columns','fwd_rows','pointwise','inv_rows','inv_columns')})" 2>/dev/null || tail -n 2 $f; done
exit $rc

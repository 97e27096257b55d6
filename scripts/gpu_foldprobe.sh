#!/bin/bash
# Round 6: timing probes of k_combine_red (wrong products by design, A/B builds only): fp1 = no limb below the
# block (fold_limb), fp2 = no mask carries, fp4 = no A / B terms; against the shipped library, C3 x2 and C4.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/fp_$1.log 2>&1
}
for rep in 1 2; do
  for v in cur fp1 fp2 fp4; do
    so=$L/libmpfft.so; [ $v != cur ] && so=$L/libmpfft_$v.so
    run c3_${v}_$rep $so C3 10 || { rc=$?; break 2; }
  done
done
if [ $rc = 0 ]; then
  for v in cur fp1 fp2 fp4; do
    so=$L/libmpfft.so; [ $v != cur ] && so=$L/libmpfft_$v.so
    run c4_$v $so C4 3 || { rc=$?; break; }
  done
fi
echo "rc=$rc"
for f in gpurun_out/fp_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], 'combine', round(d['stages_ms']['combine'],3))" 2>/dev/null || tail -n 3 $f; done
exit $rc

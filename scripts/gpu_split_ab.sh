#!/bin/bash
# Round 6: the fused-split regression on one lease.  Libraries:
#   head    = round-5 HEAD (clamped loads for every slot and pair, 4 slots in flight)
#   r4split = e3f876c^ (the round-4 guarded per-slot loads)
#   new     = in-tree libmpfft.so (clamped loads, wave-uniform skip of zero slots and dead waves)
#   wsb1/2  = new with 1 / 2 slots in flight
# C3 x 2 interleaved for all, C4 once for head / r4split / new / wsb1; rocprof kernel stats of C3
# for head / r4split / new.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
run() {   # tag lib cfg steps
  MPFFT_LIB=$L/libmpfft_$2.so timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 > gpurun_out/sab_$1.log 2>&1
}
rc=0
for rep in 1 2; do
  for lib in head r4split new wsb1 wsb2; do
    run c3_${lib}_$rep $lib C3 10 || { rc=$?; break 2; }
  done
done
if [ $rc = 0 ]; then
  for lib in head r4split new wsb1; do run c4_${lib} $lib C4 3 || { rc=$?; break; }; done
fi
if [ $rc = 0 ]; then
  for lib in head r4split new; do
    MPFFT_LIB=$L/libmpfft_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/sab_prof_$lib -o c3 -- python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline \
      --no-check --e2e-reps 0 > gpurun_out/sab_prof_$lib.log 2>&1 || { rc=$?; break; }
  done
fi
echo "rc=$rc"
for f in gpurun_out/sab_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null || tail -3 $f; done
exit $rc

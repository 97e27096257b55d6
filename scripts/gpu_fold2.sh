#!/bin/bash
# Round 6: fold kernels -- tests, benches (base = no fold), kernel trace, and SQ counters of the
# combine kernels of both libraries (separate --pmc passes, C3 only: --no-twin).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fold.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/fold2_pytest.log 2>&1 || rc=$?
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/fold2_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_base_$rep $L/libmpfft_base.so C3 10 || { rc=$?; break; }
    run c3_fold_$rep $L/libmpfft.so C3 10 || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c4_fold $L/libmpfft.so C4 3 || rc=$?; }
for lib in base fold; do
  [ $rc = 0 ] || break
  so=$L/libmpfft.so; [ $lib = base ] && so=$L/libmpfft_base.so
  MPFFT_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fold2_prof_$lib -o c3 -- \
    python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin > gpurun_out/fold2_prof_$lib.log 2>&1 || { rc=$?; break; }
  MPFFT_LIB=$so timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/fold2_pmc_$lib -o c3 -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline \
    --no-check --e2e-reps 0 --no-twin > gpurun_out/fold2_pmc_$lib.log 2>&1 || { rc=$?; break; }
done
echo "rc=$rc"
for f in gpurun_out/fold2_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null || tail -n 3 $f; done
tail -n 3 gpurun_out/fold2_pytest.log
exit $rc

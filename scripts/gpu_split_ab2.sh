#!/bin/bash
# Round 6: fused-split A/B, second lease: new = wave-uniform skip + whole-operand loads without the
# slice address arithmetic; wsb1 = the same, one slot in flight; r4split = e3f876c^.  Then the
# multi-GPU tests (event graph changes) and the split-pass parity tests on the new library.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
run() {   # tag lib cfg steps
  MPFFT_LIB=$L/libmpfft_$2.so timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 > gpurun_out/sab2_$1.log 2>&1
}
rc=0
for rep in 1 2; do
  for lib in r4split new wsb1; do run c3_${lib}_$rep $lib C3 10 || { rc=$?; break 2; }; done
done
[ $rc = 0 ] && for lib in r4split new wsb1; do run c4_${lib} $lib C4 3 || { rc=$?; break; }; done
[ $rc = 0 ] && { MPFFT_LIB=$L/libmpfft_new.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/sab2_prof_new -o c3 -- python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline \
      --no-check --e2e-reps 0 > gpurun_out/sab2_prof_new.log 2>&1 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 900 python3 -u -m pytest tests/test_multi_gpu.py tests/test_c_abi.py -x -v --timeout 300 \
      --timeout-method thread > gpurun_out/sab2_pytest_multi.log 2>&1 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
      -k "stages_exact or c2_c3 or fill_fold or mfa_split or bench_configs" > gpurun_out/sab2_pytest_parity.log 2>&1 || rc=$?; }
echo "rc=$rc"
for f in gpurun_out/sab2_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null || tail -3 $f; done
tail -n 3 gpurun_out/sab2_pytest_multi.log gpurun_out/sab2_pytest_parity.log
exit $rc

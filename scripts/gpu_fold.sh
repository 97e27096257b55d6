#!/bin/bash
# Round 6: f4 fold (fold.hpp) -- its tests first, then base (HEAD without the fold) vs fold benches,
# kernel stats of the folded C3, and the parity subset that runs whole products.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fold.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/fold_pytest.log 2>&1 || rc=$?
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 > gpurun_out/fold_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_base_$rep $L/libmpfft_base.so C3 10 || { rc=$?; break; }
    run c3_fold_$rep $L/libmpfft.so C3 10 || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c2_base $L/libmpfft_base.so C2 10 && run c2_fold $L/libmpfft.so C2 10 && \
  run c4_base $L/libmpfft_base.so C4 3 && run c4_fold $L/libmpfft.so C4 3 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fold_prof -o c3 -- \
    python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/fold_prof.log 2>&1 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_c_abi.py -x -v --timeout 300 \
    --timeout-method thread -k "random_sweep or adversarial or golden or c2_c3 or bench_configs or fill_fold or mfa_split or quad or l4096 or caller or spill_branch" \
    > gpurun_out/fold_pytest_parity.log 2>&1 || rc=$?; }
echo "rc=$rc"
for f in gpurun_out/fold_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null || tail -n 3 $f; done
tail -n 5 gpurun_out/fold_pytest.log; tail -n 3 gpurun_out/fold_pytest_parity.log
exit $rc

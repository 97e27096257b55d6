#!/bin/bash
# Round 6: the inverse MFA twiddle + scaling on load in the column blocks' first passes (ltw) --
# tests first, then C3/C4 benches: base (no fold), diag lib with MPFFT_LTW=0 (fold, twiddle in the
# rows' last pass) and =1, the shipped lib; kernel stats of the shipped lib.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "fold or c2_c3 or bench_configs or golden or random_sweep or adversarial or fill_fold or mfa_split" \
  > gpurun_out/ltw_pytest.log 2>&1 || rc=$?
run() {   # tag lib cfg steps [env]
  env $5 MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/ltw_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_base_$rep $L/libmpfft_base.so C3 10 "" || { rc=$?; break; }
    run c3_noltw_$rep diag C3 10 MPFFT_LTW=0 || { rc=$?; break; }
    run c3_ltw_$rep diag C3 10 MPFFT_LTW=1 || { rc=$?; break; }
    run c3_cur_$rep $L/libmpfft.so C3 10 "" || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c4_noltw diag C4 3 MPFFT_LTW=0 && run c4_cur $L/libmpfft.so C4 3 "" && run c2_cur $L/libmpfft.so C2 10 "" || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ltw_prof -o c3 -- \
    python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/ltw_prof.log 2>&1 || rc=$?; }
echo "rc=$rc"
for f in gpurun_out/ltw_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null || tail -n 3 $f; done
tail -n 3 gpurun_out/ltw_pytest.log
exit $rc

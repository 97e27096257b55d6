#!/bin/bash
# Round 6: k_combine_red persistent (a resident-sized grid taking tickets, the next one requested under the
# current one's loads) against the previous library (libmpfft_prev.so): fold / parity subset, C3 x2 / C4 / C2, rocprof.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_parity.py tests/test_c_abi.py -x -q \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/pe_pytest.log 2>&1 || rc=$?
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/pe_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_old_$rep $L/libmpfft_prev.so C3 10 || { rc=$?; break; }
    run c3_new_$rep $L/libmpfft.so C3 10 || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c4_old $L/libmpfft_prev.so C4 3 && run c4_new $L/libmpfft.so C4 3 && run c2_old $L/libmpfft_prev.so C2 10 && run c2_new $L/libmpfft.so C2 10 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pe_prof -o c -- \
    python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/pe_prof.log 2>&1 || rc=$?; }
echo "rc=$rc"
tail -n 2 gpurun_out/pe_pytest.log
for f in gpurun_out/pe_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], 'combine', round(d['stages_ms']['combine'],3))" 2>/dev/null || tail -n 3 $f; done
[ $rc = 0 ] && python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/pe_prof/c_kernel_stats.csv")):
    if "cmeta" in r["Name"] or "combine_red" in r["Name"]:
        print(r["Name"][:30], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
exit $rc

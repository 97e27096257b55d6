#!/bin/bash
# Round 6: k_rpass persistent (a grid of the resident workgroup count, each workgroup looping over groups)
# against the previous library (libmpfft_prev.so): the whole GPU suite, C3 x2 / C4 / C2 / C1 / C0, rocprof at C3.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 900 python3 -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/rpp_pytest.log 2>&1 || rc=$?
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/rpp_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_old_$rep $L/libmpfft_prev.so C3 10 || { rc=$?; break; }
    run c3_new_$rep $L/libmpfft.so C3 10 || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c4_old $L/libmpfft_prev.so C4 3 && run c4_new $L/libmpfft.so C4 3 && run c2_old $L/libmpfft_prev.so C2 10 && run c2_new $L/libmpfft.so C2 10 || rc=$?; }
[ $rc = 0 ] && { run c1_old $L/libmpfft_prev.so C1 20 && run c1_new $L/libmpfft.so C1 20 && run c0_old $L/libmpfft_prev.so C0 20 && run c0_new $L/libmpfft.so C0 20 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rpp_prof -o c -- \
    python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/rpp_prof.log 2>&1 || rc=$?; }
echo "rc=$rc"
tail -n 2 gpurun_out/rpp_pytest.log
for f in gpurun_out/rpp_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], 'fwd_columns', round(d['stages_ms']['fwd_columns'],3))" 2>/dev/null || tail -n 3 $f; done
[ $rc = 0 ] && python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/rpp_prof/c_kernel_stats.csv")):
    if "k_rpass<" in r["Name"]:
        print(r["Name"][:30], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
exit $rc

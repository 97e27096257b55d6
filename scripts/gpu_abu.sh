#!/bin/bash
# Round 6: k_combine_red's A / B terms at a wave-uniform position (one lane, one limb, a uniform switch):
# fold + parity subset through the shipped library, then C3 x2 / C4 / C2 stage times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_parity.py tests/test_c_abi.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/abu_pytest.log 2>&1 || rc=$?
run() {   # tag cfg steps
  timeout -k 10 300 python3 -u bench.py --config $2 --steps $3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/abu_$1.log 2>&1
}
[ $rc = 0 ] && { run c3_1 C3 10 && run c3_2 C3 10 && run c4 C4 3 && run c2 C2 10 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abu_prof -o c -- \
    python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/abu_prof.log 2>&1 || rc=$?; }
echo "rc=$rc"
tail -n 2 gpurun_out/abu_pytest.log
for f in gpurun_out/abu_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" 2>/dev/null || tail -n 3 $f; done
[ $rc = 0 ] && python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/abu_prof/c_kernel_stats.csv")):
    if "combine_red" in r["Name"] or "cmeta" in r["Name"] or "k_rpass<4, 2, 0, 2>" in r["Name"]:
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
exit $rc

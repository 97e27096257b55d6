#!/bin/bash
# Round 6: timing probes (wrong products by design, A/B builds only) and the combine's one-pass A/B
# terms.  noh1 = k_pwss without the LDS round of its h = 1 levels (bounds what two pieces per thread
# could save); splitprobe = the split pass without its source loads.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -m gpu -k "fold or c2_c3 or golden or split" > gpurun_out/pr_pytest.log 2>&1 || rc=$?
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/pr_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_cur_$rep $L/libmpfft.so C3 10 || { rc=$?; break; }
    run c3_noh1_$rep $L/libmpfft_noh1.so C3 10 || { rc=$?; break; }
    run c3_sp_$rep $L/libmpfft_splitprobe.so C3 10 || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c4_cur $L/libmpfft.so C4 3 && run c4_noh1 $L/libmpfft_noh1.so C4 3 && run c4_sp $L/libmpfft_splitprobe.so C4 3 || rc=$?; }
for v in cur sp; do
  [ $rc = 0 ] || break
  so=$L/libmpfft.so; [ $v = sp ] && so=$L/libmpfft_splitprobe.so
  MPFFT_LIB=$so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pr_prof_$v -o c -- \
    python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/pr_prof_$v.log 2>&1 || rc=$?
done
echo "rc=$rc"
tail -n 2 gpurun_out/pr_pytest.log
for f in gpurun_out/pr_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})" 2>/dev/null || tail -n 3 $f; done
for v in cur sp; do python3 - $v <<'PY'
import csv,sys
v=sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/pr_prof_{v}/c_kernel_stats.csv")):
    if "k_rpass<4, 2, 0" in r["Name"] or "combine_red" in r["Name"] or "cmeta" in r["Name"]:
        print(v, r["Name"][:40], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
done
exit $rc

#!/bin/bash
# Round 6: the split pass's zero-partner skip (RP_SPLIT_ZSKIP, libmpfft.so) against
# the same sources without it (libmpfft_nozskip.so): parity through the shipped library, then C3 / C4
# benches alternating and rocprof kernel stats of both at C3.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_c_abi.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/zs_pytest.log 2>&1 || rc=$?
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/zs_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_nz_$rep $L/libmpfft_nozskip.so C3 10 || { rc=$?; break; }
    run c3_zs_$rep $L/libmpfft.so C3 10 || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c4_nz $L/libmpfft_nozskip.so C4 3 && run c4_zs $L/libmpfft.so C4 3 && run c2_nz $L/libmpfft_nozskip.so C2 10 && run c2_zs $L/libmpfft.so C2 10 || rc=$?; }
for v in nozskip zskip; do
  [ $rc = 0 ] || break
  so=$L/libmpfft.so; [ $v = nozskip ] && so=$L/libmpfft_nozskip.so
  MPFFT_LIB=$so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zs_prof_$v -o c -- \
    python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/zs_prof_$v.log 2>&1 || rc=$?
done
echo "rc=$rc"
tail -n 2 gpurun_out/zs_pytest.log
for f in gpurun_out/zs_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], 'fwd_columns', round(d['stages_ms']['fwd_columns'],3))" 2>/dev/null || tail -n 3 $f; done
for v in nozskip zskip; do grep -h "k_rpass<4, 2, 0, 2>\|k_rpass<3, 4, 0, 2>" gpurun_out/zs_prof_$v/*kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$v /"; done
exit $rc

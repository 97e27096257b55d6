#!/bin/bash
# A/B of pointwise kernel builds (mpir-fft_amd/lib_<tag>.so, untracked) on C3 and C4, then the
# C3 bench and the GPU suite on the default build.  usage: scripts/gpu_pwab.sh "<tags>" <run-tag>
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && R=${2:-ab} && : > gpurun_out/pwab_$R.log && \
for cfg in C3 C4; do for t in $1 default; do
  if [ $t = default ]; then L=""; else L=$PWD/mpir-fft_amd/lib_$t.so; fi
  MPFFT_LIB=$L timeout -k 10 240 python3 -u scripts/pw_time.py $cfg 5 >> gpurun_out/pwab_$R.log 2>&1 || exit 1
  echo "  ^ lib=$t" >> gpurun_out/pwab_$R.log
done; done && cat gpurun_out/pwab_$R.log && \
timeout -k 10 300 python3 -u bench.py --steps 10 --cpu-reps 1 --cpu-warmup 0 --e2e-reps 1 > gpurun_out/bench_$R.log 2>&1 && \
tail -c 1200 gpurun_out/bench_$R.log && \
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_$R.log 2>&1
rc=$?; echo "rc=$rc"; tail -4 gpurun_out/pytest_$R.log; exit $rc

#!/bin/bash
# round 4, call B: the FILL mutant check, the fwd1k A/B, the bench lines with their C4 twins
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
MPFFT_LIB=libmpfft_mutfill.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -v \
  --timeout 200 --timeout-method thread -k "fill_fold" > gpurun_out/r4b_mutant.log 2>&1
rc=$?; echo "mutant pytest rc=$rc (1 = the test caught the defect)"; tail -5 gpurun_out/r4b_mutant.log
grep -c "AssertionError" gpurun_out/r4b_mutant.log; grep -c "AttributeError\|ImportError" gpurun_out/r4b_mutant.log
[ $rc -ne 1 ] && exit 3
bash scripts/gpu_libab.sh fwd1k libmpfft_fwd1k.so "C3 C2 C4" || exit $?
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4b_bench.log 2>&1 || exit $?
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r4b_share2.log 2>&1
rc=$?; echo "share2 rc=$rc"; tail -c 3000 gpurun_out/r4b_share2.log; exit $rc

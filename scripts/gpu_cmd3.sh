cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; \
echo "pytest rc=$?" ; \
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_wave.log 2>&1 && \
MPFFT_WAVE=0 timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_nowave.log 2>&1 && \
MPFFT_WLOGG=2 timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_wlogg2.log 2>&1 && \
MPFFT_WLOGG=1 timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_wlogg1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof3.log 2>&1

cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; \
echo "pytest rc=$?" ; tail -3 gpurun_out/pytest_gpu.log; \
for ab in 0 2; do for lg in 1 2 3; do MPFFT_ABLATE=$ab MPFFT_WLOGG=$lg timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/ab_${ab}_${lg}.log 2>&1 || exit 1; done; done && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof5.log 2>&1

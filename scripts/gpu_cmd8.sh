cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; \
echo "pytest rc=$?" ; tail -3 gpurun_out/pytest_gpu.log; \
for lg in 3 4 5; do MPFFT_WLOGG=$lg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p8_${lg} -o c1 -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-check > gpurun_out/ab8_${lg}.log 2>&1 || exit 1; done && \
timeout -k 10 300 python3 -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench8_c2.log 2>&1

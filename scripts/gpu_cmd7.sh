cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stages or sweep" > gpurun_out/pytest_gpu.log 2>&1 ; \
echo "pytest rc=$?" ; tail -2 gpurun_out/pytest_gpu.log; \
for ab in 0 2; do for lg in 2 3; do MPFFT_ABLATE=$ab MPFFT_WLOGG=$lg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p7_${ab}_${lg} -o c1 -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-check > gpurun_out/ab7_${ab}_${lg}.log 2>&1 || exit 1; done; done; \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc7_sq -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/pmc7_sq.log 2>&1

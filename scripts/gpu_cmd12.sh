cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sweep or golden or adversarial or bench_configs" > gpurun_out/pytest_gpu.log 2>&1 ; \
rc=$?; echo "pytest rc=$rc" ; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; \
for ab in 0 1; do MPFFT_PWABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p12_$ab -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/p12_$ab.log 2>&1 || exit 1; done

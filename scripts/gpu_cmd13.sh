cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sweep or golden or adversarial or bench_configs or c2 or pointwise" > gpurun_out/pytest_gpu.log 2>&1 ; \
rc=$?; echo "pytest rc=$rc" ; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p13 -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/p13.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/b13_c2_def.log 2>&1 && \
MPFFT_PWM2_MAXL=4096 MPFFT_PWM2_D2=1 timeout -k 10 200 python3 -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/b13_c2_d2.log 2>&1 && \
MPFFT_PWM2_MAXL=4096 timeout -k 10 200 python3 -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/b13_c2_d4.log 2>&1

cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pointwise or stages or sweep or c2" > gpurun_out/pytest_gpu.log 2>&1 ; \
rc=$?; echo "pytest rc=$rc" ; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p11 -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/p11.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench11_c2.log 2>&1

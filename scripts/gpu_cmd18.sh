# Balanced pass level splits: full GPU suite, C1 bench, rocprof stats, C2 bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu18.log 2>&1 ; \
rc=$?; echo "pytest rc=$rc" ; tail -5 gpurun_out/pytest_gpu18.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; \
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 > gpurun_out/b18_c1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p18 -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/p18.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b18_c2.log 2>&1

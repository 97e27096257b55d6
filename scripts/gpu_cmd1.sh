cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1

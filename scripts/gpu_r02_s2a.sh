cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "pytest_gpu:900:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "bench:400:python3 -u bench.py" \
 "p_c3:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c3 -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check"

cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "pytest_gpu:900:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "bench:400:python3 -u bench.py" \
 "bench_sh:400:python3 -u bench.py --mode sharded --config C4 --steps 2 --warmup 1"

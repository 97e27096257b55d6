cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "b_c4:400:python3 -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --e2e-reps 0" \
 "b_c4_sh:400:python3 -u bench.py --mode sharded --config C4 --steps 2 --warmup 1" \
 "t_c4:600:python -u -m pytest tests/test_c_abi.py -x -q --timeout 500 --timeout-method thread -k c4"

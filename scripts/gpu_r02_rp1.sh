cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "t_stages:600:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k 'stages_exact'" \
 "t_c23:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'c2_c3 or golden or random_sweep'" \
 "b_c3:300:python3 bench.py --config C3 --steps 5 --warmup 2 --no-cpu-baseline --e2e-reps 0"

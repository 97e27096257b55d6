cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "t_stages:600:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'stages_exact or c2_c3 or golden'" \
 "b_c3:300:python3 bench.py --config C3 --steps 5 --warmup 2 --no-cpu-baseline --e2e-reps 0" \
 "b_c3_l2:300:MPFFT_BLOGG=2 python3 bench.py --config C3 --steps 5 --warmup 2 --no-cpu-baseline --e2e-reps 0" \
 "p_c3:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c3 -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0"

cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c3 -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/p_c3.log 2>&1

cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "b_c3:300:python3 -u bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check" \
 "p_c3:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c3 -o c3 -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-check" \
 "b_c4:400:python3 -u bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-check"

cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
MPFFT_RP_STAMPS=1 timeout -k 10 200 python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 2>&1 | grep stamps

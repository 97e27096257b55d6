cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "st_bp:200:MPFFT_BP_STAMPS=1 python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0" \
 "st_pw:200:MPFFT_PW_STAMPS=1 python3 bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0"

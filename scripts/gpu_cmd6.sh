cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
for ab in 2 3 4; do for lg in 1 3; do MPFFT_ABLATE=$ab MPFFT_WLOGG=$lg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p6_${ab}_${lg} -o c1 -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-check > gpurun_out/ab6_${ab}_${lg}.log 2>&1 || exit 1; done; done

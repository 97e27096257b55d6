cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
MPFFT_RPASS_OFF=6 timeout -k 10 120 python -u tests/dbg_rpass.py 8 512 140000 140000 cols

cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "t_big:300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'stages_exact and (1024 or 4096 or 256-4000)'" \
 "t_c23:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'c2_c3'" \
 "t_c4:400:python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu -k 'c4'" \
 "stamps:200:MPFFT_PW_STAMPS=1 python3 bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-check" \
 "b_c3:300:python3 bench.py --config C3 --steps 5 --warmup 2 --no-cpu-baseline"

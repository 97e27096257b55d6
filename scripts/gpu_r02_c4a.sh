cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
scripts/gpu_run.sh \
 "t_big:300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'stages_exact and (1024 or 4096 or 256-4000)'" \
 "t_c23:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'c2_c3'" \
 "st_c3:300:MPFFT_BP_STAMPS=1 python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check" \
 "p_c3:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c3g -o c3 -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-check" \
 "t_c4:600:python -u -m pytest tests/test_c_abi.py -x -q --timeout 500 --timeout-method thread -k 'c4'" \
 "b_c4:400:python3 -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-check"

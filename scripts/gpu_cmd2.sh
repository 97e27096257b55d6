# C2/C3/C4 timings + C1 PMC passes
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 200 python -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/bench_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/bench_c4.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/pmc_write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_sq -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/pmc_sq.log 2>&1

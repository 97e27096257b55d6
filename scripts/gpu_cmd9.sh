cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench9.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p9 -o c1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/p9.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc9_fetch -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/pmc9_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc9_write -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/pmc9_write.log 2>&1

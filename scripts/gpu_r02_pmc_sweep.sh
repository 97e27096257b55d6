cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 400 python3 -u scripts/chooser_sweep.py gpurun_out/chooser_sweep.json > gpurun_out/sweep.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o c3 -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc_f.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o c3 -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc_w.log 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/pmc_f gpurun_out/pmc_f.json > /dev/null && python3 scripts/pmc_summary.py gpurun_out/pmc_w gpurun_out/pmc_w.json > /dev/null && echo pmc-ok

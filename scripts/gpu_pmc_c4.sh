#!/bin/bash
# C4 (one GPU): kernel stats and FETCH/WRITE PMC passes (separate runs) -> profiles/pmc_C4.json
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c4 -o c4 -- python3 bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/p_c4.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc4_f -o c4 -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc4_f.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc4_w -o c4 -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc4_w.log 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/pmc4_f gpurun_out/pmc4_f.json > /dev/null && python3 scripts/pmc_summary.py gpurun_out/pmc4_w gpurun_out/pmc4_w.json > /dev/null
rc=$?; echo "rc=$rc"; exit $rc

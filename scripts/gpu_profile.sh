#!/bin/bash
# Evidence for profiles/: rocprofv3 kernel stats of the C3 bench, FETCH/WRITE PMC passes
# (separate runs), and the new_mpn_mul6 bench lines (C3 operands, test_mul4's shape).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_default.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_c3 -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/p_c3.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o c3 -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc_f.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o c3 -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc_w.log 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/pmc_f gpurun_out/pmc_f.json > /dev/null && python3 scripts/pmc_summary.py gpurun_out/pmc_w gpurun_out/pmc_w.json > /dev/null && \
timeout -k 10 200 python3 -u bench.py --mul6 --steps 5 > gpurun_out/bench_mul6_c3.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --mul6 --config M4 --steps 10 > gpurun_out/bench_mul6_m4.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/bench_mul6_c3.log | cut -c1-400; tail -1 gpurun_out/bench_mul6_m4.log | cut -c1-400; exit $rc

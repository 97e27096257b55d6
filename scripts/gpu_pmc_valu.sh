#!/bin/bash
# VALU issue counters of the C3 kernels (one --pmc pass of its own): SQ_INSTS_VALU, SQ_INSTS_LDS,
# SQ_WAVES, GRBM_GUI_ACTIVE -> VALU utilisation = 4 SQ_INSTS_VALU / (1024 SIMDs x cycles).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_v -o c3 -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc_v.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_vt -o c3 -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/pmc_vt.log 2>&1
rc=$?; echo "rc=$rc"; python3 scripts/pmc_summary.py gpurun_out/pmc_v gpurun_out/pmc_v.json > /dev/null; exit $rc

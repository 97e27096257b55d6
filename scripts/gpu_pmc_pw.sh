#!/bin/bash
# Limiter counters of the C3 kernels, the pointwise k_pwss first:
# counter list, then two SQ passes with GRBM_GUI_ACTIVE each (durations from a kernel-trace
# pass of the same command; clocks only ever derived inside one pass).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
B="python3 bench.py --config ${CFG:-C3} --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0" && \
(timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true) && \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sqa -o c -- $B > gpurun_out/pmc_sqa.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sqb -o c -- $B > gpurun_out/pmc_sqb.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_kt -o c -- $B > gpurun_out/pmc_kt.log 2>&1
rc=$?; echo "rc=$rc"
python3 scripts/pmc_summary.py gpurun_out/pmc_sqa gpurun_out/pmc_sqa.json > /dev/null 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmc_sqb gpurun_out/pmc_sqb.json > /dev/null 2>&1
grep -i -E "^(SQ_|GRBM_)|SQ_ACTIVE|SQ_WAIT|LDS" gpurun_out/counters_list.txt | head -80
exit $rc

#!/bin/bash
# Per-kernel counters for profiles/pmc_<CFG>.json: FETCH_SIZE, WRITE_SIZE and two SQ limiter sets,
# each in a rocprofv3 --pmc pass of its own over `bench.py --config <CFG> --steps 1 --warmup 0`.
# usage: scripts/gpu_pmc_all.sh C3 [C4 ...]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
for CFG in "$@"; do
  B="python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin"
  for P in "f:FETCH_SIZE" "w:WRITE_SIZE" \
           "sqa:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "sqb:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    t=${P%%:*}; c=${P#*:}
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${CFG}_$t -o c -- $B > gpurun_out/pmc_${CFG}_$t.log 2>&1 || exit 1
    python3 scripts/pmc_summary.py gpurun_out/pmc_${CFG}_$t gpurun_out/pmc_${CFG}_$t.json > /dev/null || exit 1
  done
  python3 scripts/pmc_merge.py $CFG gpurun_out/pmc_${CFG}_f.json gpurun_out/pmc_${CFG}_w.json gpurun_out/pmc_$CFG.json \
      gpurun_out/pmc_${CFG}_sqa.json gpurun_out/pmc_${CFG}_sqb.json || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$CFG -o c -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin > gpurun_out/ks_$CFG.log 2>&1 || exit 1
  echo "== $CFG"; python3 scripts/kstats.py gpurun_out/ks_$CFG 12
done

#!/bin/bash
# SQ limiter counters of the pointwise stage alone (scripts/pw_time.py) per MPFFT_POINTWISE kind.
# usage: scripts/gpu_pmc_pw.sh C3 "pwss pwss2"
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
CFG=${1:-C3}
for k in ${2:-pwss pwss2}; do
  for P in "sqa:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "sqb:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    t=${P%%:*}; c=${P#*:}; d=gpurun_out/pmcpw_${CFG}_${k}_$t
    MPFFT_POINTWISE=$k timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $d -o c -- python3 scripts/pw_time.py $CFG 1 > $d.log 2>&1 || exit 1
    python3 scripts/pmc_summary.py $d $d.json > /dev/null || exit 1
  done
done
python3 - "$CFG" ${2:-pwss pwss2} <<'PY'
import json, sys, glob
cfg = sys.argv[1]
for k in sys.argv[2:]:
    m = {}
    for t in ("sqa", "sqb"):
        for name, v in json.load(open(f"gpurun_out/pmcpw_{cfg}_{k}_{t}.json")).items():
            if "k_pw" in name:
                m.setdefault(name[:24], {}).update(v)
    for name, v in m.items():
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        print(k, name, {a: round(b) for a, b in sorted(v.items())})
        # the formulas of scripts/pmc_merge.py
        print("   valu_issue", round(2 * v["SQ_INSTS_VALU"] / (1024 * cyc), 3),
              "valu_cyc_est", round((2 * (v["SQ_INSTS_VALU"] - v["SQ_INSTS_VALU_INT64"]) + 8 * v["SQ_INSTS_VALU_INT64"]) / (1024 * cyc), 3),
              "lds_util", round(v["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 3),
              "waves/simd", round(4 * v["SQ_WAVE_CYCLES"] / (1024 * cyc), 2),
              "wait_inst", round(v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"], 3),
              "wait_any", round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 3),
              "bank_conf/idx", round(v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"]), 3),
              "dur_ms", round(v["duration_ns"] / 1e6, 3))
PY

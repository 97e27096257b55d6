#!/bin/bash
# Round 6: SQ counters of the combine kernels, k_combine1 (base library, no fold) vs k_cmeta +
# k_combine_red (shipped), C3 (separate --pmc passes, --no-twin: C3 only).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
for lib in base cur; do
  so=$L/libmpfft.so; [ $lib = base ] && so=$L/libmpfft_base.so
  for P in "sqa:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "sqb:SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "tcc:FETCH_SIZE GRBM_GUI_ACTIVE"; do
    t=${P%%:*}; c=${P#*:}; d=gpurun_out/cpmc_${lib}_$t
    MPFFT_LIB=$so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $d -o c -- python3 bench.py --config C3 --steps 1 \
      --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin > $d.log 2>&1 || { rc=$?; break 2; }
    python3 scripts/pmc_summary.py $d $d.json > /dev/null || { rc=$?; break 2; }
  done
done
echo "rc=$rc"
[ $rc = 0 ] && python3 - <<'PY'
import json
for lib in ("base", "cur"):
    m = {}
    for t in ("sqa", "sqb", "tcc"):
        for name, v in json.load(open(f"gpurun_out/cpmc_{lib}_{t}.json")).items():
            if "combine" in name or "cmeta" in name or "rscale" in name:
                m.setdefault(name[:32], {}).update(v)
    for name, v in m.items():
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        print(lib, name, "valu_issue", round(2 * v["SQ_INSTS_VALU"] / (1024 * cyc), 3),
              "waves/simd", round(4 * v["SQ_WAVE_CYCLES"] / (1024 * cyc), 2),
              "wait_inst", round(v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"], 3),
              "wait_any", round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 3),
              "insts_valu", round(v["SQ_INSTS_VALU"]), "insts_lds", round(v["SQ_INSTS_LDS"]),
              "insts_vmem", round(v.get("SQ_INSTS_VMEM", 0)), "insts_salu", round(v.get("SQ_INSTS_SALU", 0)),
              "fetch_MB", round(2 * 1024 * v.get("FETCH_SIZE", 0) / 1e6, 1), "dur_us", round(v["duration_ns"] / 1e3, 1))
PY
exit $rc

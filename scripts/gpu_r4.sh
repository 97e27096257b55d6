#!/bin/bash
# Round 6: k_pwss with two DIT levels per exchange (libmpfft_r4inv.so,
# -DPW_R4_INV=1) against the shipped library: pointwise parity through the variant, C3 / C2
# benches alternating, and the SQ limiter counters of the pointwise stage for both.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && L=$GRAFT_REPO_ROOT/mpir-fft_amd
rc=0
for v in r4inv r4both; do
  MPFFT_LIB=$L/libmpfft_$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 \
    --timeout-method thread -k "pointwise_direct or nested or c2_c3 or golden or quad" > gpurun_out/r4_pytest_$v.log 2>&1 || { rc=$?; break; }
done
run() {   # tag lib cfg steps
  MPFFT_LIB=$2 timeout -k 10 300 python3 -u bench.py --config $3 --steps $4 --warmup 1 \
    --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/r4_$1.log 2>&1
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    run c3_cur_$rep $L/libmpfft.so C3 10 || { rc=$?; break; }
    run c3_r4_$rep $L/libmpfft_r4inv.so C3 10 || { rc=$?; break; }
    run c3_r4b_$rep $L/libmpfft_r4both.so C3 10 || { rc=$?; break; }
  done
fi
[ $rc = 0 ] && { run c2_cur $L/libmpfft.so C2 10 && run c2_r4 $L/libmpfft_r4inv.so C2 10 && run c2_r4b $L/libmpfft_r4both.so C2 10 || rc=$?; }
for lib in cur r4 r4b; do
  [ $rc = 0 ] || break
  so=$L/libmpfft.so; [ $lib = r4 ] && so=$L/libmpfft_r4inv.so; [ $lib = r4b ] && so=$L/libmpfft_r4both.so
  for P in "sqa:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "sqb:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    t=${P%%:*}; c=${P#*:}; d=gpurun_out/r4pmc_${lib}_$t
    MPFFT_LIB=$so timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $d -o c -- python3 scripts/pw_time.py C3 1 > $d.log 2>&1 || { rc=$?; break 2; }
    python3 scripts/pmc_summary.py $d $d.json > /dev/null || { rc=$?; break 2; }
  done
done
echo "rc=$rc"
for f in gpurun_out/r4_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], 'pointwise', round(d['stages_ms']['pointwise'],3))" 2>/dev/null || tail -n 3 $f; done
tail -n 2 gpurun_out/r4_pytest_*.log
[ $rc = 0 ] && python3 - <<'PY'
import json
for lib in ("cur", "r4", "r4b"):
    m = {}
    for t in ("sqa", "sqb"):
        for name, v in json.load(open(f"gpurun_out/r4pmc_{lib}_{t}.json")).items():
            if "k_pw" in name:
                m.setdefault(name[:24], {}).update(v)
    for name, v in m.items():
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        print(lib, name, "valu_issue", round(2 * v["SQ_INSTS_VALU"] / (1024 * cyc), 3),
              "lds_util", round(v["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 3),
              "waves/simd", round(4 * v["SQ_WAVE_CYCLES"] / (1024 * cyc), 2),
              "wait_inst", round(v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"], 3),
              "insts_valu", round(v["SQ_INSTS_VALU"]), "insts_lds", round(v["SQ_INSTS_LDS"]),
              "dur_ms", round(v["duration_ns"] / 1e6, 3))
PY
exit $rc

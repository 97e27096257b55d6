#!/bin/bash
# Pointwise A/B (w1 vs np: product phase stubbed, timing only) and a third SQ counter pass on C3
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && : > gpurun_out/pwab_c.log && \
for t in np default; do
  if [ $t = default ]; then L=""; else L=$PWD/mpir-fft_amd/lib_$t.so; fi
  MPFFT_LIB=$L timeout -k 10 240 python3 -u scripts/pw_time.py C3 5 >> gpurun_out/pwab_c.log 2>&1 || exit 1
  echo "  ^ lib=$t" >> gpurun_out/pwab_c.log
done && cat gpurun_out/pwab_c.log && \
B="python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0" && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU2 SQ_IFETCH SQ_IFETCH_LEVEL SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sqc -o c -- $B > gpurun_out/pmc_sqc.log 2>&1
rc=$?; echo "rc=$rc"; python3 scripts/pmc_summary.py gpurun_out/pmc_sqc gpurun_out/pmc_sqc.json > /dev/null 2>&1
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_sqc.json'))
for k,v in d.items():
    if 'pwss' in k or 'rpass<3, 2, 0, 0>' in k: print(k[:40], {a: v[a] for a in sorted(v) if a.startswith(('SQ','GRBM','dur'))})
" 2>/dev/null; tail -3 gpurun_out/pmc_sqc.log; exit $rc

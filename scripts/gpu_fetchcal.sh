#!/bin/bash
# FETCH_SIZE calibration of the pointwise load pattern (tests/microbench/fetch_cal.hip)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetchcal -o c -- tests/microbench/fetch_cal > gpurun_out/fetchcal.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob('gpurun_out/fetchcal/**/*counter_collection.csv', recursive=True):
    rows += list(csv.DictReader(open(f)))
tot = {}
for r in rows:
    k = r.get('Kernel_Name') or r.get('Kernel-Name') or r.get('KernelName')
    v = float(r.get('Counter_Value') or r.get('Counter-Value') or 0)
    tot[k] = tot.get(k, 0.0) + v
B = 2 << 30
for k, v in tot.items():
    print(f"{k[:40]:40s} FETCH_SIZE x 1024 = {v * 1024:.4e} B, true {B:.4e} B, correction x{B / (v * 1024):.3f}")
PY

#!/bin/bash
# Round 6: combine / cmeta tuning -- fold tests, C3 x2 / C2 / C4 benches, C3 kernel trace, and the
# combine kernels' SQ counters.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
rc=0
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "fold or c2_c3 or bench_configs or golden or adversarial" > gpurun_out/f3_pytest.log 2>&1 || rc=$?
run() { timeout -k 10 300 python3 -u bench.py --config $2 --steps $3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin \
  > gpurun_out/f3_$1.log 2>&1; }
[ $rc = 0 ] && { run c3_1 C3 10 && run c3_2 C3 10 && run c2 C2 10 && run c4 C4 3 || rc=$?; }
[ $rc = 0 ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f3_prof -o c3 -- \
    python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin > gpurun_out/f3_prof.log 2>&1 || rc=$?; }
[ $rc = 0 ] && { timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/f3_pmc -o c -- python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-check \
    --e2e-reps 0 --no-twin > gpurun_out/f3_pmc.log 2>&1 && python3 scripts/pmc_summary.py gpurun_out/f3_pmc gpurun_out/f3_pmc.json > /dev/null || rc=$?; }
echo "rc=$rc"
for f in gpurun_out/f3_c*.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), d['exact'], {k: round(v,3) for k,v in d['stages_ms'].items()})" 2>/dev/null || tail -n 3 $f; done
tail -n 2 gpurun_out/f3_pytest.log
[ $rc = 0 ] && python3 - <<'PY'
import json, csv, collections
d = collections.defaultdict(list)
for x in csv.DictReader(open('gpurun_out/f3_prof/c3_kernel_trace.csv')):
    n = x['Kernel_Name']
    if 'cmeta' in n or 'combine' in n: d[n[:40]].append((int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1000)
for k, v in d.items(): print(k, [round(t) for t in v])
for name, v in json.load(open('gpurun_out/f3_pmc.json')).items():
    if 'combine' in name or 'cmeta' in name:
        cyc = v['GRBM_GUI_ACTIVE'] / 8
        print(name[:40], 'insts_valu', round(v['SQ_INSTS_VALU']), 'valu_issue', round(2 * v['SQ_INSTS_VALU'] / (1024 * cyc), 3),
              'wait_any', round(v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES'], 3), 'dur_us', round(v['duration_ns'] / 1e3, 1))
PY
exit $rc

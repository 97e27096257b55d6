#!/bin/bash
# Round-6 validation, part A: the whole GPU suite, smoke(), the driver's default bench line (C3 +
# cpu_baseline incl. ncore + C4 twin + e2e), C1 / C2 / C4 lines.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r6} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 && \
timeout -k 10 700 python3 -u bench.py > gpurun_out/bench_default_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C1 --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/bench_c1_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/bench_c2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 1 --no-twin > gpurun_out/bench_c4_$T.log 2>&1
rc=$?; echo "rc=$rc"
for c in default c1 c2 c4; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), {k: round(x,3) for k,x in (d.get('stages_ms') or {}).items()})" 2>/dev/null; done
exit $rc

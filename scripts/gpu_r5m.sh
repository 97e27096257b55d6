#!/bin/bash
# Round 5, call M: the forward transforms' first level with its compile-time rotation (E = N'/2):
# pointwise parity tests, the pointwise stage alone at C3 / C4 (twice), C3 / C4 benches.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5m} && \
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
for c in C3 C4 C3 C4; do timeout -k 10 120 python3 -u scripts/pw_time.py $c 10 2>/dev/null || exit 1; done && \
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/bench_c3_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin > gpurun_out/bench_c4_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for c in c3 c4; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), {k: round(x,3) for k,x in (d.get('stages_ms') or {}).items()})" 2>/dev/null; done
exit $rc

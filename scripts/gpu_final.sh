#!/bin/bash
# Round-end validation on one MI355X: the whole GPU suite, every BASELINE config's bench
# (C1, C2, C3 headline, C4; digest-checked), world-1 sharded C4, mul6 timings, C3 kernel stats.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-x} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C1 --steps 20 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c1_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c2_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C3 --steps 20 --no-cpu-baseline --e2e-reps 2 > gpurun_out/bench_c3_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --mode sharded --config C4 --steps 2 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4s_$T.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/time_mul6.py gpurun_out/mul6_$T.json > gpurun_out/mul6_$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$T -o c3 -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-check --e2e-reps 0 > gpurun_out/ks_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pytest_$T.log
for c in c1 c2 c3 c4 c4s; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_${c}_$T.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), {k: round(x,3) for k,x in (d.get('stages_ms') or d.get('phases_ms') or {}).items()})" 2>/dev/null; done
tail -4 gpurun_out/mul6_$T.log
exit $rc

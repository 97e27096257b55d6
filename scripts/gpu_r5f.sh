#!/bin/bash
# Round 5, call F: the pointwise product's limbs staged in LDS (no Z registers beside the
# digits): GPU parity tests, C3 and C4 benches with stage times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5f} && \
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mul6.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/bench_c3_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for c in c3 c4; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), {k: round(x,3) for k,x in (d.get('stages_ms') or {}).items()})" 2>/dev/null; done
exit $rc

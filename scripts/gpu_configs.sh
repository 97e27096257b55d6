#!/bin/bash
# The other BASELINE configurations on one MI355X (C1, C2, C4), default bench settings otherwise.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 200 python3 -u bench.py --config C1 --steps 20 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c1.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c2.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "rc=$rc"
for c in c1 c2 c4; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d['exact'], {k: round(x,3) for k,x in d['stages_ms'].items()})"; done
exit $rc

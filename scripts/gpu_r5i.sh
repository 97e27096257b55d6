#!/bin/bash
# Round 5, call I: replicated forward columns computed for the rank's own rows only (DIF
# subtrees skipped after the first column pass): multi / sharded GPU tests, the C entry at
# C4 with 2 ranks on one device (device-resident time; round-5 baseline 109 ms).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5i} && \
timeout -k 10 900 python3 -u -m pytest tests/test_multi_gpu.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 2 --multi-share --steps 3 --warmup 1 --e2e-reps 1 > gpurun_out/bench_multi2_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_multi2_$T.log') if x.startswith('{')][-1]); print('multi2', round(d['ms_per_step'],3), d.get('exact'), d.get('host_pointer_ms'))"
exit $rc

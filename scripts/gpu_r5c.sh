#!/bin/bash
# Round 5, call C: the host-pointer multi-GPU entry with whole-operand H2D (replicated columns)
# and one pinned D2H per rank; the out-of-place pass ceiling (tests/microbench/pass_bw.hip).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5c} && \
timeout -k 10 600 python3 -u -m pytest tests/test_multi_gpu.py tests/test_c_abi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 2 --multi-share --steps 3 --warmup 1 --e2e-reps 2 > gpurun_out/bench_multi2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 8 --multi-share --steps 3 --warmup 1 --e2e-reps 2 > gpurun_out/bench_multi8_$T.log 2>&1 && \
timeout -k 10 120 tests/microbench/pass_bw > gpurun_out/pass_bw_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for c in multi2 multi8; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), d.get('host_pointer_ms'), d.get('host_pack_ms_python'))" 2>/dev/null; done
cat gpurun_out/pass_bw_$T.log
exit $rc

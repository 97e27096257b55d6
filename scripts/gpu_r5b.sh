#!/bin/bash
# Round 5, call B: the striped column-layout combine (exchange #3 removed) -- multi-GPU, sharded
# and C-ABI GPU tests, the default bench line, the C entry rehearsed on one device at C4 with 2
# and 8 ranks (device-resident and host-pointer times), the two-rank sharded rehearsal.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5b} && \
timeout -k 10 900 python3 -u -m pytest tests/test_multi_gpu.py tests/test_sharded_gpu.py tests/test_c_abi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-twin > gpurun_out/bench_default_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 2 --multi-share --steps 3 --warmup 1 --e2e-reps 1 > gpurun_out/bench_multi2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 8 --multi-share --steps 3 --warmup 1 --e2e-reps 1 > gpurun_out/bench_multi8_$T.log 2>&1 && \
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_$T.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$T.log
for c in default multi2 multi8 share2; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), d.get('host_pointer_ms'), {k: round(x,3) for k,x in (d.get('stages_ms') or d.get('phases_ms') or {}).items()}, d.get('c_entry'))" 2>/dev/null; done
exit $rc

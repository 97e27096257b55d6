#!/bin/bash
# Round 5, call AA: the two-rank share rehearsal, normal and with the sharded run failing on purpose
# (rank 0 falls back to the C entry's line).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5aa} && \
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_$T.log 2>&1 && \
MPFFT_BENCH_SHARE_GPU=1 MPFFT_BENCH_FAIL_SHARDED=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_fail_$T.log 2>&1
rc=$?; echo "rc=$rc"
for f in share2 share2_fail; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${f}_$T.log') if x.startswith('{')][-1]); print('$f', d.get('ms_per_step'), d.get('value'), d.get('exact'), d.get('sharded_error'), (d.get('c_entry') or {}).get('ms_per_step'), d.get('n1_twin', {}) and d['n1_twin'].get('ms_per_step'))"; done
exit $rc

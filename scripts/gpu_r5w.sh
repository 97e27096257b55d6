#!/bin/bash
# Round 5, call W: the two-rank share rehearsal with rank 0's C-entry sub-record from a child process.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5w} && \
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_$T.log 2>&1
rc=$?; echo "rc=$rc"
python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_share2_$T.log') if x.startswith('{')][-1]); print(round(d['ms_per_step'],3), d.get('exact'), json.dumps(d.get('c_entry'))[:600])"
exit $rc

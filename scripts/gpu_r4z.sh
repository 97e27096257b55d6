#!/bin/bash
# round 4, call Z4: the chunked row phase after the desc fix -- sharded + multi GPU tests, the
# two-rank bench rehearsal
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_sharded_gpu.py tests/test_multi_gpu.py tests/test_c_abi.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_chunk.log 2>&1 || { tail -40 gpurun_out/pytest_chunk.log; exit 1; }
tail -2 gpurun_out/pytest_chunk.log
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_chunk.log 2>&1 || { tail -30 gpurun_out/bench_share2_chunk.log; exit 1; }
python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/bench_share2_chunk.log') if x.startswith('{')][-1]); print('share2', round(d['ms_per_step'],1), d.get('exact'), {k: round(v,1) for k,v in d['phases_ms'].items()})"

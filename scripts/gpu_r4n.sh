#!/bin/bash
# round 4, call N: exchange #1 overlapping operand 2's column passes (C entry and sharded.py),
# the l = 2048 small-depth case-b split tests, mfma at l = 2048 case b; the share rehearsal
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multi_gpu.py tests/test_sharded_gpu.py tests/test_c_abi.py tests/test_gpu_parity.py -m gpu -k "multi or sharded or c_abi or c_caller or mfa_split or every_pointwise or stages_exact" > gpurun_out/pytest_xover.log 2>&1 || { tail -40 gpurun_out/pytest_xover.log; exit 1; }
tail -2 gpurun_out/pytest_xover.log
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_xover.log 2>&1 || { tail -30 gpurun_out/bench_share2_xover.log; exit 1; }
python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/bench_share2_xover.log') if x.startswith('{')][-1]); print('share2', round(d['ms_per_step'],1), d.get('exact'), {k: round(v,1) for k,v in d['phases_ms'].items()})"

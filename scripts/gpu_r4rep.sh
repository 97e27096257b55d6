#!/bin/bash
# replicated forward columns at world 2: parity (ranks sharing one GPU) and the share2 rehearsal
T=${1:-r4rep}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_sharded_gpu.py -k "ranks_one_gpu" > gpurun_out/pytest_rep_$T.log 2>&1 && \
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_$T.log 2>&1 && \
MPFFT_BENCH_SHARE_GPU=1 MPFFT_REPLICATE_COLUMNS=0 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_norep_$T.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_rep_$T.log
for c in share2 share2_norep; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), d.get('exact'), {k: round(x,3) for k,x in (d.get('phases_ms') or {}).items()})" 2>/dev/null; done
exit $rc

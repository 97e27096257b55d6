#!/bin/bash
# Round-6 validation, part B: world-1 sharded C4, the two-rank share rehearsal (gloo + the C entry
# sub-record), the C entry alone at 2 and 8 ranks on device 0, mul6; PMC passes + kernel stats of C3, C4.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r6} && \
timeout -k 10 400 python3 -u bench.py --mode sharded --config C4 --steps 2 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin --no-c-entry > gpurun_out/bench_c4s_$T.log 2>&1 && \
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 2 --multi-share --steps 3 --warmup 1 --e2e-reps 1 > gpurun_out/bench_multi2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 8 --multi-share --steps 3 --warmup 1 --e2e-reps 1 > gpurun_out/bench_multi8_$T.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/time_mul6.py gpurun_out/mul6_$T.json > gpurun_out/mul6_$T.log 2>&1 && \
bash scripts/gpu_pmc_all.sh C3 C4 > gpurun_out/pmc_all_$T.log 2>&1
rc=$?; echo "rc=$rc"
for c in c4s share2 multi2 multi8; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), {k: round(x,3) for k,x in (d.get('stages_ms') or d.get('phases_ms') or {}).items()})" 2>/dev/null; done
tail -4 gpurun_out/mul6_$T.log; tail -30 gpurun_out/pmc_all_$T.log
exit $rc

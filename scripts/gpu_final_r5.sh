#!/bin/bash
# Round-5 validation on one MI355X: the whole GPU suite, smoke(), the driver's default bench line
# (C3 + cpu_baseline + C4 twin), C1 / C2 / C4 lines, world-1 sharded C4, the two-rank share
# rehearsal (gloo + the C entry sub-record), the C entry alone at 2 and 8 ranks on device 0.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && T=${1:-r5} && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 && \
tail -2 gpurun_out/pytest_$T.log && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 && \
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_default_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C1 --steps 20 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/bench_c1_$T.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --config C2 --steps 10 --no-cpu-baseline --no-twin --e2e-reps 0 > gpurun_out/bench_c2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 1 --no-twin > gpurun_out/bench_c4_$T.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --mode sharded --config C4 --steps 2 --warmup 1 --no-cpu-baseline --e2e-reps 0 --no-twin --no-c-entry > gpurun_out/bench_c4s_$T.log 2>&1 && \
MPFFT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_share2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 2 --multi-share --steps 3 --warmup 1 --e2e-reps 1 > gpurun_out/bench_multi2_$T.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --mode multi --config C4 --multi-ranks 8 --multi-share --steps 3 --warmup 1 --e2e-reps 1 > gpurun_out/bench_multi8_$T.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/time_mul6.py gpurun_out/mul6_$T.json > gpurun_out/mul6_$T.log 2>&1
rc=$?; echo "rc=$rc"
for c in default c1 c2 c4 c4s share2 multi2 multi8; do python3 -c "import json; d=json.loads([x for x in open('gpurun_out/bench_${c}_$T.log') if x.startswith('{')][-1]); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], d.get('exact'), {k: round(x,3) for k,x in (d.get('stages_ms') or d.get('phases_ms') or {}).items()})" 2>/dev/null; done
tail -4 gpurun_out/mul6_$T.log
exit $rc

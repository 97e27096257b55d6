#!/bin/bash
# round 4, call T: rocprofv3 kernel statistics of the driver's bench command itself (N = 1:
# C3 + the C4 twin), to set beside the line's roofline.avg_ms for k_pwss
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_default -o c -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ks_default.log 2>&1 || { tail -20 gpurun_out/ks_default.log; exit 1; }
grep '^{' gpurun_out/ks_default.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); r=d['roofline']; print('bench', round(d['ms_per_step'],3), r['kernel'], 'avg_ms', round(r['avg_ms'],4), 'frac', round(r['frac'],4))"
python3 scripts/kstats.py gpurun_out/ks_default 8

#!/bin/bash
# Round 6: the driver's round-end sequence on the final tree: the GPU suite, smoke(), then the N = 1 bench
# exactly as the driver runs it (python3 bench.py --gpus 1 --steps 20 --warmup 5).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/rehearsal_pytest.log 2>&1 && \
tail -1 gpurun_out/rehearsal_pytest.log && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rehearsal_smoke.log 2>&1 && \
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rehearsal_bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/rehearsal_smoke.log
python3 -c "import json; d=json.loads([x for x in open('gpurun_out/rehearsal_bench.log') if x.startswith('{')][-1]); print(round(d['ms_per_step'],3), '%.4g' % d['value'], d['exact'], d['roofline']['frac'], d['c4_single']['ms_per_step'])"
exit $rc

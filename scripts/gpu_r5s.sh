#!/bin/bash
# Round 5, call S: where C4's k_pwss traffic comes from -- FETCH_SIZE / WRITE_SIZE of the pointwise
# with the quad row fusion (default) and without it (diag MPFFT_NO_FUSE2: k_pwss<20,9,0>, one slot per WG).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out || exit 1
B="python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-check --e2e-reps 0 --no-twin"
for v in fuse2 nofuse2; do
  for P in "f:FETCH_SIZE" "w:WRITE_SIZE"; do
    t=${P%%:*}; c=${P#*:}
    if [ $v = nofuse2 ]; then export MPFFT_LIB=diag MPFFT_NO_FUSE2=1; fi
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcx_${v}_$t -o c -- $B > gpurun_out/pmcx_${v}_$t.log 2>&1 || exit 1
    python3 scripts/pmc_summary.py gpurun_out/pmcx_${v}_$t gpurun_out/pmcx_${v}_$t.json > /dev/null || exit 1
  done
done
python3 - <<'PY'
import json
for v in ("fuse2", "nofuse2"):
    f = json.load(open(f"gpurun_out/pmcx_{v}_f.json")); w = json.load(open(f"gpurun_out/pmcx_{v}_w.json"))
    for k in f:
        if "pwss" in k or "rpass<3, 4, 0, 1>" in k or "rpass<2, 4, 0, 1>" in k:
            print(v, k[:34], json.dumps(f[k])[:300], json.dumps(w.get(k, {}))[:200])
PY

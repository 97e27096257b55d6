#!/bin/bash
# Round 6: the l = 2048 MFA split re-swept after the live-group launches (scripts/split_sweep.py, diag library):
# reference split vs the doubled-column split over truncation ratios, alternating twice.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && D=$GRAFT_REPO_ROOT/mpir-fft_amd/libmpfft_diag.so
rc=0
for rep in 1 2; do
  for sp in ref alt; do
    MPFFT_LIB=$D MPFFT_SPLIT=$sp timeout -k 10 300 python3 -u scripts/split_sweep.py > gpurun_out/ss2_${sp}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
echo "rc=$rc"
python3 - <<'PY'
import json, glob, collections
t = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ss2_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); t[(d["depth"], d["w"], d["n"], d["ratio"], d["split"])].append(d["ms"])
keys = sorted({k[:4] for k in t})
for k in keys:
    r, a = min(t.get(k + ("ref",), [0])), min(t.get(k + ("alt",), [0]))
    print(k, "ref", r, "alt", a, "alt/ref", round(a / r, 3) if r else None)
PY
exit $rc

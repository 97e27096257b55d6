#!/bin/bash
# Run GPU steps on the box; stop at the first crash/timeout (never retry).
# usage: scripts/gpu_run.sh "<label>:<seconds>:<command>" ...
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $label (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$label.log" 2>&1
  rc=$?
  echo "=== $label rc=$rc"; tail -5 "$OUT/$label.log"
  case $rc in
    0|1|2|5) ;;                       # ok, test failures, usage errors: keep going
    *) echo "=== stopping after $label (rc=$rc)"; exit $rc ;;
  esac
done

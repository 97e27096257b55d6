#!/usr/bin/env python3
"""Merge the FETCH_SIZE and WRITE_SIZE pass summaries (pmc_summary.py outputs) into the
per-kernel HBM bytes file bench.py reads (profiles/pmc_<config>.json).
usage: pmc_merge.py <config> <fetch.json> <write.json> <out.json>"""
import json
import sys

cfg, fj, wj, out = sys.argv[1:5]
f, w = json.load(open(fj)), json.load(open(wj))
kern = {}
for k in sorted(set(f) | set(w)):
    rd = f.get(k, {}).get("hbm_read_bytes_corrected")
    wr = w.get(k, {}).get("hbm_write_bytes")
    rec = {"dispatches": f.get(k, w.get(k, {})).get("dispatches")}
    if rd is not None:
        rec["hbm_read_bytes_per_launch"] = rd
    if wr is not None:
        rec["hbm_write_bytes_per_launch"] = wr
    if rd is not None and wr is not None:
        rec["hbm_bytes_per_launch"] = rd + wr
    kern[k] = rec
json.dump({"config": cfg,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over `bench.py --config "
                     f"{cfg} --steps 1 --warmup 0`; read = 2*1024*FETCH_SIZE (gfx950 half-count correction for "
                     "16-byte streaming loads, MI355X_MICROARCH.md HBM), write = 1024*WRITE_SIZE; per dispatch averages",
           "source": f"{fj}, {wj}", "kernels": kern}, open(out, "w"), indent=1)

#!/usr/bin/env python3
"""Per-kernel average of rocprofv3 --pmc counters (counter_collection.csv).
usage: pmc_summary.py <dir-with-csv> [out.json]
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced read (MI355X_MICROARCH.md "HBM"), so hbm_read_bytes = 2 * 1024 * FETCH_SIZE.
duration_ns: the dispatch's own start/end stamps in the same (profiled) pass."""
import collections
import csv
import glob
import json
import os
import sys

files = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for fn in files:
    with open(fn) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (fn, r["Dispatch_Id"])
            if key not in disp[k] and r.get("End_Timestamp"):
                acc[k]["duration_ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            disp[k].add(key)
out = {}
for k, cs in acc.items():
    n = len(disp[k])
    d = {c: v / n for c, v in cs.items()}
    d["dispatches"] = n
    if "FETCH_SIZE" in d:
        d["hbm_read_bytes_corrected"] = 2 * 1024 * d["FETCH_SIZE"]
    if "WRITE_SIZE" in d:
        d["hbm_write_bytes"] = 1024 * d["WRITE_SIZE"]
    out[k] = d
s = json.dumps(out, indent=1, sort_keys=True)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(s)
print(s)

#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel_stats.csv compactly: calls, average us, share.
usage: kstats.py <dir-or-csv> [rows]"""
import csv
import glob
import os
import sys

p = sys.argv[1]
if os.path.isdir(p):
    p = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in list(csv.DictReader(open(p)))[:n]:
    print("%-60s %5s %10.1f us %6.2f%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3,
                                          float(r["Percentage"])))

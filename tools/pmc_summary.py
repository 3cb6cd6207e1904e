#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 counter CSVs: python tools/pmc_summary.py <dir> [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "k_"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("ebd::", "")
        if filt not in name:
            continue
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
for k, v in agg.items():
    n = len(disp[k])
    print(k, f"dispatches={n}", {c: f"{x / n:.4g}" for c, x in sorted(v.items())})

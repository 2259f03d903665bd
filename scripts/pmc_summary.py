"""Summarise rocprofv3 CSV outputs under a directory: per kernel (name filter) mean counter values per
dispatch and mean kernel duration. usage: pmc_summary.py DIR [name-substring]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if pat in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if pat in row["Name"]:
            print(f"{row['Name'][:90]}: calls {row['Calls']} avg {float(row['AverageNs']) / 1e3:.1f} us")
for k, v in sorted(vals.items()):
    print(f"{k:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")

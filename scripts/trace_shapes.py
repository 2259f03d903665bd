#!/usr/bin/env python3
"""Group a rocprofv3 kernel_trace.csv by (kernel, grid) -> per-step time (diagnostic)."""
import collections
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 13
pat = sys.argv[3] if len(sys.argv) > 3 else ""
d = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    n = r['Kernel_Name']
    if pat in n:
        d[(n[:70], int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])), int(r['Grid_Size_Y']))].append(
            (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/steps:8.1f}us/step n={len(v)/steps:5.1f} avg={sum(v)/len(v):7.1f} min={min(v):7.1f} wg={k[1]}x{k[2]} {k[0]}")

#!/usr/bin/env python3
"""Per-step kernel time summary of a rocprofv3 kernel_stats.csv (diagnostic)."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 13
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{float(r['TotalDurationNs'])/steps/1e3:9.1f}us/step {int(r['Calls'])/steps:6.1f} calls "
          f"{float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
print(f"{tot/steps/1e6:.3f} ms/step total kernel time")

#!/usr/bin/env python3
"""Where a kernel's launches sit in the step (diagnostics): from a rocprofv3 kernel trace, for every launch of the
kernels whose name contains PATTERN within the last `window_ms`, the kernels launched just before and after it on
the same queue, with its duration and grid, counted by (before, after) pair.
usage: trace_neighbors.py <dir with *kernel_trace.csv> PATTERN [window_ms]"""
import collections
import csv
import glob
import os
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n[:70]


def main():
    root, pat = sys.argv[1], sys.argv[2]
    win = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(r)
    key = "Correlation_Id" if rows and "Correlation_Id" in rows[0] else "Dispatch_Id"
    rows.sort(key=lambda r: int(r[key]))
    t_end = max(int(r["End_Timestamp"]) for r in rows)
    t0 = t_end - int(win * 1e6)
    by_q = collections.defaultdict(list)
    for r in rows:
        by_q[r.get("Queue_Id", "0")].append(r)
    pairs = collections.Counter()
    tot = collections.Counter()
    for q, lst in by_q.items():
        for i, r in enumerate(lst):
            if pat not in r["Kernel_Name"] or int(r["Start_Timestamp"]) < t0:
                continue
            prev = short(lst[i - 1]["Kernel_Name"]) if i else "-"
            nxt = short(lst[i + 1]["Kernel_Name"]) if i + 1 < len(lst) else "-"
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
            pairs[(q, prev, nxt, grid)] += 1
            tot[(q, prev, nxt, grid)] += us
    for k, n in pairs.most_common():
        q, prev, nxt, grid = k
        print(f"{n:4d} x {tot[k] / n:7.1f} us grid {grid:>8s} q{q}: after {prev} | before {nxt}")


if __name__ == "__main__":
    main()

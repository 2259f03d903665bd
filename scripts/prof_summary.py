"""Compact per-kernel summary of a rocprofv3 --kernel-trace CSV (found under DIR): calls, total / average duration,
workgroups per launch, workgroup size, VGPRs (arch + accumulation), LDS bytes — the inputs of a CU-time estimate.
usage: prof_summary.py DIR OUT.csv [--delete-trace]. Diagnostic only."""
import collections
import csv
import glob
import os
import sys

d, out = sys.argv[1], sys.argv[2]
paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
assert paths, f"no kernel_trace.csv under {d}"
agg = collections.defaultdict(lambda: [0, 0.0, 0, 0, 0, 0])
for p in paths:
    with open(p) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "?")
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 1)) or 1)
            gy = int(r.get("Grid_Size_Y", 1) or 1)
            gz = int(r.get("Grid_Size_Z", 1) or 1)
            wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
            wy = int(r.get("Workgroup_Size_Y", 1) or 1)
            wz = int(r.get("Workgroup_Size_Z", 1) or 1)
            wgs = (gx // max(wx, 1)) * (gy // max(wy, 1)) * (gz // max(wz, 1))
            a = agg[name]
            a[0] += 1
            a[1] += dur
            a[2] += wgs
            a[3] = wx * wy * wz
            a[4] = int(r.get("Arch_VGPR_Count", r.get("VGPR_Count", 0)) or 0) + int(r.get("Accum_VGPR_Count", 0) or 0)
            a[5] = int(r.get("LDS_Block_Size", r.get("LDS_Size", 0)) or 0)
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "calls", "total_ms", "avg_us", "avg_workgroups", "wg_size", "vgpr", "lds_bytes"])
    for name, (n, tot, wgs, wgsz, vg, lds) in rows:
        w.writerow([name[:160], n, round(tot / 1e3, 3), round(tot / n, 2), round(wgs / n, 1), wgsz, vg, lds])
if "--delete-trace" in sys.argv:
    for p in glob.glob(os.path.join(d, "**", "*_trace.csv"), recursive=True):
        os.remove(p)
print(f"{len(rows)} kernels -> {out}")

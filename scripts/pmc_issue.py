#!/usr/bin/env python3
"""Per-kernel issue profile from rocprofv3 SQ counter passes over the same command (diagnostics): where each kernel's
wave time goes. usage: pmc_issue.py <dir with pass subdirs> [out.json] [min_us]

Per kernel (mean per dispatch): wave-cycles, and as fractions of them the busy / waiting shares; instruction counts per
wave; MFMA busy per SIMD-cycle; LDS bank-conflict share of LDS-active cycles. SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_*
count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE cycles (MI355X_MICROARCH.md constants table)."""
import csv
import glob
import json
import os
import sys


def counters(root):
    per = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (f, r.get("Dispatch_Id"))
            ent = per.setdefault(key, {"name": r.get("Kernel_Name", ""), "c": {}})
            c = r["Counter_Name"]
            ent["c"][c] = ent["c"].get(c, 0.0) + float(r["Counter_Value"])
    agg = {}
    for ent in per.values():
        a = agg.setdefault(ent["name"], {})
        for c, v in ent["c"].items():
            s = a.setdefault(c, [0, 0.0])
            s[0] += 1
            s[1] += v
    return {k: {c: s[1] / s[0] for c, s in v.items()} for k, v in agg.items()}


def durations(root):
    out = {}
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a = out.setdefault(r.get("Kernel_Name", ""), [0, 0.0])
            a[0] += 1
            a[1] += t
    return {k: (v[0], v[1] / v[0]) for k, v in out.items()}


def main():
    root = sys.argv[1]
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    merged, dur = {}, {}
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(d):
            continue
        for k, v in counters(d).items():
            merged.setdefault(k, {}).update(v)
        for k, v in durations(d).items():
            dur.setdefault(k, v)
    rows = []
    for k, c in merged.items():
        n, us = dur.get(k, (0, 0.0))
        if us < min_us:
            continue
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        waves = max(c.get("SQ_WAVES", 1.0), 1.0)
        row = {"kernel": k[:100], "calls": n, "avg_us": round(us, 1), "waves": int(waves)}
        if wc:
            for name in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                         "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS", "SQ_INST_CYCLES_VMEM"):
                if name in c:
                    row[name.replace("SQ_", "").lower() + "_frac"] = round(c[name] / wc, 3)
        for name in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if name in c:
                row[name.replace("SQ_INSTS_", "").lower() + "_per_wave"] = round(c[name] / waves, 1)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"]:
            row["mfma_busy_per_simd"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] * 1024), 3)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 3)
        rows.append(row)
    rows.sort(key=lambda r: -r["avg_us"] * r["calls"])
    for r in rows:
        print(json.dumps(r))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel HBM traffic table from two rocprofv3 PMC passes over the same command (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950): bytes per launch, measured ÷ compulsory where the compulsory
bytes of a kernel are known for the bench workload (B = 8 images, N = 21 prompts, vit-b), and the
implied HBM rate over the launch's duration from the kernel trace of the fetch pass. `--rescore <table.json>`
recomputes a saved table's compulsory columns with the formulas below.

FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE is doubled (gfx950 reports half the bytes of wide 16-B/lane
streaming reads, MI355X_MICROARCH.md §HBM). Usage: pmc_kernels.py <dir with fetch/ write/> [out.json]"""
import csv
import glob
import json
import os
import sys

B, N = 8, 21
P = B * N
HW_OUT = 496 * 512
MB = 1e6

# compulsory bytes per launch (read once + written once) for the bench workload
COMPULSORY = {
    # low-res fp32 in, post-processed fp32 masks out, u8 gt read for the Dice partials
    "postproc_fwd_kernel": P * 256 * 256 * 4 + P * HW_OUT * 4 + P * HW_OUT,
    # masks fp32 + gt u8 in, dmask fp32 out
    "dicece_bwd_kernel": P * HW_OUT * 4 + P * HW_OUT + P * HW_OUT * 4,
    # dmask fp32 in, row-pass tmp [P, 496, 256] fp32 out
    "pp_bwd_rows_kernel": P * HW_OUT * 4 + P * 496 * 256 * 4,
    # tmp in, dlow [P, 256, 256] fp32 out
    "pp_bwd_cols_kernel": P * 496 * 256 * 4 + P * 256 * 256 * 4,
    # up1 bf16 [P * 16384, 64] (upmask.hip layout): forward reads it and writes the fp32 low-res masks; backward
    # reads up1 and d masks and writes d up1 (the W2 / b2 / hyper partials are small)
    "upmask_bwd_kernel": P * 16384 * 64 * 2 * 2 + P * 256 * 256 * 4,
    # the form with the LayerNorm2d + GELU backward fused in (the step's default, upmask_bwd_kernel<1, true>): it also
    # reads the ConvT1 output x (bf16, the up1 shape) and its per-row mean / rstd, and writes d x instead of d up1
    "upmask_bwd_kernelILi1ELb1E": P * 16384 * 64 * 2 * 3 + P * 16384 * 4 * 2 + P * 256 * 256 * 4,
    "upmask_bwd_kernel<1, true>": P * 16384 * 64 * 2 * 3 + P * 16384 * 4 * 2 + P * 256 * 256 * 4,
    "upmask_fwd_kernel": P * 16384 * 64 * 2 + P * 256 * 256 * 4,
    # DiceCE backward fused with the row pass: masks fp32 + gt u8 in, row-pass tmp [P, 496, 256] fp32 out
    "dicece_pp_rows_kernel": P * HW_OUT * 4 + P * HW_OUT + P * 496 * 256 * 4,
    # first-block backwards with the prompt sums fused in: per-image K / V (resp. Q) rows in and gradients out once,
    # per-prompt dO rows (i2t) in once, the fp32 dQ / dK-dV partials out
    "t2i_bwd_sum_kernel": B * 4096 * 256 * 2 * 2 + P * (4096 // 64) * 4 * 256 * 4,
    "i2t_bwd_sum_kernel": B * 4096 * 128 * 2 * 2 + P * 4096 * 128 * 2 + (4096 // 64) * P * 2 * 7 * 128 * 4,
}


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if counter not in r.get("Counter_Name", ""):
                continue
            key = (r.get("Dispatch_Id"), r.get("Agent_Id"))
            k = r.get("Kernel_Name", "")
            ent = per.setdefault(key, [k, 0.0])
            ent[1] += float(r["Counter_Value"])
    agg = {}
    for k, v in per.values():
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += v
    return agg


def durations(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    out = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a = out.setdefault(k, [0, 0.0])
            a[0] += 1
            a[1] += t
    return out


def short(k):
    s = k.replace("(anonymous namespace)::", "").replace("void ", "")
    return s.split("(")[0][:60]


def rescore(path):
    """Recompute the compulsory columns of a saved table (the measured bytes are kept) with this file's formulas."""
    rows = json.load(open(path))
    for row in rows:
        row.pop("compulsory_MB", None)
        row.pop("measured_over_compulsory", None)
        for name, c in COMPULSORY.items():
            if name in row["kernel"]:
                row["compulsory_MB"] = round(c / MB, 2)
                row["measured_over_compulsory"] = round(row["hbm_MB"] * MB / c, 3)
    json.dump(rows, open(path, "w"), indent=1)
    for r in rows[:40]:
        print(json.dumps(r))


def main():
    if sys.argv[1] == "--rescore":  # pmc_kernels.py --rescore <table.json> (prints the text table)
        rescore(sys.argv[2])
        return
    d = sys.argv[1]
    fetch, write, dur = load(os.path.join(d, "fetch"), "FETCH_SIZE"), load(os.path.join(d, "write"), "WRITE_SIZE"), \
        durations(os.path.join(d, "fetch"))
    rows = []
    for k, (n, v) in fetch.items():
        fb = 2 * 1024 * v / n
        wn, wv = write.get(k, [1, 0.0])
        wb = 1024 * wv / max(wn, 1)
        dn, dt = dur.get(k, [0, 0.0])
        us = dt / dn if dn else None
        row = {"kernel": short(k), "launches": n, "fetch_MB": round(fb / MB, 2), "write_MB": round(wb / MB, 2),
               "hbm_MB": round((fb + wb) / MB, 2), "avg_us_profiled": round(us, 2) if us else None}
        if us:
            row["hbm_GBps"] = round((fb + wb) / us / 1e3, 1)
        for name, c in COMPULSORY.items():
            if name in k:
                row["compulsory_MB"] = round(c / MB, 2)
                row["measured_over_compulsory"] = round((fb + wb) / c, 3)
        rows.append(row)
    rows.sort(key=lambda r: -(r["hbm_MB"] * r["launches"]))
    for r in rows[:40]:
        print(json.dumps(r))
    if len(sys.argv) > 2:
        json.dump(rows, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()

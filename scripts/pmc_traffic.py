#!/usr/bin/env python3
"""HBM traffic per launch of a kernel from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE cannot
share a pass on gfx950; MI355X_MICROARCH.md §HBM, §rocprofv3 PMC slots):

  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir>/fetch -o run -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <dir>/write -o run -- python3 bench.py ...

FETCH_SIZE / WRITE_SIZE are in KiB. gfx950 correction: FETCH_SIZE reports half the bytes of wide
(16 B/lane) streaming reads, global_load_lds included -> doubled; WRITE_SIZE is exact for 16-B stores.
Usage: pmc_traffic.py <dir> <kernel-name-substring[,substring...]> [out.json]
A comma-separated list sums the dispatches of every listed kernel (bench.py's roofline family, octsam_gemm path 2:
gemm8_kernel,gemm8p_kernel,gemm4w_kernel -- the same launch set as its compulsory_bytes_per_launch)."""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, knames):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if counter not in r.get("Counter_Name", "") or not any(k in r.get("Kernel_Name", "") for k in knames):
                continue
            key = (r.get("Dispatch_Id"), r.get("Agent_Id"))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    d, kname = sys.argv[1], sys.argv[2]
    knames = [k for k in kname.split(",") if k]
    fetch = per_dispatch(os.path.join(d, "fetch"), "FETCH_SIZE", knames)
    write = per_dispatch(os.path.join(d, "write"), "WRITE_SIZE", knames)
    res = {"kernel": kname, "dispatches": [len(fetch), len(write)],
           "fetch_bytes_per_launch": 2 * 1024 * sum(fetch) / max(len(fetch), 1),
           "write_bytes_per_launch": 1024 * sum(write) / max(len(write), 1)}
    res["hbm_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
    s = json.dumps(res, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()

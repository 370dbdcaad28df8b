#!/usr/bin/env python3
"""Summarize a tools/profile.sh run into the files committed under profiles/.

usage: tools/pmc_summary.py <prof_dir> <kernel-substring> <out.json> [--stats-out kernel_stats.csv]

<prof_dir> holds trace/run_kernel_stats.csv, fetch/run_counter_collection.csv and
write/run_counter_collection.csv (rocprofv3 --output-format csv). The HBM bytes per launch of the
named kernel follow MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half of a wide coalesced
streaming read on gfx950, WRITE_SIZE counts 16-B streaming stores exactly, both in KB, so
hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes.
"""
import csv
import json
import os
import shutil
import sys


def counters(path, kernel, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    return vals


def stats_row(path, kernel):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                return row
    return None


def main():
    prof, kernel, out = sys.argv[1], sys.argv[2], sys.argv[3]
    stats_out = sys.argv[sys.argv.index("--stats-out") + 1] if "--stats-out" in sys.argv else None
    res = {"kernel": kernel}
    st = stats_row(os.path.join(prof, "trace", "run_kernel_stats.csv"), kernel)
    if st:
        res["trace"] = {"calls": int(st["Calls"]), "avg_ms": float(st["AverageNs"]) / 1e6,
                        "min_ms": float(st["MinNs"]) / 1e6, "max_ms": float(st["MaxNs"]) / 1e6,
                        "pct_of_gpu_time": float(st["Percentage"])}
    mean = {}
    for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        v = counters(os.path.join(prof, sub, "run_counter_collection.csv"), kernel, name)
        if v:
            mean[name] = sum(v) / len(v)
            res[name] = {"launches": len(v), "mean_kb": mean[name], "first_kb": v[0],
                         "last_kb": v[-1], "min_kb": min(v), "max_kb": max(v)}
    if len(mean) == 2:
        res["hbm_bytes_per_launch"] = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
        res["note"] = ("rocprofv3 --pmc, one pass per counter; FETCH_SIZE reads 1/2 of wide "
                       "coalesced streams on gfx950 (MI355X_MICROARCH.md §HBM) -> hbm bytes = "
                       "(2*FETCH_SIZE + WRITE_SIZE) * 1024")
    json.dump(res, open(out, "w"), indent=1)
    if stats_out:
        shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"), stats_out)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

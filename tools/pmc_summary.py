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
    # SQ / GRBM passes (optional): LDS, VALU and the clock held under load
    for sub, names in (("sq", ("SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT",
                               "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU",
                               "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES")),
                       ("grbm", ("GRBM_GUI_ACTIVE", "GRBM_COUNT"))):
        path = os.path.join(prof, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for name in names:
            v = counters(path, kernel, name)
            if v:
                mean[name] = sum(v) / len(v)
                res.setdefault("pmc_mean_per_launch", {})[name] = mean[name]
    # the GRBM pass carries its own kernel trace: under --pmc launches are serialized, so the
    # clock is taken over the durations of those same launches
    gst = stats_row(os.path.join(prof, "grbm", "run_kernel_stats.csv"), kernel) \
        if os.path.exists(os.path.join(prof, "grbm", "run_kernel_stats.csv")) else None
    if "GRBM_GUI_ACTIVE" in mean and gst:
        # MI355X_MICROARCH.md 'DVFS give-back': clock ~= GRBM_GUI_ACTIVE / 8 (XCDs) / wall time
        gdur = float(gst["AverageNs"]) * 1e-9
        res["pmc_serialized_avg_ms"] = gdur * 1e3
        res["clock_ghz"] = mean["GRBM_GUI_ACTIVE"] / 8.0 / gdur / 1e9
        if "SQ_LDS_IDX_ACTIVE" in mean:
            cyc = mean["GRBM_GUI_ACTIVE"] / 8.0
            res["lds_array_busy_frac"] = mean["SQ_LDS_IDX_ACTIVE"] / (cyc * 256.0)
            res["lds_note"] = ("SQ_LDS_IDX_ACTIVE (all LDS-array cycles, summed over CUs) / "
                               "(GRBM_GUI_ACTIVE / 8 x 256 CUs)")
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
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

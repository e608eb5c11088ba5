"""Per-kernel HBM bytes per launch from a tools/gpu_profile.sh directory
(trace/ kernel durations, pmc_fetch/ FETCH_SIZE and pmc_write/ WRITE_SIZE
passes), in the format bench.py reads (profiles/rNN/traffic_all_kernels.json):
raw = (FETCH_SIZE + WRITE_SIZE) KiB, corrected = 2 FETCH_SIZE + WRITE_SIZE
(MI355X_MICROARCH.md's gfx950 FETCH_SIZE correction).

    python tools/traffic_json.py gpurun_out/prof_r02c > profiles/r02/traffic_all_kernels.json
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

KEEP = ("refine_kernel", "fast_kernel")


def per_dispatch(path, counter):
    acc = defaultdict(float)
    name = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            acc[d] += float(r["Counter_Value"])  # summed over XCD / SE instances
            name[d] = r["Kernel_Name"]
    out = defaultdict(list)
    for d, v in acc.items():
        out[name[d]].append(v)
    return out


def main(d):
    durs = defaultdict(list)
    with open(os.path.join(d, "trace", "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    fetch = per_dispatch(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(d, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k, ts in durs.items():
        if not any(s in k for s in KEEP) or k not in fetch or k not in write:
            continue
        fk, wk = statistics.fmean(fetch[k]), statistics.fmean(write[k])
        res[k] = {"fetch_kb": fk, "write_kb": wk, "raw_bytes": 1024.0 * (fk + wk),
                  "corrected_bytes": 1024.0 * (2.0 * fk + wk), "avg_ns": statistics.fmean(ts),
                  "median_ns": statistics.median(ts), "launches": len(ts)}
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])

#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + PMC passes) per kernel.

usage: summarize_profile.py <prof_dir> [out.json] [refine_traffic.json]
HBM bytes per launch follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and
WRITE_SIZE are KiB; gfx950 FETCH_SIZE reads 1/2 of the bytes of wide coalesced
streams, so the corrected read bytes are 2*FETCH_SIZE*1024 (the correction is
uncalibrated for dword gathers: both numbers are reported).
"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return name.rsplit("(", 1)[0] if name.endswith(")") else name


def main():
    d = sys.argv[1]
    out = {"kernels": {}}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            out["kernels"].setdefault(k, {})["stats"] = {
                "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"]),
                "pct": float(r["Percentage"])}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            e = out["kernels"].setdefault(k, {}).setdefault("counters", {})
            c = e.setdefault(r["Counter_Name"], [])
            c.append(float(r["Counter_Value"]))
            meta = out["kernels"][k].setdefault("meta", {})
            for m in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Workgroup_Size", "Grid_Size"):
                meta[m] = r.get(m)
    for k, e in out["kernels"].items():
        cs = e.get("counters", {})
        e["counters"] = {n: sum(v) / len(v) for n, v in cs.items()}
        if "FETCH_SIZE" in e["counters"] or "WRITE_SIZE" in e["counters"]:
            f = e["counters"].get("FETCH_SIZE", 0.0) * 1024
            w = e["counters"].get("WRITE_SIZE", 0.0) * 1024
            e["hbm_bytes_per_launch_raw"] = f + w
            e["hbm_bytes_per_launch"] = 2 * f + w
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js)
    # traffic of the bench's dominant kernel (the expansion refine kernel) per launch
    if len(sys.argv) > 3:
        cand = {k: e for k, e in out["kernels"].items() if k.startswith("dpk::refine_kernel<4") and
                "hbm_bytes_per_launch" in e}
        if cand:
            k, e = max(cand.items(), key=lambda kv: kv[1].get("stats", {}).get("total_ns", 0.0))
            open(sys.argv[3], "w").write(json.dumps({
                "kernel": k, "batch": int(sys.argv[4]) if len(sys.argv) > 4 else None,
                "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                "hbm_bytes_per_launch_raw": e["hbm_bytes_per_launch_raw"],
                "avg_ns": e.get("stats", {}).get("avg_ns"),
                "method": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM/rocprofv3), "
                          "separate --pmc passes"}, indent=1))
    print(js)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel summary of a tools/r03_profile.sh directory: launch durations
(the trace pass), and per launch every PMC counter summed over its
instances (XCD / SE rows of one dispatch) and averaged over the kernel's
dispatches; derived HBM bytes (raw = (FETCH_SIZE + WRITE_SIZE) KiB, corrected
= 2 FETCH_SIZE + WRITE_SIZE per MI355X_MICROARCH.md) and VALU issue figures.

    python tools/profile_json.py gpurun_out/prof_r03/fast7 [more dirs] > profiles/r03/kernel_counters.json
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

KEEP = ("refine_kernel", "fast_kernel")
SIMDS = 256 * 4          # MI355X: 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4          # max clock (MI355X_MICROARCH.md)


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.rsplit("(", 1)[0] if name.endswith(")") else name


def one(d):
    out = {}
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    stats = {}
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                       "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    ctr = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(float)
        name = {}
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            name[key] = short(r["Kernel_Name"])
        for (disp, cn), v in acc.items():
            ctr[name[(disp, cn)]][cn].append(v)
    args = open(os.path.join(d, "args.txt")).read().strip() if os.path.exists(os.path.join(d, "args.txt")) else ""
    toks = args.split()
    steps = int(toks[toks.index("--steps") + 1]) if "--steps" in toks else 5
    # the library the profiled bench loaded, and the same process's own HIP-event
    # time of its timed launches: its JSON line in the trace log
    lib_sha = None
    ev_ms, ev_list = None, None
    if os.path.exists(os.path.join(d, "trace.log")):
        for line in open(os.path.join(d, "trace.log")):
            if line.startswith("{"):
                try:
                    j = json.loads(line)
                except ValueError:
                    continue
                lib_sha = j.get("lib_sha256", lib_sha)
                ev_ms = j.get("kernel_ms_per_launch", ev_ms)
                ev_list = j.get("kernel_ms_events", ev_list)
    # bench.py's full result (the stdout line is a compact summary since r06)
    det = os.path.join(d, "detail.json")
    if os.path.exists(det):
        try:
            j = json.load(open(det))
            lib_sha = j.get("lib_sha256", lib_sha)
            ev_ms = j.get("kernel_ms_per_launch", ev_ms)
            ev_list = j.get("kernel_ms_events", ev_list)
        except ValueError:
            pass
    for k in set(durs) | set(ctr):
        if not any(s in k for s in KEEP):
            continue
        e = {"command": "python3 bench.py " + args, "lib_sha256": lib_sha}
        if k in durs:
            # the bench's timed launches are the last --steps of the kernel's
            # dispatches (the first are its untimed warm-up, clocks settling)
            timed = durs[k][-steps:] if len(durs[k]) > steps else durs[k]
            e["trace_avg_ns"] = statistics.fmean(timed)
            e["trace_launches"] = len(timed)
            e["trace_avg_all_ns"] = statistics.fmean(durs[k])
            e["trace_launches_all"] = len(durs[k])
            e["trace_timed_ns"] = timed
            if ev_ms:
                # the profiled process's own HIP events around the same launches
                # (bench.py records them on the launch stream; they also cover
                # the refine's dequeue-ordering kernels and the launch gaps)
                e["events_avg_ns_same_process"] = ev_ms * 1e6
                e["events_ms_same_process"] = ev_list
                e["trace_over_events"] = e["trace_avg_ns"] / (ev_ms * 1e6)
        if k in stats:
            e["stats"] = stats[k]
        c = {n: statistics.fmean(v) for n, v in ctr.get(k, {}).items()}
        e["counters_per_launch"] = c
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_raw"] = 1024.0 * (c["FETCH_SIZE"] + c["WRITE_SIZE"])
            e["hbm_bytes_corrected"] = 1024.0 * (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"])
        if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c and "trace_avg_ns" in e:
            t = e["trace_avg_ns"] * 1e-9
            clk = c["GRBM_GUI_ACTIVE"] / 8.0 / t / 1e9  # GHz: summed over the 8 XCDs
            e["valu"] = {
                "insts_per_launch": c["SQ_INSTS_VALU"],
                "effective_clock_GHz": clk,
                "busy_frac": 4.0 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / (SIMDS * clk * 1e9 * t),
                "issue_peak_at_effective_clock_Ginst_s": SIMDS * clk / 2.0,
                "issue_peak_at_2.4GHz_Ginst_s": SIMDS * CLOCK_GHZ / 2.0,
                # SIMD cycles of wall time per wave-instruction of VALU (2 = the
                # issue peak; a fp64 add/mul/fma takes 4, a transcendental 8)
                "simd_cycles_per_valu": SIMDS * clk * 1e9 * t / c["SQ_INSTS_VALU"],
            }
            wc = c.get("SQ_WAVE_CYCLES")
            if wc and "SQ_WAIT_ANY" in c and "SQ_WAIT_INST_ANY" in c and "SQ_ACTIVE_INST_ANY" in c:
                # disjoint split of wave lifetime (MI355X_MICROARCH.md, PMC slots)
                e["valu"]["wave_cycles"] = {
                    "issuing_frac": c["SQ_ACTIVE_INST_ANY"] / wc,
                    "wait_inst_frac": c["SQ_WAIT_INST_ANY"] / wc,
                    "wait_any_frac": c["SQ_WAIT_ANY"] / wc,
                }
        out[k] = e
    return out


def main():
    res = {}
    for d in sys.argv[1:]:
        res[os.path.basename(d.rstrip("/"))] = one(d)
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where a densify's non-refine time goes, from a rocprofv3 --kernel-trace
[--memory-copy-trace] directory of tools/densify_trace.py: for the LAST
repetition (from its seed_patches_kernel on), the GPU
busy time of the refine kernels, of every other kernel and of the copies,
and the idle time between them, per generation.

    python tools/densify_gaps.py gpurun_out/dtr5/fast [--generations 76]
"""
import argparse
import collections
import csv
import glob
import os

REFINE = ("fast_kernel", "refine_kernel")


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            n = n.rsplit("(", 1)[0] if n.endswith(")") else n
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
    return sorted(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--generations", type=int, default=0)
    a = ap.parse_args()
    ev = rows(a.dir)
    # the last repetition: from the last densify begin (seed_patches_kernel)
    starts = [i for i, e in enumerate(ev) if "seed_patches_kernel" in e[2]]
    ev = ev[starts[-1]:] if starts else ev
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    busy = collections.Counter()
    count = collections.Counter()
    idle = 0
    cur = t0
    for s, e, n in ev:
        kind = "refine" if any(k in n for k in REFINE) else n
        busy[kind] += e - s
        count[kind] += 1
        if s > cur:
            idle += s - cur
        cur = max(cur, e)
    span = t1 - t0
    g = a.generations or count.get("refine", 1)
    print(f"span {span / 1e6:.2f} ms, events {len(ev)}, idle {idle / 1e6:.2f} ms, per generation ({g}): "
          f"idle {idle / g / 1e3:.1f} us")
    for k, v in busy.most_common(25):
        print(f"  {v / 1e6:8.3f} ms  {count[k]:5d}x  {v / max(count[k], 1) / 1e3:8.1f} us  {v / g / 1e3:7.1f} us/gen  {k[-70:]}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Parity-kernel staging study: how far do a refine's
window ROIs (Optimization::GetProjectedTextures, optimization.cpp:14-56) move
from the first evaluation's ROI during Nelder-Mead, and what would staging
each visible view's footprint in LDS cost?

Runs the oracle (single-threaded, ROI trace on) on Expand::ExpandPatch
children of bench.py's parents (the parity seed stage's survivors) and, per
(candidate, view), the margin M (px) that the first ROI must be grown by to
contain every later ROI of that view's NM evaluations (the filter's
re-staged evaluation excluded: it is centred on the refined position).
Prints one JSON line: the margin distribution, the fraction of window
evaluations inside first-ROI + M for M = 0..16, and the BGRA8 LDS bytes per
candidate that a tile of first-ROI + M per view needs.

    python tools/roi_footprint.py [--config cfg3_32view_4k] [--seeds 1500]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import densepoints_amd as dp  # noqa: E402
from densepoints_amd import synth  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3_32view_4k")
    ap.add_argument("--seeds", type=int, default=1500)
    ap.add_argument("--parents", type=int, default=200)
    a = ap.parse_args()
    cfg = synth.named(a.config)
    P, imgs, seeds = synth.scene_host(cfg)
    S = orc.Scene(P, imgs, dp.Options())
    rng = np.random.default_rng(5)
    pick = np.sort(rng.choice(len(seeds), size=min(a.seeds, len(seeds)), replace=False))
    sp = S.seeds_to_patches(seeds[pick])
    ok = S.refine(sp, 16, orc.MODE_SEED, nthreads=0)
    parents = np.ascontiguousarray(sp[ok == 1][: a.parents])
    cap = 20_000_000
    buf = np.zeros(5 * cap, dtype=np.int32)
    orc.lib.or_trace_set(buf.ctypes.data, cap)
    kids, acc = S.expand(parents, nthreads=1)
    n = int(orc.lib.or_trace_count())
    orc.lib.or_trace_set(None, 0)
    rec = buf[: 5 * n].reshape(n, 5)
    marks = np.flatnonzero(rec[:, 0] == -1)
    margins, inside = [], np.zeros(17)
    total_windows = 0
    lds = {m: [] for m in (0, 2, 4, 8)}
    evals = kids["evals"]
    for ci, (lo, hi) in enumerate(zip(marks, list(marks[1:]) + [n])):
        r = rec[lo + 1: hi]
        if len(r) == 0:
            continue
        # the NM evaluations are all but the filter's last (one window per view)
        nv = len(np.unique(r[:, 0]))
        nm = r[: max(len(r) - nv, 0)]
        first = {}
        need = {}
        for v, tx, ty, bx, by in nm:
            if v not in first:
                first[v] = (tx, ty, bx, by)
                need[v] = 0
                continue
            f = first[v]
            m = max(f[0] - tx, f[1] - ty, bx - f[2], by - f[3], 0)
            need[v] = max(need[v], m)
            total_windows += 1
            for M in range(17):
                inside[M] += m <= M
        margins += list(need.values())
        for M in lds:
            lds[M].append(sum(4 * (f[2] - f[0] + 1 + 2 * M + 1) * (f[3] - f[1] + 1 + 2 * M + 1)
                              for f in first.values()))
    mg = np.array(margins)
    out = {"config": a.config, "parents": int(len(parents)), "candidates": int(len(kids)),
           "E_mean": round(float(evals[evals > 0].mean()), 2), "views_per_candidate": round(len(mg) / max(len(marks), 1), 2),
           "margin_px_needed": {"median": float(np.median(mg)), "p90": float(np.percentile(mg, 90)),
                                "p99": float(np.percentile(mg, 99)), "max": int(mg.max())},
           "windows_inside_first_roi_plus_M": {str(M): round(float(inside[M] / max(total_windows, 1)), 4)
                                               for M in (0, 1, 2, 3, 4, 6, 8, 12, 16)},
           "lds_bytes_per_candidate_bgra8": {str(M): {"median": float(np.median(v)), "p90": float(np.percentile(v, 90))}
                                             for M, v in lds.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Performance-mode refine variants on the CPU spec (oracle/or_fast.c):
forward-difference gradient (spec v3, gradient = 0) against the analytic
gradient (spec v4, gradient = 1) at several CG iteration counts.  Parents: the
performance pipeline's own (seed patches refined by the same variant at
n = 16); children: Expand::ExpandPatch refined at `--cell`.  Quality of the
accepted children against the synthetic ground truth (as bench.py reports
it), E and the evaluations with a gradient.  Prints one JSON line per variant.

    python tools/fast_gradient_quality.py [--config cfg2_8view_1080p] [--parents 2000]
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


def quality(cfg, kids, acc):
    k = kids[acc == 1]
    if len(k) == 0:
        return {"accepted": 0}
    z, nrm = synth.surface(cfg, k["pos"][:, :2].astype(np.float64))
    nn = k["normal"].astype(np.float64)
    nn /= np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-30)
    ang = np.degrees(np.arccos(np.clip(np.abs((nn * nrm).sum(1)), 0.0, 1.0)))
    dz = np.abs(k["pos"][:, 2] - z)
    return {"accepted": int(len(k)), "median_abs_dz": float(np.median(dz)), "p90_abs_dz": float(np.percentile(dz, 90)),
            "median_normal_err_deg": round(float(np.median(ang)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2_8view_1080p")
    ap.add_argument("--parents", type=int, default=2000)
    ap.add_argument("--cell", type=int, default=11)
    ap.add_argument("--variants", default="0:4,1:2,1:3,1:4", help="gradient:iters,...")
    ap.add_argument("--parents-from", default="fast", choices=["fast", "parity"],
                    help="parents: the variant's own seed stage (fast) or the parity Nelder-Mead seed stage "
                         "(bench.py's headline parents)")
    a = ap.parse_args()
    cfg = synth.named(a.config)
    P, imgs, seeds = synth.scene_host(cfg)
    S = orc.Scene(P, imgs, dp.Options(expand_cell_size=a.cell))
    rng = np.random.default_rng(3)
    pick = np.sort(rng.choice(len(seeds), size=min(len(seeds), 3 * a.parents), replace=False))
    raw = S.seeds_to_patches(seeds[pick])
    for v in a.variants.split(","):
        gr, it = (int(x) for x in v.split(":"))
        fo = orc.fast_options(iters=it, gradient=gr)
        par = raw.copy()
        ok = S.fast_refine(par, 16, fo=fo) if a.parents_from == "fast" else S.refine(par, 16, orc.MODE_SEED)
        parents = np.ascontiguousarray(par[ok == 1][: a.parents])
        kids, acc = S.fast_expand(parents, fo)
        E = kids["evals"].astype(np.float64)
        print(json.dumps({"config": a.config, "cell": a.cell, "gradient": gr, "iters": it,
                          "parents": int(len(parents)), "parents_quality": quality(cfg, parents, np.ones(len(parents), np.uint8)),
                          "E_mean": round(float(E[E > 0].mean()), 3), "children": quality(cfg, kids, acc)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Calibration of the visibility / neighbourhood filter (PMVS::FilterPatches,
methods/pmvs/pmvs.h:27 -- declared, never defined; spec in
include/densepoints.h) against the synthetic scene's ground truth.

On BASELINE config 4 (64 views 4K) it densifies once per refine mode (parity
Nelder-Mead, performance-mode CG) and runs the filter under several settings;
for each it reports the kept fraction and the median / 90th-percentile depth
error |z - z_true| and normal error (deg) of the kept and of the removed
patches (dp_synth_surface).  Prints one JSON object.

    python tools/filter_calibration.py [--config cfg4_64view_4k] > out.json
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def errors(cfg, p):
    from densepoints_amd import synth

    z, nrm = synth.surface(cfg, p["pos"][:, :2].astype(np.float64))
    nn = p["normal"].astype(np.float64)
    nn /= np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-30)
    ang = np.degrees(np.arccos(np.clip(np.abs((nn * nrm).sum(1)), 0.0, 1.0)))
    return np.abs(p["pos"][:, 2] - z), ang


def stats(dz, ang):
    if len(dz) == 0:
        return {"n": 0}
    return {"n": int(len(dz)), "dz_median": float(np.median(dz)), "dz_p90": float(np.percentile(dz, 90)),
            "normal_deg_median": round(float(np.median(ang)), 3),
            "normal_deg_p90": round(float(np.percentile(ang, 90)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4_64view_4k")
    args = ap.parse_args()
    import densepoints_amd as dp
    from densepoints_amd import _native as N
    from densepoints_amd import synth

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    cfg = synth.named(args.config)
    P = synth.cameras(cfg)
    V, W, H = cfg.n_views, cfg.width, cfg.height
    out = {"config": args.config}
    settings = [("default (both passes, frac 0.25)", 3, 0.25), ("visibility only", 1, 0.25),
                ("neighbours only, frac 0.25", 2, 0.25), ("both, frac 0.125", 3, 0.125),
                ("both, frac 0.0625", 3, 0.0625)]
    with dp.Engine(dp.Options(), device=0) as eng:
        planes = torch.empty((V, H, W), dtype=torch.int32, device="cuda")
        for v in range(V):
            N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(cfg), N.ptr(P), v, planes[v].data_ptr(),
                                                 stream.cuda_stream), eng.handle)
        torch.cuda.synchronize()
        eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
        seeds = synth.seeds(cfg, P)
        for mode in ("parity", "fast"):
            eng.set_fast_options(dp.FastOptions(densify=1 if mode == "fast" else 0))
            pat, st = eng.densify(seeds)
            dz, ang = errors(cfg, pat)
            res = {"patches": int(len(pat)), "all": stats(dz, ang)}
            for name, passes, frac in settings:
                keep = eng.filter_patches(np.ascontiguousarray(pat), passes=passes, min_neighbor_frac=frac) == 1
                res[name] = {"kept_frac": round(float(keep.mean()), 4), "kept": stats(dz[keep], ang[keep]),
                             "removed": stats(dz[~keep], ang[~keep])}
            # the neighbourhood test's sensitivity to normal error: patches binned by normal error
            keep = eng.filter_patches(np.ascontiguousarray(pat), passes=2, min_neighbor_frac=0.25) == 1
            bins = [0, 5, 10, 20, 30, 45, 90]
            res["neighbours_kept_by_normal_error"] = {
                f"{a}-{b} deg": {"n": int(((ang >= a) & (ang < b)).sum()),
                                 "kept_frac": round(float(keep[(ang >= a) & (ang < b)].mean()), 4)
                                 if ((ang >= a) & (ang < b)).any() else None}
                for a, b in zip(bins[:-1], bins[1:])}
            out[mode] = res
        eng.set_fast_options(dp.FastOptions())
        del planes
    print(json.dumps(out))


if __name__ == "__main__":
    main()

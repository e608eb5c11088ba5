#!/usr/bin/env python3
"""The whole performance-mode densify (dp_densify with dp_fast_options.densify)
on a BASELINE config in both refine specs -- forward differences (v3,
gradient 0) and the analytic gradient (v4, gradient 1) -- at several CG
iteration counts: wall time, patches, and the geometry of every stored patch
against the synthetic ground truth (dp_synth_surface).  One JSON line per run.

    python tools/fast_densify_quality.py [--config cfg4_64view_4k] [--variants 0:4,1:4,1:3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def geometry(cfg, p):
    from densepoints_amd import synth

    z, nrm = synth.surface(cfg, p["pos"][:, :2].astype(np.float64))
    nn = p["normal"].astype(np.float64)
    nn /= np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-30)
    ang = np.degrees(np.arccos(np.clip(np.abs((nn * nrm).sum(1)), 0.0, 1.0)))
    dz = np.abs(p["pos"][:, 2] - z)
    return {"n": int(len(p)), "median_abs_dz": float(np.median(dz)), "p90_abs_dz": float(np.percentile(dz, 90)),
            "median_normal_err_deg": round(float(np.median(ang)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4_64view_4k")
    ap.add_argument("--variants", default="0:4,1:4,0:3,1:3", help="gradient:iters[:max_views],...")
    a = ap.parse_args()
    import densepoints_amd as dp
    from densepoints_amd import _native as N
    from densepoints_amd import synth

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    cfg = synth.named(a.config)
    P = synth.cameras(cfg)
    V, W, H = cfg.n_views, cfg.width, cfg.height
    with dp.Engine(dp.Options(), device=0) as eng:
        planes = torch.empty((V, H, W), dtype=torch.int32, device="cuda")
        for v in range(V):
            N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(cfg), N.ptr(P), v, planes[v].data_ptr(),
                                                 stream.cuda_stream), eng.handle)
        torch.cuda.synchronize()
        eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
        seeds = synth.seeds(cfg, P)
        for v in a.variants.split(","):
            f = [int(x) for x in v.split(":")]
            gr, it = f[0], f[1]
            mv = f[2] if len(f) > 2 else dp.FastOptions().max_views
            eng.set_fast_options(dp.FastOptions(densify=1, gradient=gr, iters=it, max_views=mv))
            eng.densify(seeds)  # warm-up (gray planes, clocks)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pat, st = eng.densify(seeds)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            keep = eng.filter_patches(np.ascontiguousarray(pat)) == 1
            print(json.dumps({"config": a.config, "gradient": gr, "iters": it, "max_views": mv, "densify_ms": round(ms, 2),
                              "candidates": int(st["seeds_in"]) + int(st["candidates"]),
                              "all": geometry(cfg, pat), "filter_kept": geometry(cfg, pat[keep])}), flush=True)
        eng.set_fast_options(dp.FastOptions())
        del planes


if __name__ == "__main__":
    main()

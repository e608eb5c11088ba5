#!/usr/bin/env python3
"""Performance-mode option sweep on the GPU, on bench.py's headline workload
(config 3, the parity seed stage's survivors as parents, 65,536 parents x 4
children): rate (HIP events on the launch stream), E, staged views per
evaluation and the accepted children's quality against the synthetic ground
truth, one JSON line per variant.

    python tools/fast_sweep.py --cell 11 --variants "iters=4;iters=3,ls_step=2.0;max_views=12"
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

import densepoints_amd as dp  # noqa: E402
from densepoints_amd import _native as N  # noqa: E402
from densepoints_amd import synth  # noqa: E402


def quality(cfg, kids, acc):
    k = kids[acc == 1]
    if len(k) == 0:
        return {"accepted": 0}
    z, nrm = synth.surface(cfg, k["pos"][:, :2].astype(np.float64))
    nn = k["normal"].astype(np.float64)
    nn /= np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-30)
    ang = np.degrees(np.arccos(np.clip(np.abs((nn * nrm).sum(1)), 0.0, 1.0)))
    dz = np.abs(k["pos"][:, 2] - z)
    return {"accepted": int(len(k)), "median_abs_dz": round(float(np.median(dz)), 6),
            "p90_abs_dz": round(float(np.percentile(dz, 90)), 5),
            "median_normal_err_deg": round(float(np.median(ang)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3_32view_4k")
    ap.add_argument("--cell", type=int, default=11)
    ap.add_argument("--parents", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--variants", default="iters=4")
    a = ap.parse_args()
    cfg = synth.named(a.config)
    V, W, H = cfg.n_views, cfg.width, cfg.height
    P = synth.cameras(cfg)
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng = dp.Engine(dp.Options(expand_cell_size=a.cell), device=0)
    planes = torch.empty((V, H, W), dtype=torch.int32, device="cuda")
    for v in range(V):
        N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(cfg), N.ptr(P), v, planes[v].data_ptr(),
                                             stream.cuda_stream), eng.handle)
    torch.cuda.synchronize()
    eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
    seeds = synth.seeds(cfg, P)
    seed_p = eng.seeds_to_patches(seeds)
    d_seed = torch.from_numpy(seed_p.view(np.uint8).copy()).to("cuda")
    d_ok = torch.empty(len(seed_p), dtype=torch.uint8, device="cuda")
    eng.refine_device(d_seed.data_ptr(), len(seed_p), 16, N.MODE_SEED, d_ok.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    seed_p = np.frombuffer(d_seed.cpu().numpy().tobytes(), dtype=N.PATCH_DTYPE)
    parents_all = seed_p[d_ok.cpu().numpy() == 1]
    NP = a.parents
    parents = np.ascontiguousarray(parents_all[np.arange(NP) % len(parents_all)])
    d_par = torch.from_numpy(parents.view(np.uint8).copy()).to("cuda")
    B = 4 * NP
    work = torch.empty(B * N.PATCH_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    accept = torch.empty(B, dtype=torch.uint8, device="cuda")
    base = None  # the first variant's accepted set: paired quality on the intersection
    for var in a.variants.split(";"):
        fo = dp.FastOptions()
        for kv in filter(None, var.split(",")):
            k, v = kv.split("=")
            setattr(fo, k, type(getattr(fo, k))(float(v)) if isinstance(getattr(fo, k), float) else int(v))
        eng.set_fast_options(fo)
        for _ in range(2):
            eng.fast_expand_device(d_par.data_ptr(), NP, work.data_ptr(), accept.data_ptr(), stream.cuda_stream)
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            eng.fast_expand_device(d_par.data_ptr(), NP, work.data_ptr(), accept.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            ms.append((e0, e1))
        torch.cuda.synchronize()
        ms = [x.elapsed_time(y) for x, y in ms]
        st = eng.fast_last_stats()
        out = np.frombuffer(work.cpu().numpy().tobytes(), dtype=N.PATCH_DTYPE)
        acc = accept.cpu().numpy()
        kms = float(np.mean(ms))
        if base is None:
            base = (out.copy(), acc.copy())
        both = (acc == 1) & (base[1] == 1)
        z, _ = synth.surface(cfg, out["pos"][both][:, :2].astype(np.float64))
        zb, _ = synth.surface(cfg, base[0]["pos"][both][:, :2].astype(np.float64))
        paired = {"n": int(both.sum()),
                  "median_abs_dz": round(float(np.median(np.abs(out["pos"][both][:, 2] - z))), 6),
                  "baseline_median_abs_dz": round(float(np.median(np.abs(base[0]["pos"][both][:, 2] - zb))), 6)}
        refined = out["evals"] > 1
        print(json.dumps({"variant": var, "paired_with_first": paired,
                          "all_refined": quality(cfg, out, refined.astype(np.uint8)), "cell": a.cell, "Mpatches_per_s": round(B / kms / 1e3, 3),
                          "kernel_ms": round(kms, 3), "E": round(st["evals"] / max(st["patches"], 1), 3),
                          "views_per_eval": round(st["view_evals"] / max(st["evals"], 1), 3),
                          "clipped_stagings_per_patch": round(st["clipped_stagings"] / max(st["patches"], 1), 4),
                          "accept_rate": round(float(acc.mean()), 4), "quality": quality(cfg, out, acc)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""End-to-end dp_densify on a named synthetic config (device-rendered views):
prints one JSON line with the densify statistics and timings."""
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

import densepoints_amd as dp  # noqa: E402
from densepoints_amd import _native as N  # noqa: E402
from densepoints_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3_32view_4k")
ap.add_argument("--max-seeds", type=int, default=0)
ap.add_argument("--max-pops", type=int, default=0)
args = ap.parse_args()
cfg = synth.named(args.config)
V, W, H = cfg.n_views, cfg.width, cfg.height
P = synth.cameras(cfg)
opts = dp.Options(max_pops=args.max_pops) if args.max_pops else dp.Options()
eng = dp.Engine(opts, device=0)
planes = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(V)]
for v in range(V):
    N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(cfg), N.ptr(P), v, planes[v].data_ptr(), None),
            eng.handle)
torch.cuda.synchronize()
eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
seeds = synth.seeds(cfg, P)
if args.max_seeds:
    seeds = seeds[: args.max_seeds]
t0 = time.perf_counter()
out, st = eng.densify(seeds)
wall = time.perf_counter() - t0
st = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}
print(json.dumps({"config": args.config, "seeds": len(seeds), "wall_s": round(wall, 3),
                  "patches_per_s": round(st["patches"] / wall, 1),
                  "candidates_per_s": round(st["candidates"] / wall, 1), **st}))

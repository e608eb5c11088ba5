#!/usr/bin/env python3
"""Seed generation (dp_generate_seeds) on a named synthetic config with
device-rendered views, plus the bare knnMatch kernel on random descriptors:
prints one JSON line (stage times, counts, kNN MFMA throughput)."""
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
from densepoints_amd import matcher as M  # noqa: E402
from densepoints_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3_32view_4k")
ap.add_argument("--views", type=int, default=0)
ap.add_argument("--repeat", type=int, default=2)
ap.add_argument("--knn", type=int, default=40000, help="rows per side of the bare kNN timing (0 = skip)")
ap.add_argument("--fast-threshold", type=int, default=20)
ap.add_argument("--detector", default="orb", choices=["orb", "akaze"])
args = ap.parse_args()
cfg = synth.named(args.config)
if args.views:
    cfg.n_views = args.views
V, W, H = cfg.n_views, cfg.width, cfg.height
P = synth.cameras(cfg)
eng = dp.Engine(dp.Options(), device=0)
planes = torch.empty((V, H, W), dtype=torch.int32, device="cuda")
for v in range(V):
    N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(cfg), N.ptr(P), v, planes[v].data_ptr(), None),
            eng.handle)
torch.cuda.synchronize()
eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
m = M.Matcher(eng, M.MatcherOptions(fast_threshold=args.fast_threshold,
                                     detector_type=M.DETECTOR_AKAZE if args.detector == "akaze" else M.DETECTOR_ORB))
walls = []
for _ in range(args.repeat):
    t0 = time.perf_counter()
    pts = m.generate_seeds()
    walls.append(time.perf_counter() - t0)
st = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in m.stats.items()}
out = {"config": args.config, "views": V, "detector": args.detector, "fast_threshold": args.fast_threshold,
       "wall_s": [round(w, 3) for w in walls], **st}
if args.knn:
    rng = np.random.default_rng(1)
    q = rng.integers(0, 256, size=(args.knn, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(args.knn, 32), dtype=np.uint8)
    ms = []
    for _ in range(3):
        M.knn_match(eng, q, t)
        ms.append(eng.last_kernel_ms())
    best = min(ms)
    pairs = float(args.knn) * args.knn
    out["knn"] = {"rows": args.knn, "kernel_ms": [round(x, 3) for x in ms], "Gpairs_per_s": round(pairs / best / 1e6, 1),
                  "int8_TOPS": round(pairs * 512 / best / 1e9, 1)}
print(json.dumps(out))

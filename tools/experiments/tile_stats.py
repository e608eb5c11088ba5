#!/usr/bin/env python3
"""LDS-tile path counters of the parity refine on bench.py's
headline batch: run with a -DDP_TILE_STATS build (DP_LIB_VARIANT); prints the
passes sampled from LDS / mixed / HBM / split-or-clamped, the staged tiles
and the per-evaluation tile lookups that hit or missed.

    DP_LIB_VARIANT=libdp_tstats.so python tools/experiments/tile_stats.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import densepoints_amd as dp  # noqa: E402
from densepoints_amd import _native as N  # noqa: E402
from densepoints_amd import synth  # noqa: E402


def main():
    cfg = synth.named("cfg3_32view_4k")
    V, W, H = cfg.n_views, cfg.width, cfg.height
    P = synth.cameras(cfg)
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng = dp.Engine(dp.Options(), device=0)
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
    st = np.zeros(8, dtype=np.uint64)
    N.lib.dp_debug_stamps(N.ptr(st))  # reset (the seed stage's counts)
    seed_p = np.frombuffer(d_seed.cpu().numpy().tobytes(), dtype=N.PATCH_DTYPE)
    parents = np.ascontiguousarray(seed_p[d_ok.cpu().numpy() == 1][:65536])
    d_par = torch.from_numpy(parents.view(np.uint8).copy()).to("cuda")
    B = 4 * len(parents)
    work = torch.empty(B * N.PATCH_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    accept = torch.empty(B, dtype=torch.uint8, device="cuda")
    eng.expand_device(d_par.data_ptr(), len(parents), work.data_ptr(), accept.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    rc = N.lib.dp_debug_stamps(N.ptr(st))
    names = ["passes_lds", "passes_mixed", "passes_hbm", "passes_split_or_clamped", "tiles_staged",
             "lookups_in_tile", "lookups_out_of_tile", "stagings"]
    out = {k: int(v) for k, v in zip(names, st)}
    out["rc"] = rc
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The config-4 partitioned densify (bench.py scaling_leg) at one rank, timed
per phase on the host: partition, refine, compaction, commit -- the replicated
part of every generation that does not shrink with the rank count.  Run under
rocprofv3 --kernel-trace --stats for per-kernel times.  Prints one JSON line.

    python tools/partition_probe.py [--mode fast|parity] [--reps 2]
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

import densepoints_amd as dp  # noqa: E402
from densepoints_amd import _native as N  # noqa: E402
from densepoints_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4_64view_4k")
    ap.add_argument("--mode", default="fast")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    cfg = synth.named(a.config)
    V, W, H = cfg.n_views, cfg.width, cfg.height
    P = synth.cameras(cfg)
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    dev = torch.device("cuda", 0)
    eng = dp.Engine(dp.Options(), device=0)
    planes = torch.empty((V, H, W), dtype=torch.int32, device="cuda")
    for v in range(V):
        N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(cfg), N.ptr(P), v, planes[v].data_ptr(),
                                             stream.cuda_stream), eng.handle)
    torch.cuda.synchronize()
    eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
    seeds = synth.seeds(cfg, P)
    eng.set_fast_options(dp.FastOptions(densify=1 if a.mode == "fast" else 0))
    rec = dp.PATCH_DTYPE.itemsize
    res = []
    for rep in range(a.reps):
        ph = {"partition": 0.0, "refine": 0.0, "compact": 0.0, "commit": 0.0}
        buf = torch.empty(8 << 20, dtype=torch.uint8, device=dev)
        acc = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
        comp = torch.empty(8 << 20, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        t_all = time.perf_counter()
        gen = eng.densify_begin(seeds)
        gens = 0
        while gen.items > 0:
            gens += 1
            t = time.perf_counter()
            d_order, counts, _ = eng.densify_partition_device(gen, 1, 64)
            ph["partition"] += time.perf_counter() - t
            n = int(counts[0])
            need = n * gen.per_item
            if need * rec > buf.numel():
                buf = torch.empty(need * rec + need * rec // 4, dtype=torch.uint8, device=dev)
                comp = torch.empty(need * rec + need * rec // 4, dtype=torch.uint8, device=dev)
                acc = torch.empty(need + need // 4, dtype=torch.uint8, device=dev)
            t = time.perf_counter()
            eng.densify_refine_items_device(gen, d_order, n, buf.data_ptr(), acc.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            ph["refine"] += time.perf_counter() - t
            t = time.perf_counter()
            nacc = eng.densify_compact_accepted_device(gen, d_order, n, buf.data_ptr(), acc.data_ptr(),
                                                       comp.data_ptr(), stream.cuda_stream)
            ph["compact"] += time.perf_counter() - t
            t = time.perf_counter()
            gen = eng.densify_commit_accepted_device(gen, comp.data_ptr(), nacc, stream.cuda_stream)
            torch.cuda.synchronize()
            ph["commit"] += time.perf_counter() - t
        wall = time.perf_counter() - t_all
        _, st = eng.densify_result()
        res.append({"wall_ms": round(wall * 1e3, 2), "generations": gens, "patches": int(st["patches"]),
                    **{k + "_ms": round(v * 1e3, 2) for k, v in ph.items()}})
    print(json.dumps({"config": a.config, "mode": a.mode, "reps": res}))


if __name__ == "__main__":
    main()

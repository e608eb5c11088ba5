#!/usr/bin/env python3
"""The config-4 densify of bench.py's scaling_leg at one rank, for a
rocprofv3 kernel trace: where the non-refine time of a densify goes (kernel
time of the partition / compaction / organizer kernels vs GPU idle between
launches).  --protocol device: the device-resident generations (dp_densify
/ dp_densify_run); slots: the multi-rank slot protocol at one rank
(dist.densify_partitioned_device one_rank_exchange); hybrid8: that protocol
on the generations an 8-rank run partitions, the rest replicated.  Prints one JSON line
per repetition: wall ms, refine ms (events), generations.

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/densify_trace.py --mode fast
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import densepoints_amd as dp  # noqa: E402
from densepoints_amd import _native as N  # noqa: E402
from densepoints_amd import dist as D  # noqa: E402
from densepoints_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4_64view_4k")
    ap.add_argument("--mode", default="fast")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--protocol", choices=["device", "slots", "hybrid8"], default="device")
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
    def run(eng, seeds, dist, dev):
        # hybrid8: the slot protocol on the generations an 8-rank run partitions, the rest replicated
        return D.densify_partitioned_device(eng, seeds, dist, dev, one_rank_exchange=a.protocol != "device",
                                            replicate_below={"slots": 0, "hybrid8": D.replicate_below_default(8)}
                                            .get(a.protocol))

    for rep in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got, st = run(eng, seeds, None, dev)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"rep": rep, "mode": a.mode, "protocol": a.protocol, "wall_ms": round(wall, 2),
                          "refine_ms": round(st["refine_ms"], 2), "non_refine_ms": round(wall - st["refine_ms"], 2),
                          "generations": int(st["generations"]), "patches": int(st["patches"]),
                          "phase_ms": st["phase_ms"]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

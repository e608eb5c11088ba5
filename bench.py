#!/usr/bin/env python3
"""Headline benchmark: Mpatches/sec through the fused NCC evaluate + refine +
filter kernel (BASELINE.json metric).

N = 1 (the driver's plain `python bench.py`): the 32-view 4K synthetic scene
(BASELINE config 3, the HBM-roofline run).  One step = one batch of expansion
candidates through the HIP kernel -- the reference's hot loop,
Expand::ExpandPatch (methods/pmvs/expand.cpp:103-143): each parent patch spawns
4 children (+-x, +-y at 8 px in its reference view), each child is Nelder-Mead
refined at n = 11 on the parent's visible set, then InitRelatedImages and the
NCC filter run -- with inputs resident in HBM.  Parents are the synthetic seeds
after the reference's seed stage (Seed::FilterPatches + OptimizePatches at
n = 16, run once untimed), so the children look exactly like the ones the BFS
produces.

N > 1 (one process per GPU, RCCL over xGMI): `value` is the SAME workload as
at N = 1 -- every rank refines its own fixed-size batch of config-3 expansion
candidates (candidates are independent, SURVEY 8e: no data-path collective),
value = all ranks' candidates / max-over-ranks time, "scaling": "weak".  So the
driver's 1/2/4/8 curve built from `value` divides like quantities.
`python bench.py --gpus N` launches the N ranks itself (torch.distributed.run,
started before anything touches the GPU) when it is not already under a
launcher; every rank checks that its world size equals --gpus.

`scaling_leg` (every N, N = 1 included): BASELINE config 4 (64 views 4K,
"reference-cell shard across 8 x MI355X with RCCL all-gather of accepted
patches").  One step = one whole densify (PMVS::Run minus matching,
pmvs.cpp:22-43) with every BFS generation partitioned by reference-view
super-tile over the ranks (dist.densify_partitioned_device: device partition,
refine of the rank's items, ONE RCCL all-gather of the accepted candidates,
replicated organizer commit); rate = every candidate refined (seed stage +
expansions) over the max-over-ranks wall time -- strong scaling, the same
densify at every N, under the same key at every N.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=None, help="default: cfg3_32view_4k (the headline at every N)")
    ap.add_argument("--densify-steps", type=int, default=2,
                    help="timed whole-densify repetitions of scaling_leg (config 4, every N)")
    ap.add_argument("--batch", type=int, default=262144, help="expansion candidates per step per GPU")
    ap.add_argument("--cell", type=int, default=11)
    ap.add_argument("--cpu-parents", type=int, default=5000,
                    help="CPU baseline sample: first N parents (4N candidates) of the batch")
    ap.add_argument("--cpu-parents-1thread", type=int, default=5000,
                    help="single-thread CPU baseline sample (a prefix of the same sample)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every usable host core")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-densify", action="store_true", help="skip the informational end-to-end densify")
    ap.add_argument("--no-seeds", action="store_true", help="skip the informational seed generation")
    ap.add_argument("--knn-rows", type=int, default=40000, help="descriptors per side of the kNN kernel timing")
    ap.add_argument("--mode", choices=["parity", "fast"], default="parity",
                    help="headline refine: parity (the reference's Nelder-Mead, bit-exact) or the performance "
                         "mode (LDS-staged fp16 gray tiles + fused CG, dp_fast_options)")
    ap.add_argument("--fast-cells", default="7,11", help="windows of the informational perf_mode sub-object")
    ap.add_argument("--fast-budgets", default="", help="tile budgets (bytes) to sweep in perf_mode; default: the "
                                                         "FastOptions default")
    ap.add_argument("--fast-iters", type=int, default=None, help="performance-mode CG iterations (default: FastOptions)")
    ap.add_argument("--fast-margins", default="", help="tile margins (px) to sweep in perf_mode")
    ap.add_argument("--fast-gradients", default="0,1",
                    help="perf_mode refine specs: 0 = forward differences (v3, the default), 1 = the analytic "
                         "gradient (v4; keys *_an)")
    ap.add_argument("--fast-extra-max-views", default="6",
                    help="perf_mode speed points: the default spec with the refine's view cap lowered to each "
                         "value (keys n*_mv<k>, headline parents)")
    ap.add_argument("--no-fast", action="store_true", help="skip the perf_mode sub-object")
    ap.add_argument("--seed-stride", type=float, default=32.0, help="synthetic seed grid stride (px)")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="side file for the full result (event arrays, every perf_mode run, partition probes, seed "
                         "generation); stdout carries only the compact line (compact())")
    return ap.parse_args()


STDOUT_LIMIT = 4096  # the driver parses the last stdout line; r05's 18,962-byte line was not parsed


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def compact(result: dict, detail_path: str | None = None) -> dict:
    """The ONE stdout line: the contract keys, the roofline and cpu_baseline
    with their attesting fields, and a one-number summary per informational
    leg.  Everything else stays in the side file (`--detail`).  Must serialise
    to <= STDOUT_LIMIT bytes (tests/test_bench_line_cpu.py)."""
    out = _pick(result, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                         "scaling", "vs_baseline", "dtype", "data"))
    cfg = result.get("config", {})
    out["config"] = _pick(cfg, ("workload", "views", "width", "height", "cell", "batch_per_gpu", "parallelism"))
    roof = result.get("roofline", {})
    out["roofline"] = _pick(roof, ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                   "bytes_per_launch_algorithmic", "profiled_launch_ms", "profile_over_events",
                                   "live_over_profiled_events", "profile_stale"))
    out["roofline"]["kernel_ms_per_launch"] = result.get("kernel_ms_per_launch")
    if "valu" in roof:
        out["roofline"]["valu_frac"] = roof["valu"].get("frac")
    out["E_mean_evals_per_patch"] = result.get("E_mean_evals_per_patch")
    out["Mevals_per_s"] = result.get("Mevals_per_s")
    if "cpu_baseline" in result:
        out["cpu_baseline"] = _pick(result["cpu_baseline"], ("value", "unit", "cores", "kind", "sample",
                                                             "value_1thread", "parity_bit_exact_on_sample"))
    pm = result.get("perf_mode")
    if pm:
        s = {}
        for k, v in pm.items():
            if isinstance(v, dict) and "Mpatches_per_s" in v and not k.endswith("_fast_seeds") and "_an" not in k:
                s[k] = {"Mpatches_per_s": v["Mpatches_per_s"], "frac": v["roofline"]["frac"],
                        "median_abs_dz": round(v["quality"].get("median_abs_dz", float("nan")), 5)}
                if "cpu_baseline" in v:
                    s[k]["cpu_exact"] = v["cpu_baseline"]["parity_bit_exact_on_sample"]
        out["perf_mode"] = s
    for k in ("densify_e2e", "densify_e2e_fast"):
        if k in result:
            out[k] = _pick(result[k], ("patches", "generations", "wall_s", "host_waits"))
    sl = result.get("scaling_leg")
    if sl:
        out["scaling_leg"] = {"n_gpus": sl.get("n_gpus"), "scaling": sl.get("scaling")}
        for m in ("parity", "fast", "fast_slots", "fast_hybrid8"):
            if m in sl:
                out["scaling_leg"][m] = _pick(sl[m], ("Mpatches_per_s", "ms_per_densify", "non_refine_ms",
                                                      "ranks_store_equal", "store_crc32"))
    sg = result.get("seed_generation")
    if sg:
        out["seed_generation"] = {"total_ms": sg.get("total_ms"), "points": sg.get("points"),
                                  "knn_frac": sg.get("knn_kernel", {}).get("roofline", {}).get("frac")}
    out["lib_sha256"] = result.get("lib_sha256")
    if detail_path:
        out["detail"] = os.path.relpath(detail_path, ROOT) if detail_path.startswith(ROOT) else detail_path
    return out


def emit(result: dict, detail_path: str | None) -> str:
    """Write the full result to the side file and print the compact line
    (the last stdout line, <= STDOUT_LIMIT bytes)."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(detail_path) or ".", exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(result, f, indent=1)
        except OSError as e:
            print(f"bench: could not write {detail_path}: {e}", file=sys.stderr)
            detail_path = None
    c = compact(result, detail_path)
    line = json.dumps(c, separators=(",", ":"))
    # never exceed the limit: shed informational legs (they stay in the side file)
    for k in ("seed_generation", "densify_e2e", "densify_e2e_fast", "perf_mode", "scaling_leg"):
        if len(line) <= STDOUT_LIMIT:
            break
        c.pop(k, None)
        line = json.dumps(c, separators=(",", ":"))
    print(line, flush=True)
    return line


def launch_ranks(args) -> int:
    """`bench.py --gpus N` outside a launcher: start N ranks of this script
    with torch.distributed.run (127.0.0.1 rendezvous on a free port) as a child
    process -- nothing here has touched the GPU -- and return its exit code.
    Rank 0 prints the JSON line; a failing rank fails the launcher."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    print("bench: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def lib_stamp(path: str) -> str:
    """sha256 (16 hex digits) of the loaded libdensepoints.so: profiles/ record
    it, and bench attaches a profile's counters only to the library they were
    measured on (the build is deterministic: same sources + flags, same bytes)."""
    import hashlib

    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    import densepoints_amd as dp
    from densepoints_amd import _native as N
    from densepoints_amd import dist as D
    from densepoints_amd import synth

    rank, world, local = D.env()
    if world != args.gpus:
        raise SystemExit(f"bench: world size {world} != --gpus {args.gpus}")
    if args.config is None:
        args.config = "cfg3_32view_4k"
    # rehearsal knobs for a 1-GPU box (never set by the driver): DP_BENCH_BACKEND=gloo
    # and DP_BENCH_ONE_DEVICE=1 run N ranks on cuda:0 over gloo
    if os.environ.get("DP_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("DP_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    # RCCL over xGMI ("nccl" on ROCm): barrier + max-over-ranks time only
    dist = D.init(backend, torch.device("cuda", local))
    coll_dev = torch.device("cuda", local) if backend == "nccl" else None

    cfg = synth.named(args.config, seed_stride_px=args.seed_stride)
    V, W, H = cfg.n_views, cfg.width, cfg.height
    P = synth.cameras(cfg)
    eng = dp.Engine(dp.Options(), device=local)
    stream = torch.cuda.Stream()  # a real (non-NULL) stream shared by torch and the library
    torch.cuda.set_stream(stream)
    # render every view straight into HBM as BGRA8 planes (replicated per GPU)
    # one pool (V x H x W): every plane within 4 GiB of the first -> narrow 32-bit tap offsets
    planes = torch.empty((V, H, W), dtype=torch.int32, device="cuda")
    for v in range(V):
        N.check(N.lib.dp_synth_render_device(eng.handle, __import__("ctypes").byref(cfg), N.ptr(P), v,
                                             planes[v].data_ptr(), stream.cuda_stream), eng.handle)
    torch.cuda.synchronize()
    eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
    # image ingest: the config's pyramid (device cv::pyrDown, untimed setup); the
    # parity patch loop samples level 0 like the reference
    levels = synth.PYRAMID_LEVELS.get(args.config, 1)
    torch.cuda.synchronize()
    tp = time.perf_counter()
    eng.build_pyramid(levels)
    pyr_s = time.perf_counter() - tp
    dims = [eng.level_info(l, 0)[:2] for l in range(levels)]
    pyr_bytes = sum(4.0 * V * (dims[l][0] * dims[l][1] + dims[l + 1][0] * dims[l + 1][1]) for l in range(levels - 1))

    seeds = synth.seeds(cfg, P)
    # seed stage once (untimed): FilterPatches + OptimizePatches at n = 16
    seed_p = eng.seeds_to_patches(seeds)
    raw_seed_p = seed_p.copy()
    d_seed = torch.from_numpy(seed_p.view(np.uint8).copy()).to("cuda")
    d_ok = torch.empty(len(seed_p), dtype=torch.uint8, device="cuda")
    eng.refine_device(d_seed.data_ptr(), len(seed_p), 16, N.MODE_SEED, d_ok.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    seed_p = np.frombuffer(d_seed.cpu().numpy().tobytes(), dtype=N.PATCH_DTYPE)
    parents_all = seed_p[d_ok.cpu().numpy() == 1]
    # this rank's shard of parents (weak scaling; wraps around the list)
    B = args.batch - args.batch % 4
    NP = B // 4
    idx = D.weak_shard(len(parents_all), NP, rank)
    parents = np.ascontiguousarray(parents_all[idx])
    d_parents = torch.from_numpy(parents.view(np.uint8).copy()).to("cuda")
    work = torch.empty(B * N.PATCH_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    accept = torch.empty(B, dtype=torch.uint8, device="cuda")

    fast = args.mode == "fast"
    if fast:
        eng.set_options(dp.Options(expand_cell_size=args.cell))
        fo = dp.FastOptions()
        if args.fast_budgets:
            fo.tile_budget = int(args.fast_budgets.split(",")[0])
        if args.fast_iters is not None:
            fo.iters = args.fast_iters
        eng.set_fast_options(fo)
    expand_fn = eng.fast_expand_device if fast else eng.expand_device

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        expand_fn(d_parents.data_ptr(), NP, work.data_ptr(), accept.data_ptr(), stream.cuda_stream)
        if ev:
            ev[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kern_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        step(ev)
        kern_ms.append(ev)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-launch kernel time: HIP events recorded on the stream the kernel runs on
    step_ms = [a.elapsed_time(b) for a, b in kern_ms]
    launch_ms = float(np.mean(step_ms))
    lib_last_ms = eng.last_kernel_ms()  # the library's own events around the last launch
    elapsed = D.max_over_ranks(elapsed, dist, coll_dev)

    out = np.frombuffer(work.cpu().numpy().tobytes(), dtype=N.PATCH_DTYPE)
    acc = accept.cpu().numpy()
    evals = out["evals"].astype(np.float64)
    pvis = np.array([bin(int(m[0])).count("1") + bin(int(m[1])).count("1") for m in parents["vis"]])
    nvis = np.repeat(pvis, 4)  # children refine on the parent's visible set
    if os.environ.get("DP_BENCH_VIS_HIST") == "1":
        # diagnostic: objective evaluations by the parent's visible-view count
        print("visible-view histogram (evaluations):", np.bincount(nvis, weights=evals).astype(np.int64).tolist(),
              file=sys.stderr)
    n1 = args.cell + 1
    if fast:
        # algorithmic bytes with fp16 texels: sum over evaluations of
        # the staged views sampled (device-counted) * (n+1)^2 * 2 B + 128 B record
        fst = eng.fast_last_stats()
        bytes_alg = float(fst["view_evals"] * n1 * n1 * 2 + 128 * B)
    else:
        # algorithmic bytes: E * sum_v (n+1)^2 * 4 B (BGRA8) + 128 B record in/out
        bytes_alg = float((evals * nvis * n1 * n1 * 4).sum() + 128 * B)
    achieved = bytes_alg / (launch_ms * 1e-3) / 1e9  # GB/s of the dominant kernel
    peak = 8000.0
    total_patches = B * args.steps * world
    value = total_patches / elapsed / 1e6

    result = {
        "metric": "Mpatches/sec (NCC eval+refine)",
        "value": round(value, 4),
        "unit": "Mpatches/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "scaling_note": "value at every N is the config-3 refine batch, weak-scaled (N x batch_per_gpu "
                        "candidates, no data-path collective); BASELINE.md's config-4 strong-scaling densify "
                        "(super-tile partition + RCCL all-gather) is scaling_leg.{parity,fast}.Mpatches_per_s",
        "vs_baseline": None,
        "dtype": "u8 gray texels in LDS (fp16 planes), fp32 sampling, int32 moments, fp64 CG" if fast else
                 "u8 texels, fp64 geometry, int32 moments",
        "data": "synthetic (deterministic 3x3-facet heightfield, rendered on device)",
        "config": {
            "workload": f"{args.config}: {V} views {W}x{H}, {B} expansion candidates/GPU/step "
                        f"({NP} refined seed parents x 4 directions), n={args.cell}, "
                        + ("performance mode: LDS-staged fp16 gray tiles + fused CG + InitRelatedImages + fast "
                           "filter" if fast else "Nelder-Mead + InitRelatedImages + NCC filter (parity mode)"),
            "views": V,
            "width": W,
            "height": H,
            "cell": args.cell,
            "batch_per_gpu": B,
            "parallelism": f"dp{world} (candidate shards, no data-path collective)",
        },
        "pyramid": {"levels": levels, "dims": dims, "build_ms_wall": round(pyr_s * 1e3, 3),
                    "bytes_algorithmic": pyr_bytes, "GBps_wall": round(pyr_bytes / max(pyr_s, 1e-9) / 1e9, 1)},
        "E_mean_evals_per_patch": round(float(evals.mean()), 3),
        "mean_visible_views": round(float(nvis.mean()), 3),
        "accept_rate": round(float(acc.mean()), 4),
        "kernel_ms_per_launch": round(launch_ms, 3),
        "kernel_ms_events": [round(x, 3) for x in step_ms],
        "kernel_ms_last_lib_events": round(lib_last_ms, 3),
        "Mevals_per_s": round(float(evals.sum()) * world * args.steps / elapsed / 1e6, 3),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": peak,
            "unit": "GB/s",
            "frac": round(achieved / peak, 4),
            "traffic": None,
            "bytes_per_launch_algorithmic": bytes_alg,
        },
    }
    if fast:
        result["fast_stats"] = {k: int(v) for k, v in fst.items()}
        result["roofline"]["bytes_per_launch_compulsory"] = float(fst["staged_bytes"] + 128 * B)
        result["quality"] = quality(cfg, out, acc)
    # the informational legs and the CPU baseline run at N = 1 only (at N > 1 the
    # partitioned densify legs below are the report)
    solo = world == 1
    if solo and not fast and not args.no_fast:
        result["perf_mode"] = perf_mode(eng, args, cfg, stream, d_parents, NP, work, accept, out, acc, parents, P,
                                        planes, raw_seed_p)
    if solo and not args.no_densify and not fast:
        # informational: the full PMVS::Run minus matching (dp_densify) on the same scene, untimed by the
        # contract; wall_s of the second (warm) densify, the store as a view of the pinned result buffer
        eng.densify(seeds, copy=False)
        t0 = time.perf_counter()
        dpat, dst = eng.densify(seeds, copy=False)
        wall = time.perf_counter() - t0
        result["densify_e2e"] = {"seeds": int(dst["seeds_in"]), "seed_patches": int(dst["seed_patches"]),
                                 "patches": int(dst["patches"]), "store_crc32": f"{zlib.crc32(dpat.tobytes()):08x}", "candidates": int(dst["candidates"]),
                                 "generations": int(dst["generations"]), "evals": int(dst["evals"]),
                                 "refine_ms": round(dst["refine_ms"], 1), "wall_s": round(wall, 3)}
        # informational: the same densify with the performance-mode refine
        # (dp_fast_options.densify: seed stage at n = 16 and expansions at n = 11)
        eng.set_fast_options(dp.FastOptions(densify=1))
        eng.densify(seeds, copy=False)
        t0 = time.perf_counter()
        fpat, fst = eng.densify(seeds, copy=False)
        wall = time.perf_counter() - t0
        eng.set_fast_options(dp.FastOptions())
        result["densify_e2e_fast"] = {"seed_patches": int(fst["seed_patches"]), "patches": int(fst["patches"]),
                                      "store_crc32": f"{zlib.crc32(fpat.tobytes()):08x}",
                                      "candidates": int(fst["candidates"]), "generations": int(fst["generations"]),
                                      "evals": int(fst["evals"]), "refine_ms": round(fst["refine_ms"], 1),
                                      "wall_s": round(wall, 3),
                                      "Mpatches_per_s_refine": round(int(fst["candidates"]) / max(fst["refine_ms"], 1e-9)
                                                                     / 1e3, 3)}
    result["scaling_curve"] = ("value: weak scaling of the config-3 refine batch (%d candidates per rank, no "
                               "data-path collective); scaling_leg.<mode>.Mpatches_per_s: strong scaling of the "
                               "config-4 partitioned densify (the same densify at every N)" % B)
    if not args.no_densify and not fast:
        result["scaling_leg"] = scaling_leg(args, stream, dist, coll_dev, torch.device("cuda", local))
    if solo and not args.no_seeds:
        result["seed_generation"] = seed_generation(eng, args)
    st = np.zeros(8, dtype=np.uint64)
    if N.lib.dp_debug_stamps(N.ptr(st)) == 0:  # -DDP_STAMPS diagnostic builds only
        tot = float(st[7]) or 1.0
        result["stamps_share"] = {k: round(float(st[i]) / tot, 4) for i, k in
                                  enumerate(["corners_maps", "view_passes", "sync", "ncc_finish"])}
        result["stamps_share"]["rest_nm_geometry"] = round(1.0 - sum(result["stamps_share"].values()), 4)
    lib_sha = lib_stamp(N.LIB_PATH)
    result["lib_sha256"] = lib_sha
    prof = profiled("parity" if not fast else "fast%d" % args.cell,
                    "refine_kernel<4, 2," if not fast else fast_kernel_tag(args.cell), B, lib_sha)
    if prof:
        attach_profile(result["roofline"], prof, B, launch_ms)

    if solo and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, cfg, P, planes, parents, out, fo if fast else None)
    if rank == 0:
        emit(result, args.detail)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


def partitioned_leg(eng, seeds, dist, coll_dev, dev, steps, warmup, fast, exchange=False, probe_worlds=(2, 8),
                    replicate_below=None):
    """`steps` whole densifies with every generation partitioned over the ranks
    (dist.densify_partitioned_device), after `warmup` untimed ones, bracketed by
    barrier + synchronize; rate = candidates refined (seed stage + expansions)
    per max-over-ranks second.  exchange: the multi-rank slot protocol even at
    one rank (its per-generation cost is what every rank of an N-rank run pays)."""
    import functools

    import densepoints_amd as dp
    from densepoints_amd import dist as D

    eng.set_fast_options(dp.FastOptions(densify=1 if fast else 0))
    # the store comes back as a view of the library's pinned result buffer (the
    # C ABI's *out contract), consumed before the next densify
    run = functools.partial(D.densify_partitioned_device, one_rank_exchange=exchange, copy_result=False,
                            replicate_below=replicate_below)
    probe = None
    for i in range(warmup):
        # the untimed warm-up also computes the partitions world sizes 2 and 8
        # would use on the same generations (statistics only)
        _, wst = run(eng, seeds, dist, dev, probe_worlds=probe_worlds if i == 0 else ())
        probe = probe or wst.get("partition_probe")
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        got, st = run(eng, seeds, dist, dev)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = D.max_over_ranks(time.perf_counter() - t0, dist, coll_dev)
    eng.set_fast_options(dp.FastOptions())
    world = dist.get_world_size() if dist else 1
    # every rank's replicated store must be the same bytes (checked after the timed region)
    crc = zlib.crc32(got.tobytes())
    crcs = [crc]
    if dist:
        t = torch.tensor([crc], dtype=torch.int64, device=coll_dev)
        allt = torch.empty(world, dtype=torch.int64, device=coll_dev)
        dist.all_gather_into_tensor(allt, t)
        crcs = [int(x) for x in allt.tolist()]
    # the visibility filter after the last generation (PMVS::FilterPatches,
    # pmvs.h:27, spec in densepoints.h): the store is replicated, so rank 0
    # filters it (informational, outside the timed region)
    vf = None
    if not dist or dist.get_rank() == 0:
        torch.cuda.synchronize()
        tf = time.perf_counter()
        keep = eng.filter_patches(np.ascontiguousarray(got))
        vf = {"patches_in": int(len(got)), "kept": int(keep.sum()),
              "ms_wall_host_arrays": round((time.perf_counter() - tf) * 1e3, 2)}
    cands = int(st["seeds_in"]) + int(st["candidates"])
    parts = st["partition"]
    gb = st["gathered_bytes"]
    return {"ranks": world, "mode": "performance" if fast else "parity", "steps": steps,
            "Mpatches_per_s": round(steps * cands / wall / 1e6, 4), "ms_per_densify": round(wall / steps * 1e3, 3),
            "candidates_per_densify": cands, "patches": int(st["patches"]), "seed_patches": int(st["seed_patches"]),
            "store_crc32": f"{crc:08x}", "ranks_store_equal": len(set(crcs)) == 1,
            "generations": int(st["generations"]), "evals": int(st["evals"]),
            "refine_ms_max_rank": round(st["refine_ms"], 1),
            # everything but the refine kernels (partition, compaction, exchange,
            # replicated organizer commit, host waits): the part that does not
            # shrink with the ranks
            "non_refine_ms": round(wall / steps * 1e3 - st["refine_ms"], 2),
            "protocol": "slots" if (world > 1 or exchange) else "dp_densify (device-resident generations)",
            "replicate_below": st.get("replicate_below"), "replicated_calls": st.get("replicated_calls"),
            # host time per phase of the last densify (each phase ends in a host sync;
            # refine_compact includes this rank's refine kernels), max over ranks
            "phase_ms_max_rank": {k: round(D.max_over_ranks(v, dist, coll_dev), 2)
                                  for k, v in st["phase_ms"].items()},
            "accepted_exchanged": int(sum(st["accepted"])),
            "gathered_MB_total": round(sum(gb) / 1e6, 3), "gathered_MB_max_generation": round(max(gb) / 1e6, 3),
            "gathered_MB_per_generation_mean": round(sum(gb) / len(gb) / 1e6, 4),
            "partition": partition_summary(parts, world),
            "partition_probe": {str(w): partition_summary(p, w) for w, p in (probe or {}).items()},
            "collective": "all_gather_into_tensor of the accepted candidates' 80-B records (+ 8-B counts), " +
                          ("RCCL over xGMI" if dist is not None and dist.get_backend() == "nccl" else
                           "none (one rank)" if dist is None else dist.get_backend()),
            "visibility_filter": vf}


def partition_summary(parts, world):
    """Per-densify summary of the super-tile partition records (items, largest
    share, items in tiles split between ranks, tiles) of every generation."""
    items = sum(p[0] for p in parts)
    big = [p for p in parts if p[0] >= 64 * world]  # generations large enough to share evenly
    return {"world": world, "generations": len(parts), "items": items,
            "tile_partitioned_item_frac": round(1.0 - sum(p[2] for p in parts) / max(items, 1), 5),
            # largest rank share / mean share over the generations with >= 64 items
            # per rank; a generation of fewer items than ranks has share `world`
            # whatever the partition, so the all-generation maximum is reported apart
            "max_share_vs_mean": round(max(p[1] * world / p[0] for p in big), 4) if big else None,
            "max_share_generations": len(big),
            "max_share_vs_mean_any_generation": round(max((p[1] * world / p[0]) for p in parts if p[0] > 0), 4)
            if parts else None,
            "item_weighted_share_vs_mean": round(sum(p[1] * world for p in parts) / max(items, 1), 4),
            "tiles_mean": round(sum(p[3] for p in parts) / max(len(parts), 1), 1)}


def scaling_leg(args, stream, dist, coll_dev, dev):
    """The strong-scaling series, under this key at every N (N = 1 included):
    BASELINE config 4 (64 views 4K), the whole densify with every large
    generation partitioned by reference-view super-tile over the ranks and the
    accepted candidates all-gathered (RCCL over xGMI), the small ones
    replicated device-resident (dist.replicate_below_default), both refine
    modes."""
    import ctypes

    import densepoints_amd as dp
    from densepoints_amd import _native as N
    from densepoints_amd import dist as D
    from densepoints_amd import synth

    cfg = synth.named("cfg4_64view_4k")
    P = synth.cameras(cfg)
    V, W, H = cfg.n_views, cfg.width, cfg.height
    world = dist.get_world_size() if dist else 1
    with dp.Engine(dp.Options(expand_cell_size=args.cell), device=dev.index) as eng:
        planes = torch.empty((V, H, W), dtype=torch.int32, device=dev)
        for v in range(V):
            N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(cfg), N.ptr(P), v, planes[v].data_ptr(),
                                                 stream.cuda_stream), eng.handle)
        torch.cuda.synchronize()
        eng.set_views_device(P, [W] * V, [H] * V, [W] * V, [p.data_ptr() for p in planes])
        seeds = synth.seeds(cfg, P)
        out = {m: partitioned_leg(eng, seeds, dist, coll_dev, dev, args.densify_steps, 1, m == "fast")
               for m in ("parity", "fast")}
        if world == 1:
            # the multi-rank protocol's per-generation cost at one rank (partition,
            # slot compaction, scatter, replicated commit, one wait per generation):
            # what bounds the N-rank strong scaling beside refine_ms / N
            out["fast_slots"] = partitioned_leg(eng, seeds, dist, coll_dev, dev, args.densify_steps, 1, True,
                                                exchange=True, probe_worlds=(), replicate_below=0)
            # the hybrid an 8-rank run uses (generations below 8,192 items on every
            # rank, device-resident): the per-rank protocol cost at N = 8 beside
            # refine_ms / 8 of the partitioned generations
            out["fast_hybrid8"] = partitioned_leg(eng, seeds, dist, coll_dev, dev, args.densify_steps, 1, True,
                                                  exchange=True, probe_worlds=(),
                                                  replicate_below=D.replicate_below_default(8))
        out["workload"] = (f"cfg4_64view_4k: {V} views {W}x{H}, one step = the whole densify (PMVS::Run minus "
                           f"matching) of {len(seeds)} seed points, every BFS generation partitioned by "
                           f"reference-view super-tile over {world} rank(s), accepted candidates all-gathered")
        out["scaling"] = "strong"
        out["n_gpus"] = world
        del planes
    return out


def seed_generation(eng, args):
    """Informational (not the headline): Matcher::GenerateSeeds on the bench's
    views with the reference's settings, and the brute-force Hamming knnMatch
    kernel at the reference's ORB budget (40000 x 40000 descriptors, one view
    pair) against the dense i8 MFMA peak.  The oracle's knnMatch on a bounded
    sample is the CPU baseline of that kernel."""
    from densepoints_amd import matcher as M

    m = M.Matcher(eng)
    m.generate_seeds()  # first call allocates
    t0 = time.perf_counter()
    m.generate_seeds()
    wall = time.perf_counter() - t0
    st = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in m.stats.items()}
    rng = np.random.default_rng(7)
    n = args.knn_rows
    q = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    ms = []
    for _ in range(3):
        M.knn_match(eng, q, t)
        ms.append(eng.last_kernel_ms())  # HIP events around the kernel, on its stream
    kms = float(np.mean(ms[1:]))
    ops = 2.0 * 256 * n * n  # i8 MACs of the Hamming GEMM, x2
    peak = 5000.0  # dense i8 MFMA TOPS: 2x the ~2.5 PF dense bf16 rate (MI355X_MICROARCH.md, Matrix cores)
    out = {"settings": "reference defaults (ORB 40000 features, 8 levels, FAST 20, 16 px cells x 4, ratio 0.7, "
                       "1.5 px epipolar)", "wall_s": round(wall, 4), **st,
           "knn_kernel": {"rows": n, "kernel_ms": round(kms, 4), "Gpairs_per_s": round(n * n / kms / 1e6, 1),
                          "roofline": {"bound": "mfma", "achieved": round(ops / kms / 1e9, 1), "peak": peak,
                                       "unit": "TOPS (i8)", "frac": round(ops / kms / 1e9 / peak, 4)}}}
    # DetectorType::AKAZE (matcher.cpp:56-60, 166-170) with AKAZE::create()'s
    # defaults, and the 512-bit kNN kernel at the same row count
    ma = M.Matcher(eng, M.MatcherOptions(detector_type=M.DETECTOR_AKAZE))
    ma.generate_seeds()
    t0 = time.perf_counter()
    ma.generate_seeds()
    wall_a = time.perf_counter() - t0
    q64 = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
    t64 = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
    ms = []
    for _ in range(3):
        M.knn_match(eng, q64, t64, width=64)
        ms.append(eng.last_kernel_ms())
    kms64 = float(np.mean(ms[1:]))
    ops64 = 2.0 * 512 * n * n
    out["akaze"] = {"settings": "AKAZE::create() defaults (MLDB 486 bits, threshold 0.001, 4 octaves x 4 "
                                "sublevels, PM_G2), the same cells / ratio / epipolar settings",
                    "wall_s": round(wall_a, 4),
                    **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in ma.stats.items()},
                    "knn_kernel_512bit": {"rows": n, "kernel_ms": round(kms64, 4),
                                          "Gpairs_per_s": round(n * n / kms64 / 1e6, 1),
                                          "roofline": {"bound": "mfma", "achieved": round(ops64 / kms64 / 1e9, 1),
                                                       "peak": peak, "unit": "TOPS (i8)",
                                                       "frac": round(ops64 / kms64 / 1e9 / peak, 4)}}}
    if not args.no_cpu:
        from oracle import pyoracle as orc

        s = 3000
        t0 = time.perf_counter()
        orc.knn_match(q[:s], t[:s])
        ct = time.perf_counter() - t0
        out["knn_kernel"]["cpu_baseline"] = {"Gpairs_per_s": round(s * s / ct / 1e9, 4), "cores": 1, "kind": "port",
                                             "sample": f"oracle knnMatch {s} x {s}, {ct:.2f} s"}
    return out


def quality(cfg, kids, acc):
    """Median |z - z_true| (world units) and normal error (deg) of the accepted
    children against the synthetic ground truth (dp_synth_surface)."""
    from densepoints_amd import synth

    k = kids[acc == 1]
    if len(k) == 0:
        return {"accepted": 0}
    z, nrm = synth.surface(cfg, k["pos"][:, :2].astype(np.float64))
    nn = k["normal"].astype(np.float64)
    nn /= np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-30)
    ang = np.degrees(np.arccos(np.clip(np.abs((nn * nrm).sum(1)), 0.0, 1.0)))
    return {"accepted": int(len(k)), "median_abs_dz": float(np.median(np.abs(k["pos"][:, 2] - z))),
            "median_normal_err_deg": round(float(np.median(ang)), 3)}


def quality_all(cfg, p):
    """quality() of every patch in p (unrefined parents, seed patches)."""
    return quality(cfg, p, np.ones(len(p), dtype=np.uint8))


def perf_mode(eng, args, cfg, stream, d_parents, NP, work, accept, parity_out, parity_acc, parents, P, planes,
              raw_seed_p):
    """Informational: the performance mode (DP_MODE_FAST_REFINE, dp_fast.hip --
    LDS-staged fp16 gray tiles, fused CG, one wavefront per candidate) per
    window size, on two parent sets: the headline's (the parity seed stage's
    survivors; keys n7, n11) and the performance pipeline's own (the seed
    stage refined in performance mode at n = 16, as dp_densify runs it with
    dp_fast_options.densify; keys n7_fast_seeds, n11_fast_seeds).  Per run:
    Mpatches/s from HIP events on the launch stream, E, the roofline on the
    algorithmic (every evaluation re-reads its windows) and compulsory (tiles
    staged once) byte models, geometry against the ground truth next to the
    parity mode's and the unrefined parents', and (headline parents) a CPU
    baseline of its spec (oracle/or_fast.c) with a bit-exact check."""
    import densepoints_amd as dp
    from densepoints_amd import _native as N
    from oracle import pyoracle as orc

    B = 4 * NP
    res = {"parity_quality_n%d" % args.cell: quality(cfg, parity_out, parity_acc)}
    # the performance pipeline's parents: raw seed patches -> fast refine at n = 16
    d_raw = torch.from_numpy(raw_seed_p.view(np.uint8).copy()).to("cuda")
    d_ok = torch.empty(len(raw_seed_p), dtype=torch.uint8, device="cuda")
    eng.set_fast_options(dp.FastOptions())
    eng.refine_device(d_raw.data_ptr(), len(raw_seed_p), 16, N.MODE_FAST_REFINE, d_ok.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    fseed = np.frombuffer(d_raw.cpu().numpy().tobytes(), dtype=N.PATCH_DTYPE)
    fpar_all = fseed[d_ok.cpu().numpy() == 1]
    fparents = np.ascontiguousarray(fpar_all[np.arange(NP) % len(fpar_all)])
    d_fparents = torch.from_numpy(fparents.view(np.uint8).copy()).to("cuda")
    res["parents_quality"] = {"raw_seed_patches": quality_all(cfg, raw_seed_p),
                              "parity_seed_stage": quality_all(cfg, parents),
                              "fast_seed_stage": quality_all(cfg, fparents)}
    # the parity mode's children of the performance pipeline's parents
    eng.set_options(dp.Options(expand_cell_size=args.cell))
    eng.expand_device(d_fparents.data_ptr(), NP, work.data_ptr(), accept.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    res["parity_quality_n%d_fast_seeds" % args.cell] = quality(
        cfg, np.frombuffer(work.cpu().numpy().tobytes(), dtype=dp.PATCH_DTYPE), accept.cpu().numpy())
    imgs = None
    budgets = [int(b) for b in args.fast_budgets.split(",") if b] or [None]
    margins = [int(b) for b in args.fast_margins.split(",") if b] or [None]
    grads = [int(x) for x in args.fast_gradients.split(",") if x]
    combos = [(int(c), b, mg, ps, gr, None) for gr in grads for ps in ("", "_fast_seeds")
              for c in args.fast_cells.split(",") if c for b in budgets for mg in margins]
    # speed points: the default spec with a smaller refine view cap (keys n*_mv<k>)
    combos += [(int(c), None, None, "", grads[0], int(mv)) for mv in args.fast_extra_max_views.split(",") if mv
               for c in args.fast_cells.split(",") if c]
    for cell, tb, mg, pset, gr, mv in combos:
        d_par = d_fparents if pset else d_parents
        fo = dp.FastOptions()
        if tb:
            fo.tile_budget = tb
        if mg is not None:
            fo.margin = mg
        if args.fast_iters is not None:
            fo.iters = args.fast_iters
        fo.gradient = gr
        if mv is not None:
            fo.max_views = mv
        eng.set_fast_options(fo)
        eng.set_options(dp.Options(expand_cell_size=cell))
        # untimed warm-up launches (the clocks settle over the first ~15 ms of a new launch shape)
        for _ in range(max(3, args.warmup)):
            eng.fast_expand_device(d_par.data_ptr(), NP, work.data_ptr(), accept.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        ms = []
        for _ in range(max(3, args.steps)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            eng.fast_expand_device(d_par.data_ptr(), NP, work.data_ptr(), accept.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            ms.append((e0, e1))
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ms]
        kms = float(np.mean(ms))
        st = eng.fast_last_stats()
        out = np.frombuffer(work.cpu().numpy().tobytes(), dtype=dp.PATCH_DTYPE)
        acc = accept.cpu().numpy()
        n1 = cell + 1
        alg = float(st["view_evals"] * n1 * n1 * 2 + 128 * B)
        comp = float(st["staged_bytes"] + 128 * B)
        r = {"Mpatches_per_s": round(B / kms / 1e3, 3), "kernel_ms_per_launch": round(kms, 3),
             "kernel_ms_events": [round(x, 3) for x in ms],
             "E_mean_evals_per_patch": round(st["evals"] / max(st["patches"], 1), 3),
             "mean_staged_views_per_eval": round(st["view_evals"] / max(st["evals"], 1), 3),
             "accept_rate": round(float(acc.mean()), 4),
             "Mevals_per_s": round(st["evals"] / kms / 1e3, 3),
             "roofline": {"bound": "hbm", "achieved": round(alg / kms / 1e6, 2), "peak": 8000.0, "unit": "GB/s",
                          "frac": round(alg / kms / 1e6 / 8000.0, 4), "traffic": None,
                          "bytes_per_launch_algorithmic": alg, "bytes_per_launch_compulsory": comp,
                          "compulsory_GBps": round(comp / kms / 1e6, 2)},
             "quality": quality(cfg, out, acc), "stats": {k: int(v) for k, v in st.items()},
             "fast_options": {k: getattr(fo, k) for k in ("iters", "margin", "tile_budget", "max_views", "gradient",
                                                          "filter_max_views")}}
        fprof = profiled("fast%d" % cell, fast_kernel_tag(cell, gr), B, lib_stamp(N.LIB_PATH)) \
            if not pset and fo.tile_budget == 6656 and fo.iters == 4 and gr == 0 and mv is None else None
        if fprof:
            attach_profile(r["roofline"], fprof, B, kms)
        if not args.no_cpu and not pset and gr == grads[0]:
            if imgs is None:
                imgs = []
                for pl in planes:
                    a = pl.cpu().numpy().view(np.uint8).reshape(cfg.height, cfg.width, 4)
                    imgs.append(np.ascontiguousarray(a[:, :, :3]))
            S = orc.Scene(P, imgs, dp.Options(expand_cell_size=cell))
            n = min(args.cpu_parents, len(parents))
            cores = args.cpu_threads or host_cores()
            t0 = time.perf_counter()
            kids, kacc = S.fast_expand(parents[:n], fo, cores)
            t = time.perf_counter() - t0
            g = out[: 4 * n]
            fields = ("pos", "normal", "ref", "vis", "cand", "score", "evals", "flags", "parent")
            r["cpu_baseline"] = {"value": round(4 * n / t / 1e6, 6), "unit": "Mpatches/s", "cores": cores,
                                 "kind": "port", "sample": f"first {n} parents ({4 * n} candidates), {t:.1f} s",
                                 "parity_bit_exact_on_sample": bool(all(kids[f].tobytes() == g[f].tobytes()
                                                                        for f in fields) and
                                                                    np.array_equal(kacc, acc[: 4 * n]))}
        res["n%d" % cell + ("_b%d" % tb if tb and len(budgets) > 1 else "") +
            ("_m%d" % mg if mg is not None and len(margins) > 1 else "") + pset + ("_an" if gr == 1 else "") +
            ("_mv%d" % mv if mv is not None else "")] = r
    eng.set_options(dp.Options(expand_cell_size=args.cell))
    eng.set_fast_options(dp.FastOptions())
    return res


def fast_kernel_tag(cell, gradient=0):
    """the performance kernel instance bench runs at this window (dp_fast.hip fast_dispatch;
    kMode 100 = the analytic-gradient refine, 6 = forward differences)"""
    mode = 100 if gradient else 6
    # a prefix of the instance name: later template parameters (build knobs) may follow
    return {7: f"fast_kernel<4, 3, true, false, 6656, {mode},",
            11: f"fast_kernel<2, 4, false, true, 6656, {mode},"}.get(cell, "?")


def profiled(workload, kernel, B, lib_sha):
    """The rocprofv3 record of `kernel` under bench workload `workload`
    (parity | fast7 | fast11) from the latest profiles/rNN/kernel_counters.json
    (tools/r04_profile.sh + tools/profile_json.py), when it was taken on this
    batch size (262,144 candidates): per-launch PMC counters and durations.
    The record carries the sha256 stamp of the library it profiled; a record
    of another library comes back with stale=True and is not attached."""
    import glob

    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "kernel_counters.json")))
    if not found or B != 4 * 65536:
        return None
    with open(found[-1]) as f:
        t = json.load(f)
    for k, v in t.get(workload, {}).items():
        if kernel in k:
            return dict(v, kernel=k, source=os.path.relpath(found[-1], ROOT),
                        stale=v.get("lib_sha256") != lib_sha)
    return None


def attach_profile(roof, prof, B, launch_ms):
    """roofline.traffic (HBM bytes per launch, 2 FETCH_SIZE + WRITE_SIZE per
    MI355X_MICROARCH.md; raw beside it) and roofline.valu: the kernel is VALU-
    issue-bound, so its second roofline is wave-instructions/s against the
    issue peak 1024 SIMDs x clock / 2 (a wave64 VALU instruction takes two
    cycles of a SIMD-32), with the profiled instructions per candidate (the
    instruction stream is deterministic for this workload) over the live launch
    time, and the profile's VALU-busy fraction, effective clock and wave-cycle
    split (issuing / waiting on a dependency or pipe / parked on s_waitcnt).
    Only a profile of the loaded library is attached (roofline.profile_stale
    says which case applies)."""
    roof["profile_source"] = prof["source"] + " [" + prof["kernel"] + "]"
    roof["profile_stale"] = bool(prof["stale"])
    if prof["stale"]:
        roof["profile_lib_sha256"] = prof.get("lib_sha256")
        return
    roof["profiled_launch_ms"] = round(prof["trace_avg_ns"] * 1e-6, 3)
    if prof.get("events_avg_ns_same_process"):
        # attestation: the profiled run's kernel trace against that same
        # process's HIP events (profiler overhead), and this run's events
        # against the profiled run's (box / run variance)
        pe = prof["events_avg_ns_same_process"] * 1e-6
        roof["profiled_events_ms"] = round(pe, 3)
        roof["profile_over_events"] = round(prof["trace_avg_ns"] * 1e-6 / pe, 4)
        roof["live_over_profiled_events"] = round(launch_ms / pe, 4)
    if "hbm_bytes_corrected" in prof:
        # per launch (counters summed over a dispatch's instances, averaged
        # over the dispatches), and as a rate over this run's launch time
        roof["traffic"] = prof["hbm_bytes_corrected"]
        roof["traffic_raw"] = prof["hbm_bytes_raw"]
        roof["traffic_GBps"] = round(prof["hbm_bytes_corrected"] / (launch_ms * 1e-3) / 1e9, 1)
    v = prof.get("valu")
    if v:
        per = v["insts_per_launch"] / B
        ach = per * B / (launch_ms * 1e-3) / 1e9
        roof["valu"] = {"insts_per_candidate": round(per, 1), "achieved_Ginst_per_s": round(ach, 1),
                        "peak_Ginst_per_s": v["issue_peak_at_2.4GHz_Ginst_s"],
                        "frac": round(ach / v["issue_peak_at_2.4GHz_Ginst_s"], 4),
                        "effective_clock_GHz": round(v["effective_clock_GHz"], 3),
                        "frac_at_effective_clock": round(ach / v["issue_peak_at_effective_clock_Ginst_s"], 4),
                        "simd_cycles_per_valu": round(v["simd_cycles_per_valu"], 3)
                        if "simd_cycles_per_valu" in v else None,
                        "busy_frac": round(v["busy_frac"], 4)}
        if "wave_cycles" in v:
            roof["valu"]["wave_cycles"] = v["wave_cycles"]


def host_cores():
    """CPUs this process may actually run on: the affinity mask, capped by a
    cgroup v2 CPU quota when one is set (on the GPU box os.cpu_count() reports
    the whole machine, of which the job gets a share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args, cfg, P, planes, parents, gpu_out, fo=None):
    """The oracle (CPU restatement, test infrastructure) on a FIXED sample --
    the first --cpu-parents parents (4x as many candidates) of the same batch --
    timed on all of this host's usable cores and on one thread (SURVEY 8d CPU
    timing); also a bit-exact parity check of the GPU children on that sample."""
    from oracle import pyoracle as orc

    imgs = []
    for pl in planes:
        a = pl.cpu().numpy().view(np.uint8).reshape(cfg.height, cfg.width, 4)
        imgs.append(np.ascontiguousarray(a[:, :, :3]))
    import densepoints_amd as dp

    S = orc.Scene(P, imgs, dp.Options(expand_cell_size=args.cell))
    cores = args.cpu_threads or host_cores()
    n = min(args.cpu_parents, len(parents))
    fast = fo is not None
    # the performance mode's spec with the SAME options as the GPU run
    expand = (lambda par, th: S.fast_expand(par, fo, th)) if fast else S.expand
    t0 = time.perf_counter()
    kids, acc = expand(parents[:n], cores)
    t = time.perf_counter() - t0
    n1 = min(args.cpu_parents_1thread, n)
    t0 = time.perf_counter()
    expand(parents[:n1], 1)
    t1 = time.perf_counter() - t0
    g = gpu_out[: 4 * n]
    fields = ("pos", "normal", "ref", "vis", "cand", "score", "evals", "flags", "parent")
    same = all(kids[f].tobytes() == g[f].tobytes() for f in fields)
    return {
        "value": round(4 * n / t / 1e6, 6),
        "unit": "Mpatches/s",
        "cores": cores,
        "kind": "port",
        "sample": f"first {n} parents ({4 * n} candidates) of the GPU batch, same cell, {t:.1f} s on {cores} threads",
        "value_1thread": round(4 * n1 / t1 / 1e6, 6),
        "sample_1thread": f"first {n1} parents ({4 * n1} candidates), {t1:.1f} s on 1 thread",
        "host_cpus_reported": os.cpu_count(),
        "parity_bit_exact_on_sample": bool(same),
        "spec": "oracle/or_fast.c (performance mode)" if fast else "oracle/oracle.c (reference restatement)",
    }


if __name__ == "__main__":
    main()

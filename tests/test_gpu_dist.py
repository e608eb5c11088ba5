"""Generation-at-a-time densify on the GPU (dp_densify_begin / refine_items /
commit / run / result) and its multi-rank drivers (densepoints_amd.dist):
one rank equals dp_densify, also when the device-resident generations run a
few at a time or stall on small buffers; two and three ranks (processes
sharing cuda:0, gloo all-gathers) equal it too -- the replicated-claims design
of SURVEY 8e, bit for bit."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import densepoints_amd as dp
from densepoints_amd import dist as D
from densepoints_amd import synth
from densepoints_amd._native import PATCH_DTYPE

pytestmark = pytest.mark.gpu

SCENES = {
    "hf6": dict(V=6, W=320, H=240, kind=1),
    "wide70": dict(V=70, W=96, H=72, kind=1, seed_stride_px=12.0),
}


def _scene(name):
    s = dict(SCENES[name])
    cfg = synth.config(s.pop("V"), s.pop("W"), s.pop("H"), s.pop("kind"), **s)
    return synth.scene_host(cfg)


@pytest.mark.parametrize("name,max_pops", [("hf6", 0), ("hf6", 37), ("wide70", 0)])
def test_generation_api_equals_dp_densify(name, max_pops):
    """The host-array generation API (dist.densify_partitioned at one rank:
    owners, refine_items, commit) and the device-resident dp_densify_run in
    batches of 1 and 3 generations equal dp_densify, statistics included."""
    P, imgs, seeds = _scene(name)
    opts = dp.Options(max_pops=max_pops) if max_pops else dp.Options()
    with dp.Engine(opts, device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        ref, rst = eng.densify(seeds)
        got, gst = D.densify_partitioned(eng, seeds, None)
        runs = []
        for k in (1, 3):
            g = eng.densify_begin(seeds)
            cand, acc = eng.densify_refine_items(g, np.arange(g.items))
            g = eng.densify_commit(g, cand, acc)
            calls = 0
            while g.items > 0:
                g = eng.densify_run(g, k)
                calls += 1
            runs.append((k, calls, eng.densify_result()))
    assert len(ref) > 20
    assert got.tobytes() == ref.tobytes()
    for k in ("patches", "seed_patches", "pops", "candidates", "generations", "evals"):
        assert gst[k] == rst[k], k
    for k, calls, (rp, rs) in runs:
        assert rp.tobytes() == ref.tobytes(), f"batch {k}"
        for key in ("patches", "seed_patches", "pops", "candidates", "generations", "evals"):
            assert rs[key] == rst[key], (k, key)
        assert calls >= rst["generations"] // k


@pytest.mark.parametrize("bound", [3, 30, 200])
def test_run_until_yields_at_the_bound(bound):
    """dp_densify_run_until hands back the first generation of >= bound items
    unrun (its items and index as the host-array path reaches them), the
    evaluations it reports add up to dp_densify's, and alternating it with
    host-driven generations (the hybrid multi-rank loop at one rank) gives
    dp_densify's store."""
    P, imgs, seeds = _scene("hf6")
    with dp.Engine(device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        ref, rst = eng.densify(seeds)
        _, hst = D.densify_partitioned(eng, seeds, None)
        sizes = [p[0] for p in hst["partition"]]  # items of generation 0, 1, ...
        g = eng.densify_begin(seeds)
        cand, acc = eng.densify_refine_items(g, np.arange(g.items))
        g = eng.densify_commit(g, cand, acc)
        evals_run, yields = 0, 0
        while g.items > 0:
            assert g.items == sizes[g.index], (g.index, g.items)
            if g.items < bound:
                idx = g.index
                g, ev = eng.densify_run_until(g, bound)
                evals_run += ev
                if g.items > 0:
                    # stopped at the bound: the returned generation is the first
                    # large one after idx, unrun
                    assert g.items >= bound and g.index > idx
                    assert all(s < bound for s in sizes[idx:g.index])
                    yields += 1
            else:
                cand, acc = eng.densify_refine_items(g, np.arange(g.items))
                g = eng.densify_commit(g, cand, acc)
        got, st = eng.densify_result()
    assert got.tobytes() == ref.tobytes()
    for k in ("patches", "seed_patches", "candidates", "generations", "evals"):
        assert st[k] == rst[k], k
    assert evals_run <= rst["evals"] and (evals_run > 0) == any(s < bound for s in sizes[1:])
    # hf6's generation sizes end 8, 3, 2, 2, 3, 3: at bound 3 the run stops before the second 3
    assert yields == (1 if bound == 3 else 0)


def test_densify_result_view_equals_copy():
    """Engine.densify(copy=False) / densify_result(copy=False): a view of the
    context's pinned result buffer (not owning its memory) with the same
    records as the copy, valid until the next densify on the engine; also
    through the partitioned driver at one rank (copy_result=False)."""
    P, imgs, seeds = _scene("hf6")
    with dp.Engine(device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        ref, rst = eng.densify(seeds)
        view, vst = eng.densify(seeds, copy=False)
        assert view.tobytes() == ref.tobytes() and vst["patches"] == rst["patches"]
        assert not view.flags.owndata
        got, _ = D.densify_partitioned_device(eng, seeds, None, torch.device("cuda", 0), copy_result=False)
        assert got.tobytes() == ref.tobytes()


def test_device_loop_stall_resumes():
    """DP_GEN_CAP caps the device-resident loop's candidate buffers, so its
    generations outgrow them: each stalls on the device (nothing runs), the
    host grows the buffers and resumes it -- the store equals the uncapped
    dp_densify's."""
    P, imgs, seeds = _scene("hf6")
    with dp.Engine(device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        ref, rst = eng.densify(seeds)
    os.environ["DP_GEN_CAP"] = "64"
    try:
        with dp.Engine(device=0) as eng:
            eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
            got, gst = eng.densify(seeds)
            assert gst["stalls"] > 0
    finally:
        del os.environ["DP_GEN_CAP"]
    assert got.tobytes() == ref.tobytes()
    for k in ("patches", "seed_patches", "candidates", "generations", "evals"):
        assert gst[k] == rst[k], k


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist = D.init("gloo")
    P, imgs, seeds = _scene("hf6")
    with dp.Engine(device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        got, st = D.densify_partitioned(eng, seeds, dist)
    np.save(out_path + f".r{rank}.npy", got.view(np.uint8), allow_pickle=False)
    with open(out_path + f".r{rank}.evals", "w") as f:
        f.write(str(st["evals"]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_host_partitioned_densify_equals_dp_densify(tmp_path):
    out = str(tmp_path / "dense")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    P, imgs, seeds = _scene("hf6")
    with dp.Engine(device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        ref, rst = eng.densify(seeds)
    for r in range(2):
        got = np.frombuffer(np.load(out + f".r{r}.npy", allow_pickle=False).tobytes(), dtype=PATCH_DTYPE)
        assert got.tobytes() == ref.tobytes(), f"rank {r}"
        # each rank refined its share of every generation; the summed evaluation count is the 1-GPU one
        assert int(open(out + f".r{r}.evals").read()) == rst["evals"]


def _worker_dev(rank, world, port, out_path, backend, exchange=False, cap=1, scene="hf6", rb=0):
    import torch
    import torch.distributed as tdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # torch's HIP runtime initialises the device before libdensepoints' (the
    # wheel bundles its own libamdhip64; bench.py uses the same order); the
    # torch default stream is the legacy NULL stream (the ABI's stream = NULL case)
    torch.cuda.set_device(0)
    group = None
    if backend:
        kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
        tdist.init_process_group(backend, rank=rank, world_size=world, **kw)
        group = tdist
    P, imgs, seeds = _scene(scene)
    with dp.Engine(dp.Options(max_patches_per_cell=cap), device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        # the same densify in the host-array form: the partitions (and their
        # statistics, read back by the async path with the commit) must agree
        _, hst = D.densify_partitioned(eng, seeds, group, torch.device("cuda", 0) if backend == "nccl" else None)
        if rb == "hybrid":
            # a bound between the expansion generations' sizes: some partitioned, some replicated
            sizes = sorted(p[0] for p in hst["partition"][1:])
            rb = max(2, sizes[len(sizes) // 2])
        got, st = D.densify_partitioned_device(eng, seeds, group, torch.device("cuda", 0), one_rank_exchange=exchange,
                                               replicate_below=rb)
    np.save(out_path + f".r{rank}.npy", got.view(np.uint8), allow_pickle=False)
    with open(out_path + f".r{rank}.json", "w") as f:
        f.write(json.dumps({"evals": st["evals"], "partition": st["partition"], "host_partition": hst["partition"],
                            "replicated_calls": st.get("replicated_calls", 0)}))
    if group:
        tdist.barrier()
        tdist.destroy_process_group()


@pytest.mark.parametrize("backend,world,exchange,cap,rb", [(None, 1, False, 1, 0), (None, 1, True, 1, 0),
                                                          ("nccl", 1, True, 1, 0), ("gloo", 2, False, 1, 0),
                                                          ("gloo", 3, False, 1, 0), ("gloo", 2, False, 2, 0),
                                                          ("gloo", 2, False, 1, "hybrid"),
                                                          ("gloo", 3, False, 2, "hybrid"),
                                                          ("nccl", 1, True, 1, "hybrid")])
def test_partitioned_densify_device(tmp_path, backend, world, exchange, cap, rb):
    """Reference-view super-tile partition of every generation: the device
    partition, refine of the rank's share with its accepted candidates
    compacted into the rank's slot, ONE all-gather of the slots and the
    scatter + commit (dist.densify_partitioned_device: one host wait per
    generation; at one rank the device-resident generations, or with
    `exchange` the slot protocol itself): every rank's store equals dp_densify
    -- also with organizer cell capacity 2 (max_patches_per_cell,
    patch_organizer.h:42-46).  The ranks run on the legacy NULL stream, and
    the partition statistics the async path reads back with the commit equal
    the synchronous host-array path's, generation by generation.  rb "hybrid":
    the generations below a median size run on every rank device-resident
    (dp_densify_run_until) and hand back the first larger one -- same store,
    evaluations counted once, the partitioned generations' statistics a
    subsequence of the host path's."""
    out = str(tmp_path / "dense")
    mp.spawn(_worker_dev, args=(world, _free_port(), out, backend, exchange, cap, "hf6", rb), nprocs=world, join=True)
    P, imgs, seeds = _scene("hf6")
    with dp.Engine(dp.Options(max_patches_per_cell=cap), device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        ref, rst = eng.densify(seeds)
    for r in range(world):
        got = np.frombuffer(np.load(out + f".r{r}.npy", allow_pickle=False).tobytes(), dtype=PATCH_DTYPE)
        assert got.tobytes() == ref.tobytes(), f"rank {r}"
        st = json.loads(open(out + f".r{r}.json").read())
        assert st["evals"] == rst["evals"]
        if rb == "hybrid":
            assert st["replicated_calls"] > 0 and 1 < len(st["partition"]) < len(st["host_partition"]), st
            it = iter(st["host_partition"])
            assert all(any(p == q for q in it) for p in st["partition"]), f"rank {r}"
        elif world > 1 or exchange:
            assert st["partition"] == st["host_partition"], f"rank {r}"


def test_partitioned_densify_more_ranks_than_items(tmp_path):
    """three ranks on the legacy NULL stream over a scene whose
    late generations have fewer items than ranks (a rank with no share
    refines nothing and still commits): the stores equal dp_densify and the
    partition statistics read back with the commit equal the synchronous
    path's."""
    world = 3
    out = str(tmp_path / "dense")
    mp.spawn(_worker_dev, args=(world, _free_port(), out, "gloo", False, 1, "wide70", 0), nprocs=world, join=True)
    P, imgs, seeds = _scene("wide70")
    with dp.Engine(device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        ref, rst = eng.densify(seeds)
    for r in range(world):
        got = np.frombuffer(np.load(out + f".r{r}.npy", allow_pickle=False).tobytes(), dtype=PATCH_DTYPE)
        assert got.tobytes() == ref.tobytes(), f"rank {r}"
        st = json.loads(open(out + f".r{r}.json").read())
        assert st["partition"] == st["host_partition"]
        assert any(items < world for items, _, _, _ in st["partition"]), st["partition"]


@pytest.mark.parametrize("world", [2, 8])
def test_owners_equal_oracle_and_host_path(orc, world):
    """dp_densify_owners (device projection, super-tile keys, sorted-order cut)
    equals the oracle's numpy statement generation by generation -- owners and
    partition statistics -- and the host-array partitioned driver
    equals dp_densify (with the pop cap)."""
    P, imgs, seeds = _scene("wide70")
    S = orc.Scene(P, imgs)
    G = orc.GenerationEngine(S)
    with dp.Engine(device=0) as eng:
        eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(P))])
        g = eng.densify_begin(seeds)
        og = G.densify_begin(seeds)
        gens = 0
        while g.items > 0:
            own, fb = eng.densify_owners(g, world)
            oown, ofb = G.densify_owners(og, world)
            assert fb == ofb and np.array_equal(own, oown), f"generation {gens}"
            assert eng.densify_partition_stats() == G.densify_partition_stats(), f"generation {gens}"
            cand, acc = eng.densify_refine_items(g, np.arange(g.items))
            g = eng.densify_commit(g, cand, acc)
            oc, oa = G.densify_refine_items(og, np.arange(og.items))
            og = G.densify_commit(og, oc, oa)
            gens += 1
        assert gens > 3
        ref, _ = eng.densify(seeds)
        got, st = D.densify_partitioned(eng, seeds, None)
    assert got.tobytes() == ref.tobytes()


def _worker_cfg4(rank, world, port, out_path, max_pops, nseeds):
    import torch
    import torch.distributed as tdist

    from test_gpu_configs import DeviceScene, spread

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    # a real (non-NULL) caller stream like bench.py's: the library's own stream and
    # the caller's must be ordered by the ABI, not by sharing the legacy stream
    torch.cuda.set_stream(torch.cuda.Stream())
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    with dp.Engine(dp.Options(max_pops=max_pops), device=0) as eng:
        sc = DeviceScene("cfg4_64view_4k", eng, host_views=[])
        seeds = spread(sc.seeds, nseeds)
        for mode in ("parity", "fast", "hybrid"):
            eng.set_fast_options(dp.FastOptions(densify=0 if mode == "parity" else 1))
            # parity / fast: every generation partitioned; hybrid: the default
            # bound (the small generations on every rank, device-resident)
            got, st = D.densify_partitioned_device(eng, seeds, tdist, torch.device("cuda", 0),
                                                   replicate_below=None if mode == "hybrid" else 0)
            np.save(out_path + f".{mode}.r{rank}.npy", got.view(np.uint8), allow_pickle=False)
            with open(out_path + f".{mode}.r{rank}.json", "w") as f:
                f.write(json.dumps({"evals": st["evals"], "partition": st["partition"],
                                    "accepted": st["accepted"], "gathered": st["gathered_bytes"]}))
    tdist.barrier()
    tdist.destroy_process_group()


def _check_partition(parts, world):
    """balanced contiguous shares, tiles rarely split (records: items, largest
    share, items in split tiles, tiles)"""
    items = sum(p[0] for p in parts)
    assert all(mx <= -(-it // world) for it, mx, _, _ in parts)
    assert sum(p[2] for p in parts) <= 0.1 * items, parts


def test_partitioned_densify_cfg4_two_ranks(tmp_path):
    """BASELINE config 4 (64 views 3840x2160) in the partitioned protocol: two
    ranks sharing cuda:0 (gloo, spawned before any GPU call), each with the
    scene rendered into its own HBM planes, densify 1,500 spread seeds with a
    pop cap -- in parity and in performance mode -- and both ranks' stores
    equal the single-process dp_densify byte for byte; every share is within
    one item of the mean and >= 90% of the items are in tiles no cut splits,
    at world 2 and (the partitions a world-8 run would use, computed on one
    rank) at world 8."""
    from test_gpu_configs import DeviceScene, spread

    out = str(tmp_path / "cfg4")
    max_pops, nseeds = 6000, 1500
    mp.spawn(_worker_cfg4, args=(2, _free_port(), out, max_pops, nseeds), nprocs=2, join=True)
    with dp.Engine(dp.Options(max_pops=max_pops), device=0) as eng:
        sc = DeviceScene("cfg4_64view_4k", eng, host_views=[])
        seeds = spread(sc.seeds, nseeds)
        for mode in ("parity", "fast", "hybrid"):
            eng.set_fast_options(dp.FastOptions(densify=0 if mode == "parity" else 1))
            ref, rst = eng.densify(seeds)
            assert rst["patches"] > 1000 and 0 < rst["pops"] <= max_pops
            for r in range(2):
                got = np.frombuffer(np.load(out + f".{mode}.r{r}.npy", allow_pickle=False).tobytes(),
                                    dtype=PATCH_DTYPE)
                assert got.tobytes() == ref.tobytes(), f"{mode} rank {r}"
            st = json.loads(open(out + f".{mode}.r0.json").read())
            assert st["evals"] == rst["evals"]
            _check_partition(st["partition"], 2)
            if mode != "hybrid":
                assert sum(st["accepted"]) >= rst["patches"]
        eng.set_fast_options(dp.FastOptions())
        _, pst = D.densify_partitioned_device(eng, seeds, None, torch.device("cuda", 0), probe_worlds=(8,))
        _check_partition(pst["partition_probe"][8], 8)


def _worker_cfg5(rank, world, port, out_path, max_pops, nseeds):
    import torch
    import torch.distributed as tdist

    from test_gpu_configs import DeviceScene, spread

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    with dp.Engine(dp.Options(max_pops=max_pops, expand_cell_size=11), device=0) as eng:
        sc = DeviceScene("cfg5_128view_8k", eng, host_views=[])
        seeds = spread(sc.seeds, nseeds)
        eng.set_fast_options(dp.FastOptions(densify=1))
        got, st = D.densify_partitioned_device(eng, seeds, tdist, torch.device("cuda", 0))
        np.save(out_path + f".r{rank}.npy", got.view(np.uint8), allow_pickle=False)
        with open(out_path + f".r{rank}.json", "w") as f:
            f.write(json.dumps({"evals": st["evals"], "partition": st["partition"], "accepted": st["accepted"]}))
    tdist.barrier()
    tdist.destroy_process_group()


def test_partitioned_densify_cfg5_two_ranks(tmp_path):
    """BASELINE config 5 (128 views 7680x4320, fp16 gray planes, 11x11 window)
    in the partitioned protocol: two ranks sharing cuda:0 (gloo, spawned before
    any GPU call), each holding the whole scene in its own HBM (17 GB of BGRA8
    levels + 8.5 GB of gray planes per rank), densify 1,200 spread seeds in
    performance mode with a pop cap; both ranks' stores equal the
    single-process dp_densify byte for byte and the super-tile partition splits
    the generations."""
    from test_gpu_configs import DeviceScene, spread

    out = str(tmp_path / "cfg5")
    max_pops, nseeds = 5000, 1200
    mp.spawn(_worker_cfg5, args=(2, _free_port(), out, max_pops, nseeds), nprocs=2, join=True)
    with dp.Engine(dp.Options(max_pops=max_pops, expand_cell_size=11), device=0) as eng:
        sc = DeviceScene("cfg5_128view_8k", eng, host_views=[])
        seeds = spread(sc.seeds, nseeds)
        eng.set_fast_options(dp.FastOptions(densify=1))
        ref, rst = eng.densify(seeds)
    assert rst["patches"] > 1000 and 0 < rst["pops"] <= max_pops
    for r in range(2):
        got = np.frombuffer(np.load(out + f".r{r}.npy", allow_pickle=False).tobytes(), dtype=PATCH_DTYPE)
        assert got.tobytes() == ref.tobytes(), f"rank {r}"
    st = json.loads(open(out + ".r0.json").read())
    assert st["evals"] == rst["evals"]
    _check_partition(st["partition"], 2)

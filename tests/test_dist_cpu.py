"""Multi-process path on CPU (gloo, world_size 2 and 3): candidates are
sharded by contiguous rank ranges (the bench's weak-scaled batch), or a
densify's generations are partitioned by reference-view super-tile
(dist.densify_partitioned, the host-array form of the device protocol); the
all-gathered results equal the single-process result bit for bit.
The per-rank refine here is the oracle (CPU test infrastructure); the GPU runs
the same protocols in bench.py and tests/test_gpu_dist.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from densepoints_amd import dist as D
from densepoints_amd import synth


def test_shard_range_partitions_exactly():
    for n in (0, 1, 7, 64, 1000, 65537):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = D.shard_range(n, r, world)
                assert 0 <= lo <= hi <= n
                assert hi - lo in ((n // world), (n // world) + 1)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


def test_weak_shard_fixed_size_and_wraps():
    for world in (1, 2, 4, 8):
        for r in range(world):
            idx = D.weak_shard(100, 64, r)
            assert len(idx) == 64
            assert idx[0] == (64 * r) % 100
            assert np.all(np.diff(idx) % 100 == 1)
    with pytest.raises(ValueError):
        D.weak_shard(0, 4, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    cfg = synth.config(4, 320, 240, 1)
    P, imgs, seeds = synth.scene_host(cfg)
    return P, imgs, seeds


def _worker(rank, world, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from oracle import pyoracle

    dist = D.init("gloo")
    P, imgs, seeds = _scene()
    S = pyoracle.Scene(P, imgs)
    parents = S.seeds_to_patches(seeds)[:48]
    lo, hi = D.shard_range(len(parents), rank, world)
    kids, acc = S.expand(parents[lo:hi], 2)
    kids = kids.copy()
    kids["flags"] = np.where(acc != 0, kids["flags"] | 0x80, kids["flags"])  # carry accept in the record
    # children of shard [lo, hi) are candidates [4 lo, 4 hi): parent indices are shard-local
    kids["parent"] = np.where(kids["parent"] != 0xFFFFFFFF, kids["parent"] + lo, kids["parent"])
    all_kids = D.allgather_patches(kids, dist)
    t = D.max_over_ranks(float(rank + 1), dist)
    if rank == 0:
        np.save(out_path, all_kids.view(np.uint8), allow_pickle=False)
        with open(out_path + ".max", "w") as f:
            f.write(repr(t))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_expand_equals_single_process(tmp_path, orc):
    world = 2
    out = str(tmp_path / "kids.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    from densepoints_amd._native import PATCH_DTYPE

    got = np.frombuffer(np.load(out, allow_pickle=False).tobytes(), dtype=PATCH_DTYPE)
    P, imgs, seeds = _scene()
    S = orc.Scene(P, imgs)
    parents = S.seeds_to_patches(seeds)[:48]
    kids, acc = S.expand(parents, 2)
    kids = kids.copy()
    kids["flags"] = np.where(acc != 0, kids["flags"] | 0x80, kids["flags"])
    assert len(got) == 4 * len(parents)
    assert got.tobytes() == kids.tobytes()
    assert float(open(out + ".max").read()) == 2.0


def _hf6():
    # 6-view tilted-facet scene, 320x240 (the GPU suite's "hf6")
    return synth.scene_host(synth.config(6, 320, 240, 1))


def test_partition_is_rank_major_and_stable():
    rng = np.random.default_rng(5)
    for world in (1, 2, 3, 8):
        own = rng.integers(0, world, 1000)
        order, counts, offsets = D.partition(own, world)
        assert sorted(order.tolist()) == list(range(1000))
        for r in range(world):
            seg = order[offsets[r]: offsets[r] + counts[r]]
            assert (own[seg] == r).all() and (np.diff(seg) > 0).all()


def _part_worker(rank, world, port, out_path, max_pops):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import densepoints_amd as dp
    from oracle import pyoracle

    dist = D.init("gloo")
    P, imgs, seeds = _hf6()
    S = pyoracle.Scene(P, imgs, dp.Options(max_pops=max_pops) if max_pops else None)
    patches, st = D.densify_partitioned(pyoracle.GenerationEngine(S), seeds, dist)
    np.save(out_path + f".r{rank}.npy", patches.view(np.uint8), allow_pickle=False)
    if rank == 0:
        with open(out_path + ".parts", "w") as f:
            f.write(repr(st["partition"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,max_pops", [(2, 0), (3, 0), (2, 23)])
def test_gloo_partitioned_densify_equals_single_process(tmp_path, orc, world, max_pops):
    """North star / SURVEY 8e: every generation partitioned by reference-view
    super-tile (items sorted by their (ref, v/64, u/64) key, the order cut into
    `world` contiguous equal shares), candidates all-gathered and put back in
    sequence order -> the 1-process densify bit for bit on every rank."""
    import ast

    import densepoints_amd as dp
    from densepoints_amd._native import PATCH_DTYPE

    out = str(tmp_path / "part")
    mp.spawn(_part_worker, args=(world, _free_port(), out, max_pops), nprocs=world, join=True)
    P, imgs, seeds = _hf6()
    S = orc.Scene(P, imgs, dp.Options(max_pops=max_pops) if max_pops else None)
    ref, st = S.densify(seeds)
    assert len(ref) > 50
    for r in range(world):
        got = np.frombuffer(np.load(out + f".r{r}.npy", allow_pickle=False).tobytes(), dtype=PATCH_DTYPE)
        assert got.tobytes() == ref.tobytes(), f"rank {r}"
    parts = ast.literal_eval(open(out + ".parts").read())
    # every share is within one item of the mean, and a big generation is cut
    # at tile boundaries except at the world - 1 cuts
    assert all(mx <= -(-items // world) for items, mx, _, _ in parts)
    assert any(items >= 100 and tiles > world and split < items / 2 for items, _, split, tiles in parts)

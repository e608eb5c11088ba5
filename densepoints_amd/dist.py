"""Multi-GPU plumbing for the patch loop: one process per GPU, torch.distributed
over RCCL (backend "nccl") on MI355X, gloo for CPU tests.

The refine/expand step has no data-path collective. Candidates are independent
(SURVEY 8e), so each rank refines its own shard. The only exchanges are
  * the barrier and max-over-ranks step time (bench.py), and
  * an all-gather of patch records, used when the accepted patches of all ranks
    are needed in one place (the 1-GPU result in order, or the per-generation
    exchange of a sharded densify).
Shards are contiguous ranges of the candidate sequence, so concatenating the
gathered shards in rank order restores the 1-GPU order bit for bit.

The densify BFS is also sharded by REFERENCE-VIEW SUPER-TILE (north star:
"reference-view grid cells shard across the 8 GPUs"):
densify_partitioned[_device] sort each generation's items by the (ref, v/64,
u/64) super-tile of their centre and hand rank r the r-th of `world`
contiguous equal shares of that order (dp_densify_owners / _partition_device),
all-gather the candidates, put them back in sequence order and commit -- still
bit-exact.
"""
from __future__ import annotations

import os

import time

import numpy as np
import torch

from ._native import PATCH_DTYPE


def env() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1 process = 1 GPU)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, device: torch.device | None = None):
    """Initialise the default process group when WORLD_SIZE > 1; returns the
    torch.distributed module, or None for a single process. MASTER_ADDR
    defaults to 127.0.0.1 (the container hostname may not resolve)."""
    rank, world, _ = env()
    if world <= 1:
        return None
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if not dist.is_initialized():
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n candidates for `rank` (sizes
    differ by at most one; every index in exactly one shard)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(int(n), world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def weak_shard(n_total: int, per_rank: int, rank: int) -> np.ndarray:
    """Indices of a fixed-size per-rank shard for weak scaling (bench.py): rank
    r takes per_rank consecutive items starting at r*per_rank, wrapping around
    the list, so every rank does the same amount of work at any world size."""
    if n_total <= 0:
        raise ValueError("empty candidate list")
    return (np.arange(per_rank, dtype=np.int64) + rank * per_rank) % n_total


def allgather_patches(local: np.ndarray, dist, device: torch.device | None = None) -> np.ndarray:
    """All-gather variable-length dp_patch arrays; returns the concatenation in
    rank order on every rank. Records travel as padded uint8 tensors (one
    count all-gather, one payload all-gather), on `device` for RCCL or on the
    CPU for gloo."""
    return allgather_array(np.ascontiguousarray(local, dtype=PATCH_DTYPE), dist, device)


def allgather_array(local: np.ndarray, dist, device: torch.device | None = None) -> np.ndarray:
    """All-gather of a variable-length 1-D array of any fixed-size dtype (rank order)."""
    local = np.ascontiguousarray(local)
    if dist is None:
        return local.copy()
    dt = local.dtype
    world = dist.get_world_size()
    dev = device if device is not None else torch.device("cpu")
    cnt = torch.tensor([len(local)], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(x.item()) for x in counts]
    cap = max(max(counts) * dt.itemsize, 1)
    buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    if len(local):
        buf[: len(local) * dt.itemsize] = torch.from_numpy(local.view(np.uint8).copy()).to(dev)
    parts = [torch.zeros(cap, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = [np.frombuffer(p.cpu().numpy()[: n * dt.itemsize].tobytes(), dtype=dt) for p, n in zip(parts, counts)]
    return np.concatenate(out) if out else np.empty(0, dtype=dt)


def densify_sharded(eng, seeds_xyz, dist, device: torch.device | None = None):
    """dp_densify with every generation sharded across ranks.

    Each rank refines its contiguous range of the generation's items
    (dp_densify_refine), the candidates and accept flags are all-gathered in
    rank order (= sequence order), and every rank commits the whole
    generation to its replicated organizer (dp_densify_commit).  The result
    equals the 1-GPU dp_densify bit for bit.  `eng` is a densepoints_amd
    Engine (or any object with the same four densify_* methods).  Returns
    (patches, stats); stats["evals"] and ["refine_ms"] are summed/maxed over
    ranks."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    gen = eng.densify_begin(seeds_xyz)
    while gen.items > 0:
        lo, hi = shard_range(gen.items, rank, world)
        cand, acc = eng.densify_refine(gen, lo, hi)
        all_cand = allgather_array(cand, dist, device)
        all_acc = allgather_array(acc, dist, device)
        gen = eng.densify_commit(gen, all_cand, all_acc)
    patches, stats = eng.densify_result()
    if dist is not None:
        dev = device if device is not None else "cpu"
        ev = torch.tensor([float(stats["evals"])], dtype=torch.float64, device=dev)
        ms = torch.tensor([float(stats["refine_ms"])], dtype=torch.float64, device=dev)
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        stats["evals"] = int(ev.item())
        stats["refine_ms"] = float(ms.item())
    return patches, stats


def _reduce_stats(stats, dist, device):
    if dist is None:
        return stats
    dev = device if (device is not None and dist.get_backend() == "nccl") else "cpu"
    ev = torch.tensor([float(stats["evals"])], dtype=torch.float64, device=dev)
    ms = torch.tensor([float(stats["refine_ms"])], dtype=torch.float64, device=dev)
    dist.all_reduce(ev, op=dist.ReduceOp.SUM)
    dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    stats["evals"] = int(ev.item())
    stats["refine_ms"] = float(ms.item())
    return stats


def densify_sharded_device(eng, seeds_xyz, dist, device: torch.device):
    """densify_sharded with the candidate records resident in HBM.

    Per generation each rank refines its contiguous item range straight into a
    device buffer (dp_densify_refine_device), the padded equal-size shards are
    all-gathered with ONE all_gather_into_tensor per array (RCCL over xGMI on
    "nccl"; staged through the host on "gloo", which the CPU-side tests use),
    trimmed back to the true shard sizes and concatenated in rank order on the
    device, and every rank commits the whole generation from device memory
    (dp_densify_commit_device).  80 B per candidate cross the links; nothing
    else moves.  Bit-identical to dp_densify (replicated deterministic claims)."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    rccl = dist is not None and dist.get_backend() == "nccl"
    rec = PATCH_DTYPE.itemsize
    stream = torch.cuda.current_stream(device)
    gen = eng.densify_begin(seeds_xyz)
    while gen.items > 0:
        per = gen.per_item
        ranges = [shard_range(gen.items, r, world) for r in range(world)]
        sizes = [(hi - lo) * per for lo, hi in ranges]
        cap = max(max(sizes), 1)
        buf = torch.empty(cap * rec, dtype=torch.uint8, device=device)
        acc = torch.zeros(cap, dtype=torch.uint8, device=device)
        lo, hi = ranges[rank]
        eng.densify_refine_device(gen, lo, hi, buf.data_ptr(), acc.data_ptr(), stream.cuda_stream)
        if dist is None:
            all_c, all_a = buf[: sizes[0] * rec], acc[: sizes[0]]
        else:
            if rccl:
                gb = torch.empty(world * cap * rec, dtype=torch.uint8, device=device)
                ga = torch.empty(world * cap, dtype=torch.uint8, device=device)
                dist.all_gather_into_tensor(gb, buf)
                dist.all_gather_into_tensor(ga, acc)
            else:
                gb = torch.empty(world * cap * rec, dtype=torch.uint8)
                ga = torch.empty(world * cap, dtype=torch.uint8)
                dist.all_gather_into_tensor(gb, buf.cpu())
                dist.all_gather_into_tensor(ga, acc.cpu())
                gb, ga = gb.to(device), ga.to(device)
            all_c = torch.cat([gb[r * cap * rec: r * cap * rec + sizes[r] * rec] for r in range(world)])
            all_a = torch.cat([ga[r * cap: r * cap + sizes[r]] for r in range(world)])
        n = sum(sizes)
        gen = eng.densify_commit_device(gen, all_c.data_ptr(), all_a.data_ptr(), n, stream.cuda_stream)
        del buf, acc, all_c, all_a
    patches, stats = eng.densify_result()
    return patches, _reduce_stats(stats, dist, device)


def partition(owners: np.ndarray, world: int):
    """Rank-major item order of a generation: (order, counts, offsets), items
    of rank r = order[offsets[r]:offsets[r] + counts[r]], ascending."""
    owners = np.asarray(owners, dtype=np.int64)
    order = np.argsort(owners, kind="stable").astype(np.int64)
    counts = np.bincount(owners, minlength=world).astype(np.int64)
    offsets = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    return order, counts, offsets


def _part_record(eng, counts) -> tuple:
    """(items, largest share, items in tiles split between ranks, tiles) of the
    partition just computed"""
    st = eng.densify_partition_stats()
    return (st["items"], int(np.max(counts)) if len(counts) else 0, st["split_items"], st["tiles"])


def densify_partitioned(eng, seeds_xyz, dist, device: torch.device | None = None, tile_px: int = 64):
    """dp_densify with every generation partitioned by reference-view super-tile
    (dp_densify_owners: items sorted by their (ref, floor(v/tile),
    floor(u/tile)) key, the order cut into `world` contiguous equal shares).  Each rank
    refines its own items (dp_densify_refine_items), the candidates are
    all-gathered in rank order, scattered back to sequence order and committed
    by every rank (dp_densify_commit): the replicated store equals dp_densify's
    bit for bit.  Host arrays: `eng` is an Engine or the oracle's
    GenerationEngine (gloo tests on the CPU).  stats gains "partition": per
    generation (items, largest share, items in split tiles, tiles)."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    gen = eng.densify_begin(seeds_xyz)
    parts = []
    while gen.items > 0:
        owners, _ = eng.densify_owners(gen, world, tile_px)
        order, counts, offsets = partition(owners, world)
        parts.append(_part_record(eng, counts))
        mine = order[offsets[rank]: offsets[rank] + counts[rank]]
        cand, acc = eng.densify_refine_items(gen, mine)
        all_cand = allgather_array(cand, dist, device)
        all_acc = allgather_array(acc, dist, device)
        per = gen.per_item
        pos = (order[:, None] * per + np.arange(per)[None, :]).ravel()
        item_cand = np.empty_like(all_cand)
        item_acc = np.empty_like(all_acc)
        item_cand[pos] = all_cand
        item_acc[pos] = all_acc
        gen = eng.densify_commit(gen, item_cand, item_acc)
    patches, stats = eng.densify_result()
    stats = _reduce_stats(stats, dist, device)
    stats["partition"] = parts
    return patches, stats


class _DeviceBuffers:
    """Device byte buffers reused across generations (grown by 25% when short)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.bufs: dict[str, torch.Tensor] = {}

    def get(self, name: str, nbytes: int) -> torch.Tensor:
        t = self.bufs.get(name)
        if t is None or t.numel() < nbytes:
            n = max(int(nbytes), 1)
            t = torch.empty(n + n // 4, dtype=torch.uint8, device=self.device)
            self.bufs[name] = t
        return t


def densify_partitioned_device(eng, seeds_xyz, dist, device: torch.device, tile_px: int = 64,
                               probe_worlds: tuple = ()):
    """dp_densify with every generation partitioned by reference-view super-tile,
    the records in HBM, only the ACCEPTED candidates exchanged, and ONE host
    wait per generation (round 5; the round-4 protocol with four is
    densify_partitioned_device_r04).  Per generation, all queued on the torch
    current stream:
      1. dp_densify_partition_async: the items sorted by their (ref, v/64, u/64)
         super-tile key, cut into `world` contiguous equal shares (the shares
         are floor(r n / world) cuts: known on the host without a read);
      2. this rank refines its slice of that order (dp_densify_refine_items_device);
      3. dp_densify_compact_accepted_async keeps the candidates whose filter
         passed (each tagged with its generation position) and leaves their
         count in device memory;
      4. one all_gather_into_tensor of the counts (8 B per rank, device to
         device) and ONE of fixed-capacity rank slots (the largest share x 4
         records, host-known) over RCCL/xGMI -- no count has to reach the host;
         with one rank there is no exchange;
      5. dp_densify_commit_gathered_device scatters the slots to sequence order,
         commits the replicated organizer step and reads the generation's
         status (next generation size, partition statistics, records
         exchanged): the one host wait.
    Every rank's store equals dp_densify bit for bit.  stats as the r04
    protocol's: "partition", "accepted" (records exchanged), "gathered_bytes",
    "phase_ms" (host time: begin; launch = the queued partition, refine,
    compaction and exchange calls; commit = the commit up to its status read,
    i.e. mostly the GPU time of the generation)."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    rccl = dist is not None and dist.get_backend() == "nccl"
    rec = PATCH_DTYPE.itemsize
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream
    pool = _DeviceBuffers(device)
    ph = {"begin": 0.0, "launch": 0.0, "commit": 0.0}
    t = time.perf_counter()
    gen = eng.densify_begin(seeds_xyz)
    ph["begin"] += time.perf_counter() - t
    parts, gathered, accepted = [], [], []
    probe = {int(w): [] for w in probe_worlds}
    d_cnt = torch.zeros(1, dtype=torch.int64, device=device)
    all_cnt = torch.zeros(world, dtype=torch.int64, device=device)
    while gen.items > 0:
        per = gen.per_item
        for w in probe:
            _, pc, _ = eng.densify_partition_device(gen, w, tile_px)
            probe[w].append(_part_record(eng, pc))
        t = time.perf_counter()
        d_order, counts = eng.densify_partition_async(gen, world, tile_px, sp)
        offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        mine = int(counts[rank])
        stride = max(int(counts.max()) * per, 1)  # fixed-capacity rank slot (records)
        buf = pool.get("cand", max(mine * per, 1) * rec)
        acc = pool.get("acc", max(mine * per, 1))
        send = pool.get("send", stride * rec)
        if mine:
            d_items = d_order + 8 * int(offs[rank])
            eng.densify_refine_items_device(gen, d_items, mine, buf.data_ptr(), acc.data_ptr(), sp)
            eng.densify_compact_accepted_async(gen, d_items, mine, buf.data_ptr(), acc.data_ptr(), send.data_ptr(),
                                               d_cnt.data_ptr(), sp)
        else:
            d_cnt.zero_()
        if dist is None:
            recv, cnts = send, d_cnt
        elif rccl:
            recv = pool.get("recv", world * stride * rec)[: world * stride * rec]
            dist.all_gather_into_tensor(all_cnt, d_cnt)
            dist.all_gather_into_tensor(recv, send[: stride * rec])
            cnts = all_cnt
        else:
            # gloo (one-device rehearsals): staged through the host
            hc = torch.empty(world, dtype=torch.int64)
            dist.all_gather_into_tensor(hc, d_cnt.cpu())
            hr = torch.empty(world * stride * rec, dtype=torch.uint8)
            dist.all_gather_into_tensor(hr, send[: stride * rec].cpu())
            recv = hr.to(device)
            all_cnt.copy_(hc.to(device))
            cnts = all_cnt
        t1 = time.perf_counter()
        ph["launch"] += t1 - t
        n_ex = eng.densify_commit_gathered_device(gen, recv.data_ptr(), stride, cnts.data_ptr(), world, sp)
        ph["commit"] += time.perf_counter() - t1
        parts.append(_part_record(eng, counts))
        gathered.append(world * (stride * rec + 8) if dist is not None else 0)
        accepted.append(n_ex)
    patches, stats = eng.densify_result()
    stats = _reduce_stats(stats, dist, device)
    stats["phase_ms"] = {k: round(v * 1e3, 2) for k, v in ph.items()}
    stats["partition"] = parts
    stats["gathered_bytes"] = gathered or [0]
    stats["accepted"] = accepted
    if probe:
        stats["partition_probe"] = probe
    return patches, stats


def densify_partitioned_device_r04(eng, seeds_xyz, dist, device: torch.device, tile_px: int = 64,
                                   probe_worlds: tuple = ()):
    """dp_densify with every generation partitioned by reference-view super-tile,
    the records in HBM and only the ACCEPTED candidates exchanged (SURVEY 8e,
    north star: "RCCL all-gather over xGMI of accepted patches").  Per
    generation:
      1. dp_densify_partition_device: the items sorted by their (ref, v/64,
         u/64) super-tile key and cut into `world` contiguous equal shares (the
         rank-major item order), on the device; the host reads `world` counts;
      2. this rank refines its slice of that order (dp_densify_refine_items_device);
      3. dp_densify_compact_accepted_device keeps the candidates whose filter
         passed, each tagged with its generation position;
      4. one all_gather_into_tensor of the accepted counts (8 B per rank) and
         ONE of the padded accepted records (RCCL over xGMI on "nccl"; host-
         staged on "gloo" for the one-device rehearsals);
      5. dp_densify_commit_accepted_device scatters them to sequence order and
         commits the replicated organizer step on every rank.
    Device buffers are reused across generations.  Every rank's store equals
    dp_densify bit for bit.  stats gains "partition" (items, largest share,
    items in split tiles, tiles), "accepted" and "gathered_bytes" per
    generation; with probe_worlds, "partition_probe" {world: the same records}
    of the partitions those world sizes would use (computed on this rank before
    the real one; statistics only), and "phase_ms": this rank's host time per
    phase summed over the generations (partition; refine + compaction, which
    ends in the accepted-count read; exchange; commit) -- each phase already
    ends in a host sync, so the split adds none."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    rccl = dist is not None and dist.get_backend() == "nccl"
    rec = PATCH_DTYPE.itemsize
    stream = torch.cuda.current_stream(device)
    pool = _DeviceBuffers(device)
    ph = {"begin": 0.0, "partition": 0.0, "refine_compact": 0.0, "exchange": 0.0, "commit": 0.0}
    t = time.perf_counter()
    gen = eng.densify_begin(seeds_xyz)
    ph["begin"] += time.perf_counter() - t
    parts, gathered, accepted = [], [], []
    probe = {int(w): [] for w in probe_worlds}
    while gen.items > 0:
        per = gen.per_item
        for w in probe:
            _, pc, _ = eng.densify_partition_device(gen, w, tile_px)
            probe[w].append(_part_record(eng, pc))
        t = time.perf_counter()
        d_order, counts, _ = eng.densify_partition_device(gen, world, tile_px)
        parts.append(_part_record(eng, counts))
        offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        mine = int(counts[rank])
        d_items = d_order + 8 * int(offs[rank])
        cap = max(mine * per, 1)
        buf = pool.get("cand", cap * rec)
        acc = pool.get("acc", cap)
        comp = pool.get("comp", cap * rec)
        nacc = 0
        t1 = time.perf_counter()
        ph["partition"] += t1 - t
        if mine:
            eng.densify_refine_items_device(gen, d_items, mine, buf.data_ptr(), acc.data_ptr(), stream.cuda_stream)
            nacc = eng.densify_compact_accepted_device(gen, d_items, mine, buf.data_ptr(), acc.data_ptr(),
                                                       comp.data_ptr(), stream.cuda_stream)
        t2 = time.perf_counter()
        ph["refine_compact"] += t2 - t1
        if dist is None:
            allr, total, gb = comp, nacc, nacc * rec
        else:
            cdev = device if rccl else torch.device("cpu")
            cnt = torch.tensor([nacc], dtype=torch.int64, device=cdev)
            all_cnt = torch.empty(world, dtype=torch.int64, device=cdev)
            dist.all_gather_into_tensor(all_cnt, cnt)
            ns = [int(x) for x in all_cnt.tolist()]
            mx = max(max(ns), 1)
            send = pool.get("send", mx * rec)[: mx * rec]
            send[: nacc * rec].copy_(comp[: nacc * rec])
            if rccl:
                recv = pool.get("recv", world * mx * rec)[: world * mx * rec]
                dist.all_gather_into_tensor(recv, send)
            else:
                recv = torch.empty(world * mx * rec, dtype=torch.uint8)
                dist.all_gather_into_tensor(recv, send.cpu())
                recv = recv.to(device)
            allr = torch.cat([recv[r * mx * rec: r * mx * rec + ns[r] * rec] for r in range(world)])
            total, gb = sum(ns), world * (mx * rec + 8)
        gathered.append(gb)
        accepted.append(total)
        t3 = time.perf_counter()
        ph["exchange"] += t3 - t2
        gen = eng.densify_commit_accepted_device(gen, allr.data_ptr(), total, stream.cuda_stream)
        ph["commit"] += time.perf_counter() - t3
    patches, stats = eng.densify_result()
    stats = _reduce_stats(stats, dist, device)
    stats["phase_ms"] = {k: round(v * 1e3, 2) for k, v in ph.items()}
    stats["partition"] = parts
    stats["gathered_bytes"] = gathered
    stats["accepted"] = accepted
    if probe:
        stats["partition_probe"] = probe
    return patches, stats


def densify_partitioned_device_all(eng, seeds_xyz, dist, device: torch.device, tile_px: int = 64):
    """densify_partitioned with the records in HBM: per generation the owners
    (identical on every rank), this rank's item list to the device, one refine
    launch over it (dp_densify_refine_items_device), ONE all_gather_into_tensor
    per array of the padded shards (RCCL over xGMI on "nccl"), trim to the true
    shard sizes, and one commit that scatters the gathered candidates back to
    sequence order on the device (dp_densify_commit_items_device).  stats gains
    "partition" (items, largest share, items in split tiles, tiles) and "gathered_bytes" per
    generation (81 B per candidate slot incl. padding)."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    rccl = dist is not None and dist.get_backend() == "nccl"
    rec = PATCH_DTYPE.itemsize
    stream = torch.cuda.current_stream(device)
    gen = eng.densify_begin(seeds_xyz)
    parts, gathered = [], []
    while gen.items > 0:
        per = gen.per_item
        owners, _ = eng.densify_owners(gen, world, tile_px)
        order, counts, offsets = partition(owners, world)
        parts.append(_part_record(eng, counts))
        sizes = [int(c) * per for c in counts]
        cap = max(max(sizes), 1)
        mine = torch.from_numpy(order[offsets[rank]: offsets[rank] + counts[rank]].copy()).to(device)
        buf = torch.empty(cap * rec, dtype=torch.uint8, device=device)
        acc = torch.zeros(cap, dtype=torch.uint8, device=device)
        eng.densify_refine_items_device(gen, mine.data_ptr(), int(counts[rank]), buf.data_ptr(), acc.data_ptr(),
                                        stream.cuda_stream)
        if dist is None:
            all_c, all_a = buf[: sizes[0] * rec], acc[: sizes[0]]
        else:
            if rccl:
                gb = torch.empty(world * cap * rec, dtype=torch.uint8, device=device)
                ga = torch.empty(world * cap, dtype=torch.uint8, device=device)
                dist.all_gather_into_tensor(gb, buf)
                dist.all_gather_into_tensor(ga, acc)
            else:
                gb = torch.empty(world * cap * rec, dtype=torch.uint8)
                ga = torch.empty(world * cap, dtype=torch.uint8)
                dist.all_gather_into_tensor(gb, buf.cpu())
                dist.all_gather_into_tensor(ga, acc.cpu())
                gb, ga = gb.to(device), ga.to(device)
            all_c = torch.cat([gb[r * cap * rec: r * cap * rec + sizes[r] * rec] for r in range(world)])
            all_a = torch.cat([ga[r * cap: r * cap + sizes[r]] for r in range(world)])
        d_order = torch.from_numpy(order).to(device)
        gathered.append(world * cap * (rec + 1))
        gen = eng.densify_commit_items_device(gen, all_c.data_ptr(), all_a.data_ptr(), d_order.data_ptr(),
                                              len(order), stream.cuda_stream)
        del buf, acc, all_c, all_a, mine, d_order
    patches, stats = eng.densify_result()
    stats = _reduce_stats(stats, dist, device)
    stats["partition"] = parts
    stats["gathered_bytes"] = gathered
    return patches, stats


def max_over_ranks(x: float, dist, device: torch.device | None = None) -> float:
    """Maximum of a per-rank scalar (the step time) over all ranks."""
    if dist is None:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

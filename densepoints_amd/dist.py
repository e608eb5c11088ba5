"""Multi-GPU plumbing for the patch loop: one process per GPU, torch.distributed
over RCCL (backend "nccl") on MI355X, gloo for CPU tests.

The refine/expand step has no data-path collective. Candidates are independent
(SURVEY 8e), so each rank refines its own shard. The exchanges are
  * the barrier and max-over-ranks step time (bench.py), and
  * the per-generation all-gather of a partitioned densify.

The densify BFS is sharded by REFERENCE-VIEW SUPER-TILE (north star:
"reference-view grid cells shard across the 8 GPUs"): each
generation's items are sorted by the (ref, v/64, u/64) super-tile of their
centre and rank r takes the r-th of `world` contiguous equal shares of that
order; the accepted candidates of every rank reach every rank, which commits
the whole generation to its replicated organizer -- bit-exact with dp_densify.
densify_partitioned is the host-array form (any engine with the generation
API, the oracle's included: the gloo CPU tests); densify_partitioned_device
is the device-resident one-wait-per-generation protocol (the bench's
scaling_leg and the GPU tests).
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


def replicate_below_default(world: int) -> int:
    """Items below which a generation runs replicated on every rank: a share of
    fewer than ~1024 parents (4,096 candidates, one resident wave per SIMD of
    the chip) leaves the refine latency-bound, so partitioning it buys nothing
    while the exchange costs a host turnaround per generation."""
    return 1024 * max(int(world), 1)


def densify_partitioned_device(eng, seeds_xyz, dist, device: torch.device, tile_px: int = 64,
                               probe_worlds: tuple = (), one_rank_exchange: bool = False, copy_result: bool = True,
                               replicate_below: int | None = None):
    """dp_densify with every generation partitioned by reference-view super-tile,
    the records in HBM, only the ACCEPTED candidates exchanged and ONE host
    wait per generation.  Per generation, all queued on the torch current
    stream:
      1. dp_densify_partition_async: the items sorted by their (ref, v/64,
         u/64) super-tile key, cut into `world` contiguous equal shares (the
         shares are floor(r n / world) cuts: known on the host without a read);
      2. dp_densify_refine_share_async: this rank refines its slice of that
         order and compacts the candidates whose filter passed into its
         exchange slot (a count header + up to `stride` records, each tagged
         with its generation position);
      3. ONE all_gather_into_tensor of the fixed-capacity slots over
         RCCL/xGMI (stride = the largest share x 4, host-known);
      4. dp_densify_commit_gathered_device scatters the slots to sequence
         order, commits the replicated organizer step and reads the next
         generation's state: the one host wait.
    With one rank there is nothing to partition or exchange: the whole densify
    is dp_densify (seed generation, then the expansion generations
    device-resident, eight per host wait), unless one_rank_exchange keeps the
    multi-rank protocol (slots, scatter) at world 1 for measurement, or
    probe_worlds asks for the partitions of every generation.  Every rank's
    store equals dp_densify bit for bit.  copy_result=False returns the store
    as a view of the library's pinned result buffer (valid until the engine's
    next densify) instead of a copy.
    Hybrid (r06): an expansion generation of fewer than `replicate_below`
    items (default replicate_below_default(world); 0 = partition every
    generation) runs on every rank at once, device-resident with no partition
    and no exchange (dp_densify_run_until, eight generations per host wait,
    handing back the first generation that reaches the bound), its
    evaluations counted on rank 0 only.  Those are the BFS's long tail: their
    refine is one candidate's latency, whatever the share.  stats gains "partition" (items, largest
    share, items in split tiles, tiles per generation), "accepted" (records
    exchanged), "gathered_bytes", "phase_ms" (host time: begin; launch = the
    queued partition, refine and exchange calls; commit = up to the status
    read, i.e. mostly the generation's GPU time; run = the device-resident
    generations) and, with probe_worlds, "partition_probe" {world: the same
    records} of the partitions those world sizes would use (statistics only)."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    if world == 1 and not one_rank_exchange and not probe_worlds:
        t = time.perf_counter()
        patches, stats = eng.densify(seeds_xyz, copy=copy_result)
        stats["phase_ms"] = {"densify": round((time.perf_counter() - t) * 1e3, 2)}
        stats["partition"] = []
        stats["gathered_bytes"] = [0]
        stats["accepted"] = []
        return patches, stats
    rccl = dist is not None and dist.get_backend() == "nccl"
    if replicate_below is None:
        replicate_below = replicate_below_default(world)
    repl_evals = 0
    rec = PATCH_DTYPE.itemsize
    stream = torch.cuda.current_stream(device)
    sp = stream.cuda_stream
    pool = _DeviceBuffers(device)
    ph = {"begin": 0.0, "launch": 0.0, "commit": 0.0, "run": 0.0, "replicated": 0.0}
    t = time.perf_counter()
    gen = eng.densify_begin(seeds_xyz)
    ph["begin"] += time.perf_counter() - t
    parts, gathered, accepted = [], [], []
    replicated_calls = 0
    probe = {int(w): [] for w in probe_worlds}
    while gen.items > 0:
        per = gen.per_item
        for w in probe:
            own, _ = eng.densify_owners(gen, w, tile_px)
            probe[w].append(_part_record(eng, np.bincount(own, minlength=w)))
        if world == 1 and gen.index >= 1 and not one_rank_exchange:
            t = time.perf_counter()
            torch.cuda.current_stream(device).synchronize()
            gen = eng.densify_run(gen)
            ph["run"] += time.perf_counter() - t
            continue
        if gen.index >= 1 and gen.items < replicate_below and not probe:
            # the small generations, on every rank, until one reaches the bound
            t = time.perf_counter()
            torch.cuda.current_stream(device).synchronize()
            gen, ev = eng.densify_run_until(gen, replicate_below)
            repl_evals += ev
            replicated_calls += 1
            ph["replicated"] += time.perf_counter() - t
            continue
        t = time.perf_counter()
        d_order, counts = eng.densify_partition_async(gen, world, tile_px, sp)
        offs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        mine = int(counts[rank])
        stride = max(int(counts.max()) * per, 1)  # fixed-capacity rank slot (records)
        slot = pool.get("slot", (stride + 1) * rec)[: (stride + 1) * rec]
        d_items = d_order + 8 * int(offs[rank]) if mine else 0
        eng.densify_refine_share_async(gen, d_items, mine, slot.data_ptr(), stride, sp)
        if dist is None:
            recv = slot
        elif rccl:
            recv = pool.get("recv", world * (stride + 1) * rec)[: world * (stride + 1) * rec]
            dist.all_gather_into_tensor(recv, slot)
        else:
            # gloo (one-device rehearsals): staged through the host
            hr = torch.empty(world * (stride + 1) * rec, dtype=torch.uint8)
            dist.all_gather_into_tensor(hr, slot.cpu())
            recv = hr.to(device)
        t1 = time.perf_counter()
        ph["launch"] += t1 - t
        n_ex = eng.densify_commit_gathered_device(gen, recv.data_ptr(), stride, world, sp)
        ph["commit"] += time.perf_counter() - t1
        parts.append(_part_record(eng, counts))
        gathered.append(world * (stride + 1) * rec if dist is not None else 0)
        accepted.append(n_ex)
    patches, stats = eng.densify_result(copy=copy_result)
    if rank != 0:
        # every rank ran the replicated generations: rank 0 counts them
        stats["evals"] -= repl_evals
    stats = _reduce_stats(stats, dist, device)
    stats["replicated_calls"] = replicated_calls
    stats["replicate_below"] = int(replicate_below)
    stats["phase_ms"] = {k: round(v * 1e3, 2) for k, v in ph.items()}
    stats["partition"] = parts
    stats["gathered_bytes"] = gathered or [0]
    stats["accepted"] = accepted
    if probe:
        stats["partition_probe"] = probe
    return patches, stats


def max_over_ranks(x: float, dist, device: torch.device | None = None) -> float:
    """Maximum of a per-rank scalar (the step time) over all ranks."""
    if dist is None:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

"""Host-side mirror of the reference's methods/pmvs + modules/core + modules/io
plugin surface, driving the HIP C ABI.

Reference interface -> here:
  View (modules/core/types.h:37-74)                  -> View
  PMVS::Options (methods/pmvs/options.h:8-21) and the
  scattered constructor defaults          -> Options
  Patch (methods/pmvs/patch.h:21-101)                -> rows of a PATCH_DTYPE array
  Optimization / OptimizationOpenCV::Optimize,
  FilterByErrorMeasurement (optimization*.h)         -> Engine.refine / Engine.filter
  NCCScore (modules/core/error_measurements.h:11)    -> ncc_score
  PMVS::AddCamera / Run / GetPointCloud (pmvs.h)     -> PMVS
  IO::JSONReader (modules/io/json_reader.h:30-37)    -> read_scene_json
  PMVS::PrintCloud (methods/pmvs/utils.cpp:9-50)     -> write_ply
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass, field

import numpy as np

from . import _native as N
from ._native import PATCH_DTYPE, check, lib, ptr

__all__ = [
    "Options",
    "FastOptions",
    "View",
    "Engine",
    "PMVS",
    "ncc_score",
    "read_scene_json",
    "write_ply",
    "empty_patches",
    "visible_list",
    "mask_from_list",
]


@dataclass
class FastOptions:
    """Performance-mode knobs (dp_fast_options; no reference counterpart: the
    mode replaces OptimizationOpenCV::Optimize, optimization_opencv.cpp:44-78,
    with a conjugate-gradient refine on LDS-staged gray tiles)."""

    iters: int = 4            # CG iterations: E <= 1 + 3 iters (gradient 1) / 1 + 5 iters (0), +1 filter evaluation
    margin: int = 2           # tile margin around the initial window, pixels (<= 7)
    tile_budget: int = 6656   # LDS bytes per patch: tiles + 64 per view (<= 16384; <= 6656: 4 waves/SIMD)
    max_views: int = 8        # staged views of the refine (<= 32; spec v5, was 32)
    fd_step: float = 0.5      # forward-difference step, scaled units (gradient 0)
    ls_step: float = 1.0      # initial line-search step, scaled units
    densify: int = 0          # 1: dp_densify expands with the fast refine
    gradient: int = 0         # 0: forward differences (spec v3); 1: analytic gradient (spec v4)
    filter_max_views: int = 32  # staged views of the filter / FAST_EVAL scoring (0 = max_views; spec v5)

    def to_c(self) -> N.DpFastOptions:
        o = N.DpFastOptions()
        for name, _ in N.DpFastOptions._fields_:
            setattr(o, name, getattr(self, name))
        return o


@dataclass
class Options:
    """Every hot-path knob with the reference's default (see include/densepoints.h)."""

    seed_cell_size: int = 16        # matcher.h:25
    expand_cell_size: int = 11      # expand.h:12
    grid_scale: int = 8             # patch_organizer.h:43
    max_patches_per_cell: int = 1   # patch_organizer.h:42
    min_visible: int = 3            # optimization.h:17
    min_expand_visible: int = 2     # expand.cpp:67
    nm_max_evals: int = 500         # optimization_opencv.cpp:60
    ncc_threshold: float = 0.6      # optimization.h:16
    visible_angle: float = 0.78     # patch.h:56
    candidate_angle: float = 1.04   # patch.h:57
    nm_step: tuple = (0.02, 0.2, 0.2)  # optimization_opencv.cpp:56
    nm_eps: float = 1e-4            # optimization_opencv.cpp:60
    ncc_denom_min: float = 0.1      # error_measurements.cpp:57
    max_pops: int = 10_000_000      # expand.cpp:95
    # reference PMVS::Options (options.h:10-15): stored, never read by the path
    scale: int = 1
    cell_size: int = 4
    expansions: int = 3

    def to_c(self) -> N.DpOptions:
        o = N.DpOptions()
        for name, _ in N.DpOptions._fields_:
            if name == "reserved0":
                continue
            v = getattr(self, name)
            if name == "nm_step":
                o.nm_step[:] = [float(x) for x in v]
            else:
                setattr(o, name, v)
        return o

    def to_numpy(self) -> np.ndarray:
        """The same POD as bytes (for handing to the oracle's identical layout)."""
        c = self.to_c()
        return np.frombuffer(bytes(c), dtype=np.uint8).copy()


class View:
    """A camera: 3x4 projection (fp64) + BGR8 image (H x W x 3)."""

    def __init__(self, P, image: np.ndarray | None = None, filename: str | None = None):
        self.P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(3, 4))
        self.image = None if image is None else np.ascontiguousarray(image, dtype=np.uint8)
        self.filename = filename
        C = np.zeros(3)
        K = np.zeros(9)
        E = np.zeros(12)
        x = np.zeros(3)
        rc = lib.dp_view_geometry(ptr(self.P), ptr(C), ptr(K), ptr(E), ptr(x))
        if rc != N.DP_OK:
            raise N.DensePointsError(rc, "singular projection matrix")
        self.camera_center = C
        self.intrinsics = K.reshape(3, 3)
        self.extrinsics = E.reshape(3, 4)
        self.x_axis = x

    @property
    def width(self) -> int:
        return int(self.image.shape[1])

    @property
    def height(self) -> int:
        return int(self.image.shape[0])

    def project_point(self, X) -> np.ndarray:
        h = self.P @ np.append(np.asarray(X, dtype=np.float64), 1.0)
        return h[:2] / h[2]

    def is_point_inside(self, X) -> bool:
        u, v = self.project_point(X)
        return bool(0 < u < self.width and 0 < v < self.height)


def empty_patches(n: int) -> np.ndarray:
    return np.zeros(n, dtype=PATCH_DTYPE)


def result_array(addr, n: int, copy: bool = True) -> np.ndarray:
    """n dp_patch records at a library-owned address (a densify's pinned result
    buffer) as a numpy array: a copy, or (copy=False) a view that stays valid
    until the library reuses the buffer"""
    if not n:
        return empty_patches(0)
    buf = (ctypes.c_char * (n * PATCH_DTYPE.itemsize)).from_address(addr)
    view = np.frombuffer(buf, dtype=PATCH_DTYPE, count=n)
    return view.copy() if copy else view


def visible_list(mask) -> list[int]:
    """Bitmask (u64[2]) -> ascending view list (Patch::GetTrullyVisibleImages)."""
    out = []
    for w in range(2):
        m = int(mask[w])
        for b in range(64):
            if (m >> b) & 1:
                out.append(64 * w + b)
    return out


def mask_from_list(views) -> np.ndarray:
    m = np.zeros(2, dtype=np.uint64)
    for v in views:
        m[v >> 6] |= np.uint64(1) << np.uint64(v & 63)
    return m


class Engine:
    """One GPU context: views resident in HBM, batched patch operators."""

    def __init__(self, options: Options | None = None, device: int = 0):
        self.options = options or Options()
        self._ctx = ctypes.c_void_p()
        copt = self.options.to_c()
        rc = lib.dp_ctx_create(ctypes.byref(copt), device, ctypes.byref(self._ctx))
        check(rc)
        self.views: list[View] = []
        self._keep = []

    @property
    def handle(self):
        return self._ctx

    def close(self):
        if self._ctx:
            lib.dp_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc):
        check(rc, self._ctx)

    def set_options(self, options: Options):
        self.options = options
        copt = options.to_c()
        self._check(lib.dp_set_options(self._ctx, ctypes.byref(copt)))

    def set_views(self, views: list[View]):
        V = len(views)
        P = np.ascontiguousarray(np.stack([v.P for v in views]).reshape(V, 12))
        imgs = (N.DpImage * V)()
        for i, v in enumerate(views):
            im = v.image
            imgs[i].width = im.shape[1]
            imgs[i].height = im.shape[0]
            imgs[i].stride = im.strides[0]
            imgs[i].bgr = im.ctypes.data
        self._check(lib.dp_set_views(self._ctx, V, ptr(P), imgs))
        self.views = list(views)

    def set_views_device(self, P: np.ndarray, widths, heights, pitches, dev_ptrs):
        V = len(dev_ptrs)
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(V, 12))
        w = np.asarray(widths, dtype=np.int32)
        h = np.asarray(heights, dtype=np.int32)
        pt = np.asarray(pitches, dtype=np.int32)
        arr = (ctypes.c_void_p * V)(*[int(p) for p in dev_ptrs])
        self._check(lib.dp_set_views_device(self._ctx, V, ptr(P), ptr(w), ptr(h), ptr(pt), arr))
        self._keep = [P, w, h, pt, arr]

    # ---- image pyramid (include/densepoints.h dp_build_pyramid / dp_set_level) ----
    def build_pyramid(self, levels: int):
        """Levels 1..levels-1 by cv::pyrDown on the device (level 0 = the views)."""
        self._check(lib.dp_build_pyramid(self._ctx, int(levels)))

    def set_level(self, level: int):
        """Run the patch loop on pyramid level `level` (P rows 0-1 scaled by 2^-level)."""
        self._check(lib.dp_set_level(self._ctx, int(level)))

    def level_info(self, level: int, view: int):
        w, h, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_void_p()
        self._check(lib.dp_level_info(self._ctx, level, view, ctypes.byref(w), ctypes.byref(h), ctypes.byref(d)))
        return w.value, h.value, d.value

    def read_level(self, level: int, view: int) -> np.ndarray:
        w, h, _ = self.level_info(level, view)
        out = np.zeros((h, w, 3), dtype=np.uint8)
        self._check(lib.dp_read_level(self._ctx, level, view, ptr(out)))
        return out

    # ---- PMVS-style filter (include/densepoints.h dp_filter_patches) ----
    def filter_patches(self, patches: np.ndarray, passes: int = 3, min_neighbor_frac: float = 0.25) -> np.ndarray:
        """Visibility-consistency + neighbourhood filter (PMVS::FilterPatches,
        pmvs.h:27, which the reference leaves undefined); returns keep flags."""
        patches = np.ascontiguousarray(patches)
        assert patches.dtype == PATCH_DTYPE
        fo = N.DpFilterOptions(passes, 0, min_neighbor_frac)
        keep = np.zeros(len(patches), dtype=np.uint8)
        self._check(lib.dp_filter_patches(self._ctx, ptr(patches), len(patches), ctypes.byref(fo), ptr(keep)))
        return keep

    def seeds_to_patches(self, xyz: np.ndarray) -> np.ndarray:
        xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 3)
        out = empty_patches(len(xyz))
        self._check(lib.dp_seeds_to_patches(self._ctx, ptr(xyz), len(xyz), ptr(out)))
        return out

    def refine(self, patches: np.ndarray, cell: int, mode: int) -> np.ndarray:
        """Fused evaluate+refine+filter over a batch, in place; returns accept flags."""
        assert patches.dtype == PATCH_DTYPE and patches.flags.c_contiguous
        acc = np.zeros(len(patches), dtype=np.uint8)
        self._check(lib.dp_refine_batch(self._ctx, ptr(patches), len(patches), cell, mode, ptr(acc)))
        return acc

    def refine_device(self, d_patches: int, n: int, cell: int, mode: int, d_accept: int | None,
                      stream: int | None = None):
        self._check(lib.dp_refine_batch_device(self._ctx, ctypes.c_void_p(d_patches), n, cell, mode,
                                               ctypes.c_void_p(d_accept) if d_accept else None,
                                               ctypes.c_void_p(stream) if stream else None))

    def expand(self, parents: np.ndarray):
        """Expand::ExpandPatch over a batch: returns (children[4n], accept[4n])."""
        parents = np.ascontiguousarray(parents)
        assert parents.dtype == PATCH_DTYPE
        kids = empty_patches(4 * len(parents))
        acc = np.zeros(4 * len(parents), dtype=np.uint8)
        self._check(lib.dp_expand_batch(self._ctx, ptr(parents), len(parents), ptr(kids), ptr(acc)))
        return kids, acc

    def expand_device(self, d_parents: int, n: int, d_children: int, d_accept: int | None,
                      stream: int | None = None):
        self._check(lib.dp_expand_batch_device(self._ctx, ctypes.c_void_p(d_parents), n,
                                               ctypes.c_void_p(d_children),
                                               ctypes.c_void_p(d_accept) if d_accept else None,
                                               ctypes.c_void_p(stream) if stream else None))

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_double()
        self._check(lib.dp_last_kernel_ms(self._ctx, ctypes.byref(ms)))
        return ms.value

    # ---- performance mode (include/densepoints.h dp_fast_options) ----
    def set_fast_options(self, fo: FastOptions):
        c = fo.to_c()
        self._check(lib.dp_set_fast_options(self._ctx, ctypes.byref(c)))

    def build_gray(self):
        """fp16 gray planes of the current level (built on demand otherwise)."""
        self._check(lib.dp_build_gray(self._ctx))

    def read_gray(self, view: int) -> np.ndarray:
        vw = self.views[view] if self.views else None
        w, h, _ = self.level_info(0, view) if vw is None else (vw.width, vw.height, 0)
        out = np.zeros((h, w), dtype=np.float16)
        self._check(lib.dp_read_gray(self._ctx, view, ptr(out)))
        return out

    def fast_refine(self, patches: np.ndarray, cell: int, mode: int = N.MODE_FAST_REFINE) -> np.ndarray:
        """Performance-mode refine (or one fast evaluation) in place; accept flags."""
        return self.refine(patches, cell, mode)

    def fast_expand(self, parents: np.ndarray):
        """Expand::ExpandPatch children refined in performance mode."""
        parents = np.ascontiguousarray(parents)
        assert parents.dtype == PATCH_DTYPE
        kids = empty_patches(4 * len(parents))
        acc = np.zeros(4 * len(parents), dtype=np.uint8)
        self._check(lib.dp_fast_expand_batch(self._ctx, ptr(parents), len(parents), ptr(kids), ptr(acc)))
        return kids, acc

    def fast_expand_device(self, d_parents: int, n: int, d_children: int, d_accept: int | None,
                           stream: int | None = None):
        self._check(lib.dp_fast_expand_batch_device(self._ctx, ctypes.c_void_p(d_parents), n,
                                                    ctypes.c_void_p(d_children),
                                                    ctypes.c_void_p(d_accept) if d_accept else None,
                                                    ctypes.c_void_p(stream) if stream else None))

    def fast_last_stats(self) -> dict:
        st = N.DpFastStats()
        self._check(lib.dp_fast_last_stats(self._ctx, ctypes.byref(st)))
        return {name: getattr(st, name) for name, _ in N.DpFastStats._fields_}

    def evaluate(self, patches: np.ndarray, cell: int) -> np.ndarray:
        out = np.zeros(len(patches), dtype=np.float32)
        self._check(lib.dp_eval_batch(self._ctx, ptr(patches), len(patches), cell, ptr(out)))
        return out

    def optimize(self, patches: np.ndarray, cell: int) -> np.ndarray:
        """OptimizationOpenCV::Optimize over a batch (always accepts)."""
        return self.refine(patches, cell, N.MODE_NM)

    def filter(self, patches: np.ndarray, cell: int) -> np.ndarray:
        """Optimization::FilterByErrorMeasurement over a batch."""
        return self.refine(patches, cell, N.MODE_FILTER)

    def densify(self, seeds_xyz: np.ndarray, copy: bool = True):
        """dp_densify: (patches, stats).  copy=False returns a view of the
        library's pinned result buffer instead of a copy -- valid until the next
        densify on this engine, the C ABI's own contract for *out
        (include/densepoints.h dp_densify)."""
        seeds = np.ascontiguousarray(seeds_xyz, dtype=np.float64).reshape(-1, 3)
        out = ctypes.c_void_p()
        n = ctypes.c_int64()
        st = N.DpDensifyStats()
        self._check(lib.dp_densify(self._ctx, ptr(seeds), len(seeds), ctypes.byref(out), ctypes.byref(n),
                                   ctypes.byref(st)))
        stats = {name: getattr(st, name) for name, _ in N.DpDensifyStats._fields_}
        return result_array(out.value, n.value, copy), stats


    # ---- one generation at a time (multi-GPU partitioning; dist.py) ----
    def densify_begin(self, seeds_xyz: np.ndarray) -> N.DpGeneration:
        seeds = np.ascontiguousarray(seeds_xyz, dtype=np.float64).reshape(-1, 3)
        g = N.DpGeneration()
        self._check(lib.dp_densify_begin(self._ctx, ptr(seeds), len(seeds), ctypes.byref(g)))
        return g

    def densify_commit(self, gen: N.DpGeneration, cand: np.ndarray, acc: np.ndarray) -> N.DpGeneration:
        cand = np.ascontiguousarray(cand, dtype=PATCH_DTYPE)
        acc = np.ascontiguousarray(acc, dtype=np.uint8)
        self._check(lib.dp_densify_commit(self._ctx, ctypes.byref(gen), ptr(cand), ptr(acc), len(cand)))
        return gen

    def densify_run(self, gen: N.DpGeneration, max_generations: int = 1 << 30) -> N.DpGeneration:
        """Up to max_generations expansion generations device-resident on this
        context (dp_densify_run: 8 per host wait)."""
        self._check(lib.dp_densify_run(self._ctx, ctypes.byref(gen), int(min(max_generations, 2**31 - 1))))
        return gen

    def densify_run_until(self, gen: N.DpGeneration, yield_items: int, max_generations: int = 1 << 30):
        """dp_densify_run_until: device-resident generations until the densify
        ends or the next generation has >= yield_items items (returned unrun);
        (gen, objective evaluations this call spent)."""
        ev = ctypes.c_int64()
        self._check(lib.dp_densify_run_until(self._ctx, ctypes.byref(gen), int(min(max_generations, 2**31 - 1)),
                                             int(yield_items), ctypes.byref(ev)))
        return gen, int(ev.value)

    # ---- partitioned generations (reference-view super-tiles) ----
    def densify_owners(self, gen: N.DpGeneration, world: int, tile_px: int = 64):
        """(owner rank per item, fallback flag -- always False since the round-4
        partition spec) of the generation: dp_densify_owners."""
        own = np.zeros(gen.items, dtype=np.int32)
        fb = ctypes.c_int32()
        self._check(lib.dp_densify_owners(self._ctx, ctypes.byref(gen), world, tile_px, ptr(own), ctypes.byref(fb)))
        return own, bool(fb.value)

    def densify_partition_stats(self) -> dict:
        """The last partition's {items, world, tiles, split_items}
        (dp_densify_partition_stats): distinct super-tiles, and items in the
        tiles a cut shares between two ranks."""
        st = np.zeros(4, dtype=np.int64)
        self._check(lib.dp_densify_partition_stats(self._ctx, ptr(st)))
        return {"items": int(st[0]), "world": int(st[1]), "tiles": int(st[2]), "split_items": int(st[3])}

    def densify_refine_items(self, gen: N.DpGeneration, items: np.ndarray):
        items = np.ascontiguousarray(items, dtype=np.int64)
        n = len(items) * gen.per_item
        cand = empty_patches(n)
        acc = np.zeros(n, dtype=np.uint8)
        self._check(lib.dp_densify_refine_items(self._ctx, ctypes.byref(gen), ptr(items), len(items), ptr(cand),
                                                ptr(acc)))
        return cand, acc

    # ---- the one-wait device protocol: everything on the caller's stream ----
    def densify_partition_async(self, gen: N.DpGeneration, world: int, tile_px: int = 64,
                                stream: int | None = None):
        """(device address of the rank-major item order, items per rank):
        dp_densify_partition_async -- queued on `stream`, no host wait (the
        shares are floor(r n / world) cuts; the statistics come back with the
        commit)."""
        d_order = ctypes.c_void_p()
        counts = np.zeros(world, dtype=np.int64)
        self._check(lib.dp_densify_partition_async(self._ctx, ctypes.byref(gen), world, tile_px,
                                                   ctypes.c_void_p(stream) if stream else None,
                                                   ctypes.byref(d_order), ptr(counts)))
        return int(d_order.value or 0), counts

    def densify_refine_share_async(self, gen: N.DpGeneration, d_items: int, n: int, d_slot: int, stride: int,
                                   stream: int | None = None) -> None:
        """Refine this rank's n items (device list d_items) and compact the
        accepted candidates into its exchange slot (header + stride records)."""
        self._check(lib.dp_densify_refine_share_async(self._ctx, ctypes.byref(gen), ctypes.c_void_p(d_items), n,
                                                      ctypes.c_void_p(d_slot), stride,
                                                      ctypes.c_void_p(stream) if stream else None))

    def densify_commit_gathered_device(self, gen: N.DpGeneration, d_recs: int, stride: int, world: int,
                                       stream: int | None = None) -> int:
        """Commit from the `world` gathered rank slots at d_recs (stride + 1
        records each); the generation's one host wait.  Returns the records
        exchanged."""
        ex = ctypes.c_int64()
        self._check(lib.dp_densify_commit_gathered_device(self._ctx, ctypes.byref(gen), ctypes.c_void_p(d_recs), stride,
                                                          world, ctypes.c_void_p(stream) if stream else None,
                                                          ctypes.byref(ex)))
        return int(ex.value)

    def densify_result(self, copy: bool = True):
        """dp_densify_result: (patches, stats); copy=False as in densify()."""
        out = ctypes.c_void_p()
        n = ctypes.c_int64()
        st = N.DpDensifyStats()
        self._check(lib.dp_densify_result(self._ctx, ctypes.byref(out), ctypes.byref(n), ctypes.byref(st)))
        stats = {name: getattr(st, name) for name, _ in N.DpDensifyStats._fields_}
        return result_array(out.value, n.value, copy), stats


class PMVS:
    """PMVS::PMVS (methods/pmvs/pmvs.h:14-35): AddCamera, Run, GetPointCloud.

    Seed points come from the caller (feature matching is out of scope; the
    reference's Matcher::GenerateSeeds output is just a list of 3-D points).
    """

    def __init__(self, options: Options | None = None, device: int = 0, fast: FastOptions | None = None):
        """fast: FastOptions with densify = 1 runs the whole loop in performance
        mode (no reference counterpart; dp_fast_options.densify)"""
        self.options = options or Options()
        self.device = device
        self.fast = fast
        self.views: list[View] = []
        self.patches = empty_patches(0)
        self.stats: dict = {}

    def add_camera(self, view: View) -> None:
        # PMVS::AddCamera (pmvs.cpp:11-20): views whose image failed to load are dropped
        if view.image is None or view.image.size == 0:
            return
        self.views.append(view)

    def run(self, seeds_xyz=None, filter_passes: int = 0, matcher_options=None) -> bool:
        """PMVS::Run (pmvs.cpp:22-43).  With seeds_xyz None the seeds come from
        Matcher::GenerateSeeds on the device (PMVS::InsertSeeds, pmvs.cpp:29-34);
        filter_passes != 0 then applies FilterPatches (pmvs.h:27; spec in
        dp_filter_patches)."""
        from .matcher import Matcher

        with Engine(self.options, self.device) as eng:
            eng.set_views(self.views)
            if self.fast is not None:
                eng.set_fast_options(self.fast)
            seed_stats = None
            if seeds_xyz is None:
                m = Matcher(eng, matcher_options)
                seeds_xyz = m.generate_seeds()
                seed_stats = m.stats
            self.patches, self.stats = eng.densify(np.asarray(seeds_xyz, dtype=np.float64))
            if seed_stats is not None:
                self.stats["seed_generation"] = seed_stats
            if filter_passes:
                keep = eng.filter_patches(self.patches, filter_passes)
                self.stats["filtered_out"] = int(len(keep) - keep.sum())
                self.patches = self.patches[keep == 1]
        return True

    def get_point_cloud(self) -> np.ndarray:
        return self.patches


def ncc_score(a: np.ndarray, b: np.ndarray, denom_min: float = 0.1) -> float:
    """NCCScore (error_measurements.cpp:36-60) on integer-valued textures: exact
    integer moments, finished by the library's fp64 NCC (same code as the
    kernels).  Empty input -> -1 like the reference."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.size == 0 or b.size == 0:
        return -1.0
    ai = a.astype(np.int64).ravel()
    bi = b.astype(np.int64).ravel()
    return float(lib.dp_probe_ncc(int(ai.size), int(ai.sum()), int((ai * ai).sum()), int(bi.sum()),
                                  int((bi * bi).sum()), int((ai * bi).sum()), float(denom_min)))


def read_scene_json(path: str) -> tuple[str, list[tuple[str, np.ndarray]]]:
    """IO::JSONReader (json_reader.cpp:9-29): {"imagesPath", "views": [{"filename",
    "projectionMatrix": [[4],[4],[4]]}]}."""
    with open(path) as f:
        d = json.load(f)
    images_path = d["imagesPath"]
    views = []
    for v in d["views"]:
        P = np.asarray(v["projectionMatrix"], dtype=np.float64).reshape(3, 4)
        views.append((os.path.join(images_path, v["filename"]), P))
    return images_path, views


def write_ply(path: str, patches: np.ndarray) -> None:
    """PMVS::PrintCloud (utils.cpp:9-50) through rplycpp's ASCII writer:
    x y z (float, %g) red green blue (uchar) nx ny nz (float)."""
    with open(path, "w") as f:
        f.write("ply\nformat ascii 1.0\n")
        f.write(f"element vertex {len(patches)}\n")
        for n in ("x", "y", "z"):
            f.write(f"property float {n}\n")
        for n in ("red", "green", "blue"):
            f.write(f"property uchar {n}\n")
        for n in ("nx", "ny", "nz"):
            f.write(f"property float {n}\n")
        f.write("end_header\n")
        for p in patches:
            x, y, z = (float(v) for v in p["pos"])
            r, g, b = (int(v) for v in p["rgb"])
            nx, ny, nz = (float(v) for v in p["normal"])
            f.write(f"{x:g} {y:g} {z:g} {r} {g} {b} {nx:g} {ny:g} {nz:g}\n")

"""ctypes wrapper of oracle/build/liboracle.so -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  It is the checker, never the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

MODE_EVAL, MODE_FILTER, MODE_NM, MODE_SEED, MODE_EXPAND, MODE_FAST_EVAL, MODE_FAST_REFINE = range(7)

PATCH_DTYPE = np.dtype(
    [
        ("pos", "<f4", 3),
        ("normal", "<f4", 3),
        ("ref", "<u4"),
        ("seq", "<u4"),
        ("vis", "<u8", 2),
        ("cand", "<u8", 2),
        ("score", "<f4"),
        ("evals", "<u4"),
        ("rgb", "u1", 3),
        ("flags", "u1"),
        ("parent", "<u4"),
    ],
    align=True,
)


class OrOptions(ctypes.Structure):
    _fields_ = [
        ("seed_cell_size", ctypes.c_int32),
        ("expand_cell_size", ctypes.c_int32),
        ("grid_scale", ctypes.c_int32),
        ("max_patches_per_cell", ctypes.c_int32),
        ("min_visible", ctypes.c_int32),
        ("min_expand_visible", ctypes.c_int32),
        ("nm_max_evals", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("ncc_threshold", ctypes.c_double),
        ("visible_angle", ctypes.c_double),
        ("candidate_angle", ctypes.c_double),
        ("nm_step", ctypes.c_double * 3),
        ("nm_eps", ctypes.c_double),
        ("ncc_denom_min", ctypes.c_double),
        ("max_pops", ctypes.c_int64),
    ]


class OrFastOptions(ctypes.Structure):
    """or_fast_options (layout of include/densepoints.h dp_fast_options)."""
    _fields_ = [
        ("iters", ctypes.c_int32),
        ("margin", ctypes.c_int32),
        ("tile_budget", ctypes.c_int32),
        ("max_views", ctypes.c_int32),
        ("fd_step", ctypes.c_float),
        ("ls_step", ctypes.c_float),
        ("densify", ctypes.c_int32),
        ("gradient", ctypes.c_int32),
        ("filter_max_views", ctypes.c_int32),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def _load():
    if not os.path.exists(LIB):
        build()
    L = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    sig = {
        "or_default_options": (None, [P]),
        "or_view_geometry": (ctypes.c_int, [P, P, P, P, P]),
        "or_ncc_int": (ctypes.c_double, [P, P, ctypes.c_int, ctypes.c_double]),
        "or_sincos": (None, [ctypes.c_double, P, P]),
        "or_acos": (ctypes.c_double, [ctypes.c_double]),
        "or_scene_create": (P, [ctypes.c_int, P, P, P, P, P]),
        "or_scene_destroy": (None, [P]),
        "or_scene_view_info": (ctypes.c_int, [P, ctypes.c_int, P, P]),
        "or_texture": (ctypes.c_int, [P, ctypes.c_int, P, ctypes.c_int, P]),
        "or_init_related": (ctypes.c_int, [P, P]),
        "or_scores": (ctypes.c_int, [P, P, P, P, ctypes.c_int, P, P]),
        "or_objective": (ctypes.c_double, [P, P, P, ctypes.c_int]),
        "or_refine_batch": (ctypes.c_int, [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]),
        "or_seeds_to_patches": (ctypes.c_int, [P, P, ctypes.c_int, P]),
        "or_expand_children": (ctypes.c_int, [P, P, P, P]),
        "or_expand_batch": (ctypes.c_int, [P, P, ctypes.c_int, P, P, ctypes.c_int]),
        "or_densify": (ctypes.c_int64, [P, P, ctypes.c_int, P, ctypes.c_int64, P, P]),
        "or_color": (None, [P, P]),
        "or_org_create": (P, [P]),
        "or_org_destroy": (None, [P]),
        "or_org_insert": (ctypes.c_int, [P, P, ctypes.c_uint32, ctypes.c_uint32, P]),
        "or_pyr_down": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, P]),
        "or_filter_patches": (ctypes.c_int, [P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_double, P]),
        # performance mode (or_fast.c)
        "or_fast_default_options": (None, [P]),
        "or_gray_plane": (ctypes.c_int, [P, ctypes.c_int, P]),
        "or_fast_refine_batch": (ctypes.c_int, [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int]),
        "or_fast_expand_batch": (ctypes.c_int, [P, P, ctypes.c_int, P, P, P, ctypes.c_int]),
        "or_fast_grad_probe": (ctypes.c_int, [P, P, ctypes.c_int, P, P, P]),
        "or_fast_grad_q24": (ctypes.c_int32, [ctypes.c_double]),
        "or_trace_set": (None, [P, ctypes.c_int64]),
        "or_trace_count": (ctypes.c_int64, []),
        # seed generation (or_seeds.c)
        "or_orb_pattern": (None, [P]),
        "or_features_per_level": (None, [ctypes.c_int, ctypes.c_double, ctypes.c_int, P]),
        "or_knn_match": (ctypes.c_int, [P, ctypes.c_int64, P, ctypes.c_int64, P, P]),
        "or_fundamental_matrix": (ctypes.c_int, [P, P, P]),
        "or_epipolar_distance": (ctypes.c_float, [P, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float]),
        "or_triangulate": (None, [ctypes.c_int64, P, P, P, P]),
        "or_seeds_run": (P, [ctypes.c_int, P, P, P, P, P]),
        "or_seeds_free": (None, [P]),
        "or_seeds_counts": (None, [P, P]),
        "or_seeds_view": (ctypes.c_int64, [P, ctypes.c_int, P, P]),
        "or_seeds_pair": (ctypes.c_int64, [P, ctypes.c_int, P, P]),
        "or_seeds_points": (None, [P, P]),
        "or_seeds_desc_bytes": (ctypes.c_int, [P]),
        "or_knn_match_w": (ctypes.c_int, [P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int, P, P]),
        # AKAZE (or_akaze.c)
        "or_akaze_levels": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, P, P]),
        "or_akaze_plane": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]),
        "or_akaze_halfsample": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.c_int]),
    }
    for k, (r, a) in sig.items():
        f = getattr(L, k)
        f.restype = r
        f.argtypes = a
    return L


lib = _load()


def _p(a):
    return None if a is None else a.ctypes.data


def default_options() -> OrOptions:
    o = OrOptions()
    lib.or_default_options(ctypes.byref(o))
    return o


def options_from(opts) -> OrOptions:
    """Copy a densepoints_amd Options (identical POD layout) or an OrOptions."""
    if isinstance(opts, OrOptions):
        return opts
    o = OrOptions()
    raw = bytes(opts.to_c())
    ctypes.memmove(ctypes.byref(o), raw, ctypes.sizeof(o))
    return o


class Scene:
    """CPU restatement of the reference's view set + patch loop."""

    def __init__(self, P, images, options=None):
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(-1, 12))
        self.V = len(P)
        self._imgs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        W = np.array([im.shape[1] for im in self._imgs], dtype=np.int32)
        H = np.array([im.shape[0] for im in self._imgs], dtype=np.int32)
        ptrs = (ctypes.c_void_p * self.V)(*[im.ctypes.data for im in self._imgs])
        self.opt = options_from(options) if options is not None else default_options()
        self._h = lib.or_scene_create(self.V, _p(P), _p(W), _p(H), ptrs, ctypes.byref(self.opt))
        if not self._h:
            raise ValueError("or_scene_create failed")
        self._keep = (P, W, H, ptrs)

    def __del__(self):
        if getattr(self, "_h", None):
            lib.or_scene_destroy(self._h)
            self._h = None

    def seeds_to_patches(self, xyz):
        xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 3)
        out = np.zeros(len(xyz), dtype=PATCH_DTYPE)
        lib.or_seeds_to_patches(self._h, _p(xyz), len(xyz), _p(out))
        return out

    def refine(self, patches, cell, mode, nthreads=0):
        acc = np.zeros(len(patches), dtype=np.uint8)
        rc = lib.or_refine_batch(self._h, _p(patches), len(patches), cell, mode, _p(acc), nthreads)
        if rc != 0:
            raise ValueError("or_refine_batch failed")
        return acc

    def texture(self, view, corners, cell):
        c = np.ascontiguousarray(corners, dtype=np.float64).reshape(12)
        g = np.zeros(cell * cell, dtype=np.int32)
        ok = lib.or_texture(self._h, view, _p(c), cell, _p(g))
        return (g.reshape(cell, cell) if ok else None)

    def objective(self, patch, x, cell):
        x = np.ascontiguousarray(x, dtype=np.float64)
        p = np.ascontiguousarray(np.array([patch], dtype=PATCH_DTYPE))
        return lib.or_objective(self._h, _p(p), _p(x), cell)

    def expand_children(self, parent):
        p = np.ascontiguousarray(np.array([parent], dtype=PATCH_DTYPE))
        out = np.zeros(4, dtype=PATCH_DTYPE)
        acc = np.zeros(4, dtype=np.uint8)
        lib.or_expand_children(self._h, _p(p), _p(out), _p(acc))
        return out, acc

    def expand(self, parents, nthreads=0):
        parents = np.ascontiguousarray(parents)
        kids = np.zeros(4 * len(parents), dtype=PATCH_DTYPE)
        acc = np.zeros(4 * len(parents), dtype=np.uint8)
        lib.or_expand_batch(self._h, _p(parents), len(parents), _p(kids), _p(acc), nthreads)
        return kids, acc

    def densify(self, seeds, cap=None):
        seeds = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1, 3)
        if cap is None:
            cap = 2_000_000
        out = np.zeros(cap, dtype=PATCH_DTYPE)
        nseed = ctypes.c_int64()
        pops = ctypes.c_int64()
        n = lib.or_densify(self._h, _p(seeds), len(seeds), _p(out), cap, ctypes.byref(nseed), ctypes.byref(pops))
        return out[: min(n, cap)].copy(), {"patches": n, "seed_patches": nseed.value, "pops": pops.value}


def fast_options(opts=None, **kw) -> OrFastOptions:
    """Copy a densepoints_amd FastOptions (identical layout), or defaults + kw."""
    o = OrFastOptions()
    if opts is not None:
        raw = bytes(opts.to_c() if hasattr(opts, "to_c") else opts)
        ctypes.memmove(ctypes.byref(o), raw, ctypes.sizeof(o))
    else:
        lib.or_fast_default_options(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _scene_fast_refine(self, patches, cell, mode=MODE_FAST_REFINE, fo=None, nthreads=0):
    """Performance-mode refine (or_fast.c spec) in place; returns accept flags."""
    fo = fast_options() if fo is None else fast_options(fo)
    acc = np.zeros(len(patches), dtype=np.uint8)
    if lib.or_fast_refine_batch(self._h, _p(patches), len(patches), cell, mode, ctypes.byref(fo), _p(acc),
                                nthreads) != 0:
        raise ValueError("or_fast_refine_batch failed")
    return acc


def _scene_fast_expand(self, parents, fo=None, nthreads=0):
    fo = fast_options() if fo is None else fast_options(fo)
    parents = np.ascontiguousarray(parents)
    kids = np.zeros(4 * len(parents), dtype=PATCH_DTYPE)
    acc = np.zeros(4 * len(parents), dtype=np.uint8)
    lib.or_fast_expand_batch(self._h, _p(parents), len(parents), ctypes.byref(fo), _p(kids), _p(acc), nthreads)
    return kids, acc


def _scene_fast_grad_probe(self, patch, cell, fo=None):
    """Spec v4 at x = 0, staged at margin 0: (staged views, objective, gradient)."""
    fo = fast_options() if fo is None else fast_options(fo)
    one = np.ascontiguousarray(np.asarray(patch).reshape(1))
    f = ctypes.c_int32()
    g = np.zeros(3, dtype=np.float32)
    m = lib.or_fast_grad_probe(self._h, _p(one), cell, ctypes.byref(fo), ctypes.byref(f), _p(g))
    return m, f.value, g


def _scene_gray(self, view):
    W, H = self._keep[1][view], self._keep[2][view]
    out = np.zeros((H, W), dtype=np.uint8)
    lib.or_gray_plane(self._h, view, _p(out))
    return out


Scene.fast_refine = _scene_fast_refine
Scene.fast_expand = _scene_fast_expand
Scene.fast_grad_probe = _scene_fast_grad_probe
Scene.gray = _scene_gray


def _scene_filter(self, patches, passes=3, min_neighbor_frac=0.25):
    """or_filter_patches: keep flags of the PMVS-style filter (dp_filter_patches spec)."""
    patches = np.ascontiguousarray(patches, dtype=PATCH_DTYPE)
    keep = np.zeros(len(patches), dtype=np.uint8)
    if lib.or_filter_patches(self._h, _p(patches), len(patches), passes, min_neighbor_frac, _p(keep)) != 0:
        raise ValueError("or_filter_patches failed")
    return keep


Scene.filter_patches = _scene_filter


class _Gen:
    """Mirror of dp_generation (include/densepoints.h)."""

    def __init__(self, items, head, per_item, cell, seq0, index):
        self.items, self.head, self.per_item, self.cell, self.seq0, self.index = (
            items, head, per_item, cell, seq0, index)


class GenerationEngine:
    """The generation-at-a-time densify protocol of the C ABI
    (dp_densify_begin/refine/commit/result) restated on the oracle: test
    infrastructure for the multi-rank driver (densepoints_amd.dist.densify_sharded)
    on the CPU.  Same sequence numbering, pop cap and organizer order as
    or_densify (which it must reproduce)."""

    def __init__(self, scene: "Scene", threads: int = 2, fast=None):
        """fast: dp_fast_options / FastOptions with densify = 1 -> the
        performance-mode densify (seed stage and expansions by the fast refine,
        or_fast.c), as dp_densify runs it"""
        self.S = scene
        self.threads = threads
        self.org = None
        self._P = scene._keep[0]
        self.fast = None if fast is None else fast_options(fast)

    def _refine_seeds(self, r, cell):
        if self.fast is not None:
            return self.S.fast_refine(r, cell, MODE_FAST_REFINE, self.fast, self.threads)
        return self.S.refine(r, cell, 3, self.threads)  # MODE_SEED

    def _expand(self, parents):
        if self.fast is not None:
            return self.S.fast_expand(parents, self.fast, self.threads)
        return self.S.expand(parents, self.threads)

    def densify_all(self, seeds):
        """every generation in turn (dp_densify's result): the store"""
        g = self.densify_begin(seeds)
        while g.items:
            cand, acc = self.densify_refine(g, 0, g.items)
            g = self.densify_commit(g, cand, acc)
        return np.array(self.store, dtype=PATCH_DTYPE)

    def __del__(self):
        if self.org:
            lib.or_org_destroy(self.org)

    def densify_begin(self, seeds):
        if self.org:
            lib.or_org_destroy(self.org)
        self.org = lib.or_org_create(self.S._h)
        seeds = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1, 3)
        self.sp = self.S.seeds_to_patches(seeds)
        self.nseeds = len(seeds)
        self.store = []
        return _Gen(len(seeds), 0, 1, self.S.opt.seed_cell_size, 0, 0)

    def densify_refine(self, g, lo, hi):
        if g.index == 0:
            r = self.sp[lo:hi].copy()
            acc = self._refine_seeds(r, g.cell)
            return r, acc
        parents = np.array(self.store[g.head + lo: g.head + hi], dtype=PATCH_DTYPE)
        kids, acc = self._expand(parents)
        q = g.head + lo + np.repeat(np.arange(hi - lo), 4)
        kids["parent"] = q.astype(np.uint32)
        acc[q >= self.S.opt.max_pops] = 0  # past the pop cap (expand.cpp:95)
        return kids, acc

    # ---- partitioned generations (dp_densify_owners spec) ----
    def densify_owners(self, g, world, tile_px=64):
        """Owner rank per item (include/densepoints.h, partition spec): the
        centre projected into the reference view (fp64, ((p0 x + p1 y) + p2 z)
        + p3 then one division), tile coordinates floored and clamped to
        [-1, TY] / [-1, TX] (TX, TY: tiles of the largest view), the dense key
        (ref (TY + 2) + ty + 1) (TX + 2) + tx + 1, items stable-sorted by key
        and cut into `world` contiguous shares lo_r = floor(r n / world).
        Returns (owners, False); densify_partition_stats() gives the
        partition's statistics."""
        items = self.sp if g.index == 0 else np.array(self.store[g.head: g.head + g.items], dtype=PATCH_DTYPE)
        n = len(items)
        P = np.stack([self._P[int(r)] for r in items["ref"]]) if n else np.zeros((0, 12))
        X = items["pos"].astype(np.float64)
        h = [((P[:, 4 * k] * X[:, 0] + P[:, 4 * k + 1] * X[:, 1]) + P[:, 4 * k + 2] * X[:, 2]) + P[:, 4 * k + 3]
             for k in range(3)]
        with np.errstate(divide="ignore", invalid="ignore"):
            u, w = h[0] / h[2], h[1] / h[2]
        Wmax, Hmax = int(max(self.S._keep[1].max(), 1)), int(max(self.S._keep[2].max(), 1))
        TX, TY = -(-Wmax // tile_px), -(-Hmax // tile_px)

        def tc(q, tmax):
            with np.errstate(invalid="ignore"):
                q = q / float(tile_px)
                ok = (q > -2.0e9) & (q < 2.0e9)
            t = np.where(ok, np.floor(np.where(ok, q, 0.0)), 0.0).astype(np.int64)
            return (np.clip(t, -1, tmax) + 1).astype(np.uint64)

        key = ((items["ref"].astype(np.uint64) * np.uint64(TY + 2) + tc(w, TY)) * np.uint64(TX + 2) + tc(u, TX))
        order = np.argsort(key, kind="stable")
        lo = np.array([(r * n) // world for r in range(world + 1)], dtype=np.int64)
        own = np.empty(n, dtype=np.int32)
        for r in range(world):
            own[order[lo[r]:lo[r + 1]]] = r
        sk = key[order]
        split = np.zeros(n, dtype=bool)
        for r in range(1, world):
            c = int(lo[r])
            if 0 < c < n and sk[c - 1] == sk[c]:
                split |= sk == sk[c]
        tiles = int(np.count_nonzero(np.diff(sk))) + 1 if n else 0
        self._pstats = {"items": n, "world": world, "tiles": tiles, "split_items": int(split.sum())}
        return own, False

    def densify_partition_stats(self):
        return dict(self._pstats)

    def densify_refine_items(self, g, items):
        items = np.asarray(items, dtype=np.int64)
        if g.index == 0:
            r = self.sp[items].copy()
            acc = self._refine_seeds(r, g.cell)
            return r, acc
        parents = np.array([self.store[g.head + int(i)] for i in items], dtype=PATCH_DTYPE)
        kids, acc = self._expand(parents)
        q = g.head + np.repeat(items, 4)
        kids["parent"] = q.astype(np.uint32)
        acc[q >= self.S.opt.max_pops] = 0  # past the pop cap (expand.cpp:95)
        return kids, acc

    def densify_commit(self, g, cand, acc):
        out = np.zeros(1, dtype=PATCH_DTYPE)
        for i in range(len(cand)):
            if not acc[i]:
                continue
            par = 0xFFFFFFFF if g.index == 0 else g.head + i // 4
            c1 = np.ascontiguousarray(cand[i:i + 1])
            if lib.or_org_insert(self.org, _p(c1), len(self.store), par, _p(out)):
                self.store.append(out[0].copy())
        head = 0 if g.index == 0 else g.head + g.items  # the store size before this generation
        np_ = len(self.store)
        items = np_ - head if (head < np_ and head < self.S.opt.max_pops) else 0
        return _Gen(items, head, 4, self.S.opt.expand_cell_size, self.nseeds + 4 * head, g.index + 1)

    def densify_result(self):
        res = np.array(self.store, dtype=PATCH_DTYPE) if self.store else np.zeros(0, dtype=PATCH_DTYPE)
        return res, {"patches": len(res), "evals": 0, "refine_ms": 0.0}


def ncc_int(a, b, denom_min=0.1):
    a = np.ascontiguousarray(a, dtype=np.int32).ravel()
    b = np.ascontiguousarray(b, dtype=np.int32).ravel()
    return lib.or_ncc_int(_p(a), _p(b), a.size, denom_min)


def view_geometry(P):
    P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(12))
    C = np.zeros(3)
    K = np.zeros(9)
    E = np.zeros(12)
    x = np.zeros(3)
    rc = lib.or_view_geometry(_p(P), _p(C), _p(K), _p(E), _p(x))
    return rc, C, K.reshape(3, 3), E.reshape(3, 4), x


def sincos(x):
    s = ctypes.c_double()
    c = ctypes.c_double()
    lib.or_sincos(float(x), ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def acos(x):
    return lib.or_acos(float(x))


def pyr_down(bgr):
    """cv::pyrDown of a BGR8 image (or_pyr_down)."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    H, W = bgr.shape[:2]
    out = np.zeros(((H + 1) // 2, (W + 1) // 2, 3), dtype=np.uint8)
    assert lib.or_pyr_down(_p(bgr), W, H, _p(out)) == 0
    return out


def level_scene(P, images, level):
    """(P_L, images_L) of the level-L scene: pyrDown^L images and projection
    rows 0-1 scaled by 2^-L (include/densepoints.h dp_set_level)."""
    P = np.asarray(P, dtype=np.float64).reshape(-1, 3, 4).copy()
    imgs = list(images)
    for _ in range(level):
        imgs = [pyr_down(im) for im in imgs]
    P[:, :2, :] *= 2.0 ** -level
    return P, imgs


# ---------------------------------------------------------------------------
# seed generation (or_seeds.c): Matcher::GenerateSeeds restated
# ---------------------------------------------------------------------------
class OrMatcherOptions(ctypes.Structure):
    _fields_ = [
        ("n_features", ctypes.c_int32),
        ("n_levels", ctypes.c_int32),
        ("scale_factor", ctypes.c_double),
        ("edge_threshold", ctypes.c_int32),
        ("fast_threshold", ctypes.c_int32),
        ("cell_size", ctypes.c_int32),
        ("max_keypoints_per_cell", ctypes.c_int32),
        ("epipolar_matching", ctypes.c_int32),
        ("max_epipolar_distance", ctypes.c_float),
        ("nn_match_ratio", ctypes.c_float),
        ("matcher_type", ctypes.c_int32),
        ("detector_type", ctypes.c_int32),
        ("akaze_threshold", ctypes.c_float),
    ]


DETECTOR_AKAZE, DETECTOR_ORB = 0, 1

KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("response", "<f4"), ("angle", "<f4"), ("octave", "<i4"), ("reserved", "<i4")]
)


def matcher_options(**kw) -> OrMatcherOptions:
    o = OrMatcherOptions(n_features=40000, n_levels=8, scale_factor=1.2, edge_threshold=31, fast_threshold=20,
                         cell_size=16, max_keypoints_per_cell=4, epipolar_matching=0, max_epipolar_distance=1.5,
                         nn_match_ratio=0.7, matcher_type=0, detector_type=DETECTOR_ORB, akaze_threshold=0.001)
    for k, v in kw.items():
        setattr(o, k, int(v) if isinstance(v, bool) else v)
    return o


def orb_pattern() -> np.ndarray:
    a = np.zeros(1024, dtype=np.int8)
    lib.or_orb_pattern(_p(a))
    return a.reshape(512, 2)


def features_per_level(n, sf, L) -> np.ndarray:
    a = np.zeros(L, dtype=np.int32)
    lib.or_features_per_level(n, sf, L, _p(a))
    return a


def knn_match(q: np.ndarray, t: np.ndarray, width: int = 32):
    q = np.ascontiguousarray(q, dtype=np.uint8).reshape(-1, width)
    t = np.ascontiguousarray(t, dtype=np.uint8).reshape(-1, width)
    idx = np.zeros((len(q), 2), dtype=np.int32)
    dist = np.zeros((len(q), 2), dtype=np.int32)
    lib.or_knn_match_w(_p(q), len(q), _p(t), len(t), width, _p(idx), _p(dist))
    return idx, dist


def akaze_levels(W: int, H: int):
    """AKAZE evolution levels: (w, h, octave, sigma_size, FED steps) rows, esigma"""
    info = np.zeros((16, 5), dtype=np.int32)
    es = np.zeros(16, dtype=np.float32)
    n = lib.or_akaze_levels(W, H, _p(info), _p(es))
    return info[:n], es[:n]


def akaze_halfsample(src: np.ndarray) -> np.ndarray:
    """AKAZE's halfsample_image (cv::resize INTER_AREA to floor(side / 2)) of
    an fp32 plane, as the oracle's scale space computes it"""
    src = np.ascontiguousarray(src, dtype=np.float32)
    sh, sw = src.shape
    out = np.zeros((sh // 2, sw // 2), dtype=np.float32)
    if lib.or_akaze_halfsample(_p(src), sw, sh, _p(out), sw // 2, sh // 2) != 0:
        raise ValueError("or_akaze_halfsample failed")
    return out


def akaze_plane(img_bgr: np.ndarray, level: int, which: int):
    """one plane of the AKAZE scale space of a BGR8 view (0 Lt, 1 Lx, 2 Ly,
    3 Ldet) and the contrast factor per level"""
    img = np.ascontiguousarray(img_bgr, dtype=np.uint8)
    H, W = img.shape[:2]
    info, _ = akaze_levels(W, H)
    w, h = int(info[level, 0]), int(info[level, 1])
    out = np.zeros((h, w), dtype=np.float32)
    kc = np.zeros(16, dtype=np.float32)
    if lib.or_akaze_plane(_p(img), W, H, level, which, _p(out), _p(kc)) != 0:
        raise ValueError("or_akaze_plane failed")
    return out, kc[: len(info)]


def fundamental_matrix(P1, P2) -> np.ndarray:
    a = np.ascontiguousarray(P1, dtype=np.float64).reshape(12)
    b = np.ascontiguousarray(P2, dtype=np.float64).reshape(12)
    F = np.zeros(9)
    lib.or_fundamental_matrix(_p(a), _p(b), _p(F))
    return F.reshape(3, 3)


def epipolar_distance(F, x1, y1, x2, y2) -> float:
    f = np.ascontiguousarray(F, dtype=np.float64).reshape(9)
    return lib.or_epipolar_distance(_p(f), x1, y1, x2, y2)


def triangulate(projections: list, observations: list) -> np.ndarray:
    off = np.zeros(len(projections) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(p) for p in projections])
    P = np.ascontiguousarray(np.concatenate([np.asarray(p, dtype=np.float64).reshape(-1, 12) for p in projections]))
    obs = np.ascontiguousarray(np.concatenate([np.asarray(o, dtype=np.float64).reshape(-1, 2) for o in observations]))
    X = np.zeros((len(projections), 3))
    lib.or_triangulate(len(projections), _p(off), _p(P), _p(obs), _p(X))
    return X


def seeds_run(P: np.ndarray, images: list, mo: OrMatcherOptions | None = None) -> dict:
    """Full GenerateSeeds on BGR8 images (H x W x 3); every stage's output."""
    mo = mo or matcher_options()
    V = len(images)
    P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(V, 12))
    imgs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
    W = np.array([im.shape[1] for im in imgs], dtype=np.int32)
    H = np.array([im.shape[0] for im in imgs], dtype=np.int32)
    ptrs = (ctypes.c_void_p * V)(*[im.ctypes.data for im in imgs])
    h = lib.or_seeds_run(V, _p(P), _p(W), _p(H), ptrs, ctypes.byref(mo))
    if not h:
        raise ValueError("or_seeds_run: image too small for the pyramid")
    try:
        c = np.zeros(7, dtype=np.int64)
        lib.or_seeds_counts(h, _p(c))
        out = {"counts": dict(zip(["views", "pairs", "detected", "keypoints", "ratio_matches", "matches", "points"],
                                  c.tolist())),
               "keypoints": [], "descriptors": [], "pairs": [], "q2t": []}
        db = lib.or_seeds_desc_bytes(h)
        for v in range(V):
            n = lib.or_seeds_view(h, v, None, None)
            kp = np.zeros(n, dtype=KEYPOINT_DTYPE)
            d = np.zeros((n, db), dtype=np.uint8)
            lib.or_seeds_view(h, v, _p(kp), _p(d))
            out["keypoints"].append(kp)
            out["descriptors"].append(d)
        for p in range(int(c[1])):
            n = lib.or_seeds_pair(h, p, None, None)
            fs = np.zeros(2, dtype=np.int32)
            q = np.zeros(n, dtype=np.int32)
            lib.or_seeds_pair(h, p, _p(fs), _p(q))
            out["pairs"].append((int(fs[0]), int(fs[1])))
            out["q2t"].append(q)
        pts = np.zeros((int(c[6]), 3))
        if len(pts):
            lib.or_seeds_points(h, _p(pts))
        out["points"] = pts
        return out
    finally:
        lib.or_seeds_free(h)

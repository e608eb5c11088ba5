"""Features::Matcher (modules/features/matcher.h:35-69) over the C ABI.

GenerateSeeds (matcher.cpp:18-43) runs entirely on the device: ORB (default)
or AKAZE detect, per-cell filter, rBRIEF / M-LDB descriptors, brute-force
Hamming kNN on MFMA, ratio and epipolar filters, multi-view DLT.  The standalone operators mirror the
reference's free functions (knnMatch, Geometry::ComputeFundamentalMatrix,
Geometry::DirectLinearTriangulation).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, fields

import numpy as np

from . import _native as N
from ._native import KEYPOINT_DTYPE, check, lib, ptr


@dataclass
class MatcherOptions:
    """MatcherOptions (matcher.h:14-33) plus the cv::ORB knobs the reference
    leaves at their defaults (ORB::create(40000), matcher.cpp:62)."""

    n_features: int = 40000
    n_levels: int = 8
    scale_factor: float = 1.2
    edge_threshold: int = 31
    fast_threshold: int = 20
    cell_size: int = 16
    max_keypoints_per_cell: int = 4
    epipolar_matching: bool = False
    max_epipolar_distance: float = 1.5
    nn_match_ratio: float = 0.7
    # MatcherType (matcher.h:12): KNN (default) or FLANN -- the LSH match() kept
    # iff distance < 30, answered exactly (include/densepoints.h DP_MATCHER_FLANN)
    matcher_type: int = 0
    # DetectorType (matcher.h:11): ORB (default) or AKAZE (AKAZE::create()
    # defaults, M-LDB 486-bit descriptors; threshold 0.001 unless set)
    detector_type: int = 1
    akaze_threshold: float = 0.001

    def to_c(self) -> N.DpMatcherOptions:
        o = N.DpMatcherOptions()
        lib.dp_default_matcher_options(ctypes.byref(o))
        for f in fields(self):
            v = getattr(self, f.name)
            setattr(o, f.name, int(v) if isinstance(v, bool) else v)
        return o


MATCHER_KNN, MATCHER_FLANN = 0, 1
DETECTOR_AKAZE, DETECTOR_ORB = 0, 1


class Matcher:
    """Seed generation on an Engine whose views are set (level 0 is used)."""

    def __init__(self, engine, options: MatcherOptions | None = None):
        self.engine = engine
        self.options = options or MatcherOptions()
        self.stats: dict = {}
        self.points = np.zeros((0, 3))

    def generate_seeds(self) -> np.ndarray:
        mo = self.options.to_c()
        out = ctypes.c_void_p()
        n = ctypes.c_int64()
        st = N.DpSeedStats()
        check(lib.dp_generate_seeds(self.engine.handle, ctypes.byref(mo), ctypes.byref(out), ctypes.byref(n),
                                    ctypes.byref(st)), self.engine.handle)
        pts = np.zeros((n.value, 3), dtype=np.float64)
        if n.value:
            ctypes.memmove(pts.ctypes.data, out.value, n.value * 24)
        self.points = pts
        self.stats = {name: getattr(st, name) for name, _ in N.DpSeedStats._fields_}
        return pts

    def keypoints(self, view: int):
        """(keypoints, descriptors) of one view after FilterKeypoints / compute."""
        kp = ctypes.c_void_p()
        desc = ctypes.c_void_p()
        n = ctypes.c_int64()
        check(lib.dp_seed_keypoints(self.engine.handle, view, ctypes.byref(kp), ctypes.byref(desc), ctypes.byref(n)),
              self.engine.handle)
        db = lib.dp_seed_descriptor_bytes(self.engine.handle)
        check(min(db, 0), self.engine.handle)
        k = np.zeros(n.value, dtype=KEYPOINT_DTYPE)
        d = np.zeros((n.value, db), dtype=np.uint8)
        if n.value:
            ctypes.memmove(k.ctypes.data, kp.value, n.value * KEYPOINT_DTYPE.itemsize)
            ctypes.memmove(d.ctypes.data, desc.value, n.value * db)
        return k, d

    def matches(self, pair: int):
        """(first view, second view, query -> train index or -1) of one pair."""
        a = ctypes.c_int32()
        b = ctypes.c_int32()
        q = ctypes.c_void_p()
        n = ctypes.c_int64()
        check(lib.dp_seed_matches(self.engine.handle, pair, ctypes.byref(a), ctypes.byref(b), ctypes.byref(q),
                                  ctypes.byref(n)), self.engine.handle)
        m = np.zeros(n.value, dtype=np.int32)
        if n.value:
            ctypes.memmove(m.ctypes.data, q.value, n.value * 4)
        return a.value, b.value, m


def knn_match(engine, query: np.ndarray, train: np.ndarray, width: int = 32):
    """BFMatcher(NORM_HAMMING).knnMatch(query, train, 2) on `width`-byte rows
    (32 ORB, 64 AKAZE): (idx2, dist2), -1 where absent."""
    q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, width)
    t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, width)
    idx = np.zeros((len(q), 2), dtype=np.int32)
    dist = np.zeros((len(q), 2), dtype=np.int32)
    check(lib.dp_knn_match_wide(engine.handle, ptr(q), len(q), ptr(t), len(t), width, ptr(idx), ptr(dist)),
          engine.handle)
    return idx, dist


def fundamental_matrix(P1, P2) -> np.ndarray:
    """Geometry::ComputeFundamentalMatrix (fundamental_matrix.cpp:6-34)."""
    a = np.ascontiguousarray(P1, dtype=np.float64).reshape(12)
    b = np.ascontiguousarray(P2, dtype=np.float64).reshape(12)
    F = np.zeros(9)
    check(lib.dp_fundamental_matrix(ptr(a), ptr(b), ptr(F)))
    return F.reshape(3, 3)


def triangulate(engine, projections: list, observations: list) -> np.ndarray:
    """Geometry::DirectLinearTriangulation (triangulation.cpp:15-34), batched:
    projections[i] is a list of 3x4 matrices, observations[i] the matching
    (x, y) list of point i."""
    off = np.zeros(len(projections) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(p) for p in projections])
    P = np.ascontiguousarray(np.concatenate([np.asarray(p, dtype=np.float64).reshape(-1, 12) for p in projections]))
    obs = np.ascontiguousarray(np.concatenate([np.asarray(o, dtype=np.float64).reshape(-1, 2) for o in observations]))
    X = np.zeros((len(projections), 3))
    check(lib.dp_triangulate(engine.handle, len(projections), ptr(off), ptr(P), ptr(obs), ptr(X)), engine.handle)
    return X

"""Deterministic synthetic scenes: cameras, renders, seed points.

Build extension -- the reference has no data generator.  Rendering runs the
same per-pixel code on the host or on the GPU (byte-identical images).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from ._native import lib, ptr

# BASELINE.json configs: name -> (views, width, height, kind)
CONFIGS = {
    "cfg1_2view_vga": (2, 640, 480, 0),
    "cfg1_4view_vga": (4, 640, 480, 0),
    "cfg2_8view_1080p": (8, 1920, 1080, 1),
    "cfg3_32view_4k": (32, 3840, 2160, 1),
    "cfg4_64view_4k": (64, 3840, 2160, 1),
    "cfg5_128view_8k": (128, 7680, 4320, 1),
}


# image pyramid levels BASELINE.json names per config (level 0 included)
PYRAMID_LEVELS = {
    "cfg1_2view_vga": 1,
    "cfg1_4view_vga": 1,
    "cfg2_8view_1080p": 3,
    "cfg3_32view_4k": 4,
    "cfg4_64view_4k": 4,
    "cfg5_128view_8k": 4,
}


def config(n_views=8, width=640, height=480, kind=1, seed=20261015, spread_deg=35.0,
           seed_stride_px=32.0, depth_noise=0.005) -> N.DpSynthConfig:
    c = N.DpSynthConfig()
    lib.dp_synth_default(ctypes.byref(c))
    c.n_views, c.width, c.height, c.kind = n_views, width, height, kind
    c.seed = seed
    c.spread_deg = spread_deg
    c.seed_stride_px = seed_stride_px
    c.depth_noise = depth_noise
    return c


def named(name: str, **kw) -> N.DpSynthConfig:
    V, W, H, kind = CONFIGS[name]
    return config(V, W, H, kind, **kw)


def cameras(cfg: N.DpSynthConfig) -> np.ndarray:
    P = np.zeros((cfg.n_views, 3, 4), dtype=np.float64)
    N.check(lib.dp_synth_cameras(ctypes.byref(cfg), ptr(P)))
    return P


def render_host(cfg: N.DpSynthConfig, P: np.ndarray, v: int) -> np.ndarray:
    img = np.zeros((cfg.height, cfg.width, 3), dtype=np.uint8)
    P = np.ascontiguousarray(P, dtype=np.float64)
    N.check(lib.dp_synth_render_host(ctypes.byref(cfg), ptr(P), v, ptr(img)))
    return img


def seeds(cfg: N.DpSynthConfig, P: np.ndarray) -> np.ndarray:
    P = np.ascontiguousarray(P, dtype=np.float64)
    n = lib.dp_synth_seeds(ctypes.byref(cfg), ptr(P), None, 0)
    if n < 0:
        N.check(int(n))
    out = np.zeros((n, 3), dtype=np.float64)
    lib.dp_synth_seeds(ctypes.byref(cfg), ptr(P), ptr(out), n)
    return out


def scene_host(cfg: N.DpSynthConfig):
    """(P[V,3,4], [BGR images], seeds[N,3]) rendered on the host."""
    P = cameras(cfg)
    imgs = [render_host(cfg, P, v) for v in range(cfg.n_views)]
    return P, imgs, seeds(cfg, P)


def surface(cfg: N.DpSynthConfig, xy: np.ndarray):
    """Ground truth of the synthetic surface at points xy (n x 2): height z and
    unit normal (dp_synth_surface) -- for scoring refine quality."""
    xy = np.ascontiguousarray(np.asarray(xy, dtype=np.float64).reshape(-1, 2))
    z = np.zeros(len(xy))
    nrm = np.zeros((len(xy), 3))
    N.check(lib.dp_synth_surface(ctypes.byref(cfg), len(xy), ptr(xy), ptr(z), ptr(nrm)))
    return z, nrm

"""ctypes binding of libdensepoints.so (the C ABI in include/densepoints.h).

The product path is the HIP library: if it is missing, importing this module
raises -- there is no CPU fallback anywhere in densepoints_amd.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DP_LIB_VARIANT=<file name in lib/>: load a differently-compiled build of the
# same sources (A/B measurements in one GPU session, tools/ab_variants.sh)
LIB_PATH = os.path.join(_HERE, "lib", os.environ.get("DP_LIB_VARIANT") or "libdensepoints.so")

# dp_patch (include/densepoints.h) -- 80 bytes
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
assert PATCH_DTYPE.itemsize == 80

DP_OK = 0
DP_E_ARG = -1
DP_E_HIP = -2
DP_E_OOM = -3
DP_E_DEGENERATE = -4
DP_E_STATE = -5
DP_E_NODEVICE = -6

MODE_EVAL, MODE_FILTER, MODE_NM, MODE_SEED, MODE_EXPAND = range(5)
MODE_FAST_EVAL, MODE_FAST_REFINE = 5, 6  # performance mode (dp_fast_options)
PATCH_ACCEPTED = 1
PATCH_DEGENERATE = 2


class DpOptions(ctypes.Structure):
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


class DpImage(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("stride", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("bgr", ctypes.c_void_p),
    ]


class DpDensifyStats(ctypes.Structure):
    _fields_ = [
        ("seeds_in", ctypes.c_int64),
        ("seed_patches", ctypes.c_int64),
        ("patches", ctypes.c_int64),
        ("pops", ctypes.c_int64),
        ("candidates", ctypes.c_int64),
        ("evals", ctypes.c_int64),
        ("generations", ctypes.c_int32),
        ("stalls", ctypes.c_int32),
        ("refine_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
    ]


class DpGeneration(ctypes.Structure):
    _fields_ = [
        ("items", ctypes.c_int64),
        ("head", ctypes.c_int64),
        ("per_item", ctypes.c_int32),
        ("cell", ctypes.c_int32),
        ("seq0", ctypes.c_uint32),
        ("index", ctypes.c_int32),
    ]


class DpFilterOptions(ctypes.Structure):
    _fields_ = [
        ("passes", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("min_neighbor_frac", ctypes.c_double),
    ]


FILTER_VISIBILITY, FILTER_NEIGHBORS = 1, 2


class DpSynthConfig(ctypes.Structure):
    _fields_ = [
        ("n_views", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("kind", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("spread_deg", ctypes.c_double),
        ("seed_stride_px", ctypes.c_double),
        ("depth_noise", ctypes.c_double),
    ]


class DpMatcherOptions(ctypes.Structure):
    """dp_matcher_options: Features::MatcherOptions (matcher.h:14-33) + cv::ORB knobs."""

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


class DpSeedStats(ctypes.Structure):
    _fields_ = [
        ("keypoints_detected", ctypes.c_int64),
        ("keypoints", ctypes.c_int64),
        ("pairs", ctypes.c_int64),
        ("ratio_matches", ctypes.c_int64),
        ("matches", ctypes.c_int64),
        ("points", ctypes.c_int64),
        ("detect_ms", ctypes.c_double),
        ("describe_ms", ctypes.c_double),
        ("match_ms", ctypes.c_double),
        ("triangulate_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
    ]


class DpFastOptions(ctypes.Structure):
    """dp_fast_options: the performance mode's knobs (include/densepoints.h)."""
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


class DpFastStats(ctypes.Structure):
    _fields_ = [("patches", ctypes.c_int64), ("evals", ctypes.c_int64), ("view_evals", ctypes.c_int64),
                ("staged_bytes", ctypes.c_int64), ("clipped_stagings", ctypes.c_int64)]


# dp_keypoint: the cv::KeyPoint fields the matcher reads
KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("response", "<f4"), ("angle", "<f4"), ("octave", "<i4"), ("reserved", "<i4")]
)

_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double

# (name, restype, argtypes) of every exported symbol in include/densepoints.h
# and include/densepoints_probe.h
SIGNATURES = [
    ("dp_default_options", None, [_P]),
    ("dp_abi_version", _I, []),
    ("dp_device_count", _I, []),
    ("dp_ctx_create", _I, [_P, _I, _P]),
    ("dp_ctx_destroy", _I, [_P]),
    ("dp_last_error", ctypes.c_char_p, [_P]),
    ("dp_set_options", _I, [_P, _P]),
    ("dp_set_views", _I, [_P, _I, _P, _P]),
    ("dp_set_views_device", _I, [_P, _I, _P, _P, _P, _P, _P]),
    ("dp_build_pyramid", _I, [_P, _I]),
    ("dp_set_level", _I, [_P, _I]),
    ("dp_level_info", _I, [_P, _I, _I, _P, _P, _P]),
    ("dp_read_level", _I, [_P, _I, _I, _P]),
    ("dp_view_geometry", _I, [_P, _P, _P, _P, _P]),
    ("dp_seeds_to_patches", _I, [_P, _P, _I, _P]),
    ("dp_eval_batch", _I, [_P, _P, _I, _I, _P]),
    ("dp_refine_batch", _I, [_P, _P, _I, _I, _I, _P]),
    ("dp_refine_batch_device", _I, [_P, _P, _I, _I, _I, _P, _P]),
    ("dp_expand_batch", _I, [_P, _P, _I, _P, _P]),
    ("dp_expand_batch_device", _I, [_P, _P, _I, _P, _P, _P]),
    ("dp_densify", _I, [_P, _P, _I, _P, _P, _P]),
    ("dp_densify_begin", _I, [_P, _P, _I, _P]),
    ("dp_densify_commit", _I, [_P, _P, _P, _P, ctypes.c_int64]),
    ("dp_densify_result", _I, [_P, _P, _P, _P]),
    ("dp_densify_run", _I, [_P, _P, ctypes.c_int32]),
    ("dp_densify_run_until", _I, [_P, _P, ctypes.c_int32, ctypes.c_int64, _P]),
    ("dp_densify_owners", _I, [_P, _P, _I, _I, _P, _P]),
    ("dp_densify_partition_stats", _I, [_P, _P]),
    ("dp_densify_refine_items", _I, [_P, _P, _P, ctypes.c_int64, _P, _P]),
    ("dp_densify_partition_async", _I, [_P, _P, _I, _I, _P, _P, _P]),
    ("dp_densify_refine_share_async", _I, [_P, _P, _P, ctypes.c_int64, _P, ctypes.c_int64, _P]),
    ("dp_densify_commit_gathered_device", _I, [_P, _P, _P, ctypes.c_int64, _I, _P, _P]),
    ("dp_default_filter_options", None, [_P]),
    ("dp_filter_patches", _I, [_P, _P, ctypes.c_int64, _P, _P]),
    ("dp_filter_patches_device", _I, [_P, _P, ctypes.c_int64, _P, _P, _P]),
    ("dp_last_kernel_ms", _I, [_P, _P]),
    ("dp_default_matcher_options", None, [_P]),
    ("dp_orb_pattern", _I, [_P]),
    ("dp_generate_seeds", _I, [_P, _P, _P, _P, _P]),
    ("dp_seed_keypoints", _I, [_P, _I, _P, _P, _P]),
    ("dp_seed_matches", _I, [_P, _I, _P, _P, _P, _P]),
    ("dp_knn_match", _I, [_P, _P, ctypes.c_int64, _P, ctypes.c_int64, _P, _P]),
    ("dp_knn_match_wide", _I, [_P, _P, ctypes.c_int64, _P, ctypes.c_int64, _I, _P, _P]),
    ("dp_seed_descriptor_bytes", _I, [_P]),
    ("dp_fundamental_matrix", _I, [_P, _P, _P]),
    ("dp_triangulate", _I, [_P, ctypes.c_int64, _P, _P, _P, _P]),
    ("dp_synth_default", None, [_P]),
    ("dp_synth_cameras", _I, [_P, _P]),
    ("dp_synth_render_host", _I, [_P, _P, _I, _P]),
    ("dp_synth_render_device", _I, [_P, _P, _P, _I, _P, _P]),
    ("dp_synth_seeds", ctypes.c_int64, [_P, _P, _P, ctypes.c_int64]),
    ("dp_synth_surface", _I, [_P, ctypes.c_int64, _P, _P, _P]),
    ("dp_default_fast_options", None, [_P]),
    ("dp_set_fast_options", _I, [_P, _P]),
    ("dp_build_gray", _I, [_P]),
    ("dp_read_gray", _I, [_P, _I, _P]),
    ("dp_fast_expand_batch", _I, [_P, _P, _I, _P, _P]),
    ("dp_fast_expand_batch_device", _I, [_P, _P, _I, _P, _P, _P]),
    ("dp_fast_last_stats", _I, [_P, _P]),
    ("dp_probe_sincos", None, [_D, _P, _P]),
    ("dp_probe_acos", _D, [_D]),
    ("dp_probe_texture", _I, [_P, ctypes.c_int32, ctypes.c_int32, _P, _P, _I, _P]),
    ("dp_probe_ncc", _D, [ctypes.c_int32] * 6 + [_D]),
    ("dp_probe_math_device", _I, [_P, _I, _P]),
    ("dp_probe_texel_device", _I, [_P, _P, _P, _I, _P]),
    ("dp_probe_recip_f32_device", _I, [_P, _I, _P]),
    ("dp_probe_grad_q24_device", _I, [_P, _I, _P]),
    ("dp_probe_lds_unaligned_device", _I, [_P]),
    ("dp_debug_stamps", _I, [_P]),
]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"densepoints_amd: HIP library {LIB_PATH} is missing; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class DensePointsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"densepoints error {code}: {msg}")
        self.code = code


def check(rc: int, ctx=None) -> None:
    if rc != DP_OK:
        msg = lib.dp_last_error(ctx).decode() if ctx else ""
        raise DensePointsError(rc, msg)


def ptr(a) -> int | None:
    if a is None:
        return None
    return a.ctypes.data


def default_options() -> DpOptions:
    o = DpOptions()
    lib.dp_default_options(ctypes.byref(o))
    return o

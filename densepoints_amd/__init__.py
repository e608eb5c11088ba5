"""densepoints_amd -- MI355X-native PMVS patch loop (seed -> expand -> filter).

The compute path is libdensepoints.so (hand-written gfx950 HIP kernels behind
the C ABI in include/densepoints.h); this package is the host-side mirror of
the reference's methods/pmvs interface.  Importing fails loudly if the HIP
library has not been built: there is no CPU fallback.
"""
from ._native import (  # noqa: F401
    MODE_EVAL,
    MODE_EXPAND,
    MODE_FAST_EVAL,
    MODE_FAST_REFINE,
    MODE_FILTER,
    MODE_NM,
    MODE_SEED,
    PATCH_ACCEPTED,
    PATCH_DEGENERATE,
    PATCH_DTYPE,
    DensePointsError,
    LIB_PATH,
)
from .pmvs import (  # noqa: F401
    PMVS,
    Engine,
    FastOptions,
    Options,
    View,
    empty_patches,
    mask_from_list,
    ncc_score,
    read_scene_json,
    visible_list,
    write_ply,
)
from . import synth  # noqa: F401

__version__ = "0.1.0"

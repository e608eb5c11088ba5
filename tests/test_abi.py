"""The C ABI library loads and exports every symbol include/*.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

import densepoints_amd as dp
from densepoints_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in ("densepoints.h", "densepoints_probe.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"\b(dp_[a-z0-9_]+)\s*\(", txt):
            syms.add(m.group(1))
    return syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(N.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in sorted(syms):
        assert hasattr(lib, s), f"missing export {s}"
    bound = {name for name, _, _ in N.SIGNATURES}
    assert syms == bound, f"ctypes table out of sync: {syms ^ bound}"


def test_abi_version_and_layouts():
    assert N.lib.dp_abi_version() == 2
    assert N.PATCH_DTYPE.itemsize == 80
    assert ctypes.sizeof(N.DpOptions) == 104
    o = N.default_options()
    assert (o.seed_cell_size, o.expand_cell_size, o.grid_scale, o.min_visible) == (16, 11, 8, 3)
    assert (o.ncc_threshold, o.visible_angle, o.candidate_angle) == (0.6, 0.78, 1.04)
    assert list(o.nm_step) == [0.02, 0.2, 0.2] and o.nm_max_evals == 500 and o.max_pops == 10_000_000
    assert bytes(dp.Options().to_c()) == bytes(o)


def test_oracle_layout_matches(orc):
    assert orc.PATCH_DTYPE == N.PATCH_DTYPE
    assert ctypes.sizeof(orc.OrOptions) == ctypes.sizeof(N.DpOptions)
    assert bytes(orc.default_options()) == bytes(N.default_options())


def test_errors_without_device_are_loud():
    # no GPU in the CPU suite: context creation must fail with a status, not fall back
    h = ctypes.c_void_p()
    rc = N.lib.dp_ctx_create(None, 0, ctypes.byref(h))
    if rc == N.DP_OK:  # running on a GPU box
        N.lib.dp_ctx_destroy(h)
    else:
        assert rc in (N.DP_E_NODEVICE, N.DP_E_HIP)

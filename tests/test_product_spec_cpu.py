"""CPU checks of the product's arithmetic spec: the host-compiled instance of
densepoints_amd/csrc/dp_geom.h + dp_detmath.h (the code the gfx950 kernels
run) against the independent oracle restatement -- bit for bit."""
import ctypes

import numpy as np
import pytest

import densepoints_amd as dp
from densepoints_amd import _native as N
from densepoints_amd import synth


def test_detmath_bitwise_equal_to_oracle(orc):
    rng = np.random.default_rng(11)
    xs = np.concatenate([rng.uniform(-3, 3, 20000), rng.normal(0, 0.05, 5000), rng.uniform(-1e3, 1e3, 2000)])
    s = ctypes.c_double()
    c = ctypes.c_double()
    for x in xs:
        N.lib.dp_probe_sincos(float(x), ctypes.byref(s), ctypes.byref(c))
        assert (s.value, c.value) == orc.sincos(x)
    for x in rng.uniform(-1.0, 1.0, 20000):
        assert N.lib.dp_probe_acos(float(x)) == orc.acos(x)


def test_view_geometry_bitwise_equal_to_oracle(orc):
    cfg = synth.config(16, 640, 480, 1)
    P = synth.cameras(cfg)
    for v in range(len(P)):
        view = dp.View(P[v])
        rc, C, K, E, x = orc.view_geometry(P[v])
        assert rc == 0
        assert view.camera_center.tobytes() == C.tobytes()
        assert view.intrinsics.tobytes() == K.tobytes()
        assert view.extrinsics.tobytes() == E.tobytes()
        assert view.x_axis.tobytes() == x.tobytes()


def test_ncc_finish_matches_oracle(orc):
    rng = np.random.default_rng(5)
    for n in (49, 121, 256):
        for _ in range(200):
            a = rng.integers(0, 256, n)
            b = rng.integers(0, 256, n) if rng.random() < 0.5 else np.clip(a + rng.integers(-20, 20, n), 0, 255)
            assert dp.ncc_score(a, b) == orc.ncc_int(a, b)
    # KAT through the product finish (modules/core test_error_functions.cpp:9-15)
    v = dp.ncc_score([1, 2, 3, -1, -2, -3, 1, 2, 3], [2, 0, 5, -4, 5, -2, -1, 0, -3])
    assert abs(v - 0.1005653) < 4 * 7.5e-9


@pytest.mark.parametrize("cell", [7, 11, 16])
def test_window_texture_bitwise_equal_to_oracle(orc, cell):
    """warpPerspective fixed point + BGR2GRAY: product (dp_probe_texture, the
    kernel's code compiled for the host) == oracle (literal 15-bit table)."""
    cfg = synth.config(3, 320, 240, 1)
    P, imgs, seeds = synth.scene_host(cfg)
    S = orc.Scene(P, imgs)
    rng = np.random.default_rng(cell)
    n_valid = 0
    for i in range(300):
        X = seeds[rng.integers(len(seeds))]
        ax = rng.normal(size=3)
        ay = rng.normal(size=3)
        s = rng.uniform(0.002, 0.03)
        ax *= s / np.linalg.norm(ax)
        ay *= s * rng.uniform(0.5, 1.5) / np.linalg.norm(ay)
        corners = np.array([X - ax - ay, X + ax - ay, X + ax + ay, X - ax + ay]).reshape(12)
        for v in range(3):
            g_o = S.texture(v, corners, cell)
            g_p = np.zeros(cell * cell, dtype=np.int32)
            ok = N.lib.dp_probe_texture(N.ptr(np.ascontiguousarray(P[v])), 320, 240, N.ptr(imgs[v]),
                                        N.ptr(corners), cell, N.ptr(g_p))
            assert ok == (g_o is not None)
            if ok:
                n_valid += 1
                assert np.array_equal(g_p.reshape(cell, cell), g_o)
    assert n_valid > 300

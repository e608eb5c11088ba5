"""The oracle (CPU restatement) pinned against the reference's own known-answer
tests -- the only golden vectors the reference holds for this path:
  tests/core/test_error_functions.cpp:9-15            NCCScore
  tests/core/test_projection_matrix_decomposition.cpp  View decomposition
plus accuracy of the fixed transcendental algorithm against glibc."""
import math

import numpy as np
import pytest


def float_eq(a, b, ulps=4):
    # gtest EXPECT_FLOAT_EQ: within 4 ULPs in single precision
    fa, fb = np.float32(a), np.float32(b)
    ia = np.array([fa]).view(np.int32)[0]
    ib = np.array([fb]).view(np.int32)[0]
    return abs(int(ia) - int(ib)) <= ulps


def test_ncc_known_answer(orc):
    a = [1, 2, 3, -1, -2, -3, 1, 2, 3]
    b = [2, 0, 5, -4, 5, -2, -1, 0, -3]
    assert float_eq(orc.ncc_int(a, b), 0.1005653)
    assert float_eq(orc.ncc_int(a, a), 1.0)


def test_ncc_denominator_clamp(orc):
    # constant textures: sigma = 0 -> denominator clamped to 0.1, numerator 0
    assert orc.ncc_int([7] * 9, [3] * 9) == 0.0
    # one flat texture: sigma_a*sigma_b = 0 < 0.1
    a = [5] * 8 + [6]
    b = list(range(9))
    num = sum((x - np.mean(a)) * (y - np.mean(b)) for x, y in zip(a, b))
    assert orc.ncc_int(a, b) == pytest.approx(num / max(0.1, np.std(a) * np.std(b)) / 9, rel=1e-12)


def test_projection_decomposition_known_answer(orc):
    P = np.array([[3.53553e2, 3.39645e2, 2.77744e2, -1.44946e6],
                  [-1.03528e2, 2.33212e1, 4.59607e2, -6.32525e5],
                  [7.07107e-1, -3.53553e-1, 6.12372e-1, -9.18559e2]])
    rc, C, K, E, x = orc.view_geometry(P)
    assert rc == 0
    assert abs(K[0, 0] - 468.2) < 0.1
    assert abs(K[1, 1] - 427.2) < 0.1
    assert abs(K[0, 2] - 300) < 0.1
    assert abs(K[1, 2] - 200) < 0.1
    assert abs(K[2, 2] - 1) < 0.1
    assert np.abs(K @ E - P).max() < 0.5
    assert np.allclose(C, [1000, 2000, 1500], atol=0.01)
    assert np.allclose(x, E[0, :3])


def test_decomposition_random_cameras(orc):
    rng = np.random.default_rng(7)
    for _ in range(50):
        A = rng.normal(size=(3, 3))
        R, _ = np.linalg.qr(A)
        if np.linalg.det(R) < 0:
            R[0] *= -1
        K = np.array([[rng.uniform(300, 2000), rng.uniform(-5, 5), rng.uniform(100, 900)],
                      [0, rng.uniform(300, 2000), rng.uniform(100, 900)], [0, 0, 1]])
        C = rng.normal(size=3) * 10
        P = K @ np.hstack([R, -R @ C[:, None]]) * rng.uniform(0.1, 10)
        rc, C2, K2, E2, x = orc.view_geometry(P)
        assert rc == 0
        assert np.allclose(C2, C, atol=1e-8 * (1 + np.abs(C).max()))
        assert np.allclose(K2, K, rtol=1e-9, atol=1e-9)
        assert np.allclose(x, R[0], atol=1e-10)


def ulp_diff(a, b):
    return abs(a - b) / math.ulp(b) if b != 0 else abs(a)


def test_transcendentals_within_one_ulp(orc):
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.uniform(-4, 4, 4000), rng.normal(0, 0.2, 4000), rng.uniform(-60, 60, 2000),
                         [0.0, -0.0, math.pi / 4, -math.pi / 4, math.pi / 2, 1e-9]])
    for x in xs:
        s, c = orc.sincos(x)
        assert ulp_diff(s, math.sin(x)) <= 1.0 and ulp_diff(c, math.cos(x)) <= 1.0
    for x in np.concatenate([rng.uniform(-1, 1, 8000), [-1.0, 1.0, 0.0, 0.5, -0.5, 0.999999]]):
        assert ulp_diff(orc.acos(x), math.acos(x)) <= 1.0
    assert math.isnan(orc.acos(float("nan")))
    assert math.isnan(orc.acos(1.5))


def _pyr_down_numpy(img):
    """Independent numpy statement of cv::pyrDown (reflect-101 = np.pad 'reflect')."""
    k = np.array([1, 4, 6, 4, 1], dtype=np.int64)
    H, W = img.shape[:2]
    a = np.pad(img.astype(np.int64), ((2, 2), (2, 2), (0, 0)), mode="reflect") if min(H, W) > 2 else None
    if a is None:
        pytest.skip("tiny image")
    rows = sum(k[j] * a[:, j:j + W, :] for j in range(5))
    full = sum(k[i] * rows[i:i + H, :, :] for i in range(5))
    return ((full[::2, ::2, :] + 128) >> 8).astype(np.uint8)


@pytest.mark.parametrize("shape", [(240, 320), (61, 97), (5, 6), (33, 4)])
def test_oracle_pyr_down_matches_numpy(orc, shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    out = orc.pyr_down(img)
    assert out.shape == ((shape[0] + 1) // 2, (shape[1] + 1) // 2, 3)
    assert np.array_equal(out, _pyr_down_numpy(img))


def test_oracle_pyr_down_constant_and_level_scene(orc):
    img = np.full((31, 45, 3), 200, dtype=np.uint8)
    assert (orc.pyr_down(img) == 200).all()
    P = np.arange(24, dtype=np.float64).reshape(2, 3, 4) + 1.0
    PL, imgs = orc.level_scene(P, [img, img], 2)
    assert np.array_equal(PL[:, 2], P[:, 2]) and np.array_equal(PL[:, :2], P[:, :2] / 4.0)
    assert imgs[0].shape == (8, 12, 3)

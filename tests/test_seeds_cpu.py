"""Seed generation on the CPU (no GPU): the oracle's restatement pinned by the
reference's own tests and by independent numpy statements, plus the parts of
the product that are host code (dp_fundamental_matrix).

Reference anchors: modules/features/matcher.cpp:18-474,
modules/geometry/fundamental_matrix.cpp:6-53, triangulation.cpp:15-34,
tests/core/test_triangulation.cpp:11-52, tests/test_data_generator.cpp:4-55.
"""
import os

import numpy as np
import pytest

from densepoints_amd import matcher as M
from densepoints_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---- TestScene (tests/test_data_generator.cpp): K fixed, R = Rx Ry Rz with
# angles uniform(-90, 90) (radians, as Eigen::AngleAxis reads them),
# t = uniform[0, 10)^3 + (0, 0, -20); points uniform[0, 10)^3
def _axis_angle(axis, a):
    c, s = np.cos(a), np.sin(a)
    if axis == 0:
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == 1:
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def random_view(rng):
    K = np.array([[1000.0, 0, 2000], [0, 1000, 1500], [0, 0, 1]])
    R = np.eye(3)
    t = np.zeros(3)
    for ax in range(3):
        R = R @ _axis_angle(ax, rng.uniform(-90, 90))
        t[ax] = rng.uniform(0, 10) + (0.0, 0.0, -20.0)[ax]
    return K @ np.hstack([R, t[:, None]])


def project(P, X):
    h = P @ np.append(X, 1.0)
    return h[:2] / h[2]


def _hamming_matrix(q, t):
    x = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2)
    return x.sum(axis=2).astype(np.int64)


def _knn_numpy(q, t):
    """knnMatch(k=2) by definition: the two smallest (distance, train index)."""
    idx = -np.ones((len(q), 2), dtype=np.int32)
    dist = -np.ones((len(q), 2), dtype=np.int32)
    if len(t) == 0:
        return idx, dist
    D = _hamming_matrix(q, t)
    for i in range(len(q)):
        order = np.lexsort((np.arange(len(t)), D[i]))[:2]
        idx[i, : len(order)] = order
        dist[i, : len(order)] = D[i, order]
    return idx, dist


def random_descriptors(rng, n, pool=None):
    d = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    if pool is not None and n:
        # plant exact duplicates so distance ties occur
        k = rng.integers(0, len(pool), size=n // 3)
        d[: len(k)] = pool[k]
    return d


@pytest.mark.parametrize("nq,nt", [(0, 5), (7, 0), (9, 1), (13, 2), (40, 97), (100, 300)])
def test_oracle_knn_is_lexicographic_top2(orc, nq, nt):
    rng = np.random.default_rng(nq * 1000 + nt)
    t = random_descriptors(rng, nt)
    q = random_descriptors(rng, nq, pool=t if nt else None)
    if nt > 3:
        t[nt // 2] = t[1]  # duplicate train rows: equal distances, lower index wins
    i_o, d_o = orc.knn_match(q, t)
    i_n, d_n = _knn_numpy(q, t)
    assert np.array_equal(i_o, i_n) and np.array_equal(d_o, d_n)


def test_reference_triangulation_2view(orc):
    """tests/core/test_triangulation.cpp:11-28 (EXPECT_NEAR 0.01), seeded."""
    rng = np.random.default_rng(11)
    for _ in range(200):
        P, Pp = random_view(rng), random_view(rng)
        X = rng.uniform(0, 10, size=3)
        Xt = orc.triangulate([[P, Pp]], [[project(P, X), project(Pp, X)]])[0]
        assert np.all(np.abs(Xt - X) < 0.01), (X, Xt)


def test_reference_triangulation_multiview(orc):
    """tests/core/test_triangulation.cpp:30-52 (3 views, EXPECT_NEAR 0.01), seeded."""
    rng = np.random.default_rng(12)
    for _ in range(200):
        Ps = [random_view(rng) for _ in range(3)]
        X = rng.uniform(0, 10, size=3)
        Xt = orc.triangulate([Ps], [[project(P, X) for P in Ps]])[0]
        assert np.all(np.abs(Xt - X) < 0.01), (X, Xt)


def test_oracle_dlt_matches_numpy_svd(orc):
    """The Givens-QR + one-sided Jacobi restatement returns Eigen's
    JacobiSVD null vector (here: numpy's SVD) on noisy observations."""
    rng = np.random.default_rng(13)
    Ps, obs, ref = [], [], []
    for _ in range(100):
        m = int(rng.integers(2, 7))
        P = [random_view(rng) for _ in range(m)]
        X = rng.uniform(0, 10, size=3)
        o = [project(p, X) + rng.normal(0, 2.0, size=2) for p in P]
        A = []
        for p, (x, y) in zip(P, o):
            x, y = float(np.float32(x)), float(np.float32(y))
            A += [x * p[2] - p[0], y * p[2] - p[1]]
        v = np.linalg.svd(np.array(A))[2][-1]
        Ps.append(P)
        obs.append(o)
        ref.append(v[:3] / v[3])
    got = orc.triangulate(Ps, obs)
    np.testing.assert_allclose(got, np.array(ref), rtol=1e-6, atol=1e-7)


def test_fundamental_matrix_product_equals_oracle_and_is_epipolar(orc):
    rng = np.random.default_rng(14)
    for _ in range(50):
        P1, P2 = random_view(rng), random_view(rng)
        F = M.fundamental_matrix(P1, P2)
        assert np.array_equal(F, orc.fundamental_matrix(P1, P2))  # bit-exact host code
        X = rng.uniform(0, 10, size=3)
        x1, x2 = project(P1, X), project(P2, X)
        r = np.append(x2, 1) @ F @ np.append(x1, 1)
        assert abs(r) < 1e-6 * np.linalg.norm(F) * np.linalg.norm(np.append(x1, 1)) * np.linalg.norm(np.append(x2, 1))
        d = orc.epipolar_distance(F, float(x1[0]), float(x1[1]), float(x2[0]), float(x2[1]))
        # the reference stores the line's y at x = 0 and x = 1 as float
        # (fundamental_matrix.cpp:44-49) and extrapolates them to x2: the distance
        # is exact up to that rounding times |x2|
        l = F @ np.append(x1, 1)
        ys = max(abs(l[2] / l[1]), abs((l[2] + l[0]) / l[1]), abs(x2[1]), 1.0)
        assert d < 1e-3 + 4 * float(np.spacing(np.float32(ys))) * (1.0 + abs(x2[0]))


def _load_make_orb_pattern():
    import importlib.util

    spec = importlib.util.spec_from_file_location("mop", os.path.join(ROOT, "tests", "golden", "make_orb_pattern.py"))
    mop = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mop)
    return mop


def test_orb_pattern_is_opencv_bit_pattern_31(orc):
    """The oracle's and the product's rBRIEF tables are OpenCV's bit_pattern_31_
    (ORB::create()->compute, matcher.cpp:171-173), read from the plain-data copy
    scikit-image ships, and the committed headers are what the script emits."""
    import ctypes

    from densepoints_amd import _native as N

    mop = _load_make_orb_pattern()
    if not os.path.exists(mop.SOURCE):
        pytest.skip("scikit-image's orb_descriptor_positions.txt is absent")
    rows = mop.read_table()
    want = np.array(rows, dtype=np.int8).reshape(512, 2)
    # OpenCV's first pairs (orb.cpp bit_pattern_31_): 8,-3, 9,5 / 4,2, 7,-12 / -11,9, -8,2
    assert want[:6].ravel().tolist() == [8, -3, 9, 5, 4, 2, 7, -12, -11, 9, -8, 2]
    assert np.array_equal(orc.orb_pattern(), want)
    prod = np.zeros(1024, dtype=np.int8)
    assert N.lib.dp_orb_pattern(prod.ctypes.data_as(ctypes.c_void_p)) == N.DP_OK
    assert np.array_equal(prod.reshape(512, 2), want)
    for path, text in ((mop.PRODUCT_H, mop.product_header(rows)), (mop.ORACLE_H, mop.oracle_header(rows))):
        assert open(path).read() == text, f"{path} is stale: rerun tests/golden/make_orb_pattern.py"


def test_orb_constants(orc):
    pat = orc.orb_pattern()
    assert pat.shape == (512, 2) and pat.min() >= -13 and pat.max() <= 13
    assert len({tuple(r) for r in pat.reshape(256, 4)}) == 256  # pairs are distinct tests
    for n, L in ((40000, 8), (3000, 4), (500, 1)):
        f = orc.features_per_level(n, 1.2, L)
        assert f.sum() == n and np.all(np.diff(f[:-1]) <= 0)


def test_oracle_seeds_lie_on_the_plane(orc):
    """End-to-end restatement on the textured plane (z = 0): triangulated
    seeds land on the surface to a fraction of a pixel."""
    cfg = synth.config(n_views=4, width=640, height=480, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    r = orc.seeds_run(P, imgs, orc.matcher_options(n_features=5000, fast_threshold=10))
    c = r["counts"]
    assert c["points"] > 500 and c["matches"] <= c["ratio_matches"] and c["keypoints"] <= c["detected"]
    z = np.abs(r["points"][:, 2])
    assert np.median(z) < 0.01 and np.percentile(z, 90) < 0.03
    # FilterKeypoints: at most max_keypoints_per_cell per 16 px cell of each view
    for kp in r["keypoints"]:
        cells = (kp["y"].astype(np.int64) // 16) * 1000 + kp["x"].astype(np.int64) // 16
        assert np.bincount(np.unique(cells, return_inverse=True)[1]).max() <= 4
        assert np.all(np.diff(kp["octave"]) >= 0)  # compute() buckets by octave


def test_golden_seeds_fixture_pins_the_oracle(orc):
    g = np.load(os.path.join(ROOT, "tests", "golden", "seeds_small.npz"))
    import importlib.util

    spec = importlib.util.spec_from_file_location("mgs", os.path.join(ROOT, "tests", "golden", "make_golden_seeds.py"))
    mgs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mgs)
    r = orc.seeds_run(g["P"], list(g["images"]), orc.matcher_options(**mgs.OPTIONS))
    assert np.array_equal(np.concatenate(r["keypoints"]), g["keypoints"])
    assert np.array_equal(np.concatenate(r["descriptors"]), g["descriptors"])
    assert np.array_equal(np.concatenate(r["q2t"]), g["q2t"])
    assert np.array_equal(r["points"], g["points"])


def test_golden_akaze_fixture_pins_the_oracle(orc):
    g = np.load(os.path.join(ROOT, "tests", "golden", "seeds_small.npz"))
    a = np.load(os.path.join(ROOT, "tests", "golden", "seeds_akaze_small.npz"))
    r = orc.seeds_run(g["P"], list(g["images"]),
                      orc.matcher_options(detector_type=orc.DETECTOR_AKAZE, akaze_threshold=0.0002))
    assert np.array_equal(np.concatenate(r["keypoints"]), a["keypoints"])
    assert np.array_equal(np.concatenate(r["descriptors"]), a["descriptors"])
    assert np.array_equal(np.concatenate(r["q2t"]), a["q2t"])
    assert np.array_equal(r["points"], a["points"])


def test_oracle_flann_matcher_is_exact_nn_below_30(orc):
    """MatcherType::FLANN (matcher.cpp:229-240: LSH match, distance < 30),
    stated as the exact Hamming nearest neighbour it approximates: every
    epipolar-filtered match of the oracle's FLANN mode is a query's brute-force
    nearest train descriptor (lowest index on ties) at distance < 30."""
    cfg = synth.config(n_views=3, width=640, height=480, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(n_features=3000, fast_threshold=10)
    r = orc.seeds_run(P, imgs, orc.matcher_options(matcher_type=1, **kw))
    rk = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    assert r["counts"]["matches"] > 100
    # the same keypoints and descriptors as the kNN mode; a different match rule
    assert np.array_equal(np.concatenate(r["descriptors"]), np.concatenate(rk["descriptors"]))
    assert r["counts"]["ratio_matches"] != rk["counts"]["ratio_matches"]
    for p, (a, b) in enumerate(r["pairs"]):
        da, db = r["descriptors"][a], r["descriptors"][b]
        ham = np.unpackbits(da[:, None, :] ^ db[None, :, :], axis=2).sum(axis=2)
        nn = ham.argmin(axis=1)
        d0 = ham[np.arange(len(da)), nn]
        q2t = r["q2t"][p]
        hit = q2t >= 0
        assert np.array_equal(q2t[hit], nn[hit]) and np.all(d0[hit] < 30)


# ---- DetectorType::AKAZE (matcher.cpp:56-60, 166-170; oracle/or_akaze.c) ----
def test_akaze_levels_and_fed_schedule(orc):
    """cv::AKAZE defaults: 4 octaves x 4 sublevels (the octave stops below
    80 x 40), esigma = 1.6 2^(j/4 + o), sigma_size = round(1.5 esigma / 2^o),
    and fed.cpp's step count n = ceil(sqrt(3 T / tau_max + 1/4) - 1/2) for the
    evolution time T between consecutive levels."""
    info, es = orc.akaze_levels(640, 480)
    assert len(info) == 16
    assert [tuple(r[:3]) for r in info[::4]] == [(640, 480, 0), (320, 240, 1), (160, 120, 2), (80, 60, 3)]
    for i, r in enumerate(info):
        o, j = divmod(i, 4)
        assert es[i] == np.float32(1.6 * 2.0 ** (j / 4 + o))
        assert r[3] == int(np.rint(np.float32(es[i] * np.float32(1.5) / np.float32(2 ** o))))
    assert info[0, 4] == 0 and np.all(info[1:, 4] >= 3) and np.all(np.diff(info[1:, 4]) >= 0)
    assert len(orc.akaze_levels(640, 150)[0]) == 8  # 160 x 37 is below 40 rows: two octaves
    # fed_tau_by_cycle_time's step count for the evolution time between levels
    et = 0.5 * es.astype(np.float64) ** 2
    n = info[1:, 4]
    assert np.all(n == np.ceil(np.sqrt(3 * np.diff(et) / 0.25 + 0.25) - 0.5 - 1e-8).astype(int))


def test_akaze_scale_space_is_diffusion(orc):
    """The evolution is a diffusion: Lt of every level keeps the image mean
    (zero-flux border, 2x2 averages between octaves) within fp32 rounding and
    never sharpens (the gradient energy falls level by level inside an
    octave); Ldet is the scaled Hessian determinant of a smoothed image."""
    cfg = synth.config(n_views=1, width=320, height=240, kind=1)
    _, imgs, _ = synth.scene_host(cfg)
    m0, _ = orc.akaze_plane(imgs[0], 0, 0)
    prev = None
    for lev in range(1, 8):
        lt, kc = orc.akaze_plane(imgs[0], lev, 0)
        assert abs(lt.mean() - m0.mean()) < 2e-3
        gx, gy = np.diff(lt, axis=1), np.diff(lt, axis=0)
        e = (gx ** 2).mean() + (gy ** 2).mean()
        if prev is not None and lev % 4 != 0:
            assert e < prev
        prev = e * (4 if lev % 4 == 3 else 1)
    assert kc[0] > 0 and np.allclose(kc[4], kc[0] * np.float32(0.75))


def _inter_area_numpy(src):
    """cv::resize(src, floor(size / 2), INTER_AREA) on an fp32 plane, stated
    independently of the oracle (OpenCV 3.4 imgproc/src/resize.cpp): the fast
    2x2 path when both sides halve exactly, else computeResizeAreaTab's cells
    per axis and the row-by-row weighted sums in fp32 (AKAZE's
    halfsample_image on odd sides)"""
    sh, sw = src.shape
    h, w = sh // 2, sw // 2
    f32 = np.float32
    if sw == 2 * w and sh == 2 * h:
        return ((src[0::2, 0::2] + src[0::2, 1::2]) + (src[1::2, 0::2] + src[1::2, 1::2])) * f32(0.25)

    def tab(ssize, dsize):
        scale = 1.0 / (dsize / ssize)
        out = []
        for d in range(dsize):
            fs1 = d * scale
            fs2 = fs1 + scale
            cw = min(scale, ssize - fs1)
            s2 = min(int(np.floor(fs2)), ssize - 1)
            s1 = min(int(np.ceil(fs1)), s2)
            cells = []
            if s1 - fs1 > 1e-3:
                cells.append((s1 - 1, f32((s1 - fs1) / cw)))
            cells += [(q, f32(1.0 / cw)) for q in range(s1, s2)]
            if fs2 - s2 > 1e-3:
                cells.append((s2, f32(min(min(fs2 - s2, 1.0), cw) / cw)))
            out.append(cells)
        return out

    ty, tx = tab(sh, h), tab(sw, w)
    dst = np.zeros((h, w), dtype=f32)
    for y in range(h):
        for x in range(w):
            acc = f32(0)
            for sy, b in ty[y]:
                buf = f32(0)
                for sx, a in tx[x]:
                    buf = f32(buf + f32(src[sy, sx] * a))
                acc = f32(acc + f32(b * buf))
            dst[y, x] = acc
    return dst


@pytest.mark.parametrize("shape", [(40, 30), (41, 30), (40, 31), (37, 23), (75, 150), (187, 125)])
def test_akaze_halfsample_is_inter_area(orc, shape):
    """AKAZE's octave halfsample is cv::resize INTER_AREA to floor(side / 2):
    the oracle equals an independent numpy statement of OpenCV's two paths bit
    for bit -- the 2x2 box for even sides, fractional cell weights (every
    source row and column used) when a side is odd; a constant plane stays
    within one fp32 rounding per weight of the constant."""
    rng = np.random.default_rng(sum(shape))
    src = rng.random(shape, dtype=np.float32)
    got = orc.akaze_halfsample(src)
    ref = _inter_area_numpy(src)
    assert got.shape == (shape[0] // 2, shape[1] // 2)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    c = orc.akaze_halfsample(np.full(shape, 0.5, dtype=np.float32))
    assert np.abs(c - 0.5).max() < 1e-6
    if shape[0] % 2 or shape[1] % 2:
        # the odd side's last source row / column reaches the output
        bumped = src.copy()
        bumped[-1, -1] += 1.0
        assert not np.array_equal(orc.akaze_halfsample(bumped), got)


def test_akaze_oracle_keypoints_and_descriptors(orc):
    """AKAZE through GenerateSeeds: 486-bit descriptors in 64-byte rows (the
    padding bits zero), at most max_keypoints_per_cell per cell, keypoints
    inside the descriptor border of their level, and seeds on the textured
    plane (z = 0)."""
    cfg = synth.config(n_views=3, width=640, height=480, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    r = orc.seeds_run(P, imgs, orc.matcher_options(detector_type=orc.DETECTOR_AKAZE, akaze_threshold=0.0002))
    c = r["counts"]
    assert c["keypoints"] > 300 and c["points"] > 50
    info, _ = orc.akaze_levels(640, 480)
    for kp, d in zip(r["keypoints"], r["descriptors"]):
        assert d.shape[1] == 64 and not d[:, 61:].any() and not (d[:, 60] & 0xC0).any()
        cells = (kp["y"].astype(np.int64) // 16) * 1000 + kp["x"].astype(np.int64) // 16
        assert np.bincount(np.unique(cells, return_inverse=True)[1]).max() <= 4
        lev = kp["reserved"]
        assert np.all(kp["octave"] == info[lev, 2])
        ss = info[lev, 3]
        ra = 2.0 ** kp["octave"]
        border = 10 * np.sqrt(2) * ss
        assert np.all(kp["x"] / ra >= border - 1) and np.all(kp["x"] / ra <= info[lev, 0] - border)
        assert np.all((kp["angle"] >= 0) & (kp["angle"] <= 360))
    z = np.abs(r["points"][:, 2])
    assert np.median(z) < 0.02


def test_akaze_oracle_rotation_covariance(orc):
    """Rotating a view by 90 degrees rotates its AKAZE keypoints with it: the
    filters are symmetric, so the same points come out (moved) with their
    orientation turned by 90 degrees (up to the 0.15-rad window grid) and
    nearly the same rotation-invariant M-LDB descriptor."""
    cfg = synth.config(n_views=1, width=320, height=320, kind=1)
    P, imgs, _ = synth.scene_host(cfg)
    im = imgs[0]
    rot = np.ascontiguousarray(np.rot90(im))  # new[i, j] = old[j, W - 1 - i]
    kw = dict(detector_type=orc.DETECTOR_AKAZE, akaze_threshold=0.0002, max_keypoints_per_cell=1000)
    a = orc.seeds_run(P, [im], orc.matcher_options(**kw))
    b = orc.seeds_run(P, [rot], orc.matcher_options(**kw))
    ka, da = a["keypoints"][0], a["descriptors"][0]
    kb, db = b["keypoints"][0], b["descriptors"][0]
    assert len(ka) > 50
    W = im.shape[1]
    # old (x, y) -> new (y, W - 1 - x)
    ex, ey = ka["y"], (W - 1) - ka["x"]
    d2 = (ex[:, None] - kb["x"][None, :]) ** 2 + (ey[:, None] - kb["y"][None, :]) ** 2
    j = d2.argmin(axis=1)
    hit = d2[np.arange(len(ka)), j] < 0.25
    assert hit.mean() > 0.8
    # a gradient (dx, dy) becomes (dy, -dx): its angle (image axes, y down) turns by -90
    dang = (kb["angle"][j[hit]] - ka["angle"][hit] + 90.0 + 180.0) % 360.0 - 180.0
    assert np.median(np.abs(dang)) < 5.0
    ham = np.unpackbits(da[hit] ^ db[j[hit]], axis=1).sum(axis=1)
    assert np.median(ham) < 60  # of 486 bits (random pairs: ~243)

"""GPU parity of seed generation (Features::Matcher::GenerateSeeds,
modules/features/matcher.cpp:18-474): the HIP path through the C ABI against
the oracle (oracle/or_seeds.c) on the same inputs, bit-exact on every stage --
keypoints (coordinates, response, angle, octave, order), descriptors, the
query->train match table of every pair, and the triangulated points."""
import os

import numpy as np
import pytest

import densepoints_amd as dp
from densepoints_amd import matcher as M
from densepoints_amd import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def engine_with(P, imgs):
    eng = dp.Engine()
    eng.set_views([dp.View(P[v], imgs[v]) for v in range(len(imgs))])
    return eng


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def compare_run(eng, r, mo_kw, V):
    m = M.Matcher(eng, M.MatcherOptions(**mo_kw))
    pts = m.generate_seeds()
    c = r["counts"]
    st = m.stats
    assert (st["keypoints_detected"], st["keypoints"], st["ratio_matches"], st["matches"], st["points"]) == \
        (c["detected"], c["keypoints"], c["ratio_matches"], c["matches"], c["points"]), (st, c)
    for v in range(V):
        kp, d = m.keypoints(v)
        ok, od = r["keypoints"][v], r["descriptors"][v]
        assert len(kp) == len(ok), f"view {v}: {len(kp)} vs {len(ok)} keypoints"
        nb = kp.dtype.itemsize
        bad = np.flatnonzero((bits(kp).reshape(-1, nb) != bits(ok).reshape(-1, nb)).any(axis=1))
        assert bad.size == 0, f"view {v}: keypoints differ at {bad[:5]}: {kp[bad[:3]]} vs {ok[bad[:3]]}"
        assert np.array_equal(d, od), f"view {v}: descriptors differ"
    for p, (a, b) in enumerate(r["pairs"]):
        fa, fb, q2t = m.matches(p)
        assert (fa, fb) == (a, b)
        assert np.array_equal(q2t, r["q2t"][p]), f"pair {p}: match tables differ"
    assert np.array_equal(bits(pts), bits(r["points"]))
    return m


@pytest.mark.parametrize("kind", [0, 1])
def test_generate_seeds_matches_oracle(orc, kind):
    cfg = synth.config(n_views=4, width=640, height=480, kind=kind)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(n_features=5000, fast_threshold=10)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    with engine_with(P, imgs) as eng:
        m = compare_run(eng, r, kw, 4)
        assert m.stats["points"] > 300


def test_generate_seeds_reference_defaults(orc):
    """ORB::create(40000), 8 levels, FAST 20 -- the reference's own settings."""
    cfg = synth.config(n_views=3, width=960, height=720, kind=1)
    P, imgs, _ = synth.scene_host(cfg)
    r = orc.seeds_run(P, imgs, orc.matcher_options())
    with engine_with(P, imgs) as eng:
        compare_run(eng, r, {}, 3)


def test_generate_seeds_direct_epipolar(orc):
    """DirectEpipolarMatching (matcher.cpp:267-317, epipolar_matching = true)."""
    cfg = synth.config(n_views=3, width=320, height=240, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(n_features=600, n_levels=3, fast_threshold=8, epipolar_matching=True)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    with engine_with(P, imgs) as eng:
        compare_run(eng, r, kw, 3)


def test_generate_seeds_golden_fixture():
    g = np.load(os.path.join(ROOT, "tests", "golden", "seeds_small.npz"))
    import importlib.util

    spec = importlib.util.spec_from_file_location("mgs", os.path.join(ROOT, "tests", "golden", "make_golden_seeds.py"))
    mgs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mgs)
    with engine_with(g["P"], list(g["images"])) as eng:
        m = M.Matcher(eng, M.MatcherOptions(**mgs.OPTIONS))
        pts = m.generate_seeds()
        kps = np.concatenate([m.keypoints(v)[0] for v in range(3)])
        desc = np.concatenate([m.keypoints(v)[1] for v in range(3)])
        q2t = np.concatenate([m.matches(p)[2] for p in range(3)])
    assert np.array_equal(bits(kps), bits(g["keypoints"]))
    assert np.array_equal(desc, g["descriptors"])
    assert np.array_equal(q2t, g["q2t"])
    assert np.array_equal(bits(pts), bits(g["points"]))


def test_generate_seeds_akaze_golden_fixture():
    g = np.load(os.path.join(ROOT, "tests", "golden", "seeds_small.npz"))
    a = np.load(os.path.join(ROOT, "tests", "golden", "seeds_akaze_small.npz"))
    with engine_with(g["P"], list(g["images"])) as eng:
        m = M.Matcher(eng, M.MatcherOptions(detector_type=M.DETECTOR_AKAZE, akaze_threshold=0.0002))
        pts = m.generate_seeds()
        kps = np.concatenate([m.keypoints(v)[0] for v in range(3)])
        desc = np.concatenate([m.keypoints(v)[1] for v in range(3)])
        q2t = np.concatenate([m.matches(p)[2] for p in range(3)])
    assert np.array_equal(bits(kps), bits(a["keypoints"]))
    assert np.array_equal(desc, a["descriptors"])
    assert np.array_equal(q2t, a["q2t"])
    assert np.array_equal(bits(pts), bits(a["points"]))


def _random_desc(rng, n, pool=None):
    d = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    if pool is not None and len(pool) and n:
        k = rng.integers(0, len(pool), size=n // 3)
        d[: len(k)] = pool[k]
        # near-duplicates: one flipped bit (distance 1 ties across rows)
        d[len(k): 2 * len(k)] = pool[k] ^ np.eye(32, dtype=np.uint8)[rng.integers(0, 32, len(k))]
    return d


@pytest.mark.parametrize("nq,nt", [(1, 0), (5, 1), (33, 2), (257, 31), (300, 33), (513, 129), (1000, 4099),
                                   (4096, 3000)])
def test_knn_match_matches_oracle(orc, nq, nt):
    rng = np.random.default_rng(nq * 7919 + nt)
    t = _random_desc(rng, nt)
    if nt > 8:
        t[nt - 1] = t[3]  # equal rows across tiles: the lower index must win
        t[nt // 2] = t[3]
    q = _random_desc(rng, nq, pool=t)
    io, do = orc.knn_match(q, t)
    with dp.Engine() as eng:
        ig, dg = M.knn_match(eng, q, t)
    assert np.array_equal(dg, do)
    assert np.array_equal(ig, io)


def test_knn_match_extreme_distances(orc):
    # distances 0 and 256 (all bits differ) and all-equal train sets
    t = np.zeros((70, 32), dtype=np.uint8)
    t[5:] = 255
    q = np.concatenate([np.zeros((3, 32), np.uint8), np.full((3, 32), 255, np.uint8)])
    io, do = orc.knn_match(q, t)
    with dp.Engine() as eng:
        ig, dg = M.knn_match(eng, q, t)
    assert np.array_equal(ig, io) and np.array_equal(dg, do)
    assert do[0].tolist() == [0, 0] and io[0].tolist() == [0, 1] and io[3].tolist() == [5, 6]


def test_triangulate_matches_oracle_and_reference_property(orc):
    from tests.test_seeds_cpu import project, random_view

    rng = np.random.default_rng(21)
    Ps, obs, truth = [], [], []
    for i in range(500):
        m = 2 + i % 5
        P = [random_view(rng) for _ in range(m)]
        X = rng.uniform(0, 10, size=3)
        Ps.append(P)
        noise = 0.0 if i % 2 == 0 else 1.5
        obs.append([project(p, X) + rng.normal(0, noise, size=2) for p in P])
        truth.append(X)
    want = orc.triangulate(Ps, obs)
    with dp.Engine() as eng:
        got = M.triangulate(eng, Ps, obs)
    assert np.array_equal(bits(got), bits(want))
    exact = np.array(truth)[0::2]
    assert np.all(np.abs(got[0::2] - exact) < 0.01)  # test_triangulation.cpp EXPECT_NEAR 0.01


def test_pmvs_run_generates_its_own_seeds(orc):
    """PMVS::Run (pmvs.cpp:22-27): InsertSeeds (GenerateSeeds) then expansion,
    equal to the oracle's densify on the oracle's seed points."""
    cfg = synth.config(n_views=4, width=320, height=240, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(n_features=2000, n_levels=4, fast_threshold=8)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    pm = dp.PMVS()
    for v in range(4):
        pm.add_camera(dp.View(P[v], imgs[v]))
    pm.run(None, matcher_options=M.MatcherOptions(**kw))
    got = pm.get_point_cloud()
    assert pm.stats["seed_generation"]["points"] == len(r["points"])
    S = orc.Scene(P, imgs)
    want, _ = S.densify(r["points"])
    assert len(got) == len(want) and len(got) > 0
    for f in ("pos", "normal", "ref", "vis", "rgb"):
        assert np.array_equal(bits(got[f]), bits(want[f])), f


def _run_both(orc, P, imgs, kw):
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    with engine_with(P, imgs) as eng:
        m = compare_run(eng, r, kw, len(imgs))
    return r, m


def test_seeds_edge_blank_and_single_view(orc):
    cfg = synth.config(n_views=3, width=320, height=240, kind=1)
    P, imgs, _ = synth.scene_host(cfg)
    blank = [np.full_like(im, 128) for im in imgs]
    r, m = _run_both(orc, P, blank, dict(n_features=1000, n_levels=3))
    assert m.stats["keypoints_detected"] == 0 and len(m.points) == 0
    # one textured view among blank ones: keypoints but no matches
    r, m = _run_both(orc, P, [imgs[0], blank[1], blank[2]], dict(n_features=1000, n_levels=3, fast_threshold=8))
    assert m.stats["keypoints"] > 0 and m.stats["points"] == 0
    # a single view: no pairs at all
    r, m = _run_both(orc, P[:1], imgs[:1], dict(n_features=1000, n_levels=3, fast_threshold=8))
    assert m.stats["pairs"] == 0 and m.stats["points"] == 0


def test_seeds_edge_mixed_sizes_levels_and_cells(orc):
    cfg = synth.config(n_views=3, width=480, height=360, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    # view 2 cropped to 400x300 (same camera, the ORB pyramids differ per view)
    imgs = [imgs[0], imgs[1], np.ascontiguousarray(imgs[2][:300, :400])]
    _run_both(orc, P, imgs, dict(n_features=1500, n_levels=5, fast_threshold=8))
    _run_both(orc, P, imgs, dict(n_features=1500, n_levels=1, fast_threshold=8, cell_size=8,
                                 max_keypoints_per_cell=1))
    r, m = _run_both(orc, P, imgs, dict(n_features=1500, n_levels=2, fast_threshold=8, max_keypoints_per_cell=0))
    assert m.stats["keypoints"] == 0


def test_seeds_bad_options_fail_loudly():
    cfg = synth.config(n_views=2, width=160, height=120, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    with engine_with(P, imgs) as eng:
        for kw in (dict(n_levels=0), dict(edge_threshold=5), dict(scale_factor=1.0), dict(n_levels=17)):
            with pytest.raises(dp.DensePointsError):
                M.Matcher(eng, M.MatcherOptions(**kw)).generate_seeds()
    with dp.Engine() as eng:  # no views set
        with pytest.raises(dp.DensePointsError):
            M.Matcher(eng).generate_seeds()


def test_seeds_min_edge_threshold(orc):
    """edge_threshold 19 (the minimum): keypoint centres 19 px from a level's
    border, so the descriptor's patch blur reflects (BORDER_REFLECT_101) at the
    image edge exactly as the full-image blur does."""
    cfg = synth.config(n_views=3, width=320, height=240, kind=1)
    P, imgs, _ = synth.scene_host(cfg)
    r, m = _run_both(orc, P, imgs, dict(n_features=3000, n_levels=4, fast_threshold=6, edge_threshold=19))
    kp = np.concatenate([r["keypoints"][v] for v in range(3)])  # equal to the GPU's (checked above)
    assert len(kp) > 0
    # some keypoint's blur patch reaches past its level's border (reflection exercised)
    s = 1.2 ** kp["octave"].astype(np.float64)
    x, y = kp["x"] / s, kp["y"] / s
    w, h = np.rint(320 / s), np.rint(240 / s)
    assert np.any(np.minimum(np.minimum(x, y), np.minimum(w - 1 - x, h - 1 - y)) < 22)


def test_generate_seeds_flann_matcher(orc):
    """MatcherType::FLANN (matcher.cpp:229-240; DP_MATCHER_FLANN: the exact
    nearest neighbour the LSH match approximates, kept iff distance < 30):
    every stage bit-exact against the oracle's FLANN mode."""
    cfg = synth.config(n_views=4, width=640, height=480, kind=1)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(n_features=5000, fast_threshold=10, matcher_type=M.MATCHER_FLANN)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    with engine_with(P, imgs) as eng:
        m = compare_run(eng, r, kw, 4)
        assert m.stats["points"] > 100


# ---- DetectorType::AKAZE (matcher.cpp:56-60, 166-170; oracle/or_akaze.c) ----
@pytest.mark.parametrize("kind,thr", [(0, 0.0002), (1, 0.001)])
def test_generate_seeds_akaze_matches_oracle(orc, kind, thr):
    """AKAZE detect + FilterKeypoints + M-LDB + kNN on 512-bit rows + DLT:
    every stage bit-exact against the oracle (threshold 0.001 is
    AKAZE::create()'s default)."""
    cfg = synth.config(n_views=3, width=640, height=480, kind=kind)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(detector_type=M.DETECTOR_AKAZE, akaze_threshold=thr)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    assert r["counts"]["keypoints"] > 20
    with engine_with(P, imgs) as eng:
        m = compare_run(eng, r, kw, 3)
        assert m.keypoints(0)[1].shape[1] == 64


@pytest.mark.parametrize("size", [(500, 375), (333, 250)])
def test_akaze_odd_octave_sides(orc, size):
    """Views whose octaves halve an odd side (375 -> 187 -> 93, 333 -> 166 ->
    83): the device halfsample takes cv::resize INTER_AREA's general
    fractional-weight path like the oracle, keypoints,
    descriptors and seeds bit-exact."""
    cfg = synth.config(n_views=3, width=size[0], height=size[1], kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(detector_type=M.DETECTOR_AKAZE, akaze_threshold=0.0002)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    assert r["counts"]["keypoints"] > 20
    with engine_with(P, imgs) as eng:
        compare_run(eng, r, kw, 3)


def test_akaze_chunks_and_mixed_sizes(orc, monkeypatch):
    """Views of different sizes (different level counts: 400 x 150 has two
    octaves) and a chunk budget that puts every view in its own chunk give
    the same keypoints, descriptors and seeds."""
    cfg = synth.config(n_views=3, width=480, height=360, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    imgs = [imgs[0], np.ascontiguousarray(imgs[1][:150, :400]), imgs[2]]
    kw = dict(detector_type=M.DETECTOR_AKAZE, akaze_threshold=0.0002, max_keypoints_per_cell=2, cell_size=24)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    with engine_with(P, imgs) as eng:
        compare_run(eng, r, kw, 3)
    monkeypatch.setenv("DP_AKAZE_CHUNK_BYTES", "1")
    with engine_with(P, imgs) as eng:
        compare_run(eng, r, kw, 3)


@pytest.mark.parametrize("steps", [1, 2, 3, 6])
def test_akaze_fed_steps_per_launch_equal(orc, monkeypatch, steps):
    """The FED steps of a level grouped 1, 2, 3 or 6 per launch (the default is 4;
    DP_AKAZE_FED_STEPS) give the oracle's values bit for bit: the multi-step
    LDS tiles recompute their halo with the single step's expressions."""
    cfg = synth.config(n_views=2, width=640, height=480, kind=0)
    P, imgs, _ = synth.scene_host(cfg)
    kw = dict(detector_type=M.DETECTOR_AKAZE, akaze_threshold=0.0002)
    r = orc.seeds_run(P, imgs, orc.matcher_options(**kw))
    monkeypatch.setenv("DP_AKAZE_FED_STEPS", str(steps))
    with engine_with(P, imgs) as eng:
        compare_run(eng, r, kw, 2)


@pytest.mark.parametrize("nq,nt", [(1, 0), (33, 2), (300, 129), (1000, 2500)])
def test_knn_match_wide_matches_oracle(orc, nq, nt):
    """knnMatch on 64-byte rows (the AKAZE descriptor width), ties included."""
    rng = np.random.default_rng(nq * 31 + nt)
    t = rng.integers(0, 256, size=(nt, 64), dtype=np.uint8)
    q = rng.integers(0, 256, size=(nq, 64), dtype=np.uint8)
    if nt > 8:
        t[nt - 1] = t[3]
        q[: nq // 3] = t[rng.integers(0, nt, nq // 3)]
    io, do = orc.knn_match(q, t, width=64)
    with dp.Engine() as eng:
        ig, dg = M.knn_match(eng, q, t, width=64)
    assert np.array_equal(dg, do) and np.array_equal(ig, io)


def test_akaze_edge_blank_views_and_no_keypoints(orc):
    """A uniform view (no gradient: the contrast factor's 0.03 fallback, no
    extrema) beside textured ones, and a threshold no response reaches: the
    GPU path equals the oracle and an empty keypoint set flows through the
    matching stages."""
    cfg = synth.config(n_views=3, width=320, height=240, kind=1)
    P, imgs, _ = synth.scene_host(cfg)
    blank = np.full_like(imgs[1], 128)
    kw = dict(detector_type=M.DETECTOR_AKAZE, akaze_threshold=0.0002)
    r, m = _run_both(orc, P, [imgs[0], blank, imgs[2]], kw)
    assert r["keypoints"][1].size == 0 and m.stats["keypoints"] > 0
    kw = dict(detector_type=M.DETECTOR_AKAZE, akaze_threshold=10.0)
    r, m = _run_both(orc, P, imgs, kw)
    assert m.stats["keypoints"] == 0 and m.stats["points"] == 0

"""GPU parity: the HIP path (through the C ABI) against the oracle on the same
seeded inputs, bit-exact on every field (pose f32, masks, score, E, flags,
colour, order).  Sizes are chosen so the oracle finishes in seconds."""
import ctypes

import numpy as np
import pytest

import densepoints_amd as dp
from densepoints_amd import _native as N
from densepoints_amd import synth

pytestmark = pytest.mark.gpu

FIELDS = ("pos", "normal", "ref", "vis", "cand", "score", "evals", "flags")


def assert_same(gp, op, fields=FIELDS):
    assert len(gp) == len(op)
    for f in fields:
        a, b = gp[f], op[f]
        if a.dtype.kind == "f":
            bad = np.flatnonzero((a.view(np.uint32) != b.view(np.uint32)).reshape(len(a), -1).any(axis=1))
        else:
            bad = np.flatnonzero((a != b).reshape(len(a), -1).any(axis=1))
        assert bad.size == 0, f"field {f}: {bad.size} of {len(a)} patches differ, first {bad[:5]}: " \
                              f"{a[bad[0]]} vs {b[bad[0]]}"


class SceneCase:
    def __init__(self, V, W, H, kind, nseeds=None, **kw):
        self.cfg = synth.config(V, W, H, kind, **kw)
        self.P, self.imgs, seeds = synth.scene_host(self.cfg)
        self.seeds = seeds if nseeds is None else seeds[:nseeds]
        self.views = [dp.View(self.P[v], self.imgs[v]) for v in range(V)]


_cache = {}


def scene(name):
    if name not in _cache:
        spec = {
            "hf6": dict(V=6, W=320, H=240, kind=1),
            "plane4": dict(V=4, W=640, H=480, kind=0),
            "plane2": dict(V=2, W=640, H=480, kind=0),
            "wide70": dict(V=70, W=96, H=72, kind=1, seed_stride_px=12.0),
        }[name]
        _cache[name] = SceneCase(**spec)
    return _cache[name]


@pytest.fixture(scope="module")
def engine():
    with dp.Engine(device=0) as eng:
        yield eng


def test_device_math_bitwise_equals_host():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-3, 3, 50000), rng.uniform(-1, 1, 50000), rng.normal(0, 1e-3, 10000),
                        rng.uniform(-2e3, 2e3, 10000)])
    out = np.zeros((len(x), 4))
    N.check(N.lib.dp_probe_math_device(N.ptr(x), len(x), N.ptr(out)))
    s = ctypes.c_double()
    c = ctypes.c_double()
    for i in range(0, len(x), 7):
        N.lib.dp_probe_sincos(float(x[i]), ctypes.byref(s), ctypes.byref(c))
        assert out[i, 0] == s.value and out[i, 1] == c.value
        assert out[i, 2] == N.lib.dp_probe_acos(float(x[i])) or (np.isnan(out[i, 2]) and abs(x[i]) > 1)
    assert np.array_equal(out[:, 3], np.sqrt(np.abs(x)))  # IEEE-correct sqrt on gfx950


def _blend_gray_spec(a, b, fx, fy):
    """warpPerspective INTER_LINEAR on CV_8UC3 (15-bit table == (sum w'p + 512) >> 10)
    then BGR2GRAY (1868, 9617, 4899) >> 14 -- DESIGN.md arithmetic spec."""
    c32 = np.uint64(32)
    wx0, wx1 = c32 - fx, fx
    wy0, wy1 = c32 - fy, fy
    ch = []
    for k in range(3):
        lo, hi, m = np.uint64(8 * k), np.uint64(32 + 8 * k), np.uint64(255)
        p00, p01 = (a >> lo) & m, (a >> hi) & m
        p10, p11 = (b >> lo) & m, (b >> hi) & m
        ch.append((wy0 * (wx0 * p00 + wx1 * p01) + wy1 * (wx0 * p10 + wx1 * p11) + np.uint64(512)) >> np.uint64(10))
    return (ch[0] * np.uint64(1868) + ch[1] * np.uint64(9617) + ch[2] * np.uint64(4899) + np.uint64(8192)) >> np.uint64(14)


def test_texel_blend_exhaustive_fractions():
    """The texel loop's 64x-scaled u16 dot-product blend (incl. the saturated
    fx = fy = 0 weight) equals the spec on every (fx, fy) with random and
    extreme pixels."""
    rng = np.random.default_rng(7)
    fx, fy = np.meshgrid(np.arange(32, dtype=np.uint64), np.arange(32, dtype=np.uint64))
    fx, fy = np.tile(fx.ravel(), 300), np.tile(fy.ravel(), 300)
    n = fx.size
    a = rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    b = rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    a[:1024], b[:1024] = np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(0xFFFFFFFFFFFFFFFF)
    a[1024:2048], b[1024:2048] = np.uint64(0), np.uint64(0)
    a[2048:3072], b[2048:3072] = np.uint64(0x00FFFFFF00000000), np.uint64(0x00000000FFFFFFFF)
    fxy = (fx | (fy << np.uint64(5))).astype(np.uint32)
    gray = np.zeros(n, np.int32)
    N.check(N.lib.dp_probe_texel_device(N.ptr(a), N.ptr(b), N.ptr(fxy), n, N.ptr(gray)))
    want = _blend_gray_spec(a, b, fx, fy).astype(np.int64)
    bad = np.flatnonzero(gray != want)
    assert bad.size == 0, f"{bad.size} texels differ, first {bad[:5]}"


def test_seed_conversion_equals_oracle(engine, orc):
    sc = scene("hf6")
    engine.set_views(sc.views)
    gp = engine.seeds_to_patches(sc.seeds)
    op = orc.Scene(sc.P, sc.imgs).seeds_to_patches(sc.seeds)
    assert gp.tobytes() == op.tobytes()


def test_seed_conversion_edge_points(engine, orc):
    """seed_patches_kernel on the points the reference's nearest-camera rule
    and InitRelatedImages are sensitive to: near-ties (two extra cameras
    mirrored about the plane x = 0 and seeds on it; strict '<', the first
    camera wins, seed.cpp:33-40), midpoints of camera pairs, points 1e-6 from a camera centre, far points,
    points behind the cameras and off every image."""
    sc = scene("hf6")
    # two extra cameras mirrored in x about x = 0 (same image): seeds with x = 0
    # are equidistant from both up to the rounding of the SVD camera centres
    Pm = []
    for s in (-1.0, 1.0):
        C = np.array([s * 0.75, 0.1, 3.0])
        K = np.array([[200.0, 0, 160], [0, 200.0, 120], [0, 0, 1]])
        R = np.eye(3)
        Pm.append(K @ np.hstack([R, -R @ C[:, None]]))
    views = [dp.View(Pm[0], sc.imgs[0]), dp.View(Pm[1], sc.imgs[0])] + sc.views
    engine.set_views(views)
    Cs = np.stack([v.camera_center for v in views])
    rng = np.random.default_rng(7)
    pts = [np.column_stack([np.zeros(64), rng.uniform(-0.5, 0.5, 64), rng.uniform(-0.3, 0.3, 64)])]
    pts.append(0.5 * (Cs[:, None, :] + Cs[None, :, :]).reshape(-1, 3))
    pts.append(Cs + 1e-6 * rng.standard_normal(Cs.shape))
    pts.append(rng.uniform(-1e6, 1e6, (32, 3)))
    pts.append(Cs + np.array([0.0, 0.0, 5.0]))
    seeds = np.ascontiguousarray(np.concatenate(pts))
    gp = engine.seeds_to_patches(seeds)
    op = orc.Scene(np.stack([v.P for v in views]), [v.image for v in views]).seeds_to_patches(seeds)
    assert gp.tobytes() == op.tobytes()


@pytest.mark.parametrize("mode", [N.MODE_EVAL, N.MODE_FILTER, N.MODE_NM, N.MODE_SEED, N.MODE_EXPAND])
@pytest.mark.parametrize("cell", [16, 11, 7])
def test_refine_modes_bit_exact(engine, orc, mode, cell):
    sc = scene("hf6")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    seeds = sc.seeds[:160]
    gp = engine.seeds_to_patches(seeds)
    op = S.seeds_to_patches(seeds)
    ga = engine.refine(gp, cell, mode)
    oa = S.refine(op, cell, mode)
    assert np.array_equal(ga, oa)
    assert_same(gp, op)
    if mode in (N.MODE_NM, N.MODE_SEED, N.MODE_EXPAND):
        assert gp["evals"].mean() > 5  # the optimiser really ran


@pytest.mark.parametrize("cell", [16, 11])
def test_wide_addressing_bit_exact(orc, monkeypatch, cell):
    """64-bit tap addresses (used when the view planes span more than 4 GiB)
    give the same bits as the default narrow 32-bit offsets."""
    monkeypatch.setenv("DP_WIDE_ADDRESSING", "1")
    sc = scene("hf6")
    S = orc.Scene(sc.P, sc.imgs)
    seeds = sc.seeds[:120]
    op = S.seeds_to_patches(seeds)
    oa = S.refine(op, cell, N.MODE_SEED)
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        gp = eng.seeds_to_patches(seeds)
        ga = eng.refine(gp, cell, N.MODE_SEED)
    assert np.array_equal(ga, oa)
    assert_same(gp, op)


def test_refine_perturbed_children_bit_exact(engine, orc):
    """Expansion children of refined seeds (the hot loop's real inputs)."""
    sc = scene("hf6")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    parents = S.seeds_to_patches(sc.seeds[:64])
    S.refine(parents, 16, orc.MODE_SEED)
    kids = []
    for p in parents:
        ch, _ = S.expand_children(p)
        kids.append(ch)
    kids = np.concatenate(kids)
    # the GPU derives child poses itself inside dp_densify (covered below); here
    # NM -> InitRelatedImages -> filter runs again on the oracle's children
    op = kids.copy()
    gp = kids.copy()
    oa = S.refine(op, 11, orc.MODE_EXPAND)
    ga = engine.refine(gp, 11, N.MODE_EXPAND)
    assert np.array_equal(ga, oa)
    assert_same(gp, op)


@pytest.mark.parametrize("name", ["hf6", "plane4"])
def test_densify_bit_exact(orc, name):
    sc = scene(name)
    S = orc.Scene(sc.P, sc.imgs)
    op, ost = S.densify(sc.seeds)
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        gp, gst = eng.densify(sc.seeds)
    assert gst["patches"] == ost["patches"] and gst["seed_patches"] == ost["seed_patches"]
    assert gst["pops"] == ost["pops"]
    assert len(gp) > 20
    assert_same(gp, op, FIELDS + ("seq", "parent", "rgb"))


@pytest.mark.parametrize("k", [2, 3])
def test_densify_cell_capacity_bit_exact(orc, k):
    """PatchOrganizerOptions::max_patches_per_cell > 1 (patch_organizer.h:42-46,
    the capacity test of PatchGrid::TryInsert, patch_organizer.cpp:21): a
    cell admits its first k claims in sequence order, claims of rejected
    patches included.  dp_densify equals the oracle's sequential organizer,
    and holds more patches than with capacity 1."""
    sc = scene("hf6")
    o = dp.Options(max_patches_per_cell=k)
    S = orc.Scene(sc.P, sc.imgs, o)
    op, ost = S.densify(sc.seeds)
    with dp.Engine(o, device=0) as eng:
        eng.set_views(sc.views)
        gp, gst = eng.densify(sc.seeds)
        eng.set_options(dp.Options())
        _, g1 = eng.densify(sc.seeds)
    assert gst["patches"] == ost["patches"] and gst["seed_patches"] == ost["seed_patches"]
    assert gst["pops"] == ost["pops"]
    assert gst["patches"] > g1["patches"] > 20
    assert_same(gp, op, FIELDS + ("seq", "parent", "rgb"))


def test_densify_two_views_is_empty(orc):
    """BASELINE config 1 (2 views): a patch needs >=3 visible non-reference
    views, so the reference yields no patches."""
    sc = scene("plane2")
    S = orc.Scene(sc.P, sc.imgs)
    op, ost = S.densify(sc.seeds)
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        gp, gst = eng.densify(sc.seeds)
    assert ost["patches"] == 0 and gst["patches"] == 0 and len(gp) == 0


def test_densify_pop_cap_bit_exact(orc):
    sc = scene("hf6")
    opts = dp.Options(max_pops=37)
    S = orc.Scene(sc.P, sc.imgs, opts)
    op, ost = S.densify(sc.seeds)
    with dp.Engine(opts, device=0) as eng:
        eng.set_views(sc.views)
        gp, gst = eng.densify(sc.seeds)
    assert ost["pops"] == 37 and gst["pops"] == 37
    assert_same(gp, op, FIELDS + ("seq", "parent", "rgb"))


def test_more_than_64_views_bit_exact(engine, orc):
    """V = 70: visible lists longer than one wavefront (two map chunks)."""
    sc = scene("wide70")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    seeds = sc.seeds[::7][:48]
    gp = engine.seeds_to_patches(seeds)
    op = S.seeds_to_patches(seeds)
    assert op["vis"][:, 1].any(), "no patch sees a view >= 64"
    for mode, cell in ((N.MODE_SEED, 7), (N.MODE_EXPAND, 5)):
        ga = engine.refine(gp, cell, mode)
        oa = S.refine(op, cell, mode)
        assert np.array_equal(ga, oa)
        assert_same(gp, op)


def test_edge_cases(engine, orc):
    sc = scene("hf6")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    # empty batch
    empty = dp.empty_patches(0)
    assert len(engine.refine(empty, 11, N.MODE_EXPAND)) == 0
    # patches with 0 and 1 visible views; off-image patch
    p = engine.seeds_to_patches(sc.seeds[:3])
    p["vis"][0] = 0
    p["vis"][1] = dp.mask_from_list(dp.visible_list(p["vis"][1])[:1])
    p["pos"][2] = [50.0, 50.0, 50.0]
    for mode in range(5):
        gp, op = p.copy(), p.copy()
        ga = engine.refine(gp, 11, mode)
        oa = S.refine(op, 11, mode)
        assert np.array_equal(ga, oa)
        assert_same(gp, op)
    with pytest.raises(dp.DensePointsError):
        engine.refine(p.copy(), 17, N.MODE_EVAL)


def test_deterministic_repeat(engine):
    sc = scene("hf6")
    engine.set_views(sc.views)
    a = engine.seeds_to_patches(sc.seeds[:200])
    b = a.copy()
    engine.refine(a, 11, N.MODE_EXPAND)
    engine.refine(b, 11, N.MODE_EXPAND)
    assert a.tobytes() == b.tobytes()


def test_expand_batch_bit_exact(engine, orc):
    """Expand::ExpandPatch over a batch of refined parents (the bench step)."""
    sc = scene("hf6")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    parents = S.seeds_to_patches(sc.seeds[:96])
    S.refine(parents, 16, orc.MODE_SEED)
    gk, ga = engine.expand(parents)
    ok, oa = S.expand(parents)
    assert np.array_equal(ga, oa)
    assert_same(gk, ok, FIELDS + ("parent", "seq"))
    assert ga.sum() > 0


def test_device_division_shortcuts_are_ieee_exact():
    """div_rn / div32_safe / recip_safe (fp32-seeded Newton + the exact-residual
    correction), sqrt_rn (rsq_f32 seed, Goldschmidt + two corrections) and the
    magic-constant rint agree bit-for-bit with '/', sqrt and rint on 4M inputs
    of varied magnitude (each input also sweeps 16 nearby denominators and
    radicands)."""
    rng = np.random.default_rng(2024)
    x = np.concatenate([rng.uniform(-1, 1, 1_000_000), rng.uniform(-2e3, 2e3, 1_000_000),
                        np.exp(rng.uniform(-30, 30, 1_000_000)) * rng.choice([-1, 1], 1_000_000),
                        rng.normal(0, 1e-3, 1_000_000)])
    out = np.zeros((len(x), 4))
    N.check(N.lib.dp_probe_math_device(N.ptr(x), len(x), N.ptr(out)))
    bad = np.flatnonzero(out[:, 3] == -1.0)
    assert bad.size == 0, f"{bad.size} mismatches, e.g. x={x[bad[:5]]}"


@pytest.mark.parametrize("levels", [4])
def test_pyramid_bit_exact(engine, orc, levels):
    """dp_build_pyramid (device cv::pyrDown, LDS-tiled SWAR) equals the oracle's
    pyrDown chain, on the hf6 views and on odd-sized random images."""
    sc = scene("hf6")
    rng = np.random.default_rng(3)
    extra = [rng.integers(0, 256, (61, 97, 3), dtype=np.uint8), rng.integers(0, 256, (130, 67, 3), dtype=np.uint8)]
    views = sc.views + [dp.View(sc.P[0], im) for im in extra]
    engine.set_views(views)
    engine.build_pyramid(levels)
    for v, vw in enumerate(views):
        ref = vw.image
        for lvl in range(1, levels):
            ref = orc.pyr_down(ref)
            got = engine.read_level(lvl, v)
            assert got.shape == ref.shape
            assert np.array_equal(got, ref), f"view {v} level {lvl}"


@pytest.mark.parametrize("level", [1, 2])
def test_densify_on_pyramid_level_bit_exact(orc, level):
    """The patch loop on level L equals the reference algorithm on the level-L
    scene (pyrDown^L images, P rows 0-1 scaled by 2^-L)."""
    sc = scene("plane4")
    PL, imgs = orc.level_scene(sc.P, sc.imgs, level)
    S = orc.Scene(PL, imgs)
    op, ost = S.densify(sc.seeds)
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        eng.build_pyramid(3)
        eng.set_level(level)
        gp, gst = eng.densify(sc.seeds)
    assert gst["patches"] == ost["patches"] and gst["pops"] == ost["pops"]
    assert len(gp) > 10
    assert_same(gp, op, FIELDS + ("seq", "parent", "rgb"))


@pytest.mark.parametrize("passes", [1, 2, 3])
def test_filter_bit_exact(orc, passes):
    """dp_filter_patches (front map by atomicMin, one thread per patch) equals
    the oracle's or_filter_patches on a densify result, with planted occluders."""
    from test_filter_cpu import with_occluders

    sc = scene("hf6")
    S = orc.Scene(sc.P, sc.imgs)
    op, _ = S.densify(sc.seeds)
    pat = with_occluders(orc, sc.P.reshape(-1, 3, 4), op, k=40)
    want = S.filter_patches(pat, passes)
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        got = eng.filter_patches(pat, passes)
    assert np.array_equal(got, want)
    if passes & 1:
        assert got[:40].sum() < 40


@pytest.mark.parametrize("cell", [16, 11, 7])
def test_eval_batch_scores_equal_oracle(engine, orc, cell):
    """dp_eval_batch (scores only, include/densepoints.h) against the oracle's
    per-patch objective evaluation at the stored pose: mean NCCScore over the
    visible views against texture 0 (error_measurements.cpp:36-60,
    optimization.cpp:14-56), -1 where no view scores; the records are not
    mutated."""
    sc = scene("hf6")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    gp = engine.seeds_to_patches(sc.seeds[:240])
    gp["vis"][:3] = 0  # no visible view: score -1
    before = gp.tobytes()
    got = engine.evaluate(gp, cell)
    assert gp.tobytes() == before
    op = gp.copy()
    S.refine(op, cell, orc.MODE_EVAL)
    assert np.array_equal(got.view(np.uint32), op["score"].view(np.uint32))
    assert (got[:3] == -1.0).all() and (got[3:] > -1.0).any()


@pytest.mark.parametrize("n_parents", [37, 96])
def test_dequeue_order_does_not_change_output(orc, monkeypatch, n_parents):
    """Longest-first dequeue (the default) and index order (a context created
    with DP_NO_LPT=1) give byte-identical children and accept flags, for a
    parent count that is not a multiple of the 4-group block."""
    sc = scene("hf6")
    S = orc.Scene(sc.P, sc.imgs)
    parents = S.seeds_to_patches(sc.seeds[:n_parents])
    S.refine(parents, 16, orc.MODE_SEED)
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        k1, a1 = eng.expand(parents)
        r1 = parents.copy()
        f1 = eng.refine(r1, 11, N.MODE_EXPAND)
    monkeypatch.setenv("DP_NO_LPT", "1")
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        k2, a2 = eng.expand(parents)
        r2 = parents.copy()
        f2 = eng.refine(r2, 11, N.MODE_EXPAND)
    assert k1.tobytes() == k2.tobytes() and np.array_equal(a1, a2)
    assert r1.tobytes() == r2.tobytes() and np.array_equal(f1, f2)

"""Performance mode on the GPU (dp_fast.hip) against its specification, the
oracle's or_fast.c, bit-exact on every field: gray planes, one fast
evaluation, the CG refine -> InitRelatedImages -> fast filter sequence, and
Expand::ExpandPatch children (expand.cpp:103-143) refined in performance mode,
from toy scenes to BASELINE config 3 at full size."""
import numpy as np
import pytest

import densepoints_amd as dp
from densepoints_amd import _native as N
from densepoints_amd import synth

from test_gpu_parity import FIELDS, assert_same, scene

pytestmark = pytest.mark.gpu


def test_recip_newton_equals_ieee_division():
    """The kernel's 1/hz (v_rcp_f32 + one Newton step) is IEEE 1.0f/hz on 4M+
    inputs over the range the spec allows (hz >= 2^-20)."""
    rng = np.random.default_rng(11)
    x = np.concatenate([
        np.exp2(rng.uniform(-20, 20, 2_000_000)).astype(np.float32),
        rng.uniform(0.25, 4.0, 2_000_000).astype(np.float32),
        # significands near all-ones / all-zeros
        (np.float32(1.0) + np.arange(1, 40001, dtype=np.float32) * np.float32(2.0 ** -23)),
        (np.float32(2.0) - np.arange(1, 40001, dtype=np.float32) * np.float32(2.0 ** -23)),
        np.array([2.0 ** -20, 1.0, 2.0, 3.0, 0.1, 1e6], dtype=np.float32),
    ]).astype(np.float32)
    out = np.zeros_like(x)
    N.check(N.lib.dp_probe_recip_f32_device(N.ptr(x), len(x), N.ptr(out)))
    want = np.float32(1.0) / x
    bad = np.flatnonzero(out.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"{bad.size} mismatches, e.g. {x[bad[:5]]}"


def test_recip_newton_exhaustive_binade():
    """v_rcp_f32 + one Newton step is IEEE 1.0f/x for EVERY fp32 significand
    (the binade [1, 2), all 2^23 values) and, being exponent-independent while
    input and result are normal, for every operand in [2^-125, 2^125]: the
    spec's reciprocals (view depths, the NCC denominator, the CG's 1/|d| and
    1/ggp) all lie there.  Spot checks of the scaling at every exponent."""
    x = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(0x3F800000)).view(np.float32)
    out = np.zeros_like(x)
    N.check(N.lib.dp_probe_recip_f32_device(N.ptr(x), len(x), N.ptr(out)))
    want = np.float32(1.0) / x
    bad = np.flatnonzero(out.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"{bad.size} mismatches in [1, 2), e.g. {x[bad[:5]]}"
    rng = np.random.default_rng(5)
    sig = x[rng.integers(0, len(x), 4096)]
    y = np.concatenate([np.ldexp(sig, e).astype(np.float32) for e in range(-125, 125)])
    out = np.zeros_like(y)
    N.check(N.lib.dp_probe_recip_f32_device(N.ptr(y), len(y), N.ptr(out)))
    want = np.float32(1.0) / y
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))


def test_gradient_quantiser_saturates_like_the_spec(orc):
    """Spec v4's rint(dncc 2^24) with the int32 saturation: the
    kernel's grad_q24 equals or_fast.c's sat_rint_i32 on the range edges, the
    non-finite values and 1M random doubles spanning |dncc| up to 2^40."""
    rng = np.random.default_rng(23)
    edge = np.array([0.0, -0.0, 0.5 / 2 ** 24, 1.5 / 2 ** 24, -2.5 / 2 ** 24, 127.99999994, 128.0, -128.0,
                     -128.00000006, 200.0, -1e9, 1e300, np.inf, -np.inf, np.nan])
    x = np.concatenate([edge, rng.standard_normal(500_000) * np.exp2(rng.uniform(-30, 40, 500_000)),
                        rng.uniform(-129, 129, 500_000)])
    out = np.zeros(len(x), dtype=np.int32)
    N.check(N.lib.dp_probe_grad_q24_device(N.ptr(x), len(x), N.ptr(out)))
    want = np.array([orc.lib.or_fast_grad_q24(float(v)) for v in x[:20_000]], dtype=np.int32)
    assert np.array_equal(out[:20_000], want)
    # the rest against the same definition in numpy (maxNum/minNum clamp)
    r = np.clip(np.rint(x * 2.0 ** 24), -2.0 ** 31, 2.0 ** 31 - 1)
    r[np.isnan(x)] = -2.0 ** 31
    assert np.array_equal(out, r.astype(np.int64).astype(np.int32))
    assert (out == 2 ** 31 - 1).sum() > 1000 and (out == -(2 ** 31)).sum() > 1000


@pytest.fixture(scope="module")
def engine():
    with dp.Engine(device=0) as eng:
        yield eng


def test_lds_unaligned_32bit_reads():
    """The sampler reads 32-bit tap pairs at 2-byte LDS alignment."""
    out = np.zeros(256, np.uint32)
    N.check(N.lib.dp_probe_lds_unaligned_device(N.ptr(out)))
    a = np.arange(512) * 3 + 1
    want = np.array([(a[l + k] & 0xFFFF) | ((a[l + k + 1] & 0xFFFF) << 16) for k in range(4) for l in range(64)],
                    dtype=np.uint32)
    assert np.array_equal(out, want)


def test_gray_planes_equal_spec(engine, orc):
    sc = scene("hf6")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    for v in range(len(sc.views)):
        g = engine.read_gray(v)
        assert np.array_equal(g.astype(np.int32) - 1024, S.gray(v).astype(np.int32)), f"view {v}"


@pytest.mark.parametrize("gradient", [1, 0])
@pytest.mark.parametrize("cell", [16, 11, 7, 5])
@pytest.mark.parametrize("mode", [N.MODE_FAST_EVAL, N.MODE_FAST_REFINE])
def test_fast_modes_bit_exact(engine, orc, cell, mode, gradient):
    """Both refine specs: the analytic gradient (v4, default) and forward
    differences (v3), at every pass shape (n = 16, 11, 7 with its tail sample, 5)."""
    sc = scene("hf6")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    seeds = sc.seeds[:200]
    gp = engine.seeds_to_patches(seeds)
    op = S.seeds_to_patches(seeds)
    fo = dp.FastOptions(gradient=gradient)
    engine.set_fast_options(fo)
    try:
        ga = engine.fast_refine(gp, cell, mode)
    finally:
        engine.set_fast_options(dp.FastOptions())
    oa = S.fast_refine(op, cell, mode, fo=orc.fast_options(fo))
    assert np.array_equal(ga, oa)
    assert_same(gp, op)
    if mode == N.MODE_FAST_REFINE:
        assert gp["evals"].mean() > 10 and ga.sum() > 0


@pytest.mark.parametrize("opts", [dict(), dict(iters=0), dict(iters=1), dict(iters=7, margin=7),
                                  dict(margin=0, tile_budget=2048), dict(max_views=3, ls_step=2.0),
                                  dict(gradient=0), dict(gradient=0, iters=7, margin=7),
                                  dict(gradient=0, max_views=3, fd_step=0.25, ls_step=2.0),
                                  dict(max_views=6), dict(filter_max_views=0),
                                  dict(max_views=6, filter_max_views=12)])
def test_fast_expand_bit_exact_options(orc, opts):
    sc = scene("hf6")
    S = orc.Scene(sc.P, sc.imgs)
    parents = S.seeds_to_patches(sc.seeds[:120])
    S.refine(parents, 16, orc.MODE_SEED)
    fo = dp.FastOptions(**opts)
    with dp.Engine(device=0) as eng:
        eng.set_views(sc.views)
        eng.set_fast_options(fo)
        gk, ga = eng.fast_expand(parents)
    ok, oa = S.fast_expand(parents, orc.fast_options(fo))
    assert np.array_equal(ga, oa)
    assert_same(gk, ok, FIELDS + ("parent",))


@pytest.mark.parametrize("gradient", [0, 1])
def test_fast_edge_cases(engine, orc, gradient):
    sc = scene("wide70")
    engine.set_views(sc.views)
    S = orc.Scene(sc.P, sc.imgs)
    p = engine.seeds_to_patches(sc.seeds[::7][:64])
    p["vis"][0] = 0                          # no visible view
    p["vis"][1] = dp.mask_from_list(dp.visible_list(p["vis"][1])[:1])
    p["pos"][2] = [50.0, 50.0, 50.0]         # off every image
    p["normal"][3] = [0.0, 0.0, 0.0]         # degenerate normal
    fo = dp.FastOptions(gradient=gradient)
    engine.set_fast_options(fo)
    try:
        for mode in (N.MODE_FAST_EVAL, N.MODE_FAST_REFINE):
            for cell in (5, 9):
                gp, op = p.copy(), p.copy()
                ga = engine.fast_refine(gp, cell, mode)
                oa = S.fast_refine(op, cell, mode, fo=orc.fast_options(fo))
                assert np.array_equal(ga, oa)
                assert_same(gp, op)
    finally:
        engine.set_fast_options(dp.FastOptions())
    assert len(engine.fast_refine(dp.empty_patches(0), 11)) == 0
    with pytest.raises(dp.DensePointsError):
        engine.set_fast_options(dp.FastOptions(margin=8))
    with pytest.raises(dp.DensePointsError):
        engine.set_fast_options(dp.FastOptions(tile_budget=32768))


@pytest.mark.parametrize("gradient", [0, 1])
def test_fast_expand_cfg3_full_scene(orc, gradient):
    """BASELINE config 3 (32 views 3840x2160): performance-mode expansion of
    2,000 refined parents equals the spec bit for bit (forward differences and
    the analytic gradient), and its geometry beats the parity mode's against
    the synthetic ground truth."""
    from test_gpu_configs import DeviceScene, spread

    with dp.Engine(device=0) as eng:
        sc = DeviceScene("cfg3_32view_4k", eng)
        S = orc.Scene(sc.P, sc.host_images())
        seeds = spread(sc.seeds, 600)
        par = eng.seeds_to_patches(seeds)
        acc = eng.refine(par, 16, N.MODE_SEED)
        par = np.ascontiguousarray(np.resize(par[acc == 1], 2000))
        fo = dp.FastOptions(gradient=gradient)
        eng.set_fast_options(fo)
        for cell in (11, 7):
            o = dp.Options(expand_cell_size=cell)
            eng.set_options(o)
            gk, ga = eng.fast_expand(par)
            S2 = orc.Scene(sc.P, sc.host_images(), o)
            ok, oa = S2.fast_expand(par, orc.fast_options(fo))
            assert np.array_equal(ga, oa)
            assert_same(gk, ok, FIELDS + ("parent",))
            assert 0.1 < ga.mean() < 0.95
        eng.set_options(dp.Options())
        nk, na = eng.expand(par)
    def err(k, a):
        k = k[a == 1]
        z, _ = synth.surface(sc.cfg, k["pos"][:, :2].astype(np.float64))
        return float(np.median(np.abs(k["pos"][:, 2] - z)))
    # cell 7 children vs the parity (Nelder-Mead, cell 11) children
    assert err(gk, ga) < err(nk, na)


def test_fast_expand_cfg5_full_scene(orc):
    """BASELINE config 5 (128 views 7680x4320, fp16 gray planes, 11x11 window)
    on one GPU: performance-mode expansion of 400 refined parents equals the
    spec bit for bit (the BGRA8 levels are 17 GB, the gray planes 8.5 GB in
    HBM); geometry within the scene's tolerance of the ground truth."""
    from test_gpu_configs import DeviceScene, spread

    o = dp.Options(expand_cell_size=11)
    with dp.Engine(device=0) as eng:
        sc = DeviceScene("cfg5_128view_8k", eng)
        seeds = spread(sc.seeds, 800)
        par = eng.seeds_to_patches(seeds)
        acc = eng.refine(par, 16, N.MODE_SEED)
        par = np.ascontiguousarray(par[acc == 1][:400])
        assert len(par) >= 200
        eng.set_options(o)
        gk, ga = eng.fast_expand(par)
        st = eng.fast_last_stats()
    S = orc.Scene(sc.P, sc.host_images(), o)
    ok, oa = S.fast_expand(par)
    assert np.array_equal(ga, oa)
    assert_same(gk, ok, FIELDS + ("parent",))
    assert 0.1 < ga.mean() < 0.95 and st["patches"] == 4 * len(par)
    k = gk[ga == 1]
    z, _ = synth.surface(sc.cfg, k["pos"][:, :2].astype(np.float64))
    print("cfg5 accepted %d of %d, median |dz| %.5f, staged views per eval %.2f"
          % (len(k), len(gk), float(np.median(np.abs(k["pos"][:, 2] - z))), st["view_evals"] / st["evals"]))


@pytest.mark.parametrize("name,max_pops,gradient", [("hf6", None, 0), ("plane4", None, 0), ("hf6", 37, 0),
                                                    ("hf6", None, 1), ("hf6", 37, 1)])
def test_fast_densify_bit_exact(orc, name, max_pops, gradient):
    """dp_densify with dp_fast_options.densify = 1: the seed stage and every
    expansion generation refined in performance mode (forward differences or
    the analytic gradient), the organizer claims as in the parity densify
    (PatchOrganizer::TryInsert in sequence order), the pop cap (expand.cpp:95);
    equal to the oracle's generation-at-a-time restatement on every stored field."""
    sc = scene(name)
    opts = dp.Options() if max_pops is None else dp.Options(max_pops=max_pops)
    fo = dp.FastOptions(densify=1, gradient=gradient)
    S = orc.Scene(sc.P, sc.imgs, opts)
    op = orc.GenerationEngine(S, threads=8, fast=fo).densify_all(sc.seeds)
    with dp.Engine(opts, device=0) as eng:
        eng.set_views(sc.views)
        eng.set_fast_options(fo)
        gp, gst = eng.densify(sc.seeds)
    assert gst["patches"] == len(op) > 20
    if max_pops is not None:
        assert gst["pops"] == max_pops
    assert_same(gp, op, FIELDS + ("seq", "parent", "rgb"))


def test_fast_densify_generation_protocol_bit_exact(orc):
    """The generation-at-a-time densify (the multi-GPU protocol) in
    performance mode: every generation's candidates refined by owner shards
    (dp_densify_owners + dp_densify_refine_items, two simulated ranks) and
    committed in sequence order equals dp_densify with the same flag."""
    sc = scene("hf6")
    opts = dp.Options(max_pops=90)
    fo = dp.FastOptions(densify=1)
    with dp.Engine(opts, device=0) as eng:
        eng.set_views(sc.views)
        eng.set_fast_options(fo)
        gp, gst = eng.densify(sc.seeds)
        g = eng.densify_begin(sc.seeds)
        while g.items:
            own, _ = eng.densify_owners(g, 2)
            per = g.per_item
            cand = np.zeros(g.items * per, dtype=N.PATCH_DTYPE)
            acc = np.zeros(g.items * per, dtype=np.uint8)
            for r in range(2):
                it = np.nonzero(own == r)[0].astype(np.int64)
                c, a = eng.densify_refine_items(g, it)
                sl = (it[:, None] * per + np.arange(per)).reshape(-1)
                cand[sl], acc[sl] = c, a
            g = eng.densify_commit(g, cand, acc)
        sp, sst = eng.densify_result()
    assert sst["patches"] == gst["patches"] > 20 and sst["pops"] == gst["pops"]
    assert sp.tobytes() == gp.tobytes()


def test_pmvs_host_mirror_fast_mode(orc):
    """PMVS(fast=FastOptions(densify=1)).run (the Python mirror of PMVS::Run,
    pmvs.cpp:22-43) in performance mode equals the oracle's restatement."""
    sc = scene("plane4")
    fo = dp.FastOptions(densify=1)
    pm = dp.PMVS(fast=fo)
    for v in sc.views:
        pm.add_camera(v)
    pm.run(sc.seeds)
    S = orc.Scene(sc.P, sc.imgs)
    op = orc.GenerationEngine(S, threads=8, fast=fo).densify_all(sc.seeds)
    assert len(pm.patches) == len(op) > 20
    assert_same(pm.patches, op, FIELDS + ("seq", "parent", "rgb"))

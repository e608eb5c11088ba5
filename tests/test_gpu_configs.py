"""BASELINE.json configs 2-4 at their real scene sizes on the HIP path, against
the oracle on bounded samples (bit-exact on every field).

The views are rendered on the device (dp_synth_render_device, as bench.py does)
and copied to the host for the oracle.  The reference anchors of the checked
steps: Seed::FilterPatches + OptimizePatches (methods/pmvs/seed.cpp:110-144),
Expand::ExpandPatch (expand.cpp:103-143) and PMVS::Run minus matching
(pmvs.cpp:22-43), on pyramid levels built by cv::pyrDown (dp_build_pyramid).

  cfg2  8 x 1920x1080, 3-level pyramid (bit-exact), densify with
        expand_cell_size = 7 on a seed subset at level 0 and level 2
  cfg3  32 x 3840x2160, 4-level pyramid (two views), seed stage on a spread
        subset, n = 11 expansion of 2,000 refined parents
  cfg4  64 x 3840x2160 (one GPU), the same kind of sample with 1,000 parents
Config 5 (fp16 gray planes, 11x11 window) is the performance mode's: its full
scene runs in tests/test_gpu_fast.py (test_fast_expand_cfg5_full_scene).
"""
import ctypes

import numpy as np
import pytest
import torch

import densepoints_amd as dp
from densepoints_amd import _native as N
from densepoints_amd import synth

from test_gpu_parity import FIELDS, assert_same

pytestmark = pytest.mark.gpu


class DeviceScene:
    """A named BASELINE config rendered straight into HBM (BGRA8 planes in one
    pool), registered with an engine, with host BGR copies for the oracle."""

    def __init__(self, name, eng, host_views=None):
        self.cfg = synth.named(name)
        c = self.cfg
        self.V, self.W, self.H = c.n_views, c.width, c.height
        self.P = synth.cameras(c)
        self.planes = torch.empty((self.V, self.H, self.W), dtype=torch.int32, device="cuda")
        for v in range(self.V):
            N.check(N.lib.dp_synth_render_device(eng.handle, ctypes.byref(c), N.ptr(self.P), v,
                                                 self.planes[v].data_ptr(), None), eng.handle)
        torch.cuda.synchronize()
        eng.set_views_device(self.P, [self.W] * self.V, [self.H] * self.V, [self.W] * self.V,
                             [p.data_ptr() for p in self.planes])
        self.seeds = synth.seeds(c, self.P)
        vs = range(self.V) if host_views is None else host_views
        self.imgs = {v: np.ascontiguousarray(self.planes[v].cpu().numpy().view(np.uint8)
                                             .reshape(self.H, self.W, 4)[:, :, :3]) for v in vs}

    def host_images(self):
        return [self.imgs[v] for v in range(self.V)]


def spread(seeds, k):
    """k seeds spread over the whole list (every nominal reference view)."""
    idx = np.linspace(0, len(seeds) - 1, k).astype(np.int64)
    return np.ascontiguousarray(seeds[idx])


def test_cfg2_pyramid_and_densify_levels(orc):
    """cfg2: 8 views 1080p, 3 pyramid levels bit-exact, densify (n = 7 expansion,
    popped-parent cap) at level 0 and level 2 equal to the oracle's."""
    opts = dp.Options(expand_cell_size=7, max_pops=1500)
    with dp.Engine(opts, device=0) as eng:
        sc = DeviceScene("cfg2_8view_1080p", eng)
        eng.build_pyramid(3)
        levels = {0: sc.host_images()}
        for lvl in (1, 2):
            levels[lvl] = [orc.pyr_down(im) for im in levels[lvl - 1]]
            for v in range(sc.V):
                got = eng.read_level(lvl, v)
                assert np.array_equal(got, levels[lvl][v]), f"view {v} level {lvl}"
        seeds = spread(sc.seeds, 400)
        for lvl in (0, 2):
            eng.set_level(lvl)
            gp, gst = eng.densify(seeds)
            PL = sc.P.reshape(-1, 3, 4).copy()
            PL[:, :2, :] *= 2.0 ** -lvl
            S = orc.Scene(PL, levels[lvl], opts)
            op, ost = S.densify(seeds)
            assert gst["patches"] == ost["patches"] and gst["pops"] == ost["pops"], (lvl, gst, ost)
            assert len(gp) > 100, (lvl, len(gp))
            assert_same(gp, op, FIELDS + ("seq", "parent", "rgb"))


def _seed_and_expand(orc, name, n_seeds, n_parents, pyramid_views=()):
    with dp.Engine(device=0) as eng:
        sc = DeviceScene(name, eng)
        if pyramid_views:
            eng.build_pyramid(4)
            for v in pyramid_views:
                ref = sc.imgs[v]
                for lvl in range(1, 4):
                    ref = orc.pyr_down(ref)
                    assert np.array_equal(eng.read_level(lvl, v), ref), f"view {v} level {lvl}"
        S = orc.Scene(sc.P, sc.host_images())
        seeds = spread(sc.seeds, n_seeds)
        # seed stage: FilterPatches + OptimizePatches at n = 16
        gp = eng.seeds_to_patches(seeds)
        op = S.seeds_to_patches(seeds)
        assert gp.tobytes() == op.tobytes()
        ga = eng.refine(gp, 16, N.MODE_SEED)
        oa = S.refine(op, 16, N.MODE_SEED)
        assert np.array_equal(ga, oa)
        assert_same(gp, op)
        # the bench step on this scene: ExpandPatch of refined parents at n = 11
        parents = gp[ga == 1]
        assert len(parents) > 100, len(parents)
        parents = np.ascontiguousarray(np.resize(parents, n_parents))
        gk, gacc = eng.expand(parents)
        ok, oacc = S.expand(parents)
        assert np.array_equal(gacc, oacc)
        assert_same(gk, ok, FIELDS + ("parent",))
        assert 0.05 < gacc.mean() < 0.95
        assert gk["evals"].mean() > 10
        return gk


def test_cfg3_32view_4k_seed_and_expand(orc):
    """cfg3 (the roofline scene): 32 views 3840x2160, 4-level pyramid on two
    views, seed stage on 600 spread seeds, n = 11 expansion of 2,000 parents."""
    _seed_and_expand(orc, "cfg3_32view_4k", 600, 2000, pyramid_views=(0, 31))


def test_cfg4_64view_4k_seed_and_expand(orc):
    """cfg4 on one GPU: 64 views 3840x2160, seed stage on 400 seeds, 1,000 parents."""
    kids = _seed_and_expand(orc, "cfg4_64view_4k", 400, 1000)
    nvis = np.array([bin(int(a)).count("1") + bin(int(b)).count("1") for a, b in kids["vis"]])
    print("cfg4 visible views per child: mean %.2f max %d" % (nvis.mean(), nvis.max()))


def test_cfg4_64view_4k_whole_densify_equals_oracle(orc):
    """cfg4 (64 views 3840x2160), the whole densify -- PMVS::Run minus matching
    (methods/pmvs/pmvs.cpp:22-43): seed stage, organizer, FIFO expansion with
    the pop cap -- on 400 spread seeds, max_pops 1,500, against the oracle's
    single-thread restatement on every field and in order.  This pins, at the
    config-4 scale, the dp_densify that the partitioned multi-rank tests
    (test_gpu_dist.py) compare their stores with."""
    opts = dp.Options(max_pops=1500)
    with dp.Engine(opts, device=0) as eng:
        sc = DeviceScene("cfg4_64view_4k", eng)
        seeds = spread(sc.seeds, 400)
        gp, gst = eng.densify(seeds)
        S = orc.Scene(sc.P, sc.host_images(), opts)
        op, ost = S.densify(seeds)
    assert gst["patches"] == ost["patches"] and gst["pops"] == ost["pops"], (gst, ost)
    assert 500 < gst["pops"] <= 1500 and len(gp) > 1000, gst
    assert_same(gp, op, FIELDS + ("seq", "parent", "rgb"))

"""Golden vectors (tests/golden/pmvs_small.npz, made by tests/golden/make_golden.py):
fixed inputs (4 BGR8 views 192x144, cameras, seed points) and the oracle's
outputs for every stage of the patch loop.

* CPU: the oracle re-run on the stored inputs reproduces every stored output
  bit for bit.  This pins the restatement against regressions between rounds;
  the restatement itself is pinned by the reference's known answers
  (test_oracle_kat.py).
* GPU: the HIP path (through the C ABI) reproduces the same vectors.
"""
import os

import numpy as np
import pytest

import densepoints_amd as dp
from densepoints_amd._native import PATCH_DTYPE

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pmvs_small.npz")
MODES = {"filter": 1, "nm": 2, "seed": 3}
CELLS = (16, 11, 7)


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _bytes(a):
    return np.ascontiguousarray(a, dtype=PATCH_DTYPE).tobytes()


def test_golden_fixture_shape(gold):
    assert gold["P"].shape == (4, 3, 4) and gold["images"].shape == (4, 144, 192, 3)
    assert len(gold["seed_patches"]) == len(gold["seeds"]) > 500
    # the filtering modes keep some and reject some patches (both branches are in the
    # vectors); Optimize alone always returns true (optimization_opencv.cpp:77)
    for cell in CELLS:
        for name in ("filter", "seed"):
            acc = gold[f"accept_{name}_{cell}"]
            assert 0 < acc.sum() < len(acc)
        assert gold[f"accept_nm_{cell}"].all()
    assert 0 < gold["expand_accept"].sum() < len(gold["expand_accept"])
    assert len(gold["densify"]) == gold["densify_stats"][0] > len(gold["expand_parents"])


def test_oracle_reproduces_golden(gold, orc):
    S = orc.Scene(gold["P"], list(gold["images"]))
    pat = S.seeds_to_patches(gold["seeds"])
    assert _bytes(pat) == _bytes(gold["seed_patches"])
    for name, mode in MODES.items():
        for cell in CELLS:
            r = pat.copy()
            acc = S.refine(r, cell, mode, 2)
            assert _bytes(r) == _bytes(gold[f"refine_{name}_{cell}"]), (name, cell)
            assert np.array_equal(acc, gold[f"accept_{name}_{cell}"]), (name, cell)
    kids, kacc = S.expand(gold["expand_parents"], 2)
    assert _bytes(kids) == _bytes(gold["expand_children"])
    assert np.array_equal(kacc, gold["expand_accept"])
    dense, st = S.densify(gold["seeds"])
    assert _bytes(dense) == _bytes(gold["densify"])
    assert [st["patches"], st["seed_patches"], st["pops"]] == list(gold["densify_stats"])


@pytest.mark.gpu
def test_hip_path_reproduces_golden(gold):
    views = [dp.View(gold["P"][v], gold["images"][v]) for v in range(len(gold["P"]))]
    with dp.Engine(device=0) as eng:
        eng.set_views(views)
        pat = eng.seeds_to_patches(gold["seeds"])
        assert _bytes(pat) == _bytes(gold["seed_patches"])
        for name, mode in MODES.items():
            for cell in CELLS:
                r = pat.copy()
                acc = eng.refine(r, cell, mode)
                assert _bytes(r) == _bytes(gold[f"refine_{name}_{cell}"]), (name, cell)
                assert np.array_equal(acc, gold[f"accept_{name}_{cell}"]), (name, cell)
        kids, kacc = eng.expand(gold["expand_parents"])
        assert _bytes(kids) == _bytes(gold["expand_children"])
        assert np.array_equal(kacc, gold["expand_accept"])
        dense, st = eng.densify(gold["seeds"])
        assert _bytes(dense) == _bytes(gold["densify"])
        assert [st["patches"], st["seed_patches"], st["pops"]] == list(gold["densify_stats"])

"""PMVS-style patch filter: the oracle's C restatement
(oracle/oracle.c or_filter_patches) against an independent pure-Python
statement of the spec in include/densepoints.h (dp_filter_patches), on the
golden densify output and on variants with planted occluders.  There is no
reference implementation (pmvs.h:27 is undefined, modules/filtering empty):
the spec is pinned by these two statements only ("parity unpinned" vs any
reference binary)."""
import math
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pmvs_small.npz")


def _proj(P, X):
    h = [((P[r, 0] * X[0] + P[r, 1] * X[1]) + P[r, 2] * X[2]) + P[r, 3] for r in range(3)]
    return h[0] / h[2], h[1] / h[2], h[2]


def _cell_index(v, scale):
    q = v / scale
    if not q > -1.0:
        return -1
    return int(q)


def _mask_views(vis):
    return [w * 64 + b for w in range(2) for b in range(64) if (int(vis[w]) >> b) & 1]


def filter_spec(P, W, H, xr, patches, passes=3, frac=0.25, gs=8):
    n = len(patches)
    gw = [w // gs for w in W]
    gh = [h // gs for h in H]
    pos = [tuple(float(c) for c in p["pos"]) for p in patches]
    nrm = [tuple(float(c) for c in p["normal"]) for p in patches]
    score = [float(p["score"]) for p in patches]

    def cell(v, i):
        u, w, _ = _proj(P[v], pos[i])
        r, c = _cell_index(w, float(gs)), _cell_index(u, float(gs))
        return (r, c) if 0 <= c < gw[v] and 0 <= r < gh[v] else None

    def rho(i):
        rv = int(patches[i]["ref"])
        u0, w0, _ = _proj(P[rv], pos[i])
        u1, w1, _ = _proj(P[rv], tuple(pos[i][k] + xr[rv][k] for k in range(3)))
        du, dw = u1 - u0, w1 - w0
        dx = math.sqrt(du * du + dw * dw)
        return gs / dx if dx > 0.0 else 0.0

    def nb(i, q, r2):
        d = [pos[q][k] - pos[i][k] for k in range(3)]
        a = (d[0] * nrm[i][0] + d[1] * nrm[i][1]) + d[2] * nrm[i][2]
        b = (d[0] * nrm[q][0] + d[1] * nrm[q][1]) + d[2] * nrm[q][2]
        return abs(a) + abs(b) < r2

    def front(alive):
        f = {}
        for i in range(n):
            if not alive[i]:
                continue
            for v in _mask_views(patches[i]["vis"]):
                c = cell(v, i)
                if c is None:
                    continue
                d = np.float32(_proj(P[v], pos[i])[2])
                if not d > 0:
                    continue
                key = (int(np.array([d], np.float32).view(np.uint32)[0]) << 32) | i
                f[(v, c)] = min(f.get((v, c), key), key)
        return f

    rhos = [rho(i) for i in range(n)]
    alive = [1] * n
    if passes & 1:
        f = front(alive)
        keep = []
        for i in range(n):
            views = _mask_views(patches[i]["vis"])
            occ = 0.0
            for v in views:
                c = cell(v, i)
                if c is None or (v, c) not in f:
                    continue
                q = f[(v, c)] & 0xFFFFFFFF
                if q == i or nb(i, q, 2.0 * rhos[i]):
                    continue
                occ = occ + float(np.float32(score[q]))
            keep.append(0 if len(views) * score[i] < occ else 1)
        alive = keep
    if passes & 2:
        f = front(alive)
        keep = []
        for i in range(n):
            if not alive[i]:
                keep.append(0)
                continue
            tot = near = 0
            for v in _mask_views(patches[i]["vis"]):
                c = cell(v, i)
                if c is None:
                    continue
                for dr in (-1, 0, 1):
                    for dc in (-1, 0, 1):
                        r, cc = c[0] + dr, c[1] + dc
                        if not (0 <= r < gh[v] and 0 <= cc < gw[v]) or (v, (r, cc)) not in f:
                            continue
                        q = f[(v, (r, cc))] & 0xFFFFFFFF
                        if q == i:
                            continue
                        tot += 1
                        near += nb(i, q, 2.0 * rhos[i])
            keep.append(0 if tot > 0 and near < frac * tot else 1)
        alive = keep
    return np.array(alive, dtype=np.uint8)


def with_occluders(orc, P, patches, k=25, pull=0.3, score=0.99):
    """For each of the first k patches and each view it is visible in, a copy
    pulled toward that view's camera (same ray: same cell, in front, not a
    neighbour) with a high score, appended after the originals."""
    extra = []
    for p in patches[:k]:
        X = p["pos"].astype(np.float64)
        for v in _mask_views(p["vis"]):
            C = orc.view_geometry(P[v])[1]
            e = p.copy()
            e["pos"] = (C + (1.0 - pull) * (X - C)).astype(np.float32)
            e["score"] = np.float32(score)
            extra.append(e)
    return np.concatenate([patches, np.array(extra, dtype=patches.dtype)])


@pytest.fixture(scope="module")
def gold(orc):
    d = np.load(GOLD)
    P = d["P"]
    imgs = [d["images"][i] for i in range(len(P))]
    xr = [orc.view_geometry(P[v])[4] for v in range(len(P))]
    return P, imgs, xr, d["densify"]


@pytest.mark.parametrize("passes", [1, 2, 3])
@pytest.mark.parametrize("occl", [False, True])
def test_oracle_filter_equals_python_spec(orc, gold, passes, occl):
    P, imgs, xr, pat = gold
    if occl:
        pat = with_occluders(orc, P, pat)
    S = orc.Scene(P, imgs)
    got = S.filter_patches(pat, passes)
    want = filter_spec(P, [im.shape[1] for im in imgs], [im.shape[0] for im in imgs], xr, pat, passes)
    assert np.array_equal(got, want)
    if occl and passes & 1:
        # planted occluders remove at least some of the occluded originals
        assert got[:25].sum() < 25


def test_filter_monotone_and_edge_cases(orc, gold):
    P, imgs, xr, pat = gold
    S = orc.Scene(P, imgs)
    k1 = S.filter_patches(pat, 1)
    k3 = S.filter_patches(pat, 3)
    assert (k3 <= k1).all()
    assert S.filter_patches(pat, 0).all()
    assert len(S.filter_patches(pat[:0], 3)) == 0
    one = S.filter_patches(pat[:1], 3)  # a lone patch has no occluder and no neighbour set
    assert one[0] == 1

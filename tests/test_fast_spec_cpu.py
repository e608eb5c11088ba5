"""The performance-mode specification (oracle/or_fast.c) on the CPU.

The mode has no reference counterpart (it replaces OptimizationOpenCV::Optimize,
methods/pmvs/optimization_opencv.cpp:44-78), so the spec is pinned here by
  - an independent numpy restatement of one fast evaluation (staging, fp32
    affine window map, 1/16-gray bilinear, integer moments, fp64 NCC),
    compared bit for bit with the C oracle's DP_MODE_FAST_EVAL scores;
  - its invariants (evaluation count E <= 1 + 5 iters + 1, three fewer per
    reused gradient, FAST_EVAL leaves the
    pose and masks alone, the tile budget), and the affine window map's
    distance from the projective quotient it replaced;
  - what it is for: against the synthetic scene's ground truth, refined
    children are closer to the surface than the unrefined ones and than the
    parity mode's Nelder-Mead children, and more CG iterations help.
"""
import numpy as np
import pytest

from densepoints_amd import synth


@pytest.fixture(scope="module")
def small_scene():
    cfg = synth.config(6, 320, 240, 1)
    P, imgs, seeds = synth.scene_host(cfg)
    return cfg, P, imgs, seeds


def _fmaf(a, b, c):
    """fmaf(a, b, c): a*b is exact in fp64 for fp32 inputs; when the fp64 sum
    is exact too, its fp32 rounding is the single rounding of fmaf, otherwise
    the exact value is rounded to fp32 (nearest, ties to even)."""
    from fractions import Fraction

    a, b, c = np.float32(a), np.float32(b), np.float32(c)
    s = np.float64(a) * np.float64(b)
    t = s + np.float64(c)
    if not np.isfinite(t):
        return np.float32(t)
    ex = Fraction(float(s)) + Fraction(float(c))
    if Fraction(float(t)) == ex:
        return np.float32(t)
    f = np.float32(t)
    best = None
    for cand in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        d = abs(Fraction(float(cand)) - ex)
        if best is None or d < best[0] or (d == best[0] and int(cand.view(np.uint32)) % 2 == 0):
            best = (d, cand)
    return np.float32(best[1])


def _f(x):
    return np.float32(x)


def _fdot(a, b):
    return _fmaf(a[2], b[2], _fmaf(a[1], b[1], _f(a[0]) * _f(b[0])))


def _gray(img):
    b, g, r = (img[..., k].astype(np.int64) for k in range(3))
    return ((1868 * b + 9617 * g + 4899 * r + 8192) >> 14).astype(np.int64)


def _fcam(orc, P, v):
    """fp32 camera (or_fast.c fcam_of): rows 0-1 of P times 32, row 2, the
    centre and the unit x-axis, each rounded once."""
    Pv = np.asarray(P[v], dtype=np.float64).reshape(12)
    Q = np.array([np.float32(32.0 * Pv[k]) if k < 8 else np.float32(Pv[k]) for k in range(12)], dtype=np.float32)
    _, C, _, _, xa = orc.view_geometry(Pv)
    xr = xa / np.sqrt(xa @ xa)
    return Q, C.astype(np.float32), xr.astype(np.float32)


def _qpt(Q, k, X):
    return _fmaf(Q[4 * k + 2], X[2], _fmaf(Q[4 * k + 1], X[1], _fmaf(Q[4 * k], X[0], Q[4 * k + 3])))


def _qdir(Q, k, w):
    return _fmaf(Q[4 * k + 2], w[2], _fmaf(Q[4 * k + 1], w[1], _f(Q[4 * k]) * _f(w[0])))


def _bf16(x):
    u = int(np.float32(x).view(np.uint32))
    return np.uint32((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).view(np.float32)


def _q16(f):
    return int(np.int16(np.uint16((int(np.float32(f).view(np.uint32)) - 0x4B400000) & 0xFFFF)))


def _i32(x):
    return ((int(x) + 2 ** 31) % 2 ** 32) - 2 ** 31


def _fast_eval_numpy(orc, S, P, imgs, p, cell, fo, grad=False):
    """Independent statement of DP_MODE_FAST_EVAL's score (include/densepoints.h
    dp_fast_options, spec v3: fp32 frame and view geometry, margin 0): returns
    the mean NCC or -1.  grad: spec v4's objective and analytic gradient at
    the staged pose instead (or_fast.c fast_objective_grad), (m, f, g)."""
    V = len(imgs)
    cams = [_fcam(orc, P, v) for v in range(V)]
    lo, hi = _f(2.0 ** -20), _f(2.0 ** 64)

    def proj(v, X):
        Q = cams[v][0]
        h2 = _qpt(Q, 2, X)
        if not (lo <= h2 <= hi):
            return None
        r = _f(1.0) / h2
        return _qpt(Q, 0, X) * r, _qpt(Q, 1, X) * r

    ref = int(p["ref"])
    Qr, Cr, xr = cams[ref]
    X = p["pos"].astype(np.float32)
    n0 = p["normal"].astype(np.float32)
    a, b = proj(ref, X), proj(ref, (X + xr).astype(np.float32))
    if a is None or b is None:
        return -1.0
    du, dv = b[0] - a[0], b[1] - a[1]
    dx = np.sqrt(_fmaf(dv, dv, du * du))
    nl = np.sqrt(_fdot(n0, n0))
    if not (dx > 0 and dx <= 2.0 ** 100 and nl > 0):
        return -1.0
    ps = _f(32.0) / dx
    inl = _f(1.0) / nl
    nn = (n0 * inl).astype(np.float32)
    xn = _fdot(xr, nn)
    e1 = np.array([_fmaf(-xn, nn[k], xr[k]) for k in range(3)], dtype=np.float32)
    el = np.sqrt(_fdot(e1, e1))
    if not el > 0:
        return -1.0
    e1 = (e1 * (_f(1.0) / el)).astype(np.float32)
    e2 = np.array([_fmaf(nn[1], e1[2], -(nn[2] * e1[1])), _fmaf(nn[2], e1[0], -(nn[0] * e1[2])),
                   _fmaf(nn[0], e1[1], -(nn[1] * e1[0]))], dtype=np.float32)
    r = (X - Cr).astype(np.float32)
    sd = ps / np.sqrt(_fdot(r, r))
    st = _f(2.0) / _f(cell - 1)
    ws = [r, (e1 * ps).astype(np.float32), (e2 * ps).astype(np.float32), (nn * ps).astype(np.float32)]
    c = _f(0.5) * _f(cell - 1)
    vis = [v for v in range(V) if (int(p["vis"][v >> 6]) >> (v & 63)) & 1][:64]
    staged = []
    for v in vis:
        Q = cams[v][0]
        H = [[_qpt(Q, k, X) for k in range(3)]] + [[_qdir(Q, k, w) for k in range(3)] for w in ws]
        s = H[0][2]
        if not (lo <= s <= hi):
            continue
        inv = _f(1.0) / s
        g = [np.array([h[0] * inv, h[1] * inv, h[2] * inv], dtype=np.float32) for h in H]
        U0, V0 = g[0][0], g[0][1]
        Ui, Vi = _fmaf(-U0, g[2][2], g[2][0]), _fmaf(-V0, g[2][2], g[2][1])
        Uj, Vj = _fmaf(-U0, g[3][2], g[3][0]), _fmaf(-V0, g[3][2], g[3][1])
        eu, ev = c * (abs(Ui) + abs(Uj)), c * (abs(Vi) + abs(Vj))
        ez = c * (abs(g[2][2]) + abs(g[3][2]))
        umin, umax, vmin, vmax = U0 - eu, U0 + eu, V0 - ev, V0 + ev
        Hh, Ww = imgs[v].shape[:2]
        if not (g[0][2] - ez > 0):
            continue
        if not (umin > 0 and umax < _f(32 * Ww) and vmin > 0 and vmax < _f(32 * Hh)):
            continue
        xa, xb = int(np.floor(umin * _f(0.03125))), int(np.floor(umax * _f(0.03125))) + 1
        ya, yb = int(np.floor(vmin * _f(0.03125))), int(np.floor(vmax * _f(0.03125))) + 1
        if xb - xa + 1 > 48 or yb - ya + 1 > 48:
            continue
        x0, y0 = max(xa, 0) & ~1, max(ya, 0)  # even left edge (32-bit fp16 pairs on the device)
        tw, th = min(xb, Ww - 1) - x0 + 1, min(yb, Hh - 1) - y0 + 1
        staged.append((v, g, x0, y0, tw, th, 4 * ((tw + 2) // 2) * (th + 1) + 64))
        # spec v5: the scoring staging (FAST_EVAL) takes up to filter_max_views
        # views (0 = max_views), the refine's (the gradient probe) max_views
        cap = fo.max_views if grad else (fo.filter_max_views or fo.max_views)
        if len(staged) == cap:
            break
    tot, keep = 0, []
    for t in staged:
        if tot + t[6] > fo.tile_budget:
            break
        tot += t[6]
        keep.append(t)
    if len(keep) < 2:
        return (len(keep), None, None) if grad else -1.0
    N = cell * cell
    samples, qs = [], []
    M = _f(1.5 * 2.0 ** 23)
    for v, g, x0, y0, tw, th, _ in keep:
        ox, oy = _f(-32.0 * x0), _f(-32.0 * y0)
        vec = [np.array([_fmaf(ox, gg[2], gg[0]), _fmaf(oy, gg[2], gg[1]), gg[2]], dtype=np.float32) for gg in g]
        gray = _gray(imgs[v])
        Hh, Ww = gray.shape
        A, B1, B2 = vec[0], vec[2], vec[3]
        # first-order map of the homography about the window centre
        rz = np.float32(1.0) / max(A[2], np.float32(2.0 ** -20))
        U0, V0 = A[0] * rz, A[1] * rz
        Ui, Vi = _fmaf(-U0, B1[2], B1[0]) * rz, _fmaf(-V0, B1[2], B1[1]) * rz
        Uj, Vj = _fmaf(-U0, B2[2], B2[0]) * rz, _fmaf(-V0, B2[2], B2[1]) * rz
        if grad:
            z1, Hn = vec[1][2], vec[4]
            dU0, dV0 = _fmaf(-U0, z1, vec[1][0]) * rz, _fmaf(-V0, z1, vec[1][1]) * rz
            dUi, dVi = _fmaf(-dU0, B1[2], -(Ui * z1)) * rz, _fmaf(-dV0, B1[2], -(Vi * z1)) * rz
            dUj, dVj = _fmaf(-dU0, B2[2], -(Uj * z1)) * rz, _fmaf(-dV0, B2[2], -(Vj * z1)) * rz
            ku, kv = _fmaf(U0, Hn[2], -Hn[0]) * rz, _fmaf(V0, Hn[2], -Hn[1]) * rz
            fd, fa = sd * _f(2.0 ** -10), st * _f(2.0 ** -10)
            cU0, cV0, cUi, cVi, cUj, cVj = (_bf16(x * fd) for x in (dU0, dV0, dUi, dVi, dUj, dVj))
            cku, ckv = _bf16(ku * fa), _bf16(kv * fa)
            qv = np.zeros((N, 3), dtype=np.int64)
        out = np.zeros(N, dtype=np.int64)
        for j in range(cell):
            tj = np.float32(j) - c
            for i in range(cell):
                ti = np.float32(i) - c
                b23 = np.float32(2.0 ** 23)
                U = min(max(_fmaf(tj, Uj, _fmaf(ti, Ui, U0)) + b23, b23), b23 + np.float32(32 * (tw - 1)))
                W = min(max(_fmaf(tj, Vj, _fmaf(ti, Vi, V0)) + b23, b23), b23 + np.float32(32 * (th - 1)))
                iu, iv = int(U - b23), int(W - b23)
                xx, fx, yy, fy = iu >> 5, iu & 31, iv >> 5, iv & 31

                def px(x, y):
                    return gray[min(y0 + y, Hh - 1), min(x0 + x, Ww - 1)]
                b = ((32 - fx) * (32 - fy) * px(xx, yy) + fx * (32 - fy) * px(xx + 1, yy) +
                     (32 - fx) * fy * px(xx, yy + 1) + fx * fy * px(xx + 1, yy + 1) + 32) >> 6
                out[j * cell + i] = b
                if grad:
                    p00, p01, p10, p11 = (int(px(xx, yy)), int(px(xx + 1, yy)), int(px(xx, yy + 1)),
                                          int(px(xx + 1, yy + 1)))
                    gx = _f((32 - fy) * (p01 - p00) + fy * (p11 - p10))
                    gy = _f((32 - fx) * (p10 - p00) + fx * (p11 - p01))
                    au, av = _fmaf(tj, cUj, _fmaf(ti, cUi, cU0)), _fmaf(tj, cVj, _fmaf(ti, cVi, cV0))
                    sl_ = _fmaf(gy, ckv, gx * cku)
                    qv[j * cell + i] = (_q16(_fmaf(gy, av, _fmaf(gx, au, M))), _q16(_fmaf(ti, sl_, M)),
                                        _q16(_fmaf(tj, sl_, M)))
        samples.append(out)
        if grad:
            qs.append(qv)
    a = samples[0]
    dmin = 0.1 * 256.0 * N * N
    if grad:
        import math
        Sa, Saa = int(a.sum()), int((a * a).sum())
        QA = qs[0]
        Da = [_i32(QA[:, p].sum()) for p in range(3)]
        Daa = [_i32((a * QA[:, p]).sum()) for p in range(3)]
        G, qsum = [0, 0, 0], 0
        for b, Q in zip(samples[1:], qs[1:]):
            Sb, Sbb, Sab = int(b.sum()), int((b * b).sum()), int((a * b).sum())
            num = float(N) * float(Sab) - float(Sa) * float(Sb)
            va = float(N) * float(Saa) - float(Sa) * float(Sa)
            vb = float(N) * float(Sbb) - float(Sb) * float(Sb)
            den32 = np.sqrt(_f(va) * _f(vb))
            r32 = _f(1.0) / (den32 if den32 > _f(dmin) else _f(dmin))
            qsum += int(np.rint((_f(num) * r32) * _f(16777216.0)))
            den = math.sqrt(va * vb)
            for p in range(3):
                dA, dAA = float(Da[p]), float(Daa[p])
                dB, dBB = float(_i32(Q[:, p].sum())), float(_i32((b * Q[:, p]).sum()))
                dAB = float(_i32((QA[:, p] * b + a * Q[:, p]).sum()))
                dnum = float(N) * dAB - dA * float(Sb) - float(Sa) * dB
                if den > dmin:
                    dva = 2.0 * (float(N) * dAA - float(Sa) * dA)
                    dvb = 2.0 * (float(N) * dBB - float(Sb) * dB)
                    dncc = dnum / den - (num / den) * (0.5 * (dva / va + dvb / vb))
                else:
                    dncc = dnum / dmin
                G[p] = _i32(G[p] + _sat_q24(dncc))
        f = (len(samples) - 1) * 16777216 - qsum
        return len(samples), f, np.array([_f(G[p]) * _f(-2.0 ** -20) for p in range(3)], dtype=np.float32)
    tot = 0.0
    for b in samples[1:]:
        num = N * int((a * b).sum()) - int(a.sum()) * int(b.sum())
        va = N * int((a * a).sum()) - int(a.sum()) ** 2
        vb = N * int((b * b).sum()) - int(b.sum()) ** 2
        den = np.sqrt(float(va) * float(vb))
        tot = tot + num / max(den, dmin)
    return float(np.float32(tot / (len(samples) - 1)))


def _sat_q24(dncc):
    """spec v4's quantiser: rint(dncc 2^24) clamped to int32 by maxNum/minNum"""
    if dncc != dncc:
        return -(2 ** 31)
    return int(min(max(np.rint(dncc * 16777216.0), -(2.0 ** 31)), 2.0 ** 31 - 1))


def test_fast_gradient_quantiser_saturates(orc):
    """a near-flat window (den just above the NCC floor, or the
    dnum / dmin branch) can give |dncc| >= 128; the spec saturates the 2^-24
    quantisation to int32 (the device's v_cvt semantics made explicit) instead
    of the C cast's undefined behaviour."""
    f = orc.lib.or_fast_grad_q24
    cases = [0.0, -0.0, 0.5 / 16777216, 1.5 / 16777216, -2.5 / 16777216, 0.3, -0.7, 127.99999994, 128.0,
             -128.0, -128.00000006, 200.0, -1e9, 1e300, float("inf"), float("-inf"), float("nan")]
    for x in cases:
        assert f(x) == _sat_q24(x), x
    assert f(1e6) == 2 ** 31 - 1 and f(-1e6) == -(2 ** 31) and f(float("nan")) == -(2 ** 31)


@pytest.mark.parametrize("cell", [7, 11])
def test_fast_eval_equals_numpy_restatement(orc, small_scene, cell):
    cfg, P, imgs, seeds = small_scene
    S = orc.Scene(P, imgs)
    p = S.seeds_to_patches(seeds[::5][:40])
    fo = orc.fast_options()
    q = p.copy()
    S.fast_refine(q, cell, orc.MODE_FAST_EVAL, fo)
    want = np.array([_fast_eval_numpy(orc, S, P, imgs, x, cell, fo) for x in p], dtype=np.float32)
    assert (want > -1).sum() > 20
    assert np.array_equal(q["score"].view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("cell", [7, 11])
def test_fast_gradient_equals_numpy_restatement(orc, small_scene, cell):
    """Spec v4's analytic gradient (bf16 window-map derivatives, 16-bit
    per-sample Q's, exact integer sums, fp64 quotient rule) restated in numpy
    equals the C oracle's at the staged pose, bit for bit, with the objective."""
    cfg, P, imgs, seeds = small_scene
    S = orc.Scene(P, imgs)
    p = S.seeds_to_patches(seeds[::9][:14])
    fo = orc.fast_options()
    n = 0
    for x in p:
        m, f, g = S.fast_grad_probe(x, cell, fo)
        mw, fw, gw = _fast_eval_numpy(orc, S, P, imgs, x, cell, fo, grad=True)
        assert m == mw
        if m >= 2:
            n += 1
            assert f == fw and g.view(np.uint32).tolist() == gw.view(np.uint32).tolist(), (g, gw)
            assert np.abs(g).max() > 0
    assert n >= 8


def test_fast_eval_does_not_mutate_pose(orc, small_scene):
    _, P, imgs, seeds = small_scene
    S = orc.Scene(P, imgs)
    p = S.seeds_to_patches(seeds[:50])
    q = p.copy()
    S.fast_refine(q, 11, orc.MODE_FAST_EVAL)
    for f in ("pos", "normal", "vis", "cand", "ref"):
        assert q[f].tobytes() == p[f].tobytes()
    assert (q["evals"] == 1).all()


@pytest.mark.parametrize("iters", [0, 2, 4])
def test_fast_evaluation_count_analytic(orc, small_scene, iters):
    """Spec v4: 1 + 2 iters + (iterations after a line search that moved x)
    evaluations, + 1 for the filter; one fewer per reused gradient."""
    _, P, imgs, seeds = small_scene
    S = orc.Scene(P, imgs)
    p = S.seeds_to_patches(seeds[:80])
    S.fast_refine(p, 11, orc.MODE_FAST_REFINE, orc.fast_options(iters=iters, gradient=1))
    ev = p["evals"]
    top = 2 + 3 * iters - (1 if iters > 0 else 0)
    assert ev.max() == top
    assert (ev[ev > 1] <= top).all()
    assert np.mean(ev == top) > 0.3
    if iters >= 4:
        assert np.mean((ev > 1) & (ev < top)) > 0.05  # gradients are reused


@pytest.mark.parametrize("iters", [0, 2, 4])
def test_fast_evaluation_count(orc, small_scene, iters):
    _, P, imgs, seeds = small_scene
    S = orc.Scene(P, imgs)
    p = S.seeds_to_patches(seeds[:80])
    S.fast_refine(p, 11, orc.MODE_FAST_REFINE, orc.fast_options(iters=iters, gradient=0))
    ev = p["evals"]
    # 1 + 5 iters (CG) + 1 (filter), less 3 for every iteration whose forward
    # differences repeat the last ones (the previous line search left x and
    # f(x) unchanged, so the gradient is reused), and fewer when the gradient
    # vanishes
    assert ev.max() == 2 + 5 * iters
    d = 2 + 5 * iters - ev[ev > 1]
    assert (d >= 0).all()
    assert np.mean(d % 3 == 0) > 0.9
    assert np.mean(ev == 2 + 5 * iters) > 0.3
    if iters >= 4:
        assert np.mean((d > 0) & (d % 3 == 0)) > 0.05  # gradients are reused


def _geom_err(cfg, k, a=None):
    """median |z - z_true| and median normal error (degrees) of patches k
    (the accepted ones when a is given) against synth.surface."""
    if a is not None:
        k = k[a == 1]
    z, nrm = synth.surface(cfg, k["pos"][:, :2].astype(np.float64))
    nn = k["normal"].astype(np.float64)
    nn /= np.linalg.norm(nn, axis=1, keepdims=True)
    ang = np.degrees(np.arccos(np.clip(np.abs((nn * nrm).sum(1)), 0.0, 1.0)))
    return float(np.median(np.abs(k["pos"][:, 2] - z))), float(np.median(ang))


@pytest.fixture(scope="module")
def quality_scene():
    cfg = synth.config(8, 640, 360, 1)
    P, imgs, seeds = synth.scene_host(cfg)
    return cfg, P, imgs, seeds


def test_fast_refine_quality_vs_ground_truth(orc, quality_scene):
    """Median |z - z_true| of accepted expansion children: performance mode
    below the unrefined children and below the parity mode's Nelder-Mead,
    improving with the iteration count (synth.surface is the ground truth)."""
    cfg, P, imgs, seeds = quality_scene
    S = orc.Scene(P, imgs)
    par = S.seeds_to_patches(seeds[::2][:400])
    acc = S.refine(par, 16, orc.MODE_SEED)
    par = par[acc == 1]
    nk, na = S.expand(par)
    e_nm = _geom_err(cfg, nk, na)[0]
    e = [_geom_err(cfg, *S.fast_expand(par, orc.fast_options(iters=it)))[0] for it in (0, 2, 4)]
    assert e[2] < e[1] < e[0]
    assert e[2] < 0.5 * e_nm


def test_fast_pipeline_improves_normals(orc, quality_scene):
    """Normals (and depths) against the ground truth, along the performance
    mode's own pipeline (dp_densify with dp_fast_options.densify):
      - the seed stage (CG refine at n = 16) takes the raw seed patches'
        camera-facing normals to well under half their error, where the parity
        mode's Nelder-Mead seed stage (initial simplex 0.02 of the depth, 0.2
        rad tilts) makes them worse;
      - expansion children refined at n = 11 from those parents have lower
        normal and far lower depth errors than the parity mode's children of
        the same parents, and more CG iterations lower the normal error."""
    cfg, P, imgs, seeds = quality_scene
    S = orc.Scene(P, imgs, _options(expand_cell_size=11))
    raw = S.seeds_to_patches(seeds[::2][:600])
    _, ang_raw = _geom_err(cfg, raw)
    nm = raw.copy()
    _, ang_nm_seed = _geom_err(cfg, nm[S.refine(nm, 16, orc.MODE_SEED) == 1])
    par = raw.copy()
    par = par[S.fast_refine(par, 16, orc.MODE_FAST_REFINE) == 1]
    assert len(par) > 150
    _, ang_seed = _geom_err(cfg, par)
    assert ang_seed < 0.5 * ang_raw and ang_seed < ang_nm_seed, (ang_seed, ang_raw, ang_nm_seed)
    dz_nm, ang_nm = _geom_err(cfg, *S.expand(par))
    dz4, ang4 = _geom_err(cfg, *S.fast_expand(par, orc.fast_options(iters=4)))
    dz8, ang8 = _geom_err(cfg, *S.fast_expand(par, orc.fast_options(iters=8)))
    assert ang4 < ang_nm and dz4 < 0.2 * dz_nm, (ang4, ang_nm, dz4, dz_nm)
    assert ang8 < ang4


def _options(**kw):
    import densepoints_amd as dp

    return dp.Options(**kw)


def test_fast_init_related_cosine_tests(orc, small_scene):
    """After the refine, InitRelatedImages runs in fp32 with its angle tests as
    squared cosine tests (x > cos(angle) <=> dn > 0 and dn^2 > cos^2 |d|^2 for
    a positive cosine, the cosines from the host libm): the candidate mask
    equals an independent numpy classification at the refined pose, and the
    filtered visible mask is a subset of the views that test visible."""
    import math

    _, P, imgs, seeds = small_scene
    S = orc.Scene(P, imgs)
    p = S.seeds_to_patches(seeds[:60])
    S.fast_refine(p, 7, orc.MODE_FAST_REFINE)
    V = len(imgs)
    cams = [_fcam(orc, P, v) for v in range(V)]
    opts = dp_options()
    cvis, ccand = _f(math.cos(opts.visible_angle)), _f(math.cos(opts.candidate_angle))
    assert cvis > 0 and ccand > 0

    def bits(m):
        return {v for v in range(128) if (int(m[v >> 6]) >> (v & 63)) & 1}

    checked = 0
    for q in p:
        if q["flags"] & 2:  # degenerate
            continue
        X = q["pos"].astype(np.float32)
        n = q["normal"].astype(np.float32)
        vis, cand = set(), set()
        for v in range(V):
            if v == int(q["ref"]):
                continue
            Q, C, _ = cams[v]
            h2 = _qpt(Q, 2, X)
            if not (_f(2.0 ** -20) <= h2 <= _f(2.0 ** 64)):
                continue
            rr = _f(1.0) / h2
            u, w = _qpt(Q, 0, X) * rr, _qpt(Q, 1, X) * rr
            H, W = imgs[v].shape[:2]
            if not (u > 0 and u < _f(32 * W) and w > 0 and w < _f(32 * H)):
                continue
            d = (X - C).astype(np.float32)
            dn, dd = _fdot(n, d), _fdot(d, d)
            if dn > 0 and dn * dn > (cvis * cvis) * dd:
                vis.add(v)
            elif dn > 0 and dn * dn > (ccand * ccand) * dd:
                cand.add(v)
        assert bits(q["cand"]) == cand
        assert bits(q["vis"]) <= vis | {int(q["ref"])}
        checked += 1
    assert checked > 40


def dp_options():
    from densepoints_amd import pmvs

    return pmvs.Options()


@pytest.mark.parametrize("cell", [7, 11, 16])
def test_affine_window_map_error_below_sample_grid(orc, small_scene, cell):
    """The spec samples each (view, pose) through the first-order map of the
    window homography about its centre (or_fast.c fast_sample) instead of the
    projective quotient hx/hz.  On this 320x240 scene (short focal length: the
    strongest perspective of the test scenes), over the patches' visible views
    and CG poses up to 3 scaled units in each axis, the largest sample offset
    stays below 1/2 px, and at the start pose the median window's worst sample
    is within 2.5/32 px (measured: n = 7 / 11 / 16 max 4.9 / 9.0 / 15.6 and
    start-pose median 0.38 / 1.05 / 2.37, in 1/32 px)."""
    _, P, imgs, seeds = small_scene
    S = orc.Scene(P, imgs)
    pats = S.seeds_to_patches(seeds[::3][:60])
    V = len(imgs)
    Pm = P.reshape(V, 3, 4)
    C = np.zeros((V, 3))
    xr = np.zeros((V, 3))
    for v in range(V):
        _, C[v], _, _, xa = orc.view_geometry(P[v])
        xr[v] = xa / np.sqrt(xa @ xa)
    c = 0.5 * (cell - 1)
    tau = np.arange(cell) - c
    ti, tj = np.meshgrid(tau, tau)
    worst, n, start = 0.0, 0, []
    for p in pats:
        ref = int(p["ref"])
        X0, n0 = p["pos"].astype(np.float64), p["normal"].astype(np.float64)

        def proj(v, X):
            h = Pm[v] @ np.append(X, 1.0)
            return np.array([h[0] / h[2], h[1] / h[2]])

        dx = np.linalg.norm(proj(ref, X0 + xr[ref]) - proj(ref, X0))
        nn = n0 / np.linalg.norm(n0)
        e1 = xr[ref] - (xr[ref] @ nn) * nn
        e1 /= np.linalg.norm(e1)
        e2 = np.cross(nn, e1)
        ps, r = 1.0 / dx, X0 - C[ref]
        sd, st = ps / np.linalg.norm(r), 2.0 / (cell - 1)
        vis = [v for v in range(V) if (int(p["vis"][v >> 6]) >> (v & 63)) & 1]
        for v in vis:
            H = [Pm[v] @ np.append(X0, 1.0)] + [Pm[v][:, :3] @ w for w in (r, e1 * ps, e2 * ps, nn * ps)]
            if not H[0][2] > 0:
                continue
            g = [np.array([32.0 * h[0], 32.0 * h[1], h[2]]) / H[0][2] for h in H]
            for x in np.array(np.meshgrid([-3, 0, 3], [-3, 0, 3], [-3, 0, 3])).reshape(3, -1).T:
                A = g[0] + x[0] * sd * g[1]
                B1 = g[2] - x[1] * st * g[4]
                B2 = g[3] - x[2] * st * g[4]
                h = A[:, None, None] + ti * B1[:, None, None] + tj * B2[:, None, None]
                if not (h[2] > 0).all() or not A[2] > 0:
                    continue
                U0 = A[:2] / A[2]
                Ui = (B1[:2] - U0 * B1[2]) / A[2]
                Uj = (B2[:2] - U0 * B2[2]) / A[2]
                aff = U0[:, None, None] + ti * Ui[:, None, None] + tj * Uj[:, None, None]
                e = float(np.abs(aff - h[:2] / h[2]).max())
                worst = max(worst, e)
                if not x.any():
                    start.append(e)
                n += 1
    assert n > 500
    assert worst < 16.0, f"affine map off by {worst:.3f} / 32 px"
    assert np.median(start) < 2.5


def test_generation_engine_densify_all(orc):
    """The oracle's generation-at-a-time densify run to the end equals
    or_densify (parity mode), and in performance mode (dp_fast_options.densify,
    the spec dp_densify follows) stores accepted patches in sequence order."""
    cfg = synth.config(6, 320, 240, 1)
    P, imgs, seeds = synth.scene_host(cfg)
    S = orc.Scene(P, imgs)
    op, ost = S.densify(seeds)
    gp = orc.GenerationEngine(S, threads=8).densify_all(seeds)
    assert len(gp) == ost["patches"] and gp.tobytes() == op.tobytes()
    fp = orc.GenerationEngine(S, threads=8, fast=orc.fast_options(densify=1)).densify_all(seeds)
    assert len(fp) > 20
    assert (fp["seq"] == np.arange(len(fp))).all()
    assert (fp["flags"] & 1).all()


def test_fast_analytic_gradient_quality(orc, quality_scene):
    """Spec v4 (analytic gradient) against v3 (forward differences) on the
    performance pipeline's own parents (the seed stage refined in performance
    mode, as dp_densify runs it), same iterations: lower depth and normal
    errors of the accepted children with fewer evaluations."""
    cfg, P, imgs, seeds = quality_scene
    S = orc.Scene(P, imgs, _options(expand_cell_size=11))
    out = {}
    for gr in (0, 1):
        fo = orc.fast_options(gradient=gr)
        par = S.seeds_to_patches(seeds[::2][:600])
        par = par[S.fast_refine(par, 16, orc.MODE_FAST_REFINE, fo) == 1]
        kids, acc = S.fast_expand(par, fo)
        out[gr] = _geom_err(cfg, kids, acc) + (float(kids["evals"][kids["evals"] > 0].mean()),)
    (dz0, ang0, e0), (dz1, ang1, e1) = out[0], out[1]
    assert dz1 < dz0 and ang1 < ang0 and e1 < 0.75 * e0, out

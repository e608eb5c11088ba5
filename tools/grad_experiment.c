/*
 * Experiment, not the specification and not shipped: the performance mode's
 * CG refine with the ANALYTIC gradient of the continuous objective in place of
 * the three forward differences per iteration, to measure
 * its effect on the refined geometry and on E before any kernel work.
 *
 * The gradient: per sample the bilinear slopes (gx, gy) of the staged fp16
 * tile at the sample's 1/32-px position, times the sample's motion under the
 * pose variables -- the affine window map's derivatives:
 *   d(U0)/d(df) = (A'x - U0 A'z) / Az             (A' = vec[1])
 *   d(Ui)/d(df) = (-U0' B1z - Ui A'z) / Az,  d(Uj)/d(df) likewise with B2
 *   d(Ui)/d(af) = d(Uj)/d(bf) = k_u = (-vec4x + U0 vec4z) / Az
 * so du/d(af) = ti k_u and du/d(bf) = tj k_u -- then NCC's quotient rule over
 * the moment derivatives (anchor and view both move with the pose).  fp64
 * throughout (an experiment of the optimiser, not of the arithmetic).
 *
 * Built by tools/grad_experiment.py together with oracle/oracle.c and
 * oracle/or_seeds.c (this file includes oracle/or_fast.c for its statics).
 */
#include "../oracle/or_fast.c"

static double g_qscale = 0.0; /* > 0: per-sample derivatives rounded to multiples of 1/g_qscale */
static int g_noclamp = 0;     /* 1: tap slopes also across a clamped edge */

/* samples (as fast_sample) and d sample / d(df, af, bf) */
static void sample_grad(const fast_view *t, int cell, fast_pose q, int32_t *out, double (*db)[3])
{
    float A[3], B1[3], B2[3];
    for (int k = 0; k < 3; ++k) {
        A[k] = fmaf(q.df, t->vec[1][k], t->vec[0][k]);
        B1[k] = fmaf(-q.af, t->vec[4][k], t->vec[2][k]);
        B2[k] = fmaf(-q.bf, t->vec[4][k], t->vec[3][k]);
    }
    const float rz = rcp_rn(fmaxf(A[2], FAST_RCP_MIN));
    const float U0 = A[0] * rz, V0 = A[1] * rz;
    const float Ui = fmaf(-U0, B1[2], B1[0]) * rz, Vi = fmaf(-V0, B1[2], B1[1]) * rz;
    const float Uj = fmaf(-U0, B2[2], B2[0]) * rz, Vj = fmaf(-V0, B2[2], B2[1]) * rz;
    const double iz = A[2] > FAST_RCP_MIN ? 1.0 / (double)A[2] : 0.0;
    const double dU0 = ((double)t->vec[1][0] - (double)U0 * t->vec[1][2]) * iz;
    const double dV0 = ((double)t->vec[1][1] - (double)V0 * t->vec[1][2]) * iz;
    const double dUi = (-dU0 * B1[2] - (double)Ui * t->vec[1][2]) * iz;
    const double dVi = (-dV0 * B1[2] - (double)Vi * t->vec[1][2]) * iz;
    const double dUj = (-dU0 * B2[2] - (double)Uj * t->vec[1][2]) * iz;
    const double dVj = (-dV0 * B2[2] - (double)Vj * t->vec[1][2]) * iz;
    const double ku = (-(double)t->vec[4][0] + (double)U0 * t->vec[4][2]) * iz;
    const double kv = (-(double)t->vec[4][1] + (double)V0 * t->vec[4][2]) * iz;
    const float c = 0.5f * (float)(cell - 1);
    for (int j = 0; j < cell; ++j) {
        const float tj = (float)j - c;
        for (int i = 0; i < cell; ++i) {
            const float ti = (float)i - c;
            const float u = fmaf(tj, Uj, fmaf(ti, Ui, U0));
            const float w = fmaf(tj, Vj, fmaf(ti, Vi, V0));
            const float Ub = fminf(fmaxf(u + 0x1p23f, 0x1p23f), 0x1p23f + t->umax);
            const float Vb = fminf(fmaxf(w + 0x1p23f, 0x1p23f), 0x1p23f + t->vmax);
            const int iu = (int)(Ub - 0x1p23f), iv = (int)(Vb - 0x1p23f);
            const int x0 = iu >> 5, fx = iu & 31, y0 = iv >> 5, fy = iv & 31;
            const uint16_t e0 = t->tile[y0 * (t->tw + 1) + x0];
            const uint16_t e1 = t->tile[y0 * (t->tw + 1) + x0 + 1];
            const int p00 = e0 & 255, p10 = e0 >> 8, p01 = e1 & 255, p11 = e1 >> 8;
            out[j * cell + i] = ((32 - fx) * (32 - fy) * p00 + fx * (32 - fy) * p01 + (32 - fx) * fy * p10 +
                                 fx * fy * p11 + 32) >> 6;
            /* slopes per 1/32 px (zero across a clamped edge) */
            const int cu = !g_noclamp && (u + 0x1p23f < 0x1p23f || u > t->umax),
                      cv = !g_noclamp && (w + 0x1p23f < 0x1p23f || w > t->vmax);
            const double gx = cu ? 0.0 : ((32 - fy) * (p01 - p00) + fy * (p11 - p10)) / 64.0;
            const double gy = cv ? 0.0 : ((32 - fx) * (p10 - p00) + fx * (p11 - p01)) / 64.0;
            const double dud = dU0 + ti * dUi + tj * dUj, dvd = dV0 + ti * dVi + tj * dVj;
            const double s = gx * ku + gy * kv;
            db[j * cell + i][0] = gx * dud + gy * dvd;
            db[j * cell + i][1] = ti * s;
            db[j * cell + i][2] = tj * s;
            if (g_qscale > 0.0)
                for (int p = 0; p < 3; ++p) db[j * cell + i][p] = rint(db[j * cell + i][p] * g_qscale) / g_qscale;
        }
    }
}

/* g = dF/dx of F = sum_k (1 - NCC_k) (NCC units per scaled pose unit) */
static void fast_grad(const fast_patch *fp, int cell, double ncc_denom_min, const float x[3], double g[3])
{
    const fast_pose q = pose_of(fp, x);
    const int m = fp->m, N = cell * cell;
    int32_t a[256], b[256];
    double da[256][3], dbv[256][3];
    sample_grad(&fp->fv[0], cell, q, a, da);
    double Sa = 0, Saa = 0, Da[3] = {0, 0, 0}, Daa[3] = {0, 0, 0};
    for (int i = 0; i < N; ++i) {
        Sa += a[i];
        Saa += (double)a[i] * a[i];
        for (int p = 0; p < 3; ++p) {
            Da[p] += da[i][p];
            Daa[p] += a[i] * da[i][p];
        }
    }
    const double dmin = ncc_denom_min * 256.0 * (double)N * (double)N;
    double dF[3] = {0, 0, 0};
    for (int k = 1; k < m; ++k) {
        sample_grad(&fp->fv[k], cell, q, b, dbv);
        double Sb = 0, Sbb = 0, Sab = 0, Db[3] = {0, 0, 0}, Dbb[3] = {0, 0, 0}, Dab[3] = {0, 0, 0};
        for (int i = 0; i < N; ++i) {
            Sb += b[i];
            Sbb += (double)b[i] * b[i];
            Sab += (double)a[i] * b[i];
            for (int p = 0; p < 3; ++p) {
                Db[p] += dbv[i][p];
                Dbb[p] += b[i] * dbv[i][p];
                Dab[p] += da[i][p] * b[i] + a[i] * dbv[i][p];
            }
        }
        const double num = N * Sab - Sa * Sb, va = N * Saa - Sa * Sa, vb = N * Sbb - Sb * Sb;
        const double den = sqrt(va * vb);
        for (int p = 0; p < 3; ++p) {
            const double dnum = N * Dab[p] - Da[p] * Sb - Sa * Db[p];
            double dncc;
            if (den > dmin && va > 0 && vb > 0) {
                const double dva = 2.0 * (N * Daa[p] - Sa * Da[p]), dvb = 2.0 * (N * Dbb[p] - Sb * Db[p]);
                dncc = dnum / den - (num / den) * 0.5 * (dva / va + dvb / vb);
            } else {
                dncc = dnum / dmin;
            }
            dF[p] -= dncc;
        }
    }
    g[0] = dF[0] * fp->sd;
    g[1] = dF[1] * fp->st;
    g[2] = dF[2] * fp->st;
}

static long g_grad_evals, g_probe_evals;

/* fast_cg with the analytic gradient; E counts probes + gradient evaluations */
static int fast_cg_an(const fast_patch *fp, int cell, double dmin0, const or_fast_options *fo, float x[3])
{
    x[0] = x[1] = x[2] = 0.0f;
    int32_t f = fast_objective(fp, cell, dmin0, pose_of(fp, x), NULL);
    int E = 1, Eg = 0;
    float alpha = fo->ls_step;
    float gp[3] = {0, 0, 0}, dp[3] = {0, 0, 0}, ggp = 0.0f;
    int moved = 1;
    for (int it = 0; it < fo->iters; ++it) {
        float g[3];
        if (moved) {
            double gd[3];
            fast_grad(fp, cell, dmin0, x, gd);
            for (int i = 0; i < 3; ++i) g[i] = (float)gd[i];
            ++Eg;
        } else {
            for (int i = 0; i < 3; ++i) g[i] = gp[i];
        }
        const float gg = fdot(g, g);
        if (gg == 0.0f) break;
        float beta = 0.0f;
        if (it > 0 && ggp > 0.0f) {
            const float dg[3] = {g[0] - gp[0], g[1] - gp[1], g[2] - gp[2]};
            beta = fdot(g, dg) * rcp_rn(ggp);
            beta = beta > 0.0f ? beta : 0.0f;
        }
        float d[3];
        for (int i = 0; i < 3; ++i) d[i] = fmaf(beta, dp[i], -g[i]);
        if (fdot(d, g) >= 0.0f)
            for (int i = 0; i < 3; ++i) d[i] = -g[i];
        const float inv_nd = 1.0f / sqrtf(fdot(d, d));
        float u[3], x1[3], x2[3];
        for (int i = 0; i < 3; ++i) u[i] = d[i] * inv_nd;
        for (int i = 0; i < 3; ++i) x1[i] = fmaf(alpha, u[i], x[i]);
        const int32_t f1 = fast_objective(fp, cell, dmin0, pose_of(fp, x1), NULL);
        moved = 1;
        if (f1 < f) {
            const float a2 = 2.0f * alpha;
            for (int i = 0; i < 3; ++i) x2[i] = fmaf(a2, u[i], x[i]);
            const int32_t f2 = fast_objective(fp, cell, dmin0, pose_of(fp, x2), NULL);
            if (f2 < f1) {
                memcpy(x, x2, sizeof(x2));
                f = f2;
                alpha = a2;
            } else {
                memcpy(x, x1, sizeof(x1));
                f = f1;
            }
        } else {
            const float a2 = 0.5f * alpha;
            for (int i = 0; i < 3; ++i) x2[i] = fmaf(a2, u[i], x[i]);
            const int32_t f2 = fast_objective(fp, cell, dmin0, pose_of(fp, x2), NULL);
            if (f2 < f) {
                memcpy(x, x2, sizeof(x2));
                f = f2;
            } else {
                moved = 0;
            }
            alpha = a2;
        }
        E += 2;
        for (int i = 0; i < 3; ++i) {
            gp[i] = g[i];
            dp[i] = d[i];
        }
        ggp = gg;
    }
#pragma omp atomic
    g_grad_evals += Eg;
#pragma omp atomic
    g_probe_evals += E;
    return E + Eg;
}

static int refine_one_an(const or_scene *s, or_patch *p, int cell, const or_fast_options *fo)
{
    fast_patch fp;
    fast_stage(s, p, cell, fo, fo->margin < 7 ? fo->margin : 7, &fp);
    if (fp.degenerate) {
        p->flags |= OR_FLAG_DEGENERATE;
        p->flags &= (uint8_t)~OR_FLAG_ACCEPTED;
        p->score = -1.0f;
        return 0;
    }
    if (fp.m >= 2) {
        float x[3];
        p->evals += (uint32_t)fast_cg_an(&fp, cell, s->opt.ncc_denom_min, fo, x);
        const float d = x[0] * fp.sd, a = x[1] * fp.st, b = x[2] * fp.st;
        float nrm[3];
        for (int k = 0; k < 3; ++k) nrm[k] = fmaf(b, fp.u2[k], fmaf(a, fp.u1[k], fp.un[k]));
        const float il = 1.0f / sqrtf(fdot(nrm, nrm));
        for (int k = 0; k < 3; ++k) {
            p->pos[k] = fmaf(d, fp.r[k], fp.X0[k]);
            p->normal[k] = nrm[k] * il;
        }
    }
    fast_free(&fp);
    fast_init_related(s, p);
    int ok = fast_filter(s, p, cell, fo);
    if (ok) p->flags |= OR_FLAG_ACCEPTED;
    else p->flags &= (uint8_t)~OR_FLAG_ACCEPTED;
    return ok;
}

/* or_fast_expand_batch with refine_one_an; stats[0..1] = gradient / probe evaluations */
void exp_set(double qscale, int noclamp)
{
    g_qscale = qscale;
    g_noclamp = noclamp;
}

int exp_fast_expand_batch_an(const or_scene *s, const or_patch *parents, int n, const or_fast_options *fo,
                             or_patch *children, uint8_t *acc, long *stats)
{
    const int cell = s->opt.expand_cell_size;
    g_grad_evals = g_probe_evals = 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int i = 0; i < n; ++i) {
        int vis[OR_MAX_VIEWS];
        const or_patch *par = &parents[i];
        const int live = decode_mask(par->vis, vis) >= s->opt.min_expand_visible;
        double pos[4][3];
        if (live) or_child_positions(s, par, pos);
        for (int dd = 0; dd < 4; ++dd) {
            or_patch c = *par;
            c.evals = 0;
            c.flags = 0;
            c.parent = (uint32_t)i;
            int ok = 0;
            if (live) {
                for (int k = 0; k < 3; ++k) c.pos[k] = (float)pos[dd][k];
                ok = refine_one_an(s, &c, cell, fo);
            }
            children[4 * i + dd] = c;
            acc[4 * i + dd] = (uint8_t)(ok > 0);
        }
    }
    stats[0] = g_grad_evals;
    stats[1] = g_probe_evals;
    return 0;
}

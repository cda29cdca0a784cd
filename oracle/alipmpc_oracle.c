/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  CPU (C, fp64) restatement of the reference ALIP-MPC-CBF NLP and
 * of the interior-point solve that stands in for cyipopt/IPOPT.  Mirrors oracle/np_oracle.py line by
 * line (same formulas, same algorithm and constants) so that the numpy and C restatements check each
 * other, and so that the CPU baseline in bench.py runs the same algorithm as the HIP kernels.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so, and only
 * as the checker / reported baseline.  libalipmpc.so (the product) never links or calls it.
 *
 * Reference anchors (file:line in /root/reference):
 *   constants A, B, W, M_A, M_B, dx_du, dP_du    MPC_LIP_modi.py:14-87   (generalised to any N)
 *   select_obs                                   MPC_LIP_modi.py:325-338
 *   cl/cu (leg parity) + detour goal             MPC_LIP_modi.py:197-271; MPC_LIP_sig_step.py:184-254
 *   objective / gradient                         MPC_LIP_modi.py:430-465, 645-655
 *   constraints / jacobian                       MPC_LIP_modi.py:468-583, 586-643
 *   rollout, p_list[0]                           MPC_LIP_modi.py:102-112, 630-634
 *   solver: IPOPT (3rd party via cyipopt, version unpinned; MPC_LIP_modi.py:274-296) — restated as a
 *   primal-dual interior point with IPOPT's defaults (monotone mu, fraction-to-boundary, inertia
 *   correction, filter line search) and a slack-reset restoration substitute.  See DESIGN.md.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/alipmpc.h"

#define OMAXN 8
#define OMAXV (5 * OMAXN)
#define OMAXO ALIPMPC_MAX_OBS
#define OMAXM (OMAXN * (6 + OMAXO))

typedef struct {
    int N, n;
    double beta;
    double A[5][5], B[5][3], W[3][5], MA[5][5], MB[5][5];
    double Phi[OMAXN + 1][5][OMAXV]; /* d x_k / du */
    double Psi[OMAXN][3][OMAXV];     /* d p_k / du */
    /* foothold parametrisation (W B = I): u(p) = [A^k x0]_k + U p, U block lower-triangular A^{k-1-j} B */
    double Ak[OMAXN + 1][5][5];
    double U[OMAXV][3 * OMAXN];
} oconsts;

typedef struct {
    const alipmpc_cfg* cfg;
    const oconsts* K;
    int N, n, m, rpk, nc, ne, modi;
    int split;   /* solver-internal: f_en row replaced by the two smooth rows vbx +- s dth <= bvx_hi */
    int dd;      /* DD (unicycle) instance: x0[0..2] = (px, py, th), decision u = (v, w) x N */
    double last_u[2];
    double x0[5], goal[2], goal_orig[2];
    double cir[OMAXO][3], elp[OMAXO][5];
    double eqa[OMAXO], eqb[OMAXO], eqc[OMAXO], ek[OMAXO];
    int sel_c[OMAXO], sel_e[OMAXO];
    double cl[OMAXM], cu[OMAXM];
    double df;   /* IPOPT's gradient-based objective scaling of the solve (osolve; 1 for the callbacks) */
} oprob;

/* ------------------------------------------------------------------------------------------------ */
int oracle_default_cfg(int32_t variant, int32_t N, alipmpc_cfg* c)
{
    memset(c, 0, sizeof(*c));
    c->N = N;
    c->nc_max = 6;
    c->ne_max = 6;
    c->variant = variant;
    /* the reference's IPOPT caps: MPC_LIP_modi.py:287, MPC_LIP_sig_step.py:269, MPC_DD_sig_step.py:183 */
    c->max_iter = variant == ALIPMPC_VARIANT_SIG_STEP ? 20 : variant == ALIPMPC_VARIANT_DD ? 40 : 30;
    c->precision = 0;
    c->select_obs = 1;
    c->detour = 1;
    c->tol = 1e-8;
    c->acceptable_tol = 1e-6;
    c->dt = 0.4;
    c->H = 1.0;
    c->g = 9.81;
    c->leg2_max = 0.09;
    c->bvx_lo = 0.4;
    c->bvx_hi = 0.8;
    c->bvy_lo = 0.15;
    c->bvy_hi = 0.35;
    c->dtheta_max = M_PI / 16;
    c->q = 1.0;
    c->p = 0.0;
    c->r = 50.0;
    c->gamma = 0.2;
    c->s = 0.024 * 180 / M_PI;
    c->detect_r2 = 16.0;
    c->dd_t = 2.0;
    c->mu_init = 0.1;
    if (variant == ALIPMPC_VARIANT_SIG_STEP) {
        c->bvy_hi = 0.30;
        c->p = 2.0;
        c->r = 15.0;
        c->gamma = 0.4;
        c->s = 0.014 * 180 / M_PI;
        c->select_obs = 0;
    } else if (variant == ALIPMPC_VARIANT_DD) {
        c->select_obs = 0;
        c->detour = 0;
    }
    return 0;
}

static void mm55(double a[5][5], double b[5][5], double out[5][5])
{
    double t[5][5];
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            double s = 0;
            for (int k = 0; k < 5; ++k) s += a[i][k] * b[k][j];
            t[i][j] = s;
        }
    memcpy(out, t, sizeof(t));
}

void oracle_consts(const alipmpc_cfg* cfg, oconsts* K)
{
    memset(K, 0, sizeof(*K));
    double b = sqrt(cfg->g / cfg->H), T = cfg->dt;
    double ch = cosh(b * T), sh = sinh(b * T);
    K->beta = b;
    K->N = cfg->N;
    K->n = 5 * cfg->N;
    double A[5][5] = {{ch, 0, sh / b, 0, 0}, {0, ch, 0, sh / b, 0}, {sh * b, 0, ch, 0, 0}, {0, sh * b, 0, ch, 0}, {0, 0, 0, 0, 1}};
    double B[5][3] = {{1 - ch, 0, 0}, {0, 1 - ch, 0}, {-sh * b, 0, 0}, {0, -sh * b, 0}, {0, 0, 1}};
    double a_ = 5.0, b_ = 1.0;
    double D = a_ * (ch - 1) * (ch - 1) + b_ * (sh * b) * (sh * b);
    double Ch = -a_ * (ch - 1) / D, Sh = -b_ * sh * b / D;
    double W[3][5] = {{Ch, 0, Sh, 0, 0}, {0, Ch, 0, Sh, 0}, {0, 0, 0, 0, 1}};
    memcpy(K->A, A, sizeof(A));
    memcpy(K->B, B, sizeof(B));
    memcpy(K->W, W, sizeof(W));
    double BW[5][5];
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += B[i][k] * W[k][j];
            BW[i][j] = s;
        }
    double BWA[5][5];
    mm55(BW, K->A, BWA);
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            K->MA[i][j] = A[i][j] - BWA[i][j];
            K->MB[i][j] = BW[i][j];
        }
    int n = K->n;
    for (int k = 1; k <= cfg->N; ++k) {
        for (int i = 0; i < 5; ++i)
            for (int j = 0; j < n; ++j) {
                double s = 0;
                for (int t = 0; t < 5; ++t) s += K->MA[i][t] * K->Phi[k - 1][t][j];
                K->Phi[k][i][j] = s;
            }
        for (int i = 0; i < 5; ++i)
            for (int j = 0; j < 5; ++j) K->Phi[k][i][5 * (k - 1) + j] += K->MB[i][j];
    }
    for (int i = 0; i < 5; ++i) K->Ak[0][i][i] = 1.0;
    for (int k = 1; k <= cfg->N; ++k) mm55(K->A, K->Ak[k - 1], K->Ak[k]);
    for (int k = 1; k <= cfg->N; ++k)
        for (int j = 0; j < k; ++j)
            for (int a = 0; a < 5; ++a)
                for (int c = 0; c < 3; ++c) {
                    double acc = 0;
                    for (int t = 0; t < 5; ++t) acc += K->Ak[k - 1 - j][a][t] * K->B[t][c];
                    K->U[5 * (k - 1) + a][3 * j + c] = acc;
                }
    for (int k = 0; k < cfg->N; ++k) {
        double WA[3][5];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 5; ++j) {
                double s = 0;
                for (int t = 0; t < 5; ++t) s += W[i][t] * A[t][j];
                WA[i][j] = s;
            }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < n; ++j) {
                double s = 0;
                for (int t = 0; t < 5; ++t) s += WA[i][t] * K->Phi[k][t][j];
                K->Psi[k][i][j] = -s;
            }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 5; ++j) K->Psi[k][i][5 * k + j] += W[i][j];
    }
}

/* ------------------------------------------------------------------------------------------------ */
/* set-up: select_obs, detour goal, cl/cu (compact reference row order) */
static void oprob_init(oprob* P, const alipmpc_cfg* cfg, const oconsts* K, const double* x0, const double* goal,
                       int leg, const double* cir, int nc, const double* elp, int ne, int split)
{
    memset(P, 0, sizeof(*P));
    P->cfg = cfg;
    P->K = K;
    P->N = cfg->N;
    P->n = 5 * cfg->N;
    P->modi = cfg->variant == ALIPMPC_VARIANT_MODI;
    P->split = split && P->modi;
    P->df = 1.0;
    memcpy(P->x0, x0, 5 * sizeof(double));
    P->goal_orig[0] = goal[0];
    P->goal_orig[1] = goal[1];
    for (int j = 0; j < nc; ++j) {
        const double* c = cir + 3 * j;
        double d = (x0[0] - c[0]) * (x0[0] - c[0]) + (x0[1] - c[1]) * (x0[1] - c[1]) - c[2] * c[2];
        if (!cfg->select_obs || d <= cfg->detect_r2) {
            memcpy(P->cir[P->nc], c, 3 * sizeof(double));
            P->sel_c[P->nc++] = j;
        }
    }
    for (int j = 0; j < ne; ++j) {
        const double* e = elp + 5 * j;
        double r = e[2] > e[3] ? e[2] : e[3];
        double d = (x0[0] - e[0]) * (x0[0] - e[0]) + (x0[1] - e[1]) * (x0[1] - e[1]) - r * r;
        if (!cfg->select_obs || d <= cfg->detect_r2) {
            memcpy(P->elp[P->ne], e, 5 * sizeof(double));
            P->sel_e[P->ne++] = j;
        }
    }
    for (int j = 0; j < P->ne; ++j) {
        const double* e = P->elp[j];
        double ce = cos(e[4]), se = sin(e[4]);
        P->eqa[j] = (e[3] * ce) * (e[3] * ce) + (e[2] * se) * (e[2] * se);
        P->eqb[j] = 2 * ce * se * (e[3] * e[3] - e[2] * e[2]);
        P->eqc[j] = (e[3] * se) * (e[3] * se) + (e[2] * ce) * (e[2] * ce);
        P->ek[j] = (e[3] * e[2]) * (e[3] * e[2]);
    }
    /* detour goal (MPC_LIP_modi.py:247-271) */
    P->goal[0] = goal[0];
    P->goal[1] = goal[1];
    if (cfg->detour) {
        for (int j = 0; j < P->nc; ++j) {
            const double* c = P->cir[j];
            double cen = (x0[0] - c[0]) * (x0[0] - c[0]) + (x0[1] - c[1]) * (x0[1] - c[1]);
            double gd = (x0[0] - goal[0]) * (x0[0] - goal[0]) + (x0[1] - goal[1]) * (x0[1] - goal[1]);
            if (cen < gd && cen < 9 * c[2] * c[2]) {
                double th = atan2(goal[1] - x0[1], goal[0] - x0[0]);
                double al = atan2(c[1] - x0[1], c[0] - x0[0]);
                double d = th - al;
                if (d < 0 && fabs(d) > M_PI)
                    d += 2 * M_PI;
                else if (d > 0 && fabs(d) > M_PI)
                    d -= 2 * M_PI;
                if (fabs(d) < M_PI / 12) {
                    double na = d < 0 ? th - M_PI / 12 : th + M_PI / 12;
                    double rr = sqrt(gd);
                    P->goal[0] = x0[0] + rr * cos(na);
                    P->goal[1] = x0[1] + rr * sin(na);
                    break;
                }
            }
        }
    }
    /* cl / cu (MPC_LIP_modi.py:205-245) */
    P->rpk = 4 + P->nc + P->ne + P->modi + P->split;
    P->m = P->N * P->rpk;
    int r = 0;
    for (int k = 0; k < P->N; ++k) {
        int pos_side = (leg > 0) == (k % 2 == 0);
        double vlo = pos_side ? cfg->bvy_lo : -cfg->bvy_hi;
        double vhi = pos_side ? cfg->bvy_hi : -cfg->bvy_lo;
        P->cl[r] = cfg->bvx_lo;
        P->cu[r++] = cfg->bvx_hi;
        P->cl[r] = vlo;
        P->cu[r++] = vhi;
        for (int j = 0; j < P->nc + P->ne; ++j) {
            P->cl[r] = 0.0;
            P->cu[r++] = INFINITY;
        }
        P->cl[r] = 0.0;
        P->cu[r++] = cfg->leg2_max;
        P->cl[r] = -cfg->dtheta_max;
        P->cu[r++] = cfg->dtheta_max;
        if (P->split) {
            /* |x| <= c  <=>  x <= c and -x <= c; the f_en lower bound is implied by the vbx row (s > 0) */
            P->cl[r] = -INFINITY;
            P->cu[r++] = cfg->bvx_hi;
            P->cl[r] = -INFINITY;
            P->cu[r++] = cfg->bvx_hi;
        } else if (P->modi) {
            P->cl[r] = cfg->bvx_lo;
            P->cu[r++] = cfg->bvx_hi;
        }
    }
}

/* rollout x_{i+1} = M_A x_i + M_B u_i, p_i = W(u_i - A x_i) */
static void rollout(const oprob* P, const double* u, double X[][5], double Pp[][3])
{
    const oconsts* K = P->K;
    memcpy(X[0], P->x0, 5 * sizeof(double));
    for (int i = 0; i < P->N; ++i) {
        const double* ui = u + 5 * i;
        double Ax[5];
        for (int a = 0; a < 5; ++a) {
            double s = 0;
            for (int b = 0; b < 5; ++b) s += K->A[a][b] * X[i][b];
            Ax[a] = s;
        }
        for (int a = 0; a < 3; ++a) {
            double s = 0;
            for (int b = 0; b < 5; ++b) s += K->W[a][b] * (ui[b] - Ax[b]);
            Pp[i][a] = s;
        }
        for (int a = 0; a < 5; ++a) {
            double s = 0;
            for (int b = 0; b < 5; ++b) s += K->MA[a][b] * X[i][b];
            double t = 0;
            for (int b = 0; b < 5; ++b) t += K->MB[a][b] * ui[b];
            X[i + 1][a] = s + t;
        }
    }
}

static void oabs(const oprob* P, double x, double* v, double* d1, double* d2)
{
    (void)P;   /* |x| with the reference's derivative sign(x) (MPC_LIP_modi.py:637-643) */
    *v = fabs(x);
    *d1 = x == 0 ? 0.0 : copysign(1.0, x);
    *d2 = 0.0;
}

static double h_obs(const oprob* P, int j, double px, double py)
{
    if (j < P->nc) {
        const double* c = P->cir[j];
        return (px - c[0]) * (px - c[0]) + (py - c[1]) * (py - c[1]) - c[2] * c[2];
    }
    int e = j - P->nc;
    double dx = px - P->elp[e][0], dy = py - P->elp[e][1];
    return P->eqa[e] * dx * dx + P->eqb[e] * dx * dy + P->eqc[e] * dy * dy - P->ek[e];
}

static void dh_obs(const oprob* P, int j, double px, double py, double* g0, double* g1)
{
    if (j < P->nc) {
        *g0 = 2 * (px - P->cir[j][0]);
        *g1 = 2 * (py - P->cir[j][1]);
        return;
    }
    int e = j - P->nc;
    double dx = px - P->elp[e][0], dy = py - P->elp[e][1];
    *g0 = 2 * P->eqa[e] * dx + P->eqb[e] * dy;
    *g1 = 2 * P->eqc[e] * dy + P->eqb[e] * dx;
}

double oracle_objective(const oprob* P, const double* u)
{
    const alipmpc_cfg* c = P->cfg;
    double X[OMAXN + 1][5], Pp[OMAXN][3];
    rollout(P, u, X, Pp);
    double f = 0;
    for (int k = 1; k <= P->N; ++k) {
        double dx = X[k][0] - P->goal[0], dy = X[k][1] - P->goal[1];
        double tar = atan2(P->goal[1] - X[k][1], P->goal[0] - X[k][0]);
        f += c->q * (dx * dx + dy * dy) + c->r * (X[k][4] - tar) * (X[k][4] - tar);
    }
    double dx = X[1][0] - P->goal[0], dy = X[1][1] - P->goal[1];
    f += c->p * (dx * dx + dy * dy);
    return f;
}

static void gradient(const oprob* P, const double* u, double* g)
{
    const alipmpc_cfg* c = P->cfg;
    const oconsts* K = P->K;
    double X[OMAXN + 1][5], Pp[OMAXN][3];
    rollout(P, u, X, Pp);
    int n = P->n;
    for (int j = 0; j < n; ++j) g[j] = 0;
    for (int k = 1; k <= P->N; ++k) {
        double w = c->q + (k == 1 ? c->p : 0.0);
        double ex = X[k][0] - P->goal[0], ey = X[k][1] - P->goal[1];
        double dxg = P->goal[0] - X[k][0], dyg = P->goal[1] - X[k][1];
        double rho2 = dxg * dxg + dyg * dyg;
        double phi = X[k][4] - atan2(dyg, dxg);
        for (int j = 0; j < n; ++j) {
            /* (p = goal exactly: the target heading's derivatives are 0 instead of 0 / 0) */
            double dtar = rho2 > 0.0 ? (dxg * (-K->Phi[k][1][j]) - dyg * (-K->Phi[k][0][j])) / rho2 : 0.0;
            g[j] += 2 * w * (ex * K->Phi[k][0][j] + ey * K->Phi[k][1][j]) + 2 * c->r * phi * (K->Phi[k][4][j] - dtar);
        }
    }
}

static void constraints(const oprob* P, const double* u, double* out)
{
    const alipmpc_cfg* c = P->cfg;
    double X[OMAXN + 1][5], Pp[OMAXN][3];
    rollout(P, u, X, Pp);
    double gm1 = c->gamma - 1.0;
    int r = 0;
    for (int i = 0; i < P->N; ++i) {
        double th = X[i + 1][4], ct = cos(th), st = sin(th);
        double vbx = ct * X[i + 1][2] + st * X[i + 1][3];
        double vby = -st * X[i + 1][2] + ct * X[i + 1][3];
        out[r++] = vbx;
        out[r++] = vby;
        for (int j = 0; j < P->nc + P->ne; ++j) out[r++] = h_obs(P, j, X[i + 1][0], X[i + 1][1]) + gm1 * h_obs(P, j, X[i][0], X[i][1]);
        out[r++] = (X[i][0] - Pp[i][0]) * (X[i][0] - Pp[i][0]) + (X[i][1] - Pp[i][1]) * (X[i][1] - Pp[i][1]);
        out[r++] = Pp[i][2];
        if (P->split) {
            out[r++] = vbx + c->s * Pp[i][2];
            out[r++] = vbx - c->s * Pp[i][2];
        } else if (P->modi) {
            double a, d1, d2;
            oabs(P, Pp[i][2], &a, &d1, &d2);
            out[r++] = c->s * a + vbx;
        }
    }
}

static void jacobian(const oprob* P, const double* u, double* J /* m x n */)
{
    const alipmpc_cfg* c = P->cfg;
    const oconsts* K = P->K;
    double X[OMAXN + 1][5], Pp[OMAXN][3];
    rollout(P, u, X, Pp);
    int n = P->n;
    double gm1 = c->gamma - 1.0;
    int r = 0;
    for (int i = 0; i < P->N; ++i) {
        const double(*F)[OMAXV] = K->Phi[i + 1];
        const double(*F0)[OMAXV] = K->Phi[i];
        const double(*Ps)[OMAXV] = K->Psi[i];
        double th = X[i + 1][4], vx = X[i + 1][2], vy = X[i + 1][3], ct = cos(th), st = sin(th);
        double a3 = -st * vx + ct * vy, b3 = -ct * vx - st * vy;
        double* rbx = J + (size_t)r * n;
        for (int j = 0; j < n; ++j) rbx[j] = ct * F[2][j] + st * F[3][j] + a3 * F[4][j];
        r++;
        for (int j = 0; j < n; ++j) J[(size_t)r * n + j] = -st * F[2][j] + ct * F[3][j] + b3 * F[4][j];
        r++;
        for (int o = 0; o < P->nc + P->ne; ++o) {
            double g0, g1, h0, h1;
            dh_obs(P, o, X[i + 1][0], X[i + 1][1], &g0, &g1);
            dh_obs(P, o, X[i][0], X[i][1], &h0, &h1);
            for (int j = 0; j < n; ++j) J[(size_t)r * n + j] = g0 * F[0][j] + g1 * F[1][j] + gm1 * (h0 * F0[0][j] + h1 * F0[1][j]);
            r++;
        }
        double ex = X[i][0] - Pp[i][0], ey = X[i][1] - Pp[i][1];
        for (int j = 0; j < n; ++j) J[(size_t)r * n + j] = 2 * ex * (F0[0][j] - Ps[0][j]) + 2 * ey * (F0[1][j] - Ps[1][j]);
        r++;
        for (int j = 0; j < n; ++j) J[(size_t)r * n + j] = Ps[2][j];
        r++;
        if (P->split) {
            for (int j = 0; j < n; ++j) J[(size_t)r * n + j] = rbx[j] + c->s * Ps[2][j];
            r++;
            for (int j = 0; j < n; ++j) J[(size_t)r * n + j] = rbx[j] - c->s * Ps[2][j];
            r++;
        } else if (P->modi) {
            double a, d1, d2;
            oabs(P, Pp[i][2], &a, &d1, &d2);
            for (int j = 0; j < n; ++j) J[(size_t)r * n + j] = c->s * d1 * Ps[2][j] + rbx[j];
            r++;
        }
    }
}

/* exact Hessian of L = of f - y^T c (of = 0: the restoration phase's constraint part) */
static void hessian_of(const oprob* P, const double* u, const double* y, double of, double* H /* n x n */)
{
    const alipmpc_cfg* c = P->cfg;
    const oconsts* K = P->K;
    double X[OMAXN + 1][5], Pp[OMAXN][3];
    rollout(P, u, X, Pp);
    int n = P->n, N = P->N;
    double Hl[OMAXN + 1][5][5];
    memset(Hl, 0, sizeof(Hl));
    for (int i = 0; i < n * n; ++i) H[i] = 0;
    for (int k = 1; k <= N && of != 0.0; ++k) {
        double w = c->q + (k == 1 ? c->p : 0.0);
        Hl[k][0][0] += 2 * w;
        Hl[k][1][1] += 2 * w;
        double dxg = P->goal[0] - X[k][0], dyg = P->goal[1] - X[k][1];
        double rho2 = dxg * dxg + dyg * dyg;
        double phi = X[k][4] - atan2(dyg, dxg);
        double gp[3] = {rho2 > 0.0 ? -dyg / rho2 : 0.0, rho2 > 0.0 ? dxg / rho2 : 0.0, 1.0};   /* (§2 item 7) */
        int idx[3] = {0, 1, 4};
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) Hl[k][idx[a]][idx[b]] += 2 * c->r * gp[a] * gp[b];
        double r4 = rho2 * rho2;
        double h00 = rho2 > 0.0 ? 2 * dxg * dyg / r4 : 0.0, h01 = rho2 > 0.0 ? (dyg * dyg - dxg * dxg) / r4 : 0.0,
               h11 = rho2 > 0.0 ? -2 * dxg * dyg / r4 : 0.0;
        Hl[k][0][0] += 2 * c->r * phi * (-h00);
        Hl[k][0][1] += 2 * c->r * phi * (-h01);
        Hl[k][1][0] += 2 * c->r * phi * (-h01);
        Hl[k][1][1] += 2 * c->r * phi * (-h11);
    }
    int nob = P->nc + P->ne;
    double gm1 = c->gamma - 1.0;
    for (int i = 0; i < N; ++i) {
        const double* yk = y + i * P->rpk;
        double th = X[i + 1][4], vx = X[i + 1][2], vy = X[i + 1][3], ct = cos(th), st = sin(th);
        double vbx = ct * vx + st * vy, vby = -st * vx + ct * vy;
        double wbx = yk[0] + (P->split ? yk[P->rpk - 2] + yk[P->rpk - 1] : P->modi ? yk[P->rpk - 1] : 0.0), wby = yk[1];
        double hvx = -wbx * (-st) - wby * (-ct);
        double hvy = -wbx * ct - wby * (-st);
        Hl[i + 1][2][4] += hvx;
        Hl[i + 1][4][2] += hvx;
        Hl[i + 1][3][4] += hvy;
        Hl[i + 1][4][3] += hvy;
        Hl[i + 1][4][4] += -wbx * (-vbx) - wby * (-vby);
        for (int o = 0; o < nob; ++o) {
            double wj = yk[2 + o];
            double q00, q01, q11;
            if (o < P->nc) {
                q00 = 2;
                q01 = 0;
                q11 = 2;
            } else {
                int e = o - P->nc;
                q00 = 2 * P->eqa[e];
                q01 = P->eqb[e];
                q11 = 2 * P->eqc[e];
            }
            Hl[i + 1][0][0] += -wj * q00;
            Hl[i + 1][0][1] += -wj * q01;
            Hl[i + 1][1][0] += -wj * q01;
            Hl[i + 1][1][1] += -wj * q11;
            if (i >= 1) {
                Hl[i][0][0] += -wj * gm1 * q00;
                Hl[i][0][1] += -wj * gm1 * q01;
                Hl[i][1][0] += -wj * gm1 * q01;
                Hl[i][1][1] += -wj * gm1 * q11;
            }
        }
        double wl = yk[2 + nob];
        for (int a = 0; a < n; ++a) {
            double e0a = K->Phi[i][0][a] - K->Psi[i][0][a], e1a = K->Phi[i][1][a] - K->Psi[i][1][a];
            for (int b = 0; b < n; ++b) {
                double e0b = K->Phi[i][0][b] - K->Psi[i][0][b], e1b = K->Phi[i][1][b] - K->Psi[i][1][b];
                H[a * n + b] += -wl * 2 * (e0a * e0b + e1a * e1b);
            }
        }
        if (P->modi && !P->split) {
            double av, d1, d2;
            oabs(P, Pp[i][2], &av, &d1, &d2);
            if (d2 != 0.0) {
                double w = -yk[P->rpk - 1] * c->s * d2;
                for (int a = 0; a < n; ++a)
                    for (int b = 0; b < n; ++b) H[a * n + b] += w * K->Psi[i][2][a] * K->Psi[i][2][b];
            }
        }
    }
    for (int k = 1; k <= N; ++k) {
        double T[5][OMAXV];
        for (int a = 0; a < 5; ++a)
            for (int j = 0; j < n; ++j) {
                double s = 0;
                for (int b = 0; b < 5; ++b) s += Hl[k][a][b] * K->Phi[k][b][j];
                T[a][j] = s;
            }
        for (int a = 0; a < n; ++a)
            for (int b = 0; b < n; ++b) {
                double s = 0;
                for (int t = 0; t < 5; ++t) s += K->Phi[k][t][a] * T[t][b];
                H[a * n + b] += s;
            }
    }
}
static void hessian(const oprob* P, const double* u, const double* y, double* H) { hessian_of(P, u, y, 1.0, H); }

/* ------------------------------------------------------------------------------------------------ */
static int chol(double* A, int n)
{
    for (int j = 0; j < n; ++j) {
        double d = A[j * n + j];
        for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
        if (!(d > 0)) return 0;
        d = sqrt(d);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = A[i * n + j];
            for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = s / d;
        }
    }
    return 1;
}

static void cholsolve(const double* L, int n, double* b)
{
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * b[k];
        b[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * b[k];
        b[i] = s / L[i * n + i];
    }
}

static void push_slacks(const double* c, const double* cl, const double* cu, int m, double* s)
{
    for (int i = 0; i < m; ++i) {
        int hl = isfinite(cl[i]), hu = isfinite(cu[i]);
        double v = c[i];
        double pl = 0, pu = 0;
        if (hl) pl = fmin(1e-2 * fmax(1.0, fabs(cl[i])), 1e-2 * (cu[i] - cl[i]));
        if (hu) pu = fmin(1e-2 * fmax(1.0, fabs(cu[i])), 1e-2 * (cu[i] - cl[i]));
        if (hl && hu)
            v = fmin(fmax(v, cl[i] + pl), cu[i] - pu);
        else if (hl)
            v = fmax(v, cl[i] + pl);
        else if (hu)
            v = fmin(v, cu[i] - pu);
        s[i] = v;
    }
}


static double barrier(double f, const double* s, const double* cl, const double* cu, int m, double mu)
{
    double acc = 0;
    for (int i = 0; i < m; ++i) {
        if (isfinite(cl[i])) {
            double d = s[i] - cl[i];
            if (!(d > 0)) return INFINITY;
            acc += log(d);
        }
        if (isfinite(cu[i])) {
            double d = cu[i] - s[i];
            if (!(d > 0)) return INFINITY;
            acc += log(d);
        }
    }
    return f - mu * acc;
}

/* ------------------------------------------------------------------------------------------------ */
/* DD variant (MPC_DD_sig_step.py): x_{i+1} = x_i + [T v_i cos th_i, T v_i sin th_i, w_i] (:355-360)   */
/* rows per step: reference [cbf circles, cbf ellipses, f_en = s|w| + v] (:131-141, :410-420); solver  */
/* (split): [cbf..., v + s w <= v_max, v - s w <= v_max, v in [v_min, v_max], w in [-w_max, w_max]]    */
/* ------------------------------------------------------------------------------------------------ */
static void oprob_init_dd(oprob* P, const alipmpc_cfg* cfg, const double* x0, const double* goal, const double* cir,
                          int nc, const double* elp, int ne, const double* last_u, int split)
{
    memset(P, 0, sizeof(*P));
    P->cfg = cfg;
    P->N = cfg->N;
    P->n = 2 * cfg->N;
    P->dd = 1;
    P->split = split;
    P->df = 1.0;
    memcpy(P->x0, x0, 3 * sizeof(double));
    P->goal[0] = P->goal_orig[0] = goal[0];
    P->goal[1] = P->goal_orig[1] = goal[1];
    P->last_u[0] = last_u ? last_u[0] : 0.0;
    P->last_u[1] = last_u ? last_u[1] : 0.0;
    for (int j = 0; j < nc; ++j) {       /* all obstacles: select_obs is commented out (:75) */
        memcpy(P->cir[P->nc], cir + 3 * j, 3 * sizeof(double));
        P->sel_c[P->nc++] = j;
    }
    for (int j = 0; j < ne; ++j) {
        memcpy(P->elp[P->ne], elp + 5 * j, 5 * sizeof(double));
        P->sel_e[P->ne++] = j;
    }
    for (int j = 0; j < P->ne; ++j) {
        const double* e = P->elp[j];
        double ce = cos(e[4]), se = sin(e[4]);
        P->eqa[j] = (e[3] * ce) * (e[3] * ce) + (e[2] * se) * (e[2] * se);
        P->eqb[j] = 2 * ce * se * (e[3] * e[3] - e[2] * e[2]);
        P->eqc[j] = (e[3] * se) * (e[3] * se) + (e[2] * ce) * (e[2] * ce);
        P->ek[j] = (e[3] * e[2]) * (e[3] * e[2]);
    }
    const int nob = P->nc + P->ne;
    P->rpk = nob + (split ? 4 : 1);
    P->m = P->N * P->rpk;
    int r = 0;
    for (int k = 0; k < P->N; ++k) {
        for (int j = 0; j < nob; ++j) {
            P->cl[r] = 0.0;
            P->cu[r++] = INFINITY;
        }
        if (split) {
            P->cl[r] = -INFINITY; P->cu[r++] = cfg->bvx_hi;
            P->cl[r] = -INFINITY; P->cu[r++] = cfg->bvx_hi;
            P->cl[r] = cfg->bvx_lo; P->cu[r++] = cfg->bvx_hi;
            P->cl[r] = -cfg->dtheta_max; P->cu[r++] = cfg->dtheta_max;
        } else {
            P->cl[r] = cfg->bvx_lo;
            P->cu[r++] = cfg->bvx_hi;
        }
    }
}

static void dd_rollout(const oprob* P, const double* u, double X[][3])
{
    const double T = P->cfg->dt;
    X[0][0] = P->x0[0]; X[0][1] = P->x0[1]; X[0][2] = P->x0[2];
    for (int i = 0; i < P->N; ++i) {
        const double v = u[2 * i], w = u[2 * i + 1], th = X[i][2];
        X[i + 1][0] = X[i][0] + T * v * cos(th);
        X[i + 1][1] = X[i][1] + T * v * sin(th);
        X[i + 1][2] = X[i][2] + w;
    }
}

/* Jp[k][c][a] = d x_k[c] / d u_a (closed forms of cal_dx_du, :534-566) */
static void dd_dpos(const oprob* P, double X[][3], double Jp[][3][2 * OMAXN])
{
    const double T = P->cfg->dt;
    const int n = P->n;
    memset(Jp, 0, sizeof(double) * (P->N + 1) * 3 * 2 * OMAXN);
    for (int k = 1; k <= P->N; ++k)
        for (int j = 0; j < k; ++j) {
            Jp[k][0][2 * j] = T * cos(X[j][2]);
            Jp[k][1][2 * j] = T * sin(X[j][2]);
            Jp[k][0][2 * j + 1] = -(X[k][1] - X[j + 1][1]);
            Jp[k][1][2 * j + 1] = X[k][0] - X[j + 1][0];
            Jp[k][2][2 * j + 1] = 1.0;
        }
    (void)n;
}

static double dd_objective(const oprob* P, const double* u)
{
    const alipmpc_cfg* c = P->cfg;
    double X[OMAXN + 1][3];
    dd_rollout(P, u, X);
    double f = 0, up0 = P->last_u[0], up1 = P->last_u[1];
    for (int i = 0; i < P->N; ++i) {
        double dx = X[i + 1][0] - P->goal[0], dy = X[i + 1][1] - P->goal[1];
        double tar = atan2(P->goal[1] - X[i + 1][1], P->goal[0] - X[i + 1][0]);
        double d0 = u[2 * i] - up0, d1 = u[2 * i + 1] - up1;
        f += c->q * (dx * dx + dy * dy) + c->r * (X[i + 1][2] - tar) * (X[i + 1][2] - tar) + c->dd_t * (d0 * d0 + d1 * d1);
        up0 = u[2 * i];
        up1 = u[2 * i + 1];
    }
    double dx = X[1][0] - P->goal[0], dy = X[1][1] - P->goal[1];
    return f + c->p * (dx * dx + dy * dy);
}

static void dd_gradient(const oprob* P, const double* u, double* g)
{
    const alipmpc_cfg* c = P->cfg;
    double X[OMAXN + 1][3], Jp[OMAXN + 1][3][2 * OMAXN];
    dd_rollout(P, u, X);
    dd_dpos(P, X, Jp);
    const int n = P->n;
    for (int a = 0; a < n; ++a) g[a] = 0;
    for (int k = 1; k <= P->N; ++k) {
        double w = c->q + (k == 1 ? c->p : 0.0);
        double dxg = P->goal[0] - X[k][0], dyg = P->goal[1] - X[k][1];
        double rho2 = dxg * dxg + dyg * dyg, phi = X[k][2] - atan2(dyg, dxg);
        for (int a = 0; a < n; ++a)
            g[a] += 2 * w * (-dxg * Jp[k][0][a] - dyg * Jp[k][1][a]) +
                    2 * c->r * phi * (Jp[k][2][a] - (rho2 > 0.0 ? (dyg * Jp[k][0][a] - dxg * Jp[k][1][a]) / rho2 : 0.0));
    }
    double up0 = P->last_u[0], up1 = P->last_u[1];
    for (int i = 0; i < P->N; ++i) {
        double d0 = u[2 * i] - up0, d1 = u[2 * i + 1] - up1;
        g[2 * i] += 2 * c->dd_t * d0;
        g[2 * i + 1] += 2 * c->dd_t * d1;
        if (i > 0) {
            g[2 * i - 2] -= 2 * c->dd_t * d0;
            g[2 * i - 1] -= 2 * c->dd_t * d1;
        }
        up0 = u[2 * i];
        up1 = u[2 * i + 1];
    }
}

static void dd_constraints(const oprob* P, const double* u, double* out)
{
    const alipmpc_cfg* c = P->cfg;
    double X[OMAXN + 1][3];
    dd_rollout(P, u, X);
    double gm1 = c->gamma - 1.0;
    int r = 0;
    for (int i = 0; i < P->N; ++i) {
        for (int j = 0; j < P->nc + P->ne; ++j) out[r++] = h_obs(P, j, X[i + 1][0], X[i + 1][1]) + gm1 * h_obs(P, j, X[i][0], X[i][1]);
        const double v = u[2 * i], w = u[2 * i + 1];
        if (P->split) {
            out[r++] = v + c->s * w;
            out[r++] = v - c->s * w;
            out[r++] = v;
            out[r++] = w;
        } else {
            out[r++] = c->s * fabs(w) + v;
        }
    }
}

static void dd_jacobian(const oprob* P, const double* u, double* J)
{
    const alipmpc_cfg* c = P->cfg;
    double X[OMAXN + 1][3], Jp[OMAXN + 1][3][2 * OMAXN];
    dd_rollout(P, u, X);
    dd_dpos(P, X, Jp);
    const int n = P->n;
    double gm1 = c->gamma - 1.0;
    int r = 0;
    for (int i = 0; i < P->N; ++i) {
        for (int o = 0; o < P->nc + P->ne; ++o) {
            double g0, g1, h0, h1;
            dh_obs(P, o, X[i + 1][0], X[i + 1][1], &g0, &g1);
            dh_obs(P, o, X[i][0], X[i][1], &h0, &h1);
            for (int a = 0; a < n; ++a)
                J[(size_t)r * n + a] = g0 * Jp[i + 1][0][a] + g1 * Jp[i + 1][1][a] + gm1 * (h0 * Jp[i][0][a] + h1 * Jp[i][1][a]);
            r++;
        }
        const double w = u[2 * i + 1];
        const int nrow = P->split ? 4 : 1;
        for (int t = 0; t < nrow; ++t)
            for (int a = 0; a < n; ++a) J[(size_t)(r + t) * n + a] = 0.0;
        if (P->split) {
            J[(size_t)r * n + 2 * i] = 1.0; J[(size_t)r * n + 2 * i + 1] = c->s; r++;
            J[(size_t)r * n + 2 * i] = 1.0; J[(size_t)r * n + 2 * i + 1] = -c->s; r++;
            J[(size_t)r * n + 2 * i] = 1.0; r++;
            J[(size_t)r * n + 2 * i + 1] = 1.0; r++;
        } else {
            J[(size_t)r * n + 2 * i] = 1.0;
            J[(size_t)r * n + 2 * i + 1] = c->s * (w == 0 ? 0.0 : copysign(1.0, w));   /* den_du :505-510 */
            r++;
        }
    }
}

/* exact Hessian of L = f - y^T c, including the second derivatives of the unicycle rollout */
static void dd_hessian(const oprob* P, const double* u, const double* y, double* H)
{
    const alipmpc_cfg* c = P->cfg;
    const double T = c->dt;
    double X[OMAXN + 1][3], Jp[OMAXN + 1][3][2 * OMAXN];
    dd_rollout(P, u, X);
    dd_dpos(P, X, Jp);
    const int n = P->n, N = P->N, nob = P->nc + P->ne;
    const double gm1 = c->gamma - 1.0;
    double Hl[OMAXN + 1][3][3], gl[OMAXN + 1][2];
    memset(Hl, 0, sizeof(Hl));
    memset(gl, 0, sizeof(gl));
    for (int k = 1; k <= N; ++k) {
        double w = c->q + (k == 1 ? c->p : 0.0);
        double dxg = P->goal[0] - X[k][0], dyg = P->goal[1] - X[k][1];
        double rho2 = dxg * dxg + dyg * dyg, phi = X[k][2] - atan2(dyg, dxg), r4 = rho2 * rho2;
        double gp[3] = {rho2 > 0.0 ? -dyg / rho2 : 0.0, rho2 > 0.0 ? dxg / rho2 : 0.0, 1.0};   /* (§2 item 7) */
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) Hl[k][a][b] += 2 * c->r * gp[a] * gp[b];
        Hl[k][0][0] += 2 * w;
        Hl[k][1][1] += 2 * w;
        double s00 = rho2 > 0.0 ? 2 * dxg * dyg / r4 : 0.0, s01 = rho2 > 0.0 ? (dyg * dyg - dxg * dxg) / r4 : 0.0,
               s11 = rho2 > 0.0 ? -2 * dxg * dyg / r4 : 0.0;
        Hl[k][0][0] -= 2 * c->r * phi * s00;
        Hl[k][0][1] -= 2 * c->r * phi * s01;
        Hl[k][1][0] -= 2 * c->r * phi * s01;
        Hl[k][1][1] -= 2 * c->r * phi * s11;
        gl[k][0] = -2 * w * dxg + 2 * c->r * phi * gp[0];
        gl[k][1] = -2 * w * dyg + 2 * c->r * phi * gp[1];
    }
    for (int i = 0; i < N; ++i) {
        const double* yk = y + i * P->rpk;
        for (int o = 0; o < nob; ++o) {
            double q00, q01, q11;
            if (o < P->nc) {
                q00 = 2; q01 = 0; q11 = 2;
            } else {
                int e = o - P->nc;
                q00 = 2 * P->eqa[e]; q01 = P->eqb[e]; q11 = 2 * P->eqc[e];
            }
            double g0, g1, h0, h1;
            dh_obs(P, o, X[i + 1][0], X[i + 1][1], &g0, &g1);
            dh_obs(P, o, X[i][0], X[i][1], &h0, &h1);
            Hl[i + 1][0][0] -= yk[o] * q00; Hl[i + 1][0][1] -= yk[o] * q01;
            Hl[i + 1][1][0] -= yk[o] * q01; Hl[i + 1][1][1] -= yk[o] * q11;
            gl[i + 1][0] -= yk[o] * g0; gl[i + 1][1] -= yk[o] * g1;
            if (i >= 1) {
                Hl[i][0][0] -= yk[o] * gm1 * q00; Hl[i][0][1] -= yk[o] * gm1 * q01;
                Hl[i][1][0] -= yk[o] * gm1 * q01; Hl[i][1][1] -= yk[o] * gm1 * q11;
                gl[i][0] -= yk[o] * gm1 * h0; gl[i][1] -= yk[o] * gm1 * h1;
            }
        }
    }
    for (int a = 0; a < n * n; ++a) H[a] = 0;
    for (int k = 1; k <= N; ++k)
        for (int a = 0; a < n; ++a)
            for (int b = 0; b < n; ++b) {
                double acc = 0;
                for (int p = 0; p < 3; ++p)
                    for (int q = 0; q < 3; ++q) acc += Jp[k][p][a] * Hl[k][p][q] * Jp[k][q][b];
                const int ja = a / 2, jb = b / 2, va = (a % 2) == 0, vb = (b % 2) == 0;
                double sxx = 0, syy = 0;
                if (va && !vb) {
                    if (jb < ja && ja < k) { sxx = -T * sin(X[ja][2]); syy = T * cos(X[ja][2]); }
                } else if (vb && !va) {
                    if (ja < jb && jb < k) { sxx = -T * sin(X[jb][2]); syy = T * cos(X[jb][2]); }
                } else if (!va && !vb) {
                    int mm = ja > jb ? ja : jb;
                    if (mm < k) { sxx = -(X[k][0] - X[mm + 1][0]); syy = -(X[k][1] - X[mm + 1][1]); }
                }
                H[a * n + b] += acc + gl[k][0] * sxx + gl[k][1] * syy;
            }
    for (int i = 0; i < N; ++i)
        for (int cc = 0; cc < 2; ++cc) {
            int a = 2 * i + cc;
            H[a * n + a] += 2 * c->dd_t * (i < N - 1 ? 2.0 : 1.0);
            if (i < N - 1) {
                H[a * n + a + 2] -= 2 * c->dd_t;
                H[(a + 2) * n + a] -= 2 * c->dd_t;
            }
        }
}

typedef struct {
    int iters, status, restorations;
} osolve_info;

/* foothold-space views of the NLP: u(p) = [A^k x0]_k + U p  (the solve runs on p, n = 3N) */
static void u_of_p(const oprob* P, const double* pv, double* u)
{
    const oconsts* K = P->K;
    const int N = P->N, np_ = 3 * N;
    for (int k = 1; k <= N; ++k)
        for (int a = 0; a < 5; ++a) {
            double acc = 0;
            for (int t = 0; t < 5; ++t) acc += K->Ak[k][a][t] * P->x0[t];
            for (int j = 0; j < np_; ++j) acc += K->U[5 * (k - 1) + a][j] * pv[j];
            u[5 * (k - 1) + a] = acc;
        }
}
/* the solve's objective carries IPOPT's scaling factor P->df (1 unless the starting point's gradient exceeds 100) */
static double pobj(const oprob* P, const double* pv)
{
    if (P->dd) return P->df * dd_objective(P, pv);
    double u[OMAXV];
    u_of_p(P, pv, u);
    return P->df * oracle_objective(P, u);
}
static void pcons(const oprob* P, const double* pv, double* c)
{
    if (P->dd) {
        dd_constraints(P, pv, c);
        return;
    }
    double u[OMAXV];
    u_of_p(P, pv, u);
    constraints(P, u, c);
}
static void pgrad(const oprob* P, const double* pv, double* gp)
{
    if (P->dd) {
        dd_gradient(P, pv, gp);
        for (int j = 0; j < P->n; ++j) gp[j] *= P->df;
        return;
    }
    double u[OMAXV], gu[OMAXV];
    u_of_p(P, pv, u);
    gradient(P, u, gu);
    const int nu = 5 * P->N, np_ = 3 * P->N;
    for (int j = 0; j < np_; ++j) {
        double acc = 0;
        for (int i = 0; i < nu; ++i) acc += P->K->U[i][j] * gu[i];
        gp[j] = P->df * acc;
    }
}
static void pjac(const oprob* P, const double* pv, double* Jp)
{
    static __thread double Ju[OMAXM * OMAXV];
    if (P->dd) {
        dd_jacobian(P, pv, Jp);
        return;
    }
    double u[OMAXV];
    u_of_p(P, pv, u);
    jacobian(P, u, Ju);
    const int nu = 5 * P->N, np_ = 3 * P->N;
    for (int r = 0; r < P->m; ++r)
        for (int j = 0; j < np_; ++j) {
            double acc = 0;
            for (int i = 0; i < nu; ++i) acc += Ju[r * nu + i] * P->K->U[i][j];
            Jp[r * np_ + j] = acc;
        }
}
/* Hessian of L = of df f - y^T c = df (of f - (y / df)^T c) */
static void phess_of(const oprob* P, const double* pv, const double* y_, double of, double* Hp)
{
    double y[OMAXM];
    for (int i = 0; i < P->m; ++i) y[i] = y_[i] / P->df;
    if (P->dd) {
        dd_hessian(P, pv, y, Hp);
        for (int i = 0; i < P->n * P->n; ++i) Hp[i] *= P->df;
        return;
    }
    double u[OMAXV], Hu[OMAXV * OMAXV], T[OMAXV * 3 * OMAXN];
    u_of_p(P, pv, u);
    hessian_of(P, u, y, of, Hu);
    const int nu = 5 * P->N, np_ = 3 * P->N;
    for (int i = 0; i < nu; ++i)
        for (int j = 0; j < np_; ++j) {
            double acc = 0;
            for (int t = 0; t < nu; ++t) acc += Hu[i * nu + t] * P->K->U[t][j];
            T[i * np_ + j] = acc;
        }
    for (int a = 0; a < np_; ++a)
        for (int b = 0; b < np_; ++b) {
            double acc = 0;
            for (int i = 0; i < nu; ++i) acc += P->K->U[i][a] * T[i * np_ + b];
            Hp[a * np_ + b] = P->df * acc;
        }
}
static void phess(const oprob* P, const double* pv, const double* y_, double* Hp) { phess_of(P, pv, y_, 1.0, Hp); }

/* IPOPT's default NLP scaling (nlp_scaling_method = gradient-based, nlp_scaling_max_gradient = 100,
   nlp_scaling_min_value = 1e-8), evaluated at the user's starting point u0 in the reference's own variables: the
   objective is scaled by 100 / max|grad f(u0)| where that maximum exceeds 100.  Constraint rows would be scaled the
   same way, but their gradients stay below 4 in u on every benchmark scene (measured max 3.5, sig_step; DESIGN.md §2
   item 9) and exceed 100 only with select_obs = 0 and large distant ellipses, where IPOPT would scale the row and this
   build does not (a stated deviation: tests/test_oracle.py::test_row_scaling_region); every dc_i is 1. */
static double obj_scaling(const oprob* P, const double* u0)
{
    double g[OMAXV];
    if (P->dd)
        dd_gradient(P, u0, g);
    else
        gradient(P, u0, g);
    double gm = 0.0;
    for (int i = 0; i < P->n; ++i) gm = fmax(gm, fabs(g[i]));
    return gm > 100.0 ? fmax(1e-8, 100.0 / gm) : 1.0;
}

#define REST_FAIL 6



/* a planned state exactly on the goal (rho2 = |g - p|^2 == 0), where the reference's cal_dtar_ang_du
   (MPC_LIP_modi.py:650-655; MPC_DD_sig_step.py:527-531) divides 0 by 0 */
static int at_goal(const oprob* P, const double* pv)
{
    if (P->dd) {
        double X[OMAXN + 1][3];
        dd_rollout(P, pv, X);
        for (int k = 1; k <= P->N; ++k) {
            double dxg = P->goal[0] - X[k][0], dyg = P->goal[1] - X[k][1];
            if (dxg * dxg + dyg * dyg == 0.0) return 1;
        }
        return 0;
    }
    double u[OMAXV], X[OMAXN + 1][5], Pp[OMAXN][3];
    u_of_p(P, pv, u);
    rollout(P, u, X, Pp);
    for (int k = 1; k <= P->N; ++k) {
        double dxg = P->goal[0] - X[k][0], dyg = P->goal[1] - X[k][1];
        if (dxg * dxg + dyg * dyg == 0.0) return 1;
    }
    return 0;
}

/* IPOPT's feasibility restoration phase (Wächter & Biegler 2006 §3.3; IPOPT's MinC_1NrmRestorationPhase, published
   defaults, version unpinned); mirrors np_oracle._resto (proximity on the footholds, D_R = 1 / max(1, |p_R|)):
     min rho sum(p + n) + zeta/2 sum_j D_j^2 (x_j - xR_j)^2  s.t.  c(x) - p + n - s = 0, cl <= s <= cu, p, n >= 0
   rho = 1000, zeta = sqrt(mu_R), mu_R from max(mu, |c - s|_inf); p, n from IPOPT eq. (33); y = 0; slack multipliers
   min(rho, current).  Returns RS_OK (back to the regular phase: x, s, zl, zu updated), RS_INFEASIBLE (restoration
   converged with the violation above 1e-4: Infeasible_Problem_Detected), RS_MAXITER, RS_FAILED; *it advances by the
   restoration's iterations. */
enum { RS_OK = 0, RS_INFEASIBLE = 1, RS_MAXITER = 2, RS_FAILED = 3 };
#define RESTO_RHO 1000.0
#define RESTO_KAPPA 0.9
#define RESTO_VIOL_TOL 1e-4
#define RESTO_MULT_RESET 1000.0

static double ftb(double v, double dv, double tau, double a) { return dv < 0 ? fmin(a, -tau * v / dv) : a; }

static int oresto(oprob* P, double* x, double* s, double* zl, double* zu, double mu_o, const double* cl,
                  const double* cu, const int* hl, const int* hu, const double* fo, int nfo, double theta_R, int* it,
                  int max_iter, double tol)
{
    const int n = 3 * P->N, m = P->m;
    const double rho = RESTO_RHO;
    double xR[OMAXV], d2[OMAXV], c[OMAXM], pp[OMAXM], nn[OMAXM], zp[OMAXM], zn[OMAXM], vl[OMAXM], vu[OMAXM];
    double y[OMAXM], s0[OMAXM], J[OMAXM * OMAXV], H[OMAXV * OMAXV], Kmat[OMAXV * OMAXV], L[OMAXV * OMAXV];
    double rhs[OMAXV], gx[OMAXV], dx[OMAXV], dl[OMAXM], du[OMAXM], D[OMAXM], b[OMAXM], dy[OMAXM], dp[OMAXM];
    double dn[OMAXM], ds[OMAXM], dzp[OMAXM], dzn[OMAXM], dvl[OMAXM], dvu[OMAXM], Sp[OMAXM], Sn[OMAXM], Ss[OMAXM];
    double xt[OMAXV], pt[OMAXM], nt[OMAXM], st[OMAXM], ct[OMAXM];
    static const double gth = 1e-5, gph = 1e-8, sth = 1.1, sph = 2.3, eta = 1e-8, gal = 0.05;
    memcpy(xR, x, sizeof(double) * n);
    for (int j = 0; j < n; ++j) {
        double dd = 1.0 / fmax(1.0, fabs(xR[j]));
        d2[j] = dd * dd;
    }
    pcons(P, x, c);
    double mu = mu_o;
    for (int i = 0; i < m; ++i) mu = fmax(mu, fabs(c[i] - s[i]));
    for (int i = 0; i < m; ++i) {
        double r = c[i] - s[i], a = (mu - rho * r) / (2 * rho);
        double sq = sqrt(a * a + mu * r / (2 * rho));
        nn[i] = a >= 0 ? a + sq : (mu * r / (2 * rho)) / (sq - a);
        pp[i] = r + nn[i];
        zp[i] = mu / pp[i];
        zn[i] = mu / nn[i];
        vl[i] = hl[i] ? fmin(rho, zl[i]) : 0.0;
        vu[i] = hu[i] ? fmin(rho, zu[i]) : 0.0;
        y[i] = 0.0;
        s0[i] = s[i];
    }
    const int maxf = max_iter + 2;
    double* ft = (double*)malloc(sizeof(double) * 2 * maxf);
    int nf = 0;
    double th0 = 0;
    for (int i = 0; i < m; ++i) th0 += fabs(c[i] - pp[i] + nn[i] - s[i]);
    const double theta_max = 1e4 * fmax(1.0, th0), theta_min = 1e-4 * fmax(1.0, th0);
    double dw_last = 0.0;
    int first = 1, nb = 2 * m, ret;
    for (int i = 0; i < m; ++i) nb += hl[i] + hu[i];
    const int nvar = n + 2 * m;
    for (;;) {
        pcons(P, x, c);
        if (!first) {
            double th_o = 0;
            for (int i = 0; i < m; ++i) th_o += fabs(c[i] - s[i]);
            double ph_o = barrier(pobj(P, x), s, cl, cu, m, mu_o);
            int acc = isfinite(ph_o) && th_o <= RESTO_KAPPA * theta_R;
            for (int q = 0; acc && q < nfo; ++q)
                if (!(th_o < fo[2 * q] || ph_o < fo[2 * q + 1])) acc = 0;
            if (acc) {
                /* back to the regular phase: slack multipliers by the complementarity Newton step over the whole
                   restoration (fraction to the boundary), reset to 1 above bound_mult_reset_threshold */
                const double tau = fmax(0.99, 1.0 - mu_o);
                double ad = 1.0, zmax = 0.0;
                double dzl[OMAXM], dzu[OMAXM];
                for (int i = 0; i < m; ++i) {
                    dzl[i] = hl[i] ? mu_o / (s0[i] - cl[i]) - zl[i] - zl[i] / (s0[i] - cl[i]) * (s[i] - s0[i]) : 0.0;
                    dzu[i] = hu[i] ? mu_o / (cu[i] - s0[i]) - zu[i] + zu[i] / (cu[i] - s0[i]) * (s[i] - s0[i]) : 0.0;
                    if (hl[i]) ad = ftb(zl[i], dzl[i], tau, ad);
                    if (hu[i]) ad = ftb(zu[i], dzu[i], tau, ad);
                }
                for (int i = 0; i < m; ++i) {
                    zl[i] += ad * dzl[i];
                    zu[i] += ad * dzu[i];
                    zmax = fmax(zmax, fmax(zl[i], zu[i]));
                }
                if (zmax > RESTO_MULT_RESET)
                    for (int i = 0; i < m; ++i) {
                        zl[i] = hl[i] ? 1.0 : 0.0;
                        zu[i] = hu[i] ? 1.0 : 0.0;
                    }
                ret = RS_OK;
                break;
            }
        }
        first = 0;
        pjac(P, x, J);
        double zeta = sqrt(mu);
        double nz = 0, ny = 0;
        for (int i = 0; i < m; ++i) {
            dl[i] = hl[i] ? s[i] - cl[i] : 1.0;
            du[i] = hu[i] ? cu[i] - s[i] : 1.0;
            ny += fabs(y[i]);
            nz += fabs(zp[i]) + fabs(zn[i]) + fabs(vl[i]) + fabs(vu[i]);
        }
        const double sd = fmax(100.0, (nz + ny) / (nvar + m)) / 100.0;
        const double sc = fmax(100.0, nz / (nb > 0 ? nb : 1)) / 100.0;
        double dual = 0, prim = 0;
        for (int j = 0; j < n; ++j) {
            double a = zeta * d2[j] * (x[j] - xR[j]);
            for (int i = 0; i < m; ++i) a -= J[i * n + j] * y[i];
            gx[j] = a;
            dual = fmax(dual, fabs(a));
        }
        for (int i = 0; i < m; ++i) {
            dual = fmax(dual, fmax(fabs(rho + y[i] - zp[i]), fabs(rho - y[i] - zn[i])));
            dual = fmax(dual, fabs(y[i] - vl[i] + vu[i]));
            prim = fmax(prim, fabs(c[i] - pp[i] + nn[i] - s[i]));
        }
#define RERR(muv)                                                                                   \
    ({                                                                                              \
        double cm_ = 0;                                                                             \
        for (int i_ = 0; i_ < m; ++i_) {                                                            \
            cm_ = fmax(cm_, fmax(fabs(pp[i_] * zp[i_] - (muv)), fabs(nn[i_] * zn[i_] - (muv))));    \
            if (hl[i_]) cm_ = fmax(cm_, fabs(dl[i_] * vl[i_] - (muv)));                             \
            if (hu[i_]) cm_ = fmax(cm_, fabs(du[i_] * vu[i_] - (muv)));                             \
        }                                                                                           \
        fmax(fmax(dual / sd, prim), cm_ / sc);                                                      \
    })
        if (RERR(0.0) <= tol) {
            double viol = 0;
            for (int i = 0; i < m; ++i) {
                if (hl[i]) viol = fmax(viol, P->cl[i] - c[i]);
                if (hu[i]) viol = fmax(viol, c[i] - P->cu[i]);
            }
            ret = viol > RESTO_VIOL_TOL ? RS_INFEASIBLE : RS_OK;
            break;
        }
        if (*it >= max_iter) {
            ret = RS_MAXITER;
            break;
        }
        const double mu_min = tol / 11.0, mu_old = mu;
        for (int t = 0; t < 8; ++t) {
            if (RERR(mu) <= 10.0 * mu && mu > mu_min)
                mu = fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu)));
            else
                break;
        }
#undef RERR
        if (mu != mu_old) {
            nf = 0;
            zeta = sqrt(mu);
            for (int j = 0; j < n; ++j) {
                double a = zeta * d2[j] * (x[j] - xR[j]);
                for (int i = 0; i < m; ++i) a -= J[i * n + j] * y[i];
                gx[j] = a;
            }
        }
        const double tau = fmax(0.99, 1.0 - mu);
        for (int i = 0; i < m; ++i) {
            Sp[i] = zp[i] / pp[i];
            Sn[i] = zn[i] / nn[i];
            Ss[i] = (hl[i] ? vl[i] / dl[i] : 0.0) + (hu[i] ? vu[i] / du[i] : 0.0);
            D[i] = 1.0 / Sp[i] + 1.0 / Sn[i] + 1.0 / Ss[i];
            const double mdl = hl[i] ? mu / dl[i] : 0.0, mdu = hu[i] ? mu / du[i] : 0.0;
            const double rc = c[i] - pp[i] + nn[i] - s[i];
            b[i] = -rc + (-rho - y[i] + mu / pp[i]) / Sp[i] - (-rho + y[i] + mu / nn[i]) / Sn[i] +
                   (-y[i] + mdl - mdu) / Ss[i];
        }
        phess_of(P, x, y, 0.0, H);
        for (int a = 0; a < n; ++a) {
            for (int bb = 0; bb < n; ++bb) {
                double acc = 0;
                for (int i = 0; i < m; ++i) acc += J[i * n + a] * J[i * n + bb] / D[i];
                Kmat[a * n + bb] = H[a * n + bb] + (a == bb ? zeta * d2[a] : 0.0) + acc;
            }
            double acc = -gx[a];
            for (int i = 0; i < m; ++i) acc += J[i * n + a] * (b[i] / D[i]);
            rhs[a] = acc;
        }
        memcpy(L, Kmat, sizeof(double) * n * n);
        if (!chol(L, n)) {
            double dw = dw_last == 0 ? 1e-4 : fmax(1e-20, dw_last / 3.0);
            int ok = 0;
            for (;;) {
                memcpy(L, Kmat, sizeof(double) * n * n);
                for (int a = 0; a < n; ++a) L[a * n + a] += dw;
                if (chol(L, n)) {
                    ok = 1;
                    break;
                }
                dw *= dw_last == 0 ? 100.0 : 8.0;
                if (dw > 1e40) break;
            }
            dw_last = dw;
            if (!ok) {
                ret = RS_FAILED;
                break;
            }
        }
        memcpy(dx, rhs, sizeof(double) * n);
        cholsolve(L, n, dx);
        double ap = 1.0, az = 1.0;
        for (int i = 0; i < m; ++i) {
            double jd = 0;
            for (int j = 0; j < n; ++j) jd += J[i * n + j] * dx[j];
            const double mdl = hl[i] ? mu / dl[i] : 0.0, mdu = hu[i] ? mu / du[i] : 0.0;
            dy[i] = (b[i] - jd) / D[i];
            dp[i] = (-rho - y[i] + mu / pp[i] - dy[i]) / Sp[i];
            dn[i] = (-rho + y[i] + mu / nn[i] + dy[i]) / Sn[i];
            ds[i] = (-y[i] + mdl - mdu - dy[i]) / Ss[i];
            dzp[i] = mu / pp[i] - zp[i] - Sp[i] * dp[i];
            dzn[i] = mu / nn[i] - zn[i] - Sn[i] * dn[i];
            dvl[i] = hl[i] ? mdl - vl[i] - vl[i] / dl[i] * ds[i] : 0.0;
            dvu[i] = hu[i] ? mdu - vu[i] + vu[i] / du[i] * ds[i] : 0.0;
            ap = ftb(pp[i], dp[i], tau, ap);
            ap = ftb(nn[i], dn[i], tau, ap);
            if (hl[i]) ap = ftb(dl[i], ds[i], tau, ap);
            if (hu[i]) ap = ftb(du[i], -ds[i], tau, ap);
            az = ftb(zp[i], dzp[i], tau, az);
            az = ftb(zn[i], dzn[i], tau, az);
            if (hl[i]) az = ftb(vl[i], dvl[i], tau, az);
            if (hu[i]) az = ftb(vu[i], dvu[i], tau, az);
        }
        double theta = 0, q0 = 0, gphi = 0, lg = 0;
        int bad = 0;
        for (int j = 0; j < n; ++j) {
            q0 += d2[j] * (x[j] - xR[j]) * (x[j] - xR[j]);
            gphi += zeta * d2[j] * (x[j] - xR[j]) * dx[j];
        }
        double spn = 0, gpn = 0, gs = 0;
        for (int i = 0; i < m; ++i) {
            theta += fabs(c[i] - pp[i] + nn[i] - s[i]);
            spn += pp[i] + nn[i];
            gpn += (rho - mu / pp[i]) * dp[i] + (rho - mu / nn[i]) * dn[i];
            gs += (hl[i] ? mu * ds[i] / dl[i] : 0.0) - (hu[i] ? mu * ds[i] / du[i] : 0.0);
            lg += log(pp[i]) + log(nn[i]);
            if (hl[i]) lg += log(dl[i]);
            if (hu[i]) lg += log(du[i]);
        }
        (void)bad;
        gphi += gpn - gs;
        const double phi = rho * spn + 0.5 * zeta * q0 - mu * lg;
        double amin;
        if (gphi < 0) {
            amin = fmin(gth, gph * theta / -gphi);
            if (theta <= theta_min) amin = fmin(amin, pow(theta, sth) / pow(-gphi, sph));
        } else
            amin = gth;
        amin *= gal;
        if (!(amin > 0.0)) amin = 8.673617379884035e-19;
        double al = ap;
        int accepted = 0, ftype = 0;
        while (al >= amin) {
            for (int j = 0; j < n; ++j) xt[j] = x[j] + al * dx[j];
            for (int i = 0; i < m; ++i) {
                pt[i] = pp[i] + al * dp[i];
                nt[i] = nn[i] + al * dn[i];
                st[i] = s[i] + al * ds[i];
            }
            pcons(P, xt, ct);
            double tht = 0, qt = 0, spt = 0, lgt = 0;
            int badt = 0;
            for (int j = 0; j < n; ++j) qt += d2[j] * (xt[j] - xR[j]) * (xt[j] - xR[j]);
            for (int i = 0; i < m; ++i) {
                tht += fabs(ct[i] - pt[i] + nt[i] - st[i]);
                spt += pt[i] + nt[i];
                if (!(pt[i] > 0) || !(nt[i] > 0)) badt = 1;
                if (hl[i] && !(st[i] - cl[i] > 0)) badt = 1;
                if (hu[i] && !(cu[i] - st[i] > 0)) badt = 1;
                if (!badt) {
                    lgt += log(pt[i]) + log(nt[i]);
                    if (hl[i]) lgt += log(st[i] - cl[i]);
                    if (hu[i]) lgt += log(cu[i] - st[i]);
                }
            }
            const double pht = badt ? INFINITY : rho * spt + 0.5 * zeta * qt - mu * lgt;
            int ok = isfinite(pht) && tht < theta_max;
            for (int q = 0; ok && q < nf; ++q)
                if (!(tht < ft[2 * q] || pht < ft[2 * q + 1])) ok = 0;
            if (ok) {
                int switching = gphi < 0 && al * pow(-gphi, sph) > pow(theta, sth);
                if (switching && theta <= theta_min) {
                    if (pht <= phi + eta * al * gphi) {
                        accepted = 1;
                        ftype = 1;
                    }
                } else if (tht <= (1 - gth) * theta || pht <= phi - gph * theta) {
                    accepted = 1;
                    ftype = 0;
                }
            }
            if (accepted) break;
            al *= 0.5;
        }
        if (!accepted) {
            ret = RS_FAILED;
            break;
        }
        if (!ftype && nf < maxf) {
            ft[2 * nf] = (1 - gth) * theta;
            ft[2 * nf + 1] = phi - gph * theta;
            nf++;
        }
        memcpy(x, xt, sizeof(double) * n);
        for (int i = 0; i < m; ++i) {
            pp[i] = pt[i];
            nn[i] = nt[i];
            s[i] = st[i];
            y[i] += al * dy[i];
            zp[i] += az * dzp[i];
            zn[i] += az * dzn[i];
            vl[i] += az * dvl[i];
            vu[i] += az * dvu[i];
            const double ks = 1e10;
            zp[i] = fmin(fmax(zp[i], mu / (ks * pp[i])), ks * mu / pp[i]);
            zn[i] = fmin(fmax(zn[i], mu / (ks * nn[i])), ks * mu / nn[i]);
            if (hl[i]) {
                double d = s[i] - cl[i];
                vl[i] = fmin(fmax(vl[i], mu / (ks * d)), ks * mu / d);
            } else
                vl[i] = 0;
            if (hu[i]) {
                double d = cu[i] - s[i];
                vu[i] = fmin(fmax(vu[i], mu / (ks * d)), ks * mu / d);
            } else
                vu[i] = 0;
        }
        ++*it;
    }
    free(ft);
    return ret;
}

/* Primal-dual interior point with IPOPT's filter line search; mirrors np_oracle.solve. */
static void osolve(oprob* P, const double* u0, double* uout, osolve_info* info)
{
    const alipmpc_cfg* cfg = P->cfg;
    const int n = P->dd ? 2 * P->N : 3 * P->N, m = P->m;
    double u[OMAXV];   /* the decision: footholds p (n = 3N), DD controls (n = 2N) */
    double cl[OMAXM], cu[OMAXM];
    int hl[OMAXM], hu[OMAXM];
    int nb = 0;
    for (int i = 0; i < m; ++i) {
        hl[i] = isfinite(P->cl[i]);
        hu[i] = isfinite(P->cu[i]);
        nb += hl[i] + hu[i];
        cl[i] = hl[i] ? P->cl[i] - 1e-8 * fmax(1.0, fabs(P->cl[i])) : -INFINITY;
        cu[i] = hu[i] ? P->cu[i] + 1e-8 * fmax(1.0, fabs(P->cu[i])) : INFINITY;
    }
    if (P->dd) {
        memcpy(u, u0, sizeof(double) * n);
    } else {
        double X0[OMAXN + 1][5], Pp0[OMAXN][3];
        rollout(P, u0, X0, Pp0);
        for (int k = 0; k < P->N; ++k)
            for (int c = 0; c < 3; ++c) u[3 * k + c] = Pp0[k][c];
    }
    P->df = obj_scaling(P, u0);
    double mu = cfg->mu_init;
    double c[OMAXM], s[OMAXM], zl[OMAXM], zu[OMAXM];
    pcons(P, u, c);
    push_slacks(c, cl, cu, m, s);
    for (int i = 0; i < m; ++i) {
        zl[i] = hl[i] ? 1.0 : 0.0;
        zu[i] = hu[i] ? 1.0 : 0.0;
    }
    double dw_last = 0.0;
    int status = -1, it = 0, n_rest = 0;
    double e0 = INFINITY;
    double th0 = 0;
    for (int i = 0; i < m; ++i) th0 += fabs(c[i] - s[i]);
    const double theta_max = 1e4 * fmax(1.0, th0), theta_min = 1e-4 * fmax(1.0, th0);
    const int maxf = cfg->max_iter + 2;
    double* ft = (double*)malloc(sizeof(double) * 2 * maxf);
    int nf = 0;
    static const double gth = 1e-5, gph = 1e-8, sth = 1.1, sph = 2.3, eta = 1e-8, gal = 0.05;
    double gf[OMAXV], J[OMAXM * OMAXV], H[OMAXV * OMAXV], Kmat[OMAXV * OMAXV], rhs[OMAXV], y[OMAXM];
    double dl[OMAXM], du[OMAXM], rc[OMAXM], Sig[OMAXM], dU[OMAXV], dS[OMAXM], dZl[OMAXM], dZu[OMAXM];
    double ut[OMAXV], st[OMAXM], ct[OMAXM];
    for (it = 0; it <= cfg->max_iter;) {
        /* cfg.goal_singular = ABORT: the reference's NaN gradient at this iterate — IPOPT's Eval_Error, status
           Invalid_Number_Detected with the iterate returned (include/alipmpc.h) */
        if (cfg->goal_singular == ALIPMPC_GOAL_SINGULAR_ABORT && at_goal(P, u)) {
            status = ALIPMPC_INVALID_NUMBER_DETECTED;
            break;
        }
        double f = pobj(P, u);
        pgrad(P, u, gf);
        pjac(P, u, J);
        double nz = 0;
        for (int i = 0; i < m; ++i) {
            dl[i] = hl[i] ? s[i] - cl[i] : 1.0;
            du[i] = hu[i] ? cu[i] - s[i] : 1.0;
            y[i] = zl[i] - zu[i];
            rc[i] = c[i] - s[i];
            nz += fabs(zl[i]) + fabs(zu[i]);
        }
        double ru_max = 0;
        for (int j = 0; j < n; ++j) {
            double a = gf[j];
            for (int i = 0; i < m; ++i) a -= J[i * n + j] * y[i];
            ru_max = fmax(ru_max, fabs(a));
        }
        double rc_max = 0;
        for (int i = 0; i < m; ++i) rc_max = fmax(rc_max, fabs(rc[i]));
        double sd = fmax(100.0, nz / (m + n)) / 100.0;
        double sc = fmax(100.0, nz / (nb > 0 ? nb : 1)) / 100.0;
#define ERR(muv)                                                                \
    ({                                                                          \
        double comp_ = 0;                                                       \
        for (int i_ = 0; i_ < m; ++i_) {                                        \
            if (hl[i_]) comp_ = fmax(comp_, fabs(dl[i_] * zl[i_] - (muv)));     \
            if (hu[i_]) comp_ = fmax(comp_, fabs(du[i_] * zu[i_] - (muv)));     \
        }                                                                       \
        fmax(fmax(ru_max / sd, rc_max), comp_ / sc);                            \
    })
        e0 = ERR(0.0);
        if (e0 <= cfg->tol) {
            status = 0;
            break;
        }
        if (it >= cfg->max_iter) break;
        /* IPOPT's floor min(tol, compl_inf_tol) / (barrier_tol_factor + 1 = 11) (MonotoneMuUpdate): tol / 11 for
           tol <= compl_inf_tol = 1e-4 (the fp32 programs' larger tolerances keep tol / 11) */
        double mu_min = cfg->tol / 11.0, mu_old = mu;
        for (int t = 0; t < 8; ++t) {
            if (ERR(mu) <= 10.0 * mu && mu > mu_min)
                mu = fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu)));
            else
                break;
        }
        if (mu != mu_old) nf = 0;
        double tau = fmax(0.99, 1.0 - mu);
        for (int i = 0; i < m; ++i) Sig[i] = (hl[i] ? zl[i] / dl[i] : 0.0) + (hu[i] ? zu[i] / du[i] : 0.0);
        phess(P, u, y, H);
        for (int a = 0; a < n; ++a) {
            for (int b = 0; b < n; ++b) {
                double acc = 0;
                for (int i = 0; i < m; ++i) acc += J[i * n + a] * Sig[i] * J[i * n + b];
                Kmat[a * n + b] = H[a * n + b] + acc;
            }
            double acc = -gf[a];
            for (int i = 0; i < m; ++i) {
                double w = (hl[i] ? mu / dl[i] : 0.0) - (hu[i] ? mu / du[i] : 0.0) - Sig[i] * rc[i];
                acc += J[i * n + a] * w;
            }
            rhs[a] = acc;
        }
        double L[OMAXV * OMAXV];
        double dw = 0.0;
        int fact_ok = 1;
        memcpy(L, Kmat, sizeof(double) * n * n);
        if (!chol(L, n)) {
            dw = dw_last == 0 ? 1e-4 : fmax(1e-20, dw_last / 3.0);
            for (;;) {
                memcpy(L, Kmat, sizeof(double) * n * n);
                for (int a = 0; a < n; ++a) L[a * n + a] += dw;
                if (chol(L, n)) break;
                dw *= dw_last == 0 ? 100.0 : 8.0;
                if (dw > 1e40) {   /* (not IPOPT's max_hessian_perturbation 1e20: DESIGN.md §2) */
                    fact_ok = 0;
                    break;
                }
            }
            dw_last = dw;
        }
        if (!fact_ok) {   /* regularisation exhausted: IPOPT's Error_In_Step_Computation, last iterate kept */
            status = -3;
            break;
        }
        memcpy(dU, rhs, sizeof(double) * n);
        cholsolve(L, n, dU);
        for (int i = 0; i < m; ++i) {
            double a = rc[i];
            for (int j = 0; j < n; ++j) a += J[i * n + j] * dU[j];
            dS[i] = a;
            dZl[i] = hl[i] ? mu / dl[i] - zl[i] - zl[i] / dl[i] * dS[i] : 0.0;
            dZu[i] = hu[i] ? mu / du[i] - zu[i] + zu[i] / du[i] * dS[i] : 0.0;
        }
        double ap = 1.0, az = 1.0;
        for (int i = 0; i < m; ++i) {
            if (hl[i] && dS[i] < 0) ap = fmin(ap, -tau * dl[i] / dS[i]);
            if (hu[i] && dS[i] > 0) ap = fmin(ap, tau * du[i] / dS[i]);
        }
        for (int i = 0; i < m; ++i) {
            if (hl[i] && dZl[i] < 0) az = fmin(az, -tau * zl[i] / dZl[i]);
            if (hu[i] && dZu[i] < 0) az = fmin(az, -tau * zu[i] / dZu[i]);
        }
        /* filter line search */
        double theta = 0;
        for (int i = 0; i < m; ++i) theta += fabs(rc[i]);
        double phi = barrier(f, s, cl, cu, m, mu);
        double gphi = 0, sl = 0, su = 0;
        for (int j = 0; j < n; ++j) gphi += gf[j] * dU[j];
        for (int i = 0; i < m; ++i) {
            if (hl[i]) sl += dS[i] / dl[i];
            if (hu[i]) su += dS[i] / du[i];
        }
        gphi -= mu * (sl - su);
        double amin;
        if (gphi < 0) {
            amin = fmin(gth, gph * theta / -gphi);
            if (theta <= theta_min) amin = fmin(amin, pow(theta, sth) / pow(-gphi, sph));
        } else
            amin = gth;
        amin *= gal;
        /* floor 2^-60 where the formula gives 0 (theta = 0 exactly): a trial sequence ap 2^-j
           never falls below 0; a positive amin, however small, is IPOPT's own */
        if (!(amin > 0.0)) amin = 8.673617379884035e-19;
        double a = ap;
        int accepted = 0, ftype = 0;
        while (a >= amin) {
            for (int j = 0; j < n; ++j) ut[j] = u[j] + a * dU[j];
            for (int i = 0; i < m; ++i) st[i] = s[i] + a * dS[i];
            pcons(P, ut, ct);
            double ftv = pobj(P, ut);
            double tht = 0;
            for (int i = 0; i < m; ++i) tht += fabs(ct[i] - st[i]);
            double pht = barrier(ftv, st, cl, cu, m, mu);
            int ok = isfinite(pht) && tht < theta_max;
            for (int q = 0; ok && q < nf; ++q)
                if (!(tht < ft[2 * q] || pht < ft[2 * q + 1])) ok = 0;
            if (ok) {
                int switching = gphi < 0 && a * pow(-gphi, sph) > pow(theta, sth);
                if (switching && theta <= theta_min) {
                    if (pht <= phi + eta * a * gphi) {
                        accepted = 1;
                        ftype = 1;
                    }
                } else if (tht <= (1 - gth) * theta || pht <= phi - gph * theta) {
                    accepted = 1;
                    ftype = 0;
                }
            }
            if (accepted) break;
            a *= 0.5;
        }
        if (accepted) {
            if (!ftype && nf < maxf) {
                ft[2 * nf] = (1 - gth) * theta;
                ft[2 * nf + 1] = phi - gph * theta;
                nf++;
            }
            memcpy(u, ut, sizeof(double) * n);
            memcpy(s, st, sizeof(double) * m);
            memcpy(c, ct, sizeof(double) * m);
        } else if (cfg->restoration == ALIPMPC_RESTORATION_IPOPT && !P->dd) {
            /* IPOPT: the current point enters the filter, then the restoration phase takes over (oresto) */
            n_rest++;
            if (nf < maxf) {
                ft[2 * nf] = (1 - gth) * theta;
                ft[2 * nf + 1] = phi - gph * theta;
                nf++;
            }
            it++;
            const int rs = oresto(P, u, s, zl, zu, mu, cl, cu, hl, hu, ft, nf, theta, &it, cfg->max_iter, cfg->tol);
            pcons(P, u, c);
            if (rs == RS_INFEASIBLE || rs == RS_FAILED) {
                status = 2;
                break;
            }
            if (rs == RS_MAXITER) break;
            for (int i = 0; i < m; ++i) {
                if (hl[i]) {
                    double d = s[i] - cl[i];
                    zl[i] = fmin(fmax(zl[i], mu / (1e10 * d)), 1e10 * mu / d);
                } else
                    zl[i] = 0;
                if (hu[i]) {
                    double d = cu[i] - s[i];
                    zu[i] = fmin(fmax(zu[i], mu / (1e10 * d)), 1e10 * mu / d);
                } else
                    zu[i] = 0;
            }
            continue;
        } else {
            n_rest++;
            a = fmax(a, amin);
            for (int j = 0; j < n; ++j) u[j] += a * dU[j];
            pcons(P, u, c);
            push_slacks(c, cl, cu, m, s);
            nf = 0;
            double viol = 0;
            for (int i = 0; i < m; ++i) {
                if (hl[i]) viol = fmax(viol, P->cl[i] - c[i]);
                if (hu[i]) viol = fmax(viol, c[i] - P->cu[i]);
            }
            if (n_rest >= REST_FAIL && viol > 1e-4) {
                status = 2;
                it++;
                break;
            }
        }
        for (int i = 0; i < m; ++i) {
            zl[i] += az * dZl[i];
            zu[i] += az * dZu[i];
            if (hl[i]) {
                double d = s[i] - cl[i];
                zl[i] = fmin(fmax(zl[i], mu / (1e10 * d)), 1e10 * mu / d);
            } else
                zl[i] = 0;
            if (hu[i]) {
                double d = cu[i] - s[i];
                zu[i] = fmin(fmax(zu[i], mu / (1e10 * d)), 1e10 * mu / d);
            } else
                zu[i] = 0;
        }
#undef ERR
        ++it;
    }
    free(ft);
    if (status != 0 && status != 2 && status != -3 && status != ALIPMPC_INVALID_NUMBER_DETECTED) {
        pcons(P, u, c);
        double viol = 0;
        for (int i = 0; i < m; ++i) {
            if (hl[i]) viol = fmax(viol, P->cl[i] - c[i]);
            if (hu[i]) viol = fmax(viol, c[i] - P->cu[i]);
        }
        if (e0 <= cfg->acceptable_tol)
            status = 1;
        else if (viol > 1e-4)
            status = 2;
    }
    if (P->dd)
        memcpy(uout, u, sizeof(double) * n);
    else
        u_of_p(P, u, uout);
    info->iters = it;
    info->status = status;
    info->restorations = n_rest;
}

/* ------------------------------------------------------------------------------------------------ */
/* batch entry points (same argument meaning as alipmpc_solve_batch / alipmpc_eval_batch, host memory) */
int oracle_rows_per_step(const alipmpc_cfg* cfg)
{
    if (cfg->variant == ALIPMPC_VARIANT_DD) return cfg->nc_max + cfg->ne_max + 1;
    return 4 + cfg->nc_max + cfg->ne_max + (cfg->variant == ALIPMPC_VARIANT_MODI);
}

int oracle_solve_batch(const alipmpc_cfg* cfg, int64_t B, const double* x0, const double* goal, const int8_t* leg,
                       const double* cir, const int32_t* nc, const double* elp, const int32_t* ne, const double* u0,
                       double* u_out, double* foot_out, double* x_pred, int32_t* status, int32_t* iters,
                       int32_t* restorations, int nthreads)
{
    if (cfg->variant == ALIPMPC_VARIANT_DD || cfg->N < 1 || cfg->N > OMAXN) return ALIPMPC_EUNSUPPORTED;
    oconsts* K = (oconsts*)malloc(sizeof(oconsts));
    oracle_consts(cfg, K);
    const int n = 5 * cfg->N;
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t b = 0; b < B; ++b) {
        oprob* P = (oprob*)malloc(sizeof(oprob));
        oprob_init(P, cfg, K, x0 + 5 * b, goal + 2 * b, leg[b], cir + (size_t)3 * cfg->nc_max * b, nc[b],
                   elp ? elp + (size_t)5 * cfg->ne_max * b : NULL, ne ? ne[b] : 0, 1);
        double u[OMAXV];
        osolve_info info;
        osolve(P, u0 + (size_t)n * b, u, &info);
        if (u_out) memcpy(u_out + (size_t)n * b, u, sizeof(double) * n);
        double X[OMAXN + 1][5], Pp[OMAXN][3];
        rollout(P, u, X, Pp);
        if (foot_out) memcpy(foot_out + 3 * b, Pp[0], 3 * sizeof(double));
        if (x_pred)
            for (int k = 0; k < cfg->N; ++k) memcpy(x_pred + ((size_t)b * cfg->N + k) * 5, X[k + 1], 5 * sizeof(double));
        if (status) status[b] = info.status;
        if (iters) iters[b] = info.iters;
        if (restorations) restorations[b] = info.restorations;
        free(P);
    }
    free(K);
    return 0;
}

int oracle_eval_batch(const alipmpc_cfg* cfg, int64_t B, const double* x0, const double* goal, const int8_t* leg,
                      const double* cir, const int32_t* nc, const double* elp, const int32_t* ne, const double* u,
                      double* f, double* grad, double* c, double* J, double* cl, double* cu, double* goal_eff,
                      int8_t* row_active)
{
    if (cfg->variant == ALIPMPC_VARIANT_DD || cfg->N < 1 || cfg->N > OMAXN) return ALIPMPC_EUNSUPPORTED;
    oconsts* K = (oconsts*)malloc(sizeof(oconsts));
    oracle_consts(cfg, K);
    const int n = 5 * cfg->N;
    const int rps = oracle_rows_per_step(cfg), mmax = cfg->N * rps;
    oprob* P = (oprob*)malloc(sizeof(oprob));
    double* Jc = (double*)malloc(sizeof(double) * OMAXM * OMAXV);
    double cc[OMAXM];
    for (int64_t b = 0; b < B; ++b) {
        oprob_init(P, cfg, K, x0 + 5 * b, goal + 2 * b, leg[b], cir + (size_t)3 * cfg->nc_max * b, nc[b],
                   elp ? elp + (size_t)5 * cfg->ne_max * b : NULL, ne ? ne[b] : 0, 0);
        const double* ub = u + (size_t)n * b;
        if (f) f[b] = oracle_objective(P, ub);
        if (grad) gradient(P, ub, grad + (size_t)n * b);
        constraints(P, ub, cc);
        jacobian(P, ub, Jc);
        /* scatter compact rows into the padded layout */
        for (int k = 0; k < cfg->N; ++k) {
            int src = k * P->rpk, dst = k * rps;
            int map[5 + 2 * OMAXO];
            int q = 0;
            map[q++] = dst + 0;
            map[q++] = dst + 1;
            for (int j = 0; j < P->nc; ++j) map[q++] = dst + 2 + j;
            for (int j = 0; j < P->ne; ++j) map[q++] = dst + 2 + cfg->nc_max + j;
            map[q++] = dst + 2 + cfg->nc_max + cfg->ne_max;
            map[q++] = dst + 3 + cfg->nc_max + cfg->ne_max;
            if (P->modi) map[q++] = dst + 4 + cfg->nc_max + cfg->ne_max;
            for (int r = dst; r < dst + rps; ++r) {
                if (c) c[(size_t)b * mmax + r] = 0;
                if (J)
                    for (int j = 0; j < n; ++j) J[((size_t)b * mmax + r) * n + j] = 0;
                if (cl) cl[(size_t)b * mmax + r] = -INFINITY;
                if (cu) cu[(size_t)b * mmax + r] = INFINITY;
                if (row_active) row_active[(size_t)b * mmax + r] = 0;
            }
            for (int t = 0; t < q; ++t) {
                int r = map[t];
                if (c) c[(size_t)b * mmax + r] = cc[src + t];
                if (J) memcpy(J + ((size_t)b * mmax + r) * n, Jc + (size_t)(src + t) * n, sizeof(double) * n);
                if (cl) cl[(size_t)b * mmax + r] = P->cl[src + t];
                if (cu) cu[(size_t)b * mmax + r] = P->cu[src + t];
                if (row_active) row_active[(size_t)b * mmax + r] = 1;
            }
        }
        if (goal_eff) {
            goal_eff[2 * b] = P->goal[0];
            goal_eff[2 * b + 1] = P->goal[1];
        }
    }
    free(Jc);
    free(P);
    free(K);
    return 0;
}

/* DD batch entry points: x0 B x 3, u0/u B x 2N, last_u B x 2; foot_out = first control [v, w, 0];
 * x_pred = x_1..x_N (B x N x 3) */
int oracle_solve_batch_dd(const alipmpc_cfg* cfg, int64_t B, const double* x0, const double* goal, const double* cir,
                          const int32_t* nc, const double* elp, const int32_t* ne, const double* u0,
                          const double* last_u, double* u_out, double* foot_out, double* x_pred, int32_t* status,
                          int32_t* iters, int32_t* restorations, int nthreads)
{
    if (cfg->variant != ALIPMPC_VARIANT_DD || cfg->N < 1 || cfg->N > OMAXN) return ALIPMPC_EUNSUPPORTED;
    const int n = 2 * cfg->N;
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t b = 0; b < B; ++b) {
        oprob* P = (oprob*)malloc(sizeof(oprob));
        oprob_init_dd(P, cfg, x0 + 3 * b, goal + 2 * b, cir + (size_t)3 * cfg->nc_max * b, nc[b],
                      elp ? elp + (size_t)5 * cfg->ne_max * b : NULL, ne ? ne[b] : 0, last_u ? last_u + 2 * b : NULL,
                      1);
        double u[OMAXV];
        osolve_info info;
        osolve(P, u0 + (size_t)n * b, u, &info);
        if (u_out) memcpy(u_out + (size_t)n * b, u, sizeof(double) * n);
        double X[OMAXN + 1][3];
        dd_rollout(P, u, X);
        if (foot_out) {
            foot_out[3 * b] = u[0];
            foot_out[3 * b + 1] = u[1];
            foot_out[3 * b + 2] = 0.0;
        }
        if (x_pred)
            for (int k = 0; k < cfg->N; ++k) memcpy(x_pred + ((size_t)b * cfg->N + k) * 3, X[k + 1], 3 * sizeof(double));
        if (status) status[b] = info.status;
        if (iters) iters[b] = info.iters;
        if (restorations) restorations[b] = info.restorations;
        free(P);
    }
    return 0;
}

/* reference DD callbacks in the padded layout [circle slots nc_max, ellipse slots ne_max, f_en] per step */
int oracle_eval_batch_dd(const alipmpc_cfg* cfg, int64_t B, const double* x0, const double* goal, const double* cir,
                         const int32_t* nc, const double* elp, const int32_t* ne, const double* u,
                         const double* last_u, double* f, double* grad, double* c, double* J, double* cl, double* cu,
                         int8_t* row_active)
{
    if (cfg->variant != ALIPMPC_VARIANT_DD || cfg->N < 1 || cfg->N > OMAXN) return ALIPMPC_EUNSUPPORTED;
    const int n = 2 * cfg->N;
    const int rps = cfg->nc_max + cfg->ne_max + 1, mmax = cfg->N * rps;
    oprob* P = (oprob*)malloc(sizeof(oprob));
    double* Jc = (double*)malloc(sizeof(double) * OMAXM * OMAXV);
    double cc[OMAXM];
    for (int64_t b = 0; b < B; ++b) {
        oprob_init_dd(P, cfg, x0 + 3 * b, goal + 2 * b, cir + (size_t)3 * cfg->nc_max * b, nc[b],
                      elp ? elp + (size_t)5 * cfg->ne_max * b : NULL, ne ? ne[b] : 0, last_u ? last_u + 2 * b : NULL,
                      0);
        const double* ub = u + (size_t)n * b;
        if (f) f[b] = dd_objective(P, ub);
        if (grad) dd_gradient(P, ub, grad + (size_t)n * b);
        dd_constraints(P, ub, cc);
        dd_jacobian(P, ub, Jc);
        for (int k = 0; k < cfg->N; ++k) {
            int src = k * P->rpk, dst = k * rps;
            int map[1 + 2 * OMAXO];
            int q = 0;
            for (int j = 0; j < P->nc; ++j) map[q++] = dst + j;
            for (int j = 0; j < P->ne; ++j) map[q++] = dst + cfg->nc_max + j;
            map[q++] = dst + cfg->nc_max + cfg->ne_max;
            for (int r = dst; r < dst + rps; ++r) {
                if (c) c[(size_t)b * mmax + r] = 0;
                if (J)
                    for (int j = 0; j < n; ++j) J[((size_t)b * mmax + r) * n + j] = 0;
                if (cl) cl[(size_t)b * mmax + r] = -INFINITY;
                if (cu) cu[(size_t)b * mmax + r] = INFINITY;
                if (row_active) row_active[(size_t)b * mmax + r] = 0;
            }
            for (int t = 0; t < q; ++t) {
                int r = map[t];
                if (c) c[(size_t)b * mmax + r] = cc[src + t];
                if (J) memcpy(J + ((size_t)b * mmax + r) * n, Jc + (size_t)(src + t) * n, sizeof(double) * n);
                if (cl) cl[(size_t)b * mmax + r] = P->cl[src + t];
                if (cu) cu[(size_t)b * mmax + r] = P->cu[src + t];
                if (row_active) row_active[(size_t)b * mmax + r] = 1;
            }
        }
    }
    free(Jc);
    free(P);
    return 0;
}

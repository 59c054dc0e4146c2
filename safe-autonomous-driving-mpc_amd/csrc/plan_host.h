// plan_host.h — host backend of libmpcplan (plan_create(..., device = -1, ...)): the planner's chunk solve in
// IEEE double on the CPU, std::thread workers over the chunks (PLAN_CPU_THREADS, default: every hardware thread).
//
// Product code (not test infrastructure): it restates the same chunk algorithm as the HIP kernel (DESIGN.md,
// "Offline planner"; plan_kernel.h) in plain sequential C++ -- Gauss-Newton / exact-Hessian SQP over
// z = [X, U, S] from the reference's initial guess (trajectory_planning.py:357-376), an L1-merit line search,
// each QP by an active-set crossover, else a Mehrotra interior point on the stage-wise Riccati recursion and
// the equality-constrained polish -- and performs oracle/plan_oracle.c's sequence of IEEE operations, so
// tests/test_plan_host.py finds the two bit-identical.  It does not include, link or call the oracle.  The
// reference's planner is CPU code (scipy SLSQP, :381-387); this is the library's CPU path of the same C ABI.
#pragma once
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/mpcplan.h"

namespace plan_host {


#define NZ 8                  /* stage variables: x (s, d, o, k, v), w (u1, u2, S) */
#define NR 11                 /* rows per stage at most */
#define MAXNP (PLAN_MAX_N + 1)
#define NZMAX (5 * (PLAN_MAX_N + 1) + 3 * PLAN_MAX_N)
#define RHO 1e8               /* penalty of the active rows in the equality-constrained solve */
#define AL_STEPS 4            /* refinement + multiplier updates of that solve */
#define AL_TOL 1e-13        /* stop the refinements once the multiplier update is at rounding level */
#define POLISH_ROUNDS 6
#define WARM_ROUNDS 5         /* active-set rounds from the previous QP's classification before the interior point */
#define MU_CHECK 1e-4         /* interior-point checkpoint: a polish is tried once mu and phi are below this ... */
#define CHECK_SEP 100.0       /* ... and every row's s and lambda differ by this factor (no near-tie to classify) */
#define CHECK_ROUNDS 2        /* polish rounds at the checkpoint (the interior point resumes if they fail) */
#define SHIFT0 1.0            /* interior-point start: s = max(row, 0) + SHIFT0, lambda = 1 */
#define TAU 0.995
#define CYCLE_REL 1e-6
#define DELTA0 1e-6           /* first Hessian regularisation when a pivot fails; x10 per retry */
#define DELTA_MAX 1e4
#define EXACT_STEP 0.1        /* exact Lagrangian Hessian once the last SQP step is at most this (max norm) ... */
#define EXACT_AFTER 20        /* ... or from this SQP iteration on (a Gauss-Newton SQP can zigzag with steps of ~0.2
                                 around an active lateral-acceleration row without ever meeting EXACT_STEP) */
#define LS_ARMIJO 1e-4        /* line search on the L1 merit f + mu * violation: sufficient decrease */
#define LS_STEPS 12           /* halvings at most (the last one is taken regardless) */
#define LS_FULL 1e-3          /* steps at most this long (max norm) are taken whole (local phase) */
#define LS_MEMORY 4           /* non-monotone line search: decrease against the largest of the last merits */

inline void default_params(plan_params* p) {
    memset(p, 0, sizeof(*p));
    p->N = 20;
    p->dt = 0.3;                                           /* trajectory_planning.py:514 */
    p->w_y = 10.0; p->w_s = 10.0; p->w_u = 0.1; p->w_slack = 100.0;   /* :14 */
    p->u_min[0] = -0.6; p->u_min[1] = -5.0;                /* :35-36 */
    p->u_max[0] = 0.6; p->u_max[1] = 4.0;
    p->k_min = -0.8; p->k_max = 0.8;                       /* :43-44 */
    p->a_max = 6.0;                                        /* :47 */
    p->v_min = 0.0;                                        /* :476-477 */
    p->defect_sign = 1.0;
    p->sqp_iters = 100;
    p->sqp_tol = 1e-9;
    p->max_iter = 100;
    p->tol = 1e-10;
}

/* ------------------------------------------------------------------------------------------------ */
/* route: k_ref_fun and v_max_fun of optimize_full_trajectory (trajectory_planning.py:437-477)       */
/* ------------------------------------------------------------------------------------------------ */
struct route {
    int M;
    double *s, *cx, *cy, *vmax;
};

inline int route_create(const double* s, int M, const double* cx, const double* cy, const double* vmax,
                     route** out) {
    if (!s || !cx || !cy || !vmax || !out || M < 2) return PLAN_E_ARG;
    for (int i = 1; i < M; ++i)
        if (!(s[i] > s[i - 1])) return PLAN_E_ARG;
    route* r = (route*)calloc(1, sizeof(route));
    r->M = M;
    r->s = (double*)malloc(sizeof(double) * M);
    r->vmax = (double*)malloc(sizeof(double) * M);
    r->cx = (double*)malloc(sizeof(double) * 4 * (M - 1));
    r->cy = (double*)malloc(sizeof(double) * 4 * (M - 1));
    memcpy(r->s, s, sizeof(double) * M);
    memcpy(r->vmax, vmax, sizeof(double) * M);
    memcpy(r->cx, cx, sizeof(double) * 4 * (M - 1));
    memcpy(r->cy, cy, sizeof(double) * 4 * (M - 1));
    *out = r;
    return PLAN_SUCCESS;
}

inline void route_destroy(route* r) {
    if (!r) return;
    free(r->s); free(r->cx); free(r->cy); free(r->vmax);
    free(r);
}

inline double route_s_total(const route* r) { return r->s[r->M - 1]; }

/* first index i with s[i] >= v (numpy searchsorted side='left') */
static int lower_bound(const double* x, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int m = (lo + hi) >> 1;
        if (x[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

/* first index i with s[i] > v (side='right') */
static int upper_bound(const double* x, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int m = (lo + hi) >> 1;
        if (x[m] <= v) lo = m + 1; else hi = m;
    }
    return lo;
}

/* k_ref_fun (:445-459): t = s_to_t(s) (interp1d linear, extrapolated, :440-442: searchsorted left, index
 * clipped to [1, M-1]); curvature of the CubicSpline pair at t (PPoly: interval floor(t) clipped to
 * [0, M-2]); first and second derivatives in s on the same pieces (t is linear in s there). */
static double route_kappa(const route* r, double s, double* dkds, double* d2kds2) {
    const int M = r->M;
    int i = lower_bound(r->s, M, s);
    if (i < 1) i = 1;
    if (i > M - 1) i = M - 1;
    const double slope = 1.0 / (r->s[i] - r->s[i - 1]);
    const double t = slope * (s - r->s[i - 1]) + (double)(i - 1);
    int j = (int)floor(t);
    if (j < 0) j = 0;
    if (j > M - 2) j = M - 2;
    const double tau = t - (double)j;
    const double* a = r->cx + 4 * j;
    const double* b = r->cy + 4 * j;
    const double x1 = (3.0 * a[0] * tau + 2.0 * a[1]) * tau + a[2], x2 = 6.0 * a[0] * tau + 2.0 * a[1], x3 = 6.0 * a[0];
    const double y1 = (3.0 * b[0] * tau + 2.0 * b[1]) * tau + b[2], y2 = 6.0 * b[0] * tau + 2.0 * b[1], y3 = 6.0 * b[0];
    const double num = x1 * y2 - y1 * x2;
    const double q = x1 * x1 + y1 * y1;
    const double sq = sqrt(q);
    double den = q * sq + 1e-9;
    const int clamp = den < 1e-8;
    if (clamp) den = 1e-8;
    const double k = num / den;
    if (dkds) {
        const double dnum = x1 * y3 - y1 * x3;
        const double dden = clamp ? 0.0 : 3.0 * sq * (x1 * x2 + y1 * y2);
        const double kt = (dnum - k * dden) / den;
        *dkds = kt * slope;
        if (d2kds2) {
            /* num'' = x2 y3 - y2 x3 (cubic pieces); den'' = 3/4 q^-1/2 q'^2 + 3/2 q^1/2 q'' */
            const double d2num = x2 * y3 - y2 * x3;
            const double qd = 2.0 * (x1 * x2 + y1 * y2), qdd = 2.0 * (x2 * x2 + x1 * x3 + y2 * y2 + y1 * y3);
            const double d2den = (clamp || sq == 0.0) ? 0.0 : 0.75 * qd * qd / sq + 1.5 * sq * qdd;
            *d2kds2 = (d2num - 2.0 * kt * dden - k * d2den) / den * slope * slope;
        }
    }
    return k;
}

inline double route_kappa_at(const route* r, double s, double* dkds) { return route_kappa(r, s, dkds, NULL); }

/* v_max_fun (:470-473): interp1d kind='previous' (below the first knot: the first limit, see mpcplan.h) */
inline double route_vmax_at(const route* r, double s) {
    const int i = upper_bound(r->s, r->M, s);
    return r->vmax[i > 0 ? i - 1 : 0];
}

/* ------------------------------------------------------------------------------------------------ */
/* the NLP's functions and derivatives                                                                */
/* ------------------------------------------------------------------------------------------------ */
static double guard_den(double den) {       /* :74-77 */
    if (fabs(den) < 1e-4) den = den > 0.0 ? 1e-4 : (den < 0.0 ? -1e-4 : 1e-4);
    return den;
}

/* TrajectoryOptimizer.dynamics (:50-89) */
inline void dynamics(const double x[5], double u1, double u2, double kref, double f[5]) {
    const double den = guard_den(1.0 - x[1] * kref);
    const double sd = (x[4] * cos(x[2])) / den;
    f[0] = sd;
    f[1] = x[4] * sin(x[2]);
    f[2] = x[4] * x[3] - sd * kref;
    f[3] = u1;
    f[4] = u2;
}

/* d f / d x with kappa = kappa(s): F row-major 5x5 (d f / d u = e3, e4 for u1, u2) */
static void dyn_jac(const double x[5], double kref, double dk, double F[25]) {
    const double d = x[1], o = x[2], k = x[3], v = x[4];
    const double raw = 1.0 - d * kref;
    const int guarded = fabs(raw) < 1e-4;
    const double den = guard_den(raw);
    const double c = cos(o), sn = sin(o);
    const double sd = v * c / den;
    double ds[5];
    ds[0] = guarded ? 0.0 : v * c * d * dk / (den * den);
    ds[1] = guarded ? 0.0 : v * c * kref / (den * den);
    ds[2] = -v * sn / den;
    ds[3] = 0.0;
    ds[4] = c / den;
    memset(F, 0, sizeof(double) * 25);
    for (int j = 0; j < 5; ++j) {
        F[j] = ds[j];
        F[10 + j] = -kref * ds[j];
    }
    F[5 + 2] = v * c;
    F[5 + 4] = sn;
    F[10 + 0] += -dk * sd;
    F[10 + 3] += v;
    F[10 + 4] += k;
}

/* W = sum_i y_i d2 f_i / dx2 at x, kappa = kappa(s) with derivatives k1, k2 (f3, f4 are linear) */
static void hess_f(const double x[5], double kr, double k1, double k2, const double y[5], double W[25]) {
    const double d = x[1], o = x[2], v = x[4];
    const double raw = 1.0 - d * kr;
    const int gu = fabs(raw) < 1e-4;
    const double g = 1.0 / guard_den(raw);
    const double c = cos(o), sn = sin(o);
    /* g = 1 / (1 - d kappa(s)) and its derivatives (constant when guarded) */
    const double gs = gu ? 0.0 : d * k1 * g * g, gd = gu ? 0.0 : kr * g * g;
    const double gss = gu ? 0.0 : d * k2 * g * g + 2.0 * d * d * k1 * k1 * g * g * g;
    const double gsd = gu ? 0.0 : k1 * g * g + 2.0 * d * k1 * kr * g * g * g;
    const double gdd = gu ? 0.0 : 2.0 * kr * kr * g * g * g;
    double Hs[25], ds[5];
    memset(Hs, 0, sizeof(Hs));
    /* s_dot = v cos(o) g */
    Hs[0] = v * c * gss;
    Hs[1] = Hs[5] = v * c * gsd;
    Hs[6] = v * c * gdd;
    Hs[2] = Hs[10] = -v * sn * gs;
    Hs[7] = Hs[11] = -v * sn * gd;
    Hs[12] = -v * c * g;
    Hs[4] = Hs[20] = c * gs;
    Hs[9] = Hs[21] = c * gd;
    Hs[14] = Hs[22] = -sn * g;
    ds[0] = v * c * gs; ds[1] = v * c * gd; ds[2] = -v * sn * g; ds[3] = 0.0; ds[4] = c * g;
    const double sd = v * c * g;
    for (int i = 0; i < 25; ++i) W[i] = (y[0] - y[2] * kr) * Hs[i];
    /* f1 = v sin(o) */
    W[12] += -y[1] * v * sn;
    W[14] += y[1] * c;
    W[22] += y[1] * c;
    /* f2 = v k - s_dot kappa(s): the v k term, and -(grad s_dot x grad kappa + transpose + s_dot kappa'') */
    W[19] += y[2];
    W[23] += y[2];
    for (int j = 0; j < 5; ++j) {
        W[j] += -y[2] * k1 * ds[j];
        W[5 * j] += -y[2] * k1 * ds[j];
    }
    W[0] += -y[2] * sd * k2;
}

/* Hermite-Simpson defect of interval k (:183-208): x_{k+1} - (x_k + sign * dt/6 (f_k + 4 f_mid + f_{k+1})) */
inline void defect(const route* r, const plan_params* p, const double xa[5], const double xb[5], double u1,
                     double u2, double def[5]) {
    const double h = p->dt;
    double fa[5], fb[5], fm[5], xm[5];
    dynamics(xa, u1, u2, route_kappa_at(r, xa[0], NULL), fa);
    dynamics(xb, u1, u2, route_kappa_at(r, xb[0], NULL), fb);
    for (int i = 0; i < 5; ++i) xm[i] = 0.5 * (xa[i] + xb[i]) + (h / 8.0) * (fa[i] - fb[i]);
    dynamics(xm, u1, u2, route_kappa_at(r, xm[0], NULL), fm);
    for (int i = 0; i < 5; ++i) def[i] = xb[i] - (xa[i] + p->defect_sign * (h / 6.0) * (fa[i] + 4.0 * fm[i] + fb[i]));
}

/* TrajectoryOptimizer.cost (:128-170) */
inline double cost(const route* r, const plan_params* p, int N, const double x0[5], const double* X,
                     const double* U, const double* S) {
    const double st = route_s_total(r);
    const double den = fmax(1.0, st - x0[0]);
    double c = 0.0;
    for (int k = 0; k < N; ++k) {
        const double* x = X + 5 * k;
        const double t1 = p->w_y * (x[1] * x[1] + x[2] * x[2]);
        const double e = (st - x[0]) / den;
        const double t2 = p->w_s * e * e;
        const double t3 = p->w_u * (U[2 * k] * U[2 * k] + U[2 * k + 1] * U[2 * k + 1]);
        const double t4 = p->w_slack * (S[k] * S[k]);
        c += t1 + t2 + t3 + t4;
    }
    return c;
}

/* ------------------------------------------------------------------------------------------------ */
/* the stage QP                                                                                       */
/* ------------------------------------------------------------------------------------------------ */
enum { ROW_VMIN, ROW_VMAX, ROW_LATP, ROW_LATM, ROW_KMIN, ROW_KMAX, ROW_U1MIN, ROW_U1MAX, ROW_U2MIN, ROW_U2MAX,
       ROW_S, ROW_STERM };

typedef struct {
    int N, fin;
    double delta;                                         /* Hessian regularisation of this QP (0 unless needed) */
    double A[MAXNP][25], B[MAXNP][15], c[MAXNP][5];      /* k < N: dx' = A dx + B dw + c (B: 5x3, S col 0) */
    double D1[MAXNP][25];                                 /* d def_k / d x_{k+1} (multiplier recovery) */
    double H[MAXNP][NZ][NZ], gq[MAXNP][NZ];               /* stage Hessian and gradient of the QP objective */
    int nr[MAXNP];
    unsigned char kind[MAXNP][NR];
    double a[MAXNP][NR][NZ], g[MAXNP][NR];                /* rows: g + a . (dx_k, dw_k) >= 0 */
    double xi0[5];                                        /* dx_0 = x0 - xbar_0 */
    double e[2];                                          /* final chunk: E dx_N = e, E = rows s, v */
} qp_t;

typedef struct {
    double K[MAXNP][15], L[MAXNP][6];                     /* dw = K dx + kk ; Hww = L L' */
    double ez[2][MAXNP][NZ];                              /* final chunk: responses to the terminal forces */
    double Em[2][2];
} fac_t;

typedef struct {
    double z[MAXNP][NZ];                                  /* QP variable (dx_k, dw_k) */
    double s[MAXNP][NR], lam[MAXNP][NR];
    double nu[2];                                         /* final chunk: terminal multipliers (last solve) */
    unsigned char act[MAXNP][NR];
} qpsol_t;

typedef struct {                                          /* NLP multipliers for the next QP's Hessian */
    double y[MAXNP][5];                                   /* defects (Lagrangian f - y.def - lam.g) */
    double lat[MAXNP][2];                                 /* lateral-acceleration rows (+, -) */
} mult_t;

/* Gaussian elimination with partial pivoting: Mx X = rhs (5 x ncol, row-major), in place; Mx destroyed */
static int solve5(double Mx[25], double* rhs, int ncol) {
    for (int c = 0; c < 5; ++c) {
        int pr = c;
        for (int i = c + 1; i < 5; ++i)
            if (fabs(Mx[5 * i + c]) > fabs(Mx[5 * pr + c])) pr = i;
        if (Mx[5 * pr + c] == 0.0) return -1;
        if (pr != c) {
            for (int j = 0; j < 5; ++j) { const double t = Mx[5 * c + j]; Mx[5 * c + j] = Mx[5 * pr + j]; Mx[5 * pr + j] = t; }
            for (int j = 0; j < ncol; ++j) { const double t = rhs[ncol * c + j]; rhs[ncol * c + j] = rhs[ncol * pr + j]; rhs[ncol * pr + j] = t; }
        }
        for (int i = c + 1; i < 5; ++i) {
            const double f = Mx[5 * i + c] / Mx[5 * c + c];
            for (int j = c; j < 5; ++j) Mx[5 * i + j] -= f * Mx[5 * c + j];
            for (int j = 0; j < ncol; ++j) rhs[ncol * i + j] -= f * rhs[ncol * c + j];
        }
    }
    for (int c = 4; c >= 0; --c)
        for (int j = 0; j < ncol; ++j) {
            double v = rhs[ncol * c + j];
            for (int k = c + 1; k < 5; ++k) v -= Mx[5 * c + k] * rhs[ncol * k + j];
            rhs[ncol * c + j] = v / Mx[5 * c + c];
        }
    return 0;
}

/* linearisation of interval k's defect at (xa, xb, u): dx_{k+1} = A dx_k + B dw + c; D1 = d def / d x_{k+1} */
static int interval_lin(const route* r, const plan_params* p, const double xa[5], const double xb[5], double u1,
                        double u2, double A[25], double B[15], double c[5], double D1o[25]) {
    const double h = p->dt, sg = p->defect_sign;
    double dka, dkb, dkm, fa[5], fb[5], fm[5], xm[5], Fa[25], Fb[25], Fm[25];
    const double ka = route_kappa(r, xa[0], &dka, NULL);
    const double kb = route_kappa(r, xb[0], &dkb, NULL);
    dynamics(xa, u1, u2, ka, fa);
    dynamics(xb, u1, u2, kb, fb);
    for (int i = 0; i < 5; ++i) xm[i] = 0.5 * (xa[i] + xb[i]) + (h / 8.0) * (fa[i] - fb[i]);
    const double km = route_kappa(r, xm[0], &dkm, NULL);
    dynamics(xm, u1, u2, km, fm);
    double def[5];
    for (int i = 0; i < 5; ++i) def[i] = xb[i] - (xa[i] + sg * (h / 6.0) * (fa[i] + 4.0 * fm[i] + fb[i]));
    dyn_jac(xa, ka, dka, Fa);
    dyn_jac(xb, kb, dkb, Fb);
    dyn_jac(xm, km, dkm, Fm);
    /* D0 = -I - sg h/6 (Fa + 4 Fm (I/2 + h/8 Fa)); D1 = I - sg h/6 (4 Fm (I/2 - h/8 Fb) + Fb); Du = -sg h G */
    double D0[25], D1[25];
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            double m0 = 0.0, m1 = 0.0;
            for (int l = 0; l < 5; ++l) {
                const double ia = (l == j ? 0.5 : 0.0) + (h / 8.0) * Fa[5 * l + j];
                const double ib = (l == j ? 0.5 : 0.0) - (h / 8.0) * Fb[5 * l + j];
                m0 += Fm[5 * i + l] * ia;
                m1 += Fm[5 * i + l] * ib;
            }
            D0[5 * i + j] = (i == j ? -1.0 : 0.0) - sg * (h / 6.0) * (Fa[5 * i + j] + 4.0 * m0);
            D1[5 * i + j] = (i == j ? 1.0 : 0.0) - sg * (h / 6.0) * (4.0 * m1 + Fb[5 * i + j]);
        }
    memcpy(D1o, D1, sizeof(D1));
    /* rhs = [-D0 | -Du | -def] = [-D0 | sg h e3, sg h e4 | -def] */
    double R[5 * 8];
    for (int i = 0; i < 5; ++i) {
        for (int j = 0; j < 5; ++j) R[8 * i + j] = -D0[5 * i + j];
        R[8 * i + 5] = i == 3 ? sg * h : 0.0;
        R[8 * i + 6] = i == 4 ? sg * h : 0.0;
        R[8 * i + 7] = -def[i];
    }
    if (solve5(D1, R, 8)) return -1;
    for (int i = 0; i < 5; ++i) {
        for (int j = 0; j < 5; ++j) A[5 * i + j] = R[8 * i + j];
        B[3 * i + 0] = R[8 * i + 5];
        B[3 * i + 1] = R[8 * i + 6];
        B[3 * i + 2] = 0.0;
        c[i] = R[8 * i + 7];
    }
    return 0;
}

/* curvature of -y . def_k (the defect's share of the Lagrangian Hessian) over (x_a, x_b): blocks aa, ab, bb.
 * d2(y.f_mid) = Jm' W_m Jm + h/8 (V_a (+) -V_b), Jm = [I/2 + h/8 F_a, I/2 - h/8 F_b] (x_mid does not
 * depend on u), W = sum y_i d2 f_i, V = sum (F_m' y)_l d2 f_l. */
static void interval_hess(const route* r, const plan_params* p, const double xa[5], const double xb[5], double u1,
                          double u2, const double y[5], double Haa[25], double Hab[25], double Hbb[25]) {
    const double h = p->dt, f6 = p->defect_sign * h / 6.0;
    double k1a, k2a, k1b, k2b, k1m, k2m, fa[5], fb[5], fm[5], xm[5], Fa[25], Fb[25], Fm[25];
    const double ka = route_kappa(r, xa[0], &k1a, &k2a);
    const double kb = route_kappa(r, xb[0], &k1b, &k2b);
    dynamics(xa, u1, u2, ka, fa);
    dynamics(xb, u1, u2, kb, fb);
    for (int i = 0; i < 5; ++i) xm[i] = 0.5 * (xa[i] + xb[i]) + (h / 8.0) * (fa[i] - fb[i]);
    const double km = route_kappa(r, xm[0], &k1m, &k2m);
    dynamics(xm, u1, u2, km, fm);
    dyn_jac(xa, ka, k1a, Fa);
    dyn_jac(xb, kb, k1b, Fb);
    dyn_jac(xm, km, k1m, Fm);
    double Wa[25], Wb[25], Wm[25], Va[25], Vb[25], yb[5], Ma[25], Mb[25], WMa[25], WMb[25];
    for (int j = 0; j < 5; ++j) {
        double v = 0.0;
        for (int i = 0; i < 5; ++i) v += Fm[5 * i + j] * y[i];
        yb[j] = v;
    }
    hess_f(xa, ka, k1a, k2a, y, Wa);
    hess_f(xb, kb, k1b, k2b, y, Wb);
    hess_f(xm, km, k1m, k2m, y, Wm);
    hess_f(xa, ka, k1a, k2a, yb, Va);
    hess_f(xb, kb, k1b, k2b, yb, Vb);
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            Ma[5 * i + j] = (i == j ? 0.5 : 0.0) + (h / 8.0) * Fa[5 * i + j];
            Mb[5 * i + j] = (i == j ? 0.5 : 0.0) - (h / 8.0) * Fb[5 * i + j];
        }
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            double va = 0.0, vb = 0.0;
            for (int l = 0; l < 5; ++l) { va += Wm[5 * i + l] * Ma[5 * l + j]; vb += Wm[5 * i + l] * Mb[5 * l + j]; }
            WMa[5 * i + j] = va;
            WMb[5 * i + j] = vb;
        }
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            double aa = 0.0, ab = 0.0, bb = 0.0;
            for (int l = 0; l < 5; ++l) {
                aa += Ma[5 * l + i] * WMa[5 * l + j];
                ab += Ma[5 * l + i] * WMb[5 * l + j];
                bb += Mb[5 * l + i] * WMb[5 * l + j];
            }
            Haa[5 * i + j] = f6 * (Wa[5 * i + j] + 4.0 * (aa + (h / 8.0) * Va[5 * i + j]));
            Hab[5 * i + j] = f6 * (4.0 * ab);
            Hbb[5 * i + j] = f6 * (Wb[5 * i + j] + 4.0 * (bb - (h / 8.0) * Vb[5 * i + j]));
        }
}

/* fold a quadratic over (x_k, x_{k+1}) into stage k's (x_k, w_k) along x_{k+1} = A x_k + B w_k + c
 * (the same objective on the QP's feasible set): Hessian T' [Haa Hab; Hab' Hbb] T with T = [I 0; A B], and
 * the linear terms T' Hbb c + E' Hab c */
static void fold_interval(qp_t* Q, int k, const double Haa[25], const double Hab[25], const double Hbb[25]) {
    const double* A = Q->A[k];
    const double* B = Q->B[k];
    const double* c = Q->c[k];
    double T[5][NZ];
    for (int i = 0; i < 5; ++i) {
        for (int j = 0; j < 5; ++j) T[i][j] = A[5 * i + j];
        for (int j = 0; j < 3; ++j) T[i][5 + j] = B[3 * i + j];
    }
    double HbT[5][NZ], HabT[5][NZ];
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < NZ; ++j) {
            double vb = 0.0, va = 0.0;
            for (int l = 0; l < 5; ++l) { vb += Hbb[5 * i + l] * T[l][j]; va += Hab[5 * i + l] * T[l][j]; }
            HbT[i][j] = vb;
            HabT[i][j] = va;
        }
    for (int i = 0; i < NZ; ++i)
        for (int j = 0; j < NZ; ++j) {
            double v = 0.0;
            for (int l = 0; l < 5; ++l) v += T[l][i] * HbT[l][j];
            if (i < 5) v += HabT[i][j];
            if (j < 5) v += HabT[j][i];
            if (i < 5 && j < 5) v += Haa[5 * i + j];
            Q->H[k][i][j] += v;
        }
    double hbc[5];
    for (int l = 0; l < 5; ++l) {
        double v = 0.0;
        for (int m = 0; m < 5; ++m) v += Hbb[5 * l + m] * c[m];
        hbc[l] = v;
    }
    for (int i = 0; i < NZ; ++i) {
        double v = 0.0;
        for (int l = 0; l < 5; ++l) v += T[l][i] * hbc[l];
        if (i < 5)
            for (int m = 0; m < 5; ++m) v += Hab[5 * i + m] * c[m];
        Q->gq[k][i] += v;
    }
}

#define ADDROW(kd, ...)                                                                                    \
    do {                                                                                                   \
        const double cf_[NZ] = {__VA_ARGS__};                                                              \
        memcpy(Q->a[k][n], cf_, sizeof(cf_));                                                              \
        Q->g[k][n] = gv;                                                                                   \
        Q->kind[k][n] = (kd);                                                                              \
        ++n;                                                                                               \
    } while (0)

/* the QP at the SQP iterate (Xb, Ub, Sb); vlim: frozen speed limits or NULL; M: multipliers for the exact
 * Lagrangian Hessian or NULL (the cost's Hessian).  Returns 0, or -1 when a defect Jacobian is singular. */
static int build_qp(const route* r, const plan_params* p, int N, const double x0[5], double s_target, int fin,
                    const double* Xb, const double* Ub, const double* Sb, const double* vlim, const mult_t* M,
                    qp_t* Q) {
    const double st = route_s_total(r);
    const double den = fmax(1.0, st - x0[0]);
    Q->N = N;
    Q->fin = fin;
    Q->delta = 0.0;
    for (int k = 0; k <= N; ++k) {
        const double* x = Xb + 5 * k;
        memset(Q->H[k], 0, sizeof(Q->H[k]));
        memset(Q->gq[k], 0, sizeof(Q->gq[k]));
        if (k < N) {
            Q->H[k][0][0] = 2.0 * p->w_s / (den * den);
            Q->H[k][1][1] = 2.0 * p->w_y;
            Q->H[k][2][2] = 2.0 * p->w_y;
            Q->H[k][5][5] = 2.0 * p->w_u;
            Q->H[k][6][6] = 2.0 * p->w_u;
            Q->H[k][7][7] = 2.0 * p->w_slack;
            Q->gq[k][0] = -2.0 * p->w_s * (st - x[0]) / (den * den);
            Q->gq[k][1] = 2.0 * p->w_y * x[1];
            Q->gq[k][2] = 2.0 * p->w_y * x[2];
            Q->gq[k][5] = 2.0 * p->w_u * Ub[2 * k];
            Q->gq[k][6] = 2.0 * p->w_u * Ub[2 * k + 1];
            Q->gq[k][7] = 2.0 * p->w_slack * Sb[k];
            if (interval_lin(r, p, x, Xb + 5 * (k + 1), Ub[2 * k], Ub[2 * k + 1], Q->A[k], Q->B[k], Q->c[k], Q->D1[k]))
                return -1;
            if (M) {
                double Haa[25], Hab[25], Hbb[25];
                interval_hess(r, p, x, Xb + 5 * (k + 1), Ub[2 * k], Ub[2 * k + 1], M->y[k], Haa, Hab, Hbb);
                fold_interval(Q, k, Haa, Hab, Hbb);
            }
        }
        const double sl = k < N ? Sb[k] : 0.0, hs = k < N ? 1.0 : 0.0;
        const double kk = x[3], v = x[4];
        int n = 0;
        double gv;
        if (!(fin && k == N)) {
            gv = v + sl - p->v_min;
            ADDROW(ROW_VMIN, 0, 0, 0, 0, 1.0, 0, 0, hs);                                  /* :251-259 */
            gv = (vlim ? vlim[k] : route_vmax_at(r, x[0])) - (v + sl);
            ADDROW(ROW_VMAX, 0, 0, 0, 0, -1.0, 0, 0, -hs);                                /* :263-271 */
            if (k > 0) {
                gv = p->a_max - kk * v * v;
                ADDROW(ROW_LATP, 0, 0, 0, -v * v, -2.0 * kk * v, 0, 0, 0);                /* :277-281 */
                gv = p->a_max + kk * v * v;
                ADDROW(ROW_LATM, 0, 0, 0, v * v, 2.0 * kk * v, 0, 0, 0);                  /* :285-289 */
                if (M) {
                    /* -lam d2 g over (k, v): g = a_max -+ k v^2 */
                    const double lp = M->lat[k][0], lm = M->lat[k][1];
                    Q->H[k][3][4] += 2.0 * v * (lp - lm);
                    Q->H[k][4][3] += 2.0 * v * (lp - lm);
                    Q->H[k][4][4] += 2.0 * kk * (lp - lm);
                }
            }
        }
        if (k > 0) {
            gv = kk - p->k_min;
            ADDROW(ROW_KMIN, 0, 0, 0, 1.0, 0, 0, 0, 0);                                   /* :296-299 */
            gv = p->k_max - kk;
            ADDROW(ROW_KMAX, 0, 0, 0, -1.0, 0, 0, 0, 0);                                  /* :303-306 */
        }
        if (k < N) {
            gv = Ub[2 * k] - p->u_min[0];
            ADDROW(ROW_U1MIN, 0, 0, 0, 0, 0, 1.0, 0, 0);                                  /* :313-316 */
            gv = p->u_max[0] - Ub[2 * k];
            ADDROW(ROW_U1MAX, 0, 0, 0, 0, 0, -1.0, 0, 0);                                 /* :320-323 */
            gv = Ub[2 * k + 1] - p->u_min[1];
            ADDROW(ROW_U2MIN, 0, 0, 0, 0, 0, 0, 1.0, 0);                                  /* :328-331 */
            gv = p->u_max[1] - Ub[2 * k + 1];
            ADDROW(ROW_U2MAX, 0, 0, 0, 0, 0, 0, -1.0, 0);                                 /* :335-338 */
            gv = Sb[k];
            ADDROW(ROW_S, 0, 0, 0, 0, 0, 0, 0, 1.0);                                      /* :343-345 */
        }
        if (k == N && !fin) {
            gv = x[0] - s_target / 2.0;
            ADDROW(ROW_STERM, 1.0, 0, 0, 0, 0, 0, 0, 0);                                  /* :241-244 */
        }
        Q->nr[k] = n;
    }
    for (int i = 0; i < 5; ++i) Q->xi0[i] = x0[i] - Xb[i];
    Q->e[0] = s_target - Xb[5 * N];          /* :223-226 */
    Q->e[1] = -Xb[5 * N + 4];                /* :231-234 */
    return 0;
}

/* stage Hessian (8x8) with row weights W, plus delta I */
static void stage_hess(const qp_t* Q, int k, const double* W, double H[NZ][NZ]) {
    memcpy(H, Q->H[k], sizeof(double) * NZ * NZ);
    const int nv = k < Q->N ? NZ : 5;
    for (int i = 0; i < nv; ++i) H[i][i] += Q->delta;
    for (int j = 0; j < Q->nr[k]; ++j) {
        const double* a = Q->a[k][j];
        if (W[j] == 0.0) continue;
        for (int u = 0; u < NZ; ++u) {
            if (a[u] == 0.0) continue;
            for (int v = 0; v < NZ; ++v) H[u][v] += W[j] * a[u] * a[v];
        }
    }
}

/* H (3 x 3, symmetric positive definite) = L D L' with L unit lower triangular, stored as {1/d0, l10, 1/d1,
 * l20, l21, 1/d2}: no square roots, three divisions per factorisation and none in the solves (the GPU kernel's
 * form and rounding).  Fails when a pivot is not positive, the Cholesky condition. */
static int chol3(const double H[3][3], double L[6]) {
    const double d0 = H[0][0];
    if (!(d0 > 0.0)) return -1;
    L[0] = 1.0 / d0;
    L[1] = H[1][0] * L[0];
    const double d1 = H[1][1] - L[1] * H[1][0];
    if (!(d1 > 0.0)) return -1;
    L[2] = 1.0 / d1;
    L[3] = H[2][0] * L[0];
    const double e21 = H[2][1] - L[3] * H[1][0];
    L[4] = e21 * L[2];
    const double d2 = H[2][2] - L[3] * H[2][0] - L[4] * e21;
    if (!(d2 > 0.0)) return -1;
    L[5] = 1.0 / d2;
    return 0;
}

/* b <- (L D L')^-1 b */
static void chol3_solve(const double L[6], double b[3]) {
    const double y0 = b[0];
    const double y1 = b[1] - L[1] * y0;
    const double y2 = b[2] - L[3] * y0 - L[4] * y1;
    b[2] = y2 * L[5];
    b[1] = y1 * L[2] - L[4] * b[2];
    b[0] = y0 * L[0] - L[1] * b[1] - L[3] * b[2];
}

static void solve_core(const qp_t* Q, const fac_t* F, const double gl[][NZ], double dz[][NZ]);

/* Riccati factorisation of the stage Hessians with row weights W[k][j] (and, for the final chunk, the
 * responses to the two terminal forces).  Returns -1 when a control pivot is not positive. */
static int factor(const qp_t* Q, const double W[][NR], fac_t* F) {
    const int N = Q->N;
    double H[NZ][NZ], P[25], PA[25], PB[15], Hww[3][3], Hwx[15];
    stage_hess(Q, N, W[N], H);
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) P[5 * i + j] = H[i][j];
    for (int k = N - 1; k >= 0; --k) {
        stage_hess(Q, k, W[k], H);
        const double* A = Q->A[k];
        const double* B = Q->B[k];
        for (int i = 0; i < 5; ++i) {
            for (int j = 0; j < 5; ++j) {
                double v = 0.0;
                for (int l = 0; l < 5; ++l) v = fma(P[5 * i + l], A[5 * l + j], v);
                PA[5 * i + j] = v;
            }
            for (int j = 0; j < 3; ++j) {
                double v = 0.0;
                for (int l = 0; l < 5; ++l) v = fma(P[5 * i + l], B[3 * l + j], v);
                PB[3 * i + j] = v;
            }
        }
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) {
                double v = H[5 + i][5 + j];
                for (int l = 0; l < 5; ++l) v = fma(B[3 * l + i], PB[3 * l + j], v);
                Hww[i][j] = v;
            }
            for (int j = 0; j < 5; ++j) {
                double v = H[5 + i][j];
                for (int l = 0; l < 5; ++l) v = fma(B[3 * l + i], PA[5 * l + j], v);
                Hwx[5 * i + j] = v;
            }
        }
        if (chol3((const double(*)[3])Hww, F->L[k])) return -1;
        for (int j = 0; j < 5; ++j) {
            double col[3] = {-Hwx[j], -Hwx[5 + j], -Hwx[10 + j]};
            chol3_solve(F->L[k], col);
            F->K[k][j] = col[0];
            F->K[k][5 + j] = col[1];
            F->K[k][10 + j] = col[2];
        }
        if (k > 0) {
            double Pn[25];
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) {
                    double v = H[i][j];
                    for (int l = 0; l < 5; ++l) v = fma(A[5 * l + i], PA[5 * l + j], v);
                    for (int l = 0; l < 3; ++l) v = fma(Hwx[5 * l + i], F->K[k][5 * l + j], v);
                    Pn[5 * i + j] = v;
                }
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) P[5 * i + j] = 0.5 * (Pn[5 * i + j] + Pn[5 * j + i]);
        }
    }
    if (Q->fin) {
        /* d z responses to unit forces on s_N and v_N (superposition, the terminal equalities) */
        static const int eidx[2] = {0, 4};
        double gl[MAXNP][NZ];
        for (int c = 0; c < 2; ++c) {
            memset(gl, 0, sizeof(double) * NZ * (N + 1));
            gl[N][eidx[c]] = 1.0;
            solve_core(Q, F, (const double(*)[NZ])gl, F->ez[c]);
        }
        for (int i = 0; i < 2; ++i)
            for (int c = 0; c < 2; ++c) F->Em[i][c] = F->ez[c][N][eidx[i]];
        const double det = F->Em[0][0] * F->Em[1][1] - F->Em[0][1] * F->Em[1][0];
        if (!(fabs(det) > 0.0) || !isfinite(det)) return -1;
    }
    return 0;
}

/* factorisation with the regularisation raised until the pivots are positive */
static int factor_reg(qp_t* Q, const double W[][NR], fac_t* F) {
    while (factor(Q, W, F)) {
        if (Q->delta >= DELTA_MAX) return -1;
        Q->delta = Q->delta > 0.0 ? 10.0 * Q->delta : DELTA0;
    }
    return 0;
}

/* LQ solve with zero initial state and homogeneous dynamics: stage linear terms gl[k] (x then w) */
static void solve_core(const qp_t* Q, const fac_t* F, const double gl[][NZ], double dz[][NZ]) {
    const int N = Q->N;
    double p[5], kk[MAXNP][3];
    for (int i = 0; i < 5; ++i) p[i] = gl[N][i];
    for (int k = N - 1; k >= 0; --k) {
        const double* A = Q->A[k];
        const double* B = Q->B[k];
        double h[3];
        for (int i = 0; i < 3; ++i) {
            double v = gl[k][5 + i];
            for (int l = 0; l < 5; ++l) v = fma(B[3 * l + i], p[l], v);
            h[i] = v;
        }
        double t[3] = {-h[0], -h[1], -h[2]};
        chol3_solve(F->L[k], t);
        kk[k][0] = t[0]; kk[k][1] = t[1]; kk[k][2] = t[2];
        if (k > 0) {
            double pn[5];
            for (int i = 0; i < 5; ++i) {
                double v = gl[k][i];
                for (int l = 0; l < 5; ++l) v = fma(A[5 * l + i], p[l], v);
                for (int l = 0; l < 3; ++l) v = fma(F->K[k][5 * l + i], h[l], v);
                pn[i] = v;
            }
            memcpy(p, pn, sizeof(p));
        }
    }
    double x[5] = {0, 0, 0, 0, 0};
    for (int k = 0; k < N; ++k) {
        double w[3];
        for (int i = 0; i < 3; ++i) {
            double v = kk[k][i];
            for (int l = 0; l < 5; ++l) v = fma(F->K[k][5 * i + l], x[l], v);
            w[i] = v;
        }
        for (int i = 0; i < 5; ++i) dz[k][i] = x[i];
        for (int i = 0; i < 3; ++i) dz[k][5 + i] = w[i];
        double xn[5];
        for (int i = 0; i < 5; ++i) {
            double v = 0.0;
            for (int l = 0; l < 5; ++l) v = fma(Q->A[k][5 * i + l], x[l], v);
            for (int l = 0; l < 3; ++l) v = fma(Q->B[k][3 * i + l], w[l], v);
            xn[i] = v;
        }
        memcpy(x, xn, sizeof(x));
    }
    for (int i = 0; i < 5; ++i) dz[N][i] = x[i];
    for (int i = 5; i < NZ; ++i) dz[N][i] = 0.0;
}

/* the full solve: also meets E dz_N = rE exactly (final chunk); nu = the terminal forces used */
static void solve(const qp_t* Q, const fac_t* F, const double gl[][NZ], const double rE[2], double dz[][NZ],
                  double nu[2]) {
    solve_core(Q, F, gl, dz);
    nu[0] = nu[1] = 0.0;
    if (!Q->fin) return;
    const int N = Q->N;
    const double b0 = rE[0] - dz[N][0], b1 = rE[1] - dz[N][4];
    const double det = F->Em[0][0] * F->Em[1][1] - F->Em[0][1] * F->Em[1][0];
    const double n0 = (b0 * F->Em[1][1] - F->Em[0][1] * b1) / det;
    const double n1 = (F->Em[0][0] * b1 - F->Em[1][0] * b0) / det;
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < NZ; ++i) dz[k][i] += n0 * F->ez[0][k][i] + n1 * F->ez[1][k][i];
    nu[0] = n0;
    nu[1] = n1;
}

static double row_val(const qp_t* Q, int k, int j, const double z[NZ]) {
    const double* a = Q->a[k][j];
    double v = Q->g[k][j];
    for (int u = 0; u < NZ; ++u) v += a[u] * z[u];
    return v;
}

/* dynamics-feasible start: dx_0 = xi0, dw = 0 (fused multiply-adds, the kernel's DPP recursion) */
static void rollout(const qp_t* Q, double z[][NZ]) {
    const int N = Q->N;
    memset(z, 0, sizeof(double) * NZ * (N + 1));
    for (int i = 0; i < 5; ++i) z[0][i] = Q->xi0[i];
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < 5; ++i) {
            double v = Q->c[k][i];
            for (int l = 0; l < 5; ++l) v = fma(Q->A[k][5 * i + l], z[k][l], v);
            z[k + 1][i] = v;
        }
}

/* gradient of the QP objective 1/2 z'(H + delta I)z + gq'z at stage k */
static void grad_f(const qp_t* Q, int k, const double z[NZ], double g[NZ]) {
    const int nv = k < Q->N ? NZ : 5;
    for (int i = 0; i < NZ; ++i) {
        double v = Q->gq[k][i] + (i < nv ? Q->delta * z[i] : 0.0);
        for (int j = 0; j < NZ; ++j) v += Q->H[k][i][j] * z[j];
        g[i] = i < nv ? v : 0.0;
    }
}

static int finite_z(const qp_t* Q, const double z[][NZ]) {
    for (int k = 0; k <= Q->N; ++k)
        for (int i = 0; i < NZ; ++i)
            if (!isfinite(z[k][i])) return 0;
    return 1;
}

/* equality-constrained QP on the rows marked active (act), by penalty RHO and multiplier updates from the
 * estimates lam (active rows); on return z, lam hold the solution and its multipliers, nu the terminal
 * ones.  KKT-consistent (active multipliers >= 0, inactive rows satisfied): returns 0; otherwise the number
 * of offending rows, whose classification is flipped in act; -1 on a breakdown. */
static int eqp(qp_t* Q, unsigned char act[][NR], double z[][NZ], double lam[][NR], double nu[2], double scale) {
    static thread_local fac_t F;
    static thread_local double W[MAXNP][NR], gl[MAXNP][NZ], dz[MAXNP][NZ], y[MAXNP][NR];
    const int N = Q->N;
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < Q->nr[k]; ++j) {
            W[k][j] = act[k][j] ? RHO : 0.0;
            y[k][j] = act[k][j] ? lam[k][j] : 0.0;
        }
    if (factor_reg(Q, (const double(*)[NR])W, &F)) return -1;
    rollout(Q, z);
    for (int it = 0; it < AL_STEPS; ++it) {
        for (int k = 0; k <= N; ++k) {
            grad_f(Q, k, z[k], gl[k]);
            for (int j = 0; j < Q->nr[k]; ++j) {
                if (!act[k][j]) continue;
                const double f = RHO * row_val(Q, k, j, z[k]) - y[k][j];
                for (int u = 0; u < NZ; ++u) gl[k][u] += f * Q->a[k][j][u];
            }
        }
        const double rE[2] = {Q->e[0] - z[N][0], Q->e[1] - z[N][4]};
        solve(Q, &F, (const double(*)[NZ])gl, rE, dz, nu);
        for (int k = 0; k <= N; ++k)
            for (int u = 0; u < NZ; ++u) z[k][u] += dz[k][u];
        double upd = 0.0, ym = 0.0;
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < Q->nr[k]; ++j)
                if (act[k][j]) {
                    const double d = RHO * row_val(Q, k, j, z[k]);
                    y[k][j] -= d;
                    upd = fmax(upd, fabs(d));
                    ym = fmax(ym, fabs(y[k][j]));
                }
        /* the multiplier update has reached rounding level: further refinements change nothing */
        if (upd <= AL_TOL * (1.0 + ym)) break;
    }
    if (!finite_z(Q, (const double(*)[NZ])z)) return -1;
    int bad = 0;
    const double tr = 1e-9 * scale, tl = 1e-9 * scale;
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < Q->nr[k]; ++j) {
            const double rv = row_val(Q, k, j, z[k]);
            if (act[k][j]) {
                lam[k][j] = y[k][j];
                if (y[k][j] < -tl || fabs(rv) > tr) { act[k][j] = 0; ++bad; }
            } else {
                lam[k][j] = 0.0;
                if (rv < -tr) { act[k][j] = 1; ++bad; }
            }
        }
    return bad;
}

/* Mehrotra predictor-corrector interior point on the QP; returns 0 converged, 1 iteration cap, -1 breakdown,
 * 2 checkpoint (first call only: mu and phi below MU_CHECK with every row's s and lambda CHECK_SEP apart).
 * resume = 1 continues from X, *iters and *phi_io. */
static int ipm(qp_t* Q, const plan_params* p, qpsol_t* X, int* iters, int resume, double* phi_io) {
    static thread_local fac_t F;
    static thread_local double W[MAXNP][NR], gl[MAXNP][NZ], dz[MAXNP][NZ], dsa[MAXNP][NR], dla[MAXNP][NR],
        rp[MAXNP][NR], ds[MAXNP][NR], dl[MAXNP][NR];
    const int N = Q->N;
    int m = 0;
    if (!resume) rollout(Q, X->z);
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < Q->nr[k]; ++j) {
            if (!resume) {
                const double rv = row_val(Q, k, j, X->z[k]);
                X->s[k][j] = (rv > 0.0 ? rv : 0.0) + SHIFT0;
                X->lam[k][j] = 1.0;
            }
            ++m;
        }
    double phi = resume ? *phi_io : 1.0;
    int it = resume ? *iters : 0, rc = 1;
    for (; it < p->max_iter; ++it) {
        double mu = 0.0;
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < Q->nr[k]; ++j) {
                rp[k][j] = row_val(Q, k, j, X->z[k]) - X->s[k][j];
                mu += X->s[k][j] * X->lam[k][j];
            }
        mu /= m;
        if (!isfinite(mu)) { rc = -1; break; }
        if (mu <= p->tol && phi <= 1e-12) { rc = 0; break; }
        if (!resume && mu <= MU_CHECK && phi <= MU_CHECK) {
            int tie = 0;
            for (int k = 0; k <= N; ++k)
                for (int j = 0; j < Q->nr[k]; ++j) {
                    const double s = X->s[k][j], l = X->lam[k][j];
                    if (!(s > CHECK_SEP * l || l > CHECK_SEP * s)) tie = 1;
                }
            if (!tie) { rc = 2; break; }
        }
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < Q->nr[k]; ++j) W[k][j] = X->lam[k][j] / X->s[k][j];
        if (factor_reg(Q, (const double(*)[NR])W, &F)) { rc = -1; break; }
        const double rE[2] = {Q->e[0] - X->z[N][0], Q->e[1] - X->z[N][4]};
        for (int pass = 0; pass < 2; ++pass) {
            double sigma_mu = 0.0;
            if (pass == 1) {
                /* sigma = (mu_aff / mu)^3 from the affine step */
                double am = 1.0;
                for (int k = 0; k <= N; ++k)
                    for (int j = 0; j < Q->nr[k]; ++j) {
                        if (dsa[k][j] < 0.0) am = fmin(am, -X->s[k][j] / dsa[k][j]);
                        if (dla[k][j] < 0.0) am = fmin(am, -X->lam[k][j] / dla[k][j]);
                    }
                double mua = 0.0;
                for (int k = 0; k <= N; ++k)
                    for (int j = 0; j < Q->nr[k]; ++j)
                        mua += (X->s[k][j] + am * dsa[k][j]) * (X->lam[k][j] + am * dla[k][j]);
                mua /= m;
                const double ratio = mua / mu;
                sigma_mu = ratio * ratio * ratio * mu;
            }
            for (int k = 0; k <= N; ++k) {
                grad_f(Q, k, X->z[k], gl[k]);
                for (int j = 0; j < Q->nr[k]; ++j) {
                    const double s = X->s[k][j], l = X->lam[k][j];
                    double rs = -s * l;
                    if (pass == 1) rs += sigma_mu - dsa[k][j] * dla[k][j];
                    const double f = l + (rs - l * rp[k][j]) / s;
                    for (int u = 0; u < NZ; ++u) gl[k][u] -= f * Q->a[k][j][u];
                }
            }
            solve(Q, &F, (const double(*)[NZ])gl, rE, dz, X->nu);
            double (*DS)[NR] = pass == 0 ? dsa : ds;
            double (*DL)[NR] = pass == 0 ? dla : dl;
            for (int k = 0; k <= N; ++k)
                for (int j = 0; j < Q->nr[k]; ++j) {
                    const double s = X->s[k][j], l = X->lam[k][j];
                    double rs = -s * l;
                    if (pass == 1) rs += sigma_mu - dsa[k][j] * dla[k][j];
                    double v = rp[k][j];
                    for (int u = 0; u < NZ; ++u) v += Q->a[k][j][u] * dz[k][u];
                    DS[k][j] = v;
                    DL[k][j] = (rs - l * v) / s;
                }
        }
        double amax = 1.0 / TAU;
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < Q->nr[k]; ++j) {
                if (ds[k][j] < 0.0) amax = fmin(amax, -X->s[k][j] / ds[k][j]);
                if (dl[k][j] < 0.0) amax = fmin(amax, -X->lam[k][j] / dl[k][j]);
            }
        const double alpha = fmin(1.0, TAU * amax);
        if (!isfinite(alpha) || !finite_z(Q, (const double(*)[NZ])dz)) { rc = -1; break; }
        for (int k = 0; k <= N; ++k) {
            for (int u = 0; u < NZ; ++u) X->z[k][u] += alpha * dz[k][u];
            for (int j = 0; j < Q->nr[k]; ++j) {
                X->s[k][j] += alpha * ds[k][j];
                X->lam[k][j] += alpha * dl[k][j];
            }
        }
        phi *= 1.0 - alpha;
    }
    *iters = it;
    *phi_io = phi;
    return rc;
}

/* one QP: active-set rounds from the previous classification (when given), else interior point + polish.
 * Returns 0 solved (exact KKT point), 1 interior-point answer without a certified polish, -1 failure. */
/* diagnostics (PLAN_TRACE=1 in the environment, tools/plan_trace.py): how the last QP was solved -- 'W' warm
 * active-set rounds (qp_path_n = rounds), 'C' checkpoint polish, 'P' polish after the interior point, 'I' the
 * interior point's answer uncertified, 'F' failure */
static thread_local char qp_path;
static thread_local int qp_path_n;
static int plan_trace(void) { return getenv("PLAN_TRACE") != NULL; }

static int qp_solve(qp_t* Q, const plan_params* p, qpsol_t* X, int have_cls, int* iters) {
    static thread_local unsigned char act[MAXNP][NR];
    static thread_local double z[MAXNP][NZ], lam[MAXNP][NR];
    const int N = Q->N;
    double scale = 1.0, nu[2];
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < Q->nr[k]; ++j) scale = fmax(scale, fabs(Q->g[k][j]));
    *iters = 0;
    if (have_cls) {
        memcpy(act, X->act, sizeof(act));
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < Q->nr[k]; ++j) lam[k][j] = X->lam[k][j];
        /* each round corrects the rows that contradict the classification (eqp), so a set that moved by a
         * few rows since the last QP is recovered in a few equality solves instead of a cold interior point */
        for (int round = 0; round < WARM_ROUNDS; ++round) {
            const int bad = eqp(Q, act, z, lam, nu, scale);
            if (bad < 0) break;
            if (bad == 0) {
                memcpy(X->z, z, sizeof(double) * NZ * (N + 1));
                memcpy(X->lam, lam, sizeof(lam));
                memcpy(X->act, act, sizeof(act));
                X->nu[0] = nu[0];
                X->nu[1] = nu[1];
                qp_path = 'W';
                qp_path_n = round + 1;
                return 0;
            }
        }
    }
    double phi = 1.0;
    int rc = ipm(Q, p, X, iters, 0, &phi);
    if (rc == 2) {
        /* checkpoint: the loose interior point's classification (no near-ties) is often already the
         * optimum's, which the polish then certifies exactly; otherwise the interior point resumes */
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < Q->nr[k]; ++j) {
                act[k][j] = X->s[k][j] < X->lam[k][j];
                lam[k][j] = X->lam[k][j];
            }
        for (int round = 0; round < CHECK_ROUNDS; ++round) {
            const int bad = eqp(Q, act, z, lam, nu, scale);
            if (bad < 0) break;
            if (bad == 0) {
                memcpy(X->z, z, sizeof(double) * NZ * (N + 1));
                memcpy(X->lam, lam, sizeof(lam));
                memcpy(X->act, act, sizeof(act));
                X->nu[0] = nu[0];
                X->nu[1] = nu[1];
                qp_path = 'C';
                qp_path_n = round + 1;
                return 0;
            }
        }
        rc = ipm(Q, p, X, iters, 1, &phi);
    }
    qp_path = 'F';
    qp_path_n = 0;
    if (rc < 0) return -1;
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < Q->nr[k]; ++j) {
            act[k][j] = X->s[k][j] < X->lam[k][j];
            lam[k][j] = X->lam[k][j];
        }
    for (int round = 0; round < POLISH_ROUNDS; ++round) {
        const int bad = eqp(Q, act, z, lam, nu, scale);
        if (bad < 0) break;
        if (bad == 0) {
            memcpy(X->z, z, sizeof(double) * NZ * (N + 1));
            memcpy(X->lam, lam, sizeof(lam));
            memcpy(X->act, act, sizeof(act));
            X->nu[0] = nu[0];
            X->nu[1] = nu[1];
            return 0;
        }
    }
    /* keep the interior-point answer; its classification seeds the next crossover */
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < Q->nr[k]; ++j) X->act[k][j] = X->s[k][j] < X->lam[k][j];
    return rc == 0 ? 1 : -1;
}

/* NLP multiplier estimates from a QP solution: rows' lam, and the defects' y_k = D1_k^-T pi_{k+1} with the
 * co-states pi (the cost-to-go gradients, pi_N = grad_N + E' nu, pi_k = grad_k + A_k' pi_{k+1}, where
 * grad = gradient of the QP objective minus sum lam a, x part) */
static void multipliers(const qp_t* Q, const qpsol_t* X, mult_t* M) {
    const int N = Q->N;
    double g[NZ], pi[5];
    memset(M, 0, sizeof(*M));
    for (int k = N; k >= 0; --k) {
        grad_f(Q, k, X->z[k], g);
        for (int j = 0; j < Q->nr[k]; ++j) {
            for (int u = 0; u < NZ; ++u) g[u] -= X->lam[k][j] * Q->a[k][j][u];
            if (Q->kind[k][j] == ROW_LATP) M->lat[k][0] = X->lam[k][j];
            if (Q->kind[k][j] == ROW_LATM) M->lat[k][1] = X->lam[k][j];
        }
        if (k == N) {
            for (int i = 0; i < 5; ++i) pi[i] = g[i];
            if (Q->fin) {
                pi[0] += X->nu[0];
                pi[4] += X->nu[1];
            }
            continue;
        }
        double D1t[25], y[5];
        for (int i = 0; i < 5; ++i)
            for (int j = 0; j < 5; ++j) D1t[5 * i + j] = Q->D1[k][5 * j + i];
        memcpy(y, pi, sizeof(y));
        if (solve5(D1t, y, 1) == 0) memcpy(M->y[k], y, sizeof(y));
        if (k > 0) {
            double pn[5];
            for (int i = 0; i < 5; ++i) {
                double v = g[i];
                for (int l = 0; l < 5; ++l) v = fma(Q->A[k][5 * l + i], pi[l], v);
                pn[i] = v;
            }
            memcpy(pi, pn, sizeof(pi));
        }
    }
}

/* L1 violation of the reference's constraints at z (defects, x_0 = x0, the rows with the speed limits vl of
 * the current linearisation, the final chunk's terminal equalities) */
static double violation(const route* r, const plan_params* p, int N, const double x0[5], double s_target, int fin,
                        const double* z, const double* vl) {
    const double* X = z;
    const double* U = z + 5 * (N + 1);
    const double* S = U + 2 * N;
    double v = 0.0, def[5];
    for (int i = 0; i < 5; ++i) v += fabs(X[i] - x0[i]);
    for (int k = 0; k < N; ++k) {
        defect(r, p, X + 5 * k, X + 5 * (k + 1), U[2 * k], U[2 * k + 1], def);
        for (int i = 0; i < 5; ++i) v += fabs(def[i]);
    }
    for (int k = 0; k <= N; ++k) {
        const double kk = X[5 * k + 3], vv = X[5 * k + 4], sl = k < N ? S[k] : 0.0;
        double g[12];
        int n = 0;
        if (!(fin && k == N)) {
            g[n++] = vv + sl - p->v_min;
            g[n++] = vl[k] - (vv + sl);
            if (k > 0) {
                g[n++] = p->a_max - kk * vv * vv;
                g[n++] = p->a_max + kk * vv * vv;
            }
        }
        if (k > 0) {
            g[n++] = kk - p->k_min;
            g[n++] = p->k_max - kk;
        }
        if (k < N) {
            g[n++] = U[2 * k] - p->u_min[0];
            g[n++] = p->u_max[0] - U[2 * k];
            g[n++] = U[2 * k + 1] - p->u_min[1];
            g[n++] = p->u_max[1] - U[2 * k + 1];
            g[n++] = S[k];
        }
        if (k == N && !fin) g[n++] = X[5 * N] - s_target / 2.0;
        for (int j = 0; j < n; ++j) v += g[j] < 0.0 ? -g[j] : 0.0;
    }
    if (fin) v += fabs(X[5 * N] - s_target) + fabs(X[5 * N + 4]);
    return v;
}

/* directional derivative of the cost at z along dz */
static double cost_dir(const route* r, const plan_params* p, int N, const double x0[5], const double* z,
                       const double* dz) {
    const double st = route_s_total(r);
    const double den = fmax(1.0, st - x0[0]);
    const double *X = z, *dX = dz, *U = z + 5 * (N + 1), *dU = dz + 5 * (N + 1), *S = U + 2 * N, *dS = dU + 2 * N;
    double v = 0.0;
    for (int k = 0; k < N; ++k) {
        v += 2.0 * p->w_y * (X[5 * k + 1] * dX[5 * k + 1] + X[5 * k + 2] * dX[5 * k + 2]);
        v += -2.0 * p->w_s * (st - X[5 * k]) / (den * den) * dX[5 * k];
        v += 2.0 * p->w_u * (U[2 * k] * dU[2 * k] + U[2 * k + 1] * dU[2 * k + 1]);
        v += 2.0 * p->w_slack * S[k] * dS[k];
    }
    return v;
}

inline int chunk(const route* r, const plan_params* p, int N, const double x0[5], double s_target,
                   int is_final, double* X, double* U, double* S, int* iters, int* sqp) {
    static thread_local qp_t Q;
    static thread_local qpsol_t sol;
    static thread_local mult_t mult;
    if (N < 1 || N > PLAN_MAX_N) return PLAN_NUMERICAL;
    const int nz = 5 * (N + 1) + 3 * N;
    double zb[NZMAX], z2[NZMAX], znew[NZMAX], dzv[NZMAX], vlim[MAXNP], vl[MAXNP], mu_m = 0.0;
    double hf[LS_MEMORY], hv[LS_MEMORY];
    int nh = 0;
    double* Xb = zb;
    double* Ub = zb + 5 * (N + 1);
    double* Sb = Ub + 2 * N;
    /* initial guess (:357-376) */
    memset(zb, 0, sizeof(double) * nz);
    const double ds = (s_target - x0[0]) / N;
    for (int k = 0; k <= N; ++k) {
        Xb[5 * k] = k == N ? s_target : x0[0] + k * ds;
        Xb[5 * k + 4] = is_final ? (k == N ? 0.0 : x0[4] + k * ((0.0 - x0[4]) / N)) : x0[4];
    }
    memcpy(z2, zb, sizeof(double) * nz);
    int status = PLAN_NOT_CONVERGED, total = 0, nq = 0, have_cls = 0, frozen = 0, since = 0;
    double last = INFINITY;
    for (int it = 0; it < p->sqp_iters; ++it, ++since) {
        int exact = last <= EXACT_STEP || it >= EXACT_AFTER, rc = -1;
        const int tot0 = total;
        for (;;) {
            if (build_qp(r, p, N, x0, s_target, is_final, Xb, Ub, Sb, frozen ? vlim : NULL, exact ? &mult : NULL, &Q)) {
                rc = -2;
                break;
            }
            int ni = 0;
            rc = qp_solve(&Q, p, &sol, have_cls, &ni);
            total += ni;
            if (rc >= 0 || !exact) break;
            exact = 0;                    /* the exact-Hessian QP failed: this QP with the cost's Hessian */
        }
        ++nq;
        if (rc == -2) { status = PLAN_NUMERICAL; break; }
        if (rc < 0) { status = PLAN_QP_FAILED; break; }
        have_cls = 1;
        multipliers(&Q, &sol, &mult);
        /* the QP step in z's layout */
        for (int k = 0; k <= N; ++k) {
            for (int i = 0; i < 5; ++i) dzv[5 * k + i] = sol.z[k][i];
            if (k < N) {
                dzv[5 * (N + 1) + 2 * k] = sol.z[k][5];
                dzv[5 * (N + 1) + 2 * k + 1] = sol.z[k][6];
                dzv[5 * (N + 1) + 2 * N + k] = sol.z[k][7];
            }
        }
        double full = 0.0;
        for (int i = 0; i < nz; ++i) full = fmax(full, fabs(dzv[i]));
        /* merit line search (L1 exact penalty), mu above the multipliers' magnitude */
        for (int k = 0; k <= N; ++k) {
            for (int i = 0; i < 5 && k < N; ++i) mu_m = fmax(mu_m, 2.0 * fabs(mult.y[k][i]));
            for (int j = 0; j < Q.nr[k]; ++j) mu_m = fmax(mu_m, 2.0 * fabs(sol.lam[k][j]));
        }
        if (is_final) mu_m = fmax(mu_m, 2.0 * fmax(fabs(sol.nu[0]), fabs(sol.nu[1])));
        double alpha = 1.0;
        if (full > LS_FULL) {
            for (int k = 0; k <= N; ++k) vl[k] = frozen ? vlim[k] : route_vmax_at(r, Xb[5 * k]);
            const double v0 = violation(r, p, N, x0, s_target, is_final, zb, vl);
            const double f0 = cost(r, p, N, x0, Xb, Ub, Sb);
            const double dd = cost_dir(r, p, N, x0, zb, dzv) - mu_m * v0;
            hf[nh % LS_MEMORY] = f0;
            hv[nh % LS_MEMORY] = v0;
            ++nh;
            double m0 = -INFINITY;
            for (int i = 0; i < (nh < LS_MEMORY ? nh : LS_MEMORY); ++i) m0 = fmax(m0, hf[i] + mu_m * hv[i]);
            for (int ls = 0; ls < LS_STEPS; ++ls) {
                for (int i = 0; i < nz; ++i) znew[i] = zb[i] + alpha * dzv[i];
                const double m1 = cost(r, p, N, x0, znew, znew + 5 * (N + 1), znew + 5 * (N + 1) + 2 * N) +
                                  mu_m * violation(r, p, N, x0, s_target, is_final, znew, vl);
                if (m1 <= m0 + LS_ARMIJO * alpha * dd || ls == LS_STEPS - 1) break;
                alpha *= 0.5;
            }
        }
        double step = 0.0, back2 = 0.0;
        int fin = 1;
        for (int i = 0; i < nz; ++i) {
            znew[i] = zb[i] + alpha * dzv[i];
            step = fmax(step, fabs(znew[i] - zb[i]));
            back2 = fmax(back2, fabs(znew[i] - z2[i]));
            fin &= isfinite(znew[i]);
        }
        if (!fin) { status = PLAN_NUMERICAL; break; }
        if (plan_trace()) {
            int nact = 0, nchg = 0;
            static thread_local unsigned char prev[MAXNP][NR];
            for (int k = 0; k <= N; ++k)
                for (int j = 0; j < Q.nr[k]; ++j) {
                    nact += sol.act[k][j];
                    nchg += it > 0 && sol.act[k][j] != prev[k][j];
                    prev[k][j] = sol.act[k][j];
                }
            fprintf(stderr, "sqp %3d %s qp %c%d ipm %4d act %3d chg %3d |dz| %.3e alpha %.4g step %.3e back2 %.3e "
                    "frozen %d delta %.1e\n", it, exact ? "exact" : "gn   ", qp_path, qp_path_n, total - tot0, nact, nchg, full, alpha,
                    step, back2, frozen, Q.delta);
        }
        memcpy(z2, zb, sizeof(double) * nz);
        memcpy(zb, znew, sizeof(double) * nz);
        last = step;
        if (step <= p->sqp_tol) { status = frozen ? PLAN_FROZEN_LIMITS : PLAN_OK; break; }
        if (since >= 2 && back2 <= CYCLE_REL * step) {             /* 2-cycle */
            if (frozen) break;
            for (int k = 0; k <= N; ++k)
                vlim[k] = fmin(route_vmax_at(r, zb[5 * k]), route_vmax_at(r, z2[5 * k]));
            frozen = 1;
            since = -1;
            memcpy(z2, zb, sizeof(double) * nz);
        }
    }
    if (status == PLAN_FROZEN_LIMITS) {
        /* the frozen answer must satisfy the reference's own speed rows at its positions */
        for (int k = 0; k <= N; ++k)
            if (Xb[5 * k + 4] + (k < N ? Sb[k] : 0.0) > route_vmax_at(r, Xb[5 * k]) + 1e-9) status = PLAN_NOT_CONVERGED;
    }
    if (X) memcpy(X, Xb, sizeof(double) * 5 * (N + 1));
    if (U) memcpy(U, Ub, sizeof(double) * 2 * N);
    if (S) memcpy(S, Sb, sizeof(double) * N);
    if (iters) *iters = total;
    if (sqp) *sqp = nq;
    return status;
}

// B chunks (the layout of plan_solve_chunks: row stride Nmax, the largest horizon; rows past a chunk's
// horizon zero), dynamic chunks of 4 over `threads` workers
inline void batch(const route* r, const plan_params* p, int B, int Nmax, const int* N, const double* x0,
                  const double* s_target, const int* is_final, double* X, double* U, double* S, int* status,
                  int* iters, int* sqp, int threads) {
    std::atomic<int> next(0);
    auto work = [&]() {
        for (;;) {
            const int b0 = next.fetch_add(4);
            if (b0 >= B) return;
            for (int b = b0; b < std::min(B, b0 + 4); ++b) {
                const int n = N ? N[b] : p->N;
                double* Xo = X ? X + (size_t)b * 5 * (Nmax + 1) : nullptr;
                double* Uo = U ? U + (size_t)b * 2 * Nmax : nullptr;
                double* So = S ? S + (size_t)b * Nmax : nullptr;
                if (Xo) memset(Xo, 0, sizeof(double) * 5 * (Nmax + 1));
                if (Uo) memset(Uo, 0, sizeof(double) * 2 * Nmax);
                if (So) memset(So, 0, sizeof(double) * Nmax);
                int it = 0, nq = 0;
                const int st = chunk(r, p, n, x0 + 5 * (size_t)b, s_target[b], is_final ? is_final[b] : 0, Xo, Uo, So,
                                     &it, &nq);
                if (status) status[b] = st;
                if (iters) iters[b] = it;
                if (sqp) sqp[b] = nq;
            }
        }
    };
    threads = std::max(1, std::min(threads, (B + 3) / 4));
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
}

// optimize_full_trajectory's receding-horizon chunk loop (trajectory_planning.py:478-559) for B plans, each on
// one worker: the loop of plan_loop_kernel (plan_kernel.h) with this file's chunk solve
inline void optimize(const route* r, const plan_params* p0, int B, int Nmax, const double* starts,
                     double max_chunk_size, int max_chunks, const double* avg, int nav, double* X, double* U, double* S,
                     int* N, int* is_final, int* status, int* iters, int* sqp, int* nchunks, int threads) {
    std::atomic<int> next(0);
    const double s_total = route_s_total(r);
    auto work = [&]() {
        std::vector<double> Xb(5 * (size_t)(Nmax + 1)), Ub(2 * (size_t)Nmax), Sb((size_t)Nmax);
        plan_params p = *p0;
        for (;;) {
            const int b = next.fetch_add(1);
            if (b >= B) return;
            double x0[5];
            for (int i = 0; i < 5; ++i) x0[i] = starts[5 * (size_t)b + i];
            int n = 0;
            bool err = false;
            for (; n < max_chunks; ++n) {
                const double rem = s_total - x0[0];
                if (!(rem > 0.1)) break;
                const int fin = rem < max_chunk_size * 2.0 ? 1 : 0;
                const double size = fin ? rem : max_chunk_size;
                // vmax[int(s / 5):] with Python's slice rules (see plan_loop_kernel)
                const double si = x0[0] / 5.0;
                if (!(si < (double)nav)) { err = true; break; }
                int idx = si <= -(double)nav ? 0 : (int)si;
                if (idx < 0) idx += nav;
                const double hz = ceil(size / avg[idx] * 2.0 / 0.3);
                if (!(hz >= 1.0 && hz <= (double)Nmax)) { err = true; break; }
                const int Nc = (int)hz;
                p.N = Nc;
                int total = 0, nq = 0;
                const int st = chunk(r, &p, Nc, x0, x0[0] + size, fin, Xb.data(), Ub.data(), Sb.data(), &total, &nq);
                const size_t slot = (size_t)b * max_chunks + n;
                for (int k = 0; k <= Nmax; ++k)
                    for (int i = 0; i < 5; ++i) X[(slot * (Nmax + 1) + k) * 5 + i] = k <= Nc ? Xb[5 * (size_t)k + i] : 0.0;
                for (int k = 0; k < Nmax; ++k) {
                    U[(slot * Nmax + k) * 2 + 0] = k < Nc ? Ub[2 * (size_t)k] : 0.0;
                    U[(slot * Nmax + k) * 2 + 1] = k < Nc ? Ub[2 * (size_t)k + 1] : 0.0;
                    S[slot * Nmax + k] = k < Nc ? Sb[k] : 0.0;
                }
                N[slot] = Nc;
                is_final[slot] = fin;
                status[slot] = st;
                iters[slot] = total;
                sqp[slot] = nq;
                const int c = fin ? Nc : Nc / 2;
                for (int i = 0; i < 5; ++i) x0[i] = Xb[5 * (size_t)c + i];
            }
            nchunks[b] = err ? -(n + 1) : n;
        }
    };
    threads = std::max(1, std::min(threads, B));
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
}

}  // namespace plan_host

/*
 * mpc_oracle.c — CPU restatement of the reference tracking-MPC hot path (plain C99, FP64).
 *
 * TEST INFRASTRUCTURE: the checker for the HIP path and the bench's CPU baseline ("port").
 * Never linked into the product.  Compile with -ffp-contract=off: the interp / predict /
 * warm-start restatements are bit-exact to the reference's numpy arithmetic.
 *
 * Reference citations (medinammartin3/Safe-Autonomous-Driving-MPC):
 *   trajectory_loader.py:26-30   strict-monotone s fix
 *   trajectory_loader.py:67-77   interp1d(kind='linear', fill_value='extrapolate'), whose
 *                                arithmetic is scipy/interpolate/_interpolate.py:457-483
 *                                (searchsorted-left, clip [1,T-1], slope*(x-x_lo)+y_lo)
 *   trajectory_loader.py:86-102  get_state / get_control
 *   trajectory_tracking.py:50-67 dynamics; :87-114 predict; :116-152 cost; :155-211 constraints;
 *   trajectory_tracking.py:224-246 warm start; :213-263 solve.
 * The QP(ubar) and its solver are SURVEY.md Appendix B / DESIGN.md section 3: Gauss-Newton
 * linearisation about ubar, elastic (L1) state rows, Mehrotra primal-dual interior point with
 * stage-wise (Riccati) Newton solves.
 */
#include "mpc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXN MPC_MAX_N
#define NROW 9      /* soft one-sided rows per stage                       */
#define NBOX 4      /* hard box rows per control stage                     */
#define TAU 0.995   /* fraction to the boundary                             */
#define START_SHIFT 3.0   /* interior-point start: slack and elastic slack beyond the row value */

struct orc_table {
    int T, Tu;
    double *s, *d, *o, *k, *v, *u1, *u2;
    double *gx, *gy, *gpsi;             /* global geometry, trajectory_loader.py:32-62 */
    double smax;
    double last[5];
};

void orc_default_params(mpc_params* p) {
    memset(p, 0, sizeof(*p));
    p->N = 5;
    p->max_obs = 0;
    p->dt = 0.2;
    p->u_min[0] = -0.6; p->u_min[1] = -5.0;
    p->u_max[0] = 0.6;  p->u_max[1] = 4.0;
    p->vehicle_radius = 1.0;
    p->w_d = 10.0; p->w_o = 10.0; p->w_v = 5.0; p->w_u1 = 0.5; p->w_u2 = 0.5;
    p->obstacle_safety_distance = 5.0;
    p->max_time_2_obs = 1.5;
    p->wheelbase = 2.8;
    p->lane_width = 3.0;
    p->safe_lane_margin = 0.1;
    p->brake_distance = 40.0;
    p->brake_accel = -2.0;
    p->linearization = 1;
    p->sqp_iters = 1;
    p->max_iter = 80;
    p->tol = 1e-9;
    p->tol_mu = 1e-10;
    p->elastic_rho = 1e5;
    p->polish = 2;
    p->sqp_tol = 1e-10;
}

static int seg(const double* x, int n, double v);
static double lin(const double* x, const double* y, int i, double v);

orc_table* orc_table_create(const double* X, int T, const double* U, int Tu) {
    if (T < 2 || Tu < 1) return NULL;
    orc_table* t = (orc_table*)calloc(1, sizeof(orc_table));
    t->T = T;
    t->Tu = Tu < T ? Tu : T;            /* limit = min(len(s), len(U))  trajectory_loader.py:73-75 */
    double* buf = (double*)malloc(sizeof(double) * (8 * T + 2 * t->Tu));
    t->s = buf; t->d = buf + T; t->o = buf + 2 * T; t->k = buf + 3 * T; t->v = buf + 4 * T;
    t->u1 = buf + 5 * T; t->u2 = buf + 5 * T + t->Tu;
    t->gx = buf + 5 * T + 2 * t->Tu; t->gy = t->gx + T; t->gpsi = t->gy + T;
    for (int i = 0; i < T; ++i) {
        double si = X[5 * i];
        if (i > 0 && si <= t->s[i - 1]) si = t->s[i - 1] + 1e-5;   /* trajectory_loader.py:28-30 */
        t->s[i] = si;
        t->d[i] = X[5 * i + 1]; t->o[i] = X[5 * i + 2]; t->k[i] = X[5 * i + 3]; t->v[i] = X[5 * i + 4];
    }
    for (int i = 0; i < t->Tu; ++i) { t->u1[i] = U[2 * i]; t->u2[i] = U[2 * i + 1]; }
    t->smax = t->s[T - 1];
    for (int j = 0; j < 5; ++j) t->last[j] = X[5 * (T - 1) + j];
    /* global pose of the reference line: heading integrates the planned curvature X[i-1,3] over ds,
     * position integrates the mean heading of each step (trajectory_loader.py:38-58) */
    t->gx[0] = t->gy[0] = t->gpsi[0] = 0.0;
    for (int i = 1; i < T; ++i) {
        double ds = t->s[i] - t->s[i - 1];
        double kk = X[5 * (i - 1) + 3];
        double psi_old = t->gpsi[i - 1];
        double psi_new = psi_old + kk * ds;
        double psi_avg = (psi_old + psi_new) / 2.0;
        t->gpsi[i] = psi_new;
        t->gx[i] = t->gx[i - 1] + cos(psi_avg) * ds;
        t->gy[i] = t->gy[i - 1] + sin(psi_avg) * ds;
    }
    return t;
}

/* TrajectoryLoader.get_global_pose(s, d) (trajectory_loader.py:104-116): clamp s to s_max, interpolate
 * the global line (linear, extrapolating below 0), offset laterally by d. */
void orc_global_pose(const orc_table* t, double s, double d, double out[3]) {
    if (s > t->smax) s = t->smax;
    int i = seg(t->s, t->T, s);
    double xr = lin(t->s, t->gx, i, s), yr = lin(t->s, t->gy, i, s), psi = lin(t->s, t->gpsi, i, s);
    out[0] = xr - d * sin(psi);
    out[1] = yr + d * cos(psi);
    out[2] = psi;
}

void orc_table_destroy(orc_table* t) {
    if (!t) return;
    free(t->s);
    free(t);
}

double orc_s_max(const orc_table* t) { return t->smax; }

/* numpy searchsorted(side='left') clipped to [1, n-1] (scipy _interpolate.py:461-466) */
static int seg(const double* x, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (x[mid] < v) lo = mid + 1; else hi = mid;
    }
    if (lo < 1) lo = 1;
    if (lo > n - 1) lo = n - 1;
    return lo;
}

static double lin(const double* x, const double* y, int i, double v) {
    double slope = (y[i] - y[i - 1]) / (x[i] - x[i - 1]);
    return slope * (v - x[i - 1]) + y[i - 1];
}

static double slope_at(const double* x, const double* y, int i) {
    return (y[i] - y[i - 1]) / (x[i] - x[i - 1]);
}

void orc_get_state(const orc_table* t, double s, double out[5]) {
    if (s >= t->smax) { memcpy(out, t->last, 5 * sizeof(double)); return; }
    int i = seg(t->s, t->T, s);
    out[0] = s;
    out[1] = lin(t->s, t->d, i, s);
    out[2] = lin(t->s, t->o, i, s);
    out[3] = lin(t->s, t->k, i, s);
    out[4] = lin(t->s, t->v, i, s);
}

void orc_get_control(const orc_table* t, double s, double out[2]) {
    if (s >= t->smax) { out[0] = 0.0; out[1] = 0.0; return; }
    int i = seg(t->s, t->Tu, s);
    out[0] = lin(t->s, t->u1, i, s);
    out[1] = lin(t->s, t->u2, i, s);
}

void orc_state_slopes(const orc_table* t, double s, double out[4]) {
    if (s >= t->smax) { out[0] = out[1] = out[2] = out[3] = 0.0; return; }
    int i = seg(t->s, t->T, s);
    out[0] = slope_at(t->s, t->d, i);
    out[1] = slope_at(t->s, t->o, i);
    out[2] = slope_at(t->s, t->k, i);
    out[3] = slope_at(t->s, t->v, i);
}

void orc_warm_start(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs,
                    int nobs, double* ubar) {
    double s_curr = x0[0], v_curr = x0[4];
    int brake = 0;
    for (int j = 0; j < p->N; ++j) {
        for (int i = 0; i < nobs; ++i)
            if ((obs[2 * i] - s_curr) < p->brake_distance) brake = 1;   /* sticky, :231-233 */
        double ur[2];
        orc_get_control(t, s_curr, ur);
        ubar[2 * j] = ur[0];
        ubar[2 * j + 1] = brake ? p->brake_accel : ur[1];
        s_curr += v_curr * p->dt;
    }
}

/* one explicit-Euler step of trajectory_tracking.py:50-67,110 */
static void euler(const mpc_params* p, const double x[5], const double u[2], double kref, double y[5]) {
    double dt = p->dt;
    double xd0 = x[4], xd1 = x[4] * x[2], xd2 = x[4] * (x[3] - kref), xd3 = u[0], xd4 = u[1];
    y[0] = x[0] + dt * xd0;
    y[1] = x[1] + dt * xd1;
    y[2] = x[2] + dt * xd2;
    y[3] = x[3] + dt * xd3;
    y[4] = x[4] + dt * xd4;
}

void orc_predict(const orc_table* t, const mpc_params* p, const double x0[5], const double* U, double* X) {
    double x[5], st[5];
    memcpy(x, x0, sizeof(x));
    memcpy(X, x0, 5 * sizeof(double));
    for (int k = 0; k < p->N; ++k) {
        orc_get_state(t, x[0], st);
        double y[5];
        euler(p, x, U + 2 * k, st[3], y);
        memcpy(x, y, sizeof(x));
        memcpy(X + 5 * (k + 1), x, sizeof(x));
    }
}

double orc_cost(const orc_table* t, const mpc_params* p, const double x0[5], const double* U) {
    double X[(MAXN + 1) * 5];
    orc_predict(t, p, x0, U, X);
    double c = 0.0, st[5];
    for (int k = 1; k <= p->N; ++k) {
        const double* x = X + 5 * k;
        orc_get_state(t, x[0], st);
        double ed = x[1] - st[1], eo = x[2] - st[2], ev = x[4] - st[4];
        c += p->w_d * (ed * ed);
        c += p->w_o * (eo * eo);
        c += p->w_v * (ev * ev);
    }
    for (int k = 0; k < p->N; ++k) {
        c += p->w_u1 * (U[2 * k] * U[2 * k]);
        c += p->w_u2 * (U[2 * k + 1] * U[2 * k + 1]);
    }
    return c;
}

static double safe_lane(const mpc_params* p) {
    return p->lane_width / 2.0 - p->vehicle_radius - p->safe_lane_margin;   /* :169 */
}

int orc_constraints(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs,
                    int nobs, const double* U, double* out) {
    double X[(MAXN + 1) * 5];
    orc_predict(t, p, x0, U, X);
    double sl = safe_lane(p);
    int r = 0;
    for (int k = 1; k <= p->N; ++k) {
        double s = X[5 * k], d = X[5 * k + 1], o = X[5 * k + 2], v = X[5 * k + 4];
        out[r++] = sl - d;
        out[r++] = d + sl;
        double vf = d + (p->wheelbase / 2.0) * o;
        out[r++] = sl - vf;
        out[r++] = vf + sl;
        double vfull = d + p->wheelbase * o;
        out[r++] = sl - vfull;
        out[r++] = vfull + sl;
        for (int i = 0; i < nobs; ++i) {
            double sop = obs[2 * i] + obs[2 * i + 1] * (k * p->dt);
            double gap = sop - s;
            double vs = v * p->max_time_2_obs;
            double ssafe = p->obstacle_safety_distance > vs ? p->obstacle_safety_distance : vs;
            out[r++] = gap - ssafe;
        }
        out[r++] = v;
    }
    return r;
}

/* ---------------------------------------------------------------------------------------
 * QP(ubar) data, stage-wise
 * ------------------------------------------------------------------------------------- */
typedef struct {
    int N, has_obs;
    double dt, rho;
    double Xbar[MAXN + 1][5];
    /* A_k = I + J'_k, k = 0..N-1 (a04 = dt) */
    double a12[MAXN], a14[MAXN], a20[MAXN], a23[MAXN], a24[MAXN];
    /* cost on (s,d,o,k,v) at k = 1..N (k-row/col zero), control cost */
    double Q[MAXN + 1][5][5], q[MAXN + 1][5];
    double R[2], r[MAXN][2];
    double c0;
    /* soft rows (>=) at k = 1..N: coefficient over 5-state, bound */
    double C[NROW][5];
    double b[MAXN + 1][NROW];
    int on[NROW];
    /* hard box rows at t = 0..N-1: +u1>=, -u1>=, +u2>=, -u2>= */
    double bb[MAXN][NBOX];
} qpdat;

static void build_stage_qp(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs,
                           int nobs, const double* ubar, qpdat* Q) {
    int N = p->N;
    double dt = p->dt;
    memset(Q, 0, sizeof(*Q));
    Q->N = N;
    Q->dt = dt;
    Q->rho = p->elastic_rho;
    Q->has_obs = nobs > 0;
    orc_predict(t, p, x0, ubar, &Q->Xbar[0][0]);          /* nominal rollout == predict(x0, ubar) */
    int gn = p->linearization != 0;
    for (int k = 0; k < N; ++k) {
        const double* x = Q->Xbar[k];
        double st[5], sl4[4];
        orc_get_state(t, x[0], st);
        orc_state_slopes(t, x[0], sl4);
        double dk = gn ? sl4[2] : 0.0;
        Q->a12[k] = dt * x[4];
        Q->a14[k] = dt * x[2];
        Q->a20[k] = dt * (-x[4] * dk);
        Q->a23[k] = dt * x[4];
        Q->a24[k] = dt * (x[3] - st[3]);
    }
    double w[3] = {p->w_d, p->w_o, p->w_v};
    int idx[3] = {1, 2, 4};
    Q->c0 = 0.0;
    for (int k = 1; k <= N; ++k) {
        const double* x = Q->Xbar[k];
        double st[5], sl4[4];
        orc_get_state(t, x[0], st);
        orc_state_slopes(t, x[0], sl4);
        double ref[3] = {st[1], st[2], st[4]};
        double dref[3] = {gn ? sl4[0] : 0.0, gn ? sl4[1] : 0.0, gn ? sl4[3] : 0.0};
        for (int j = 0; j < 3; ++j) {
            double m[5] = {0, 0, 0, 0, 0};
            m[idx[j]] = 1.0;
            m[0] = -dref[j];
            double r0 = x[idx[j]] - ref[j];
            for (int a = 0; a < 5; ++a) {
                Q->q[k][a] += 2.0 * w[j] * r0 * m[a];
                for (int bq = 0; bq < 5; ++bq) Q->Q[k][a][bq] += 2.0 * w[j] * m[a] * m[bq];
            }
            Q->c0 += w[j] * r0 * r0;
        }
    }
    Q->R[0] = 2.0 * p->w_u1;
    Q->R[1] = 2.0 * p->w_u2;
    for (int k = 0; k < N; ++k) {
        Q->r[k][0] = Q->R[0] * ubar[2 * k];
        Q->r[k][1] = Q->R[1] * ubar[2 * k + 1];
        Q->c0 += p->w_u1 * ubar[2 * k] * ubar[2 * k] + p->w_u2 * ubar[2 * k + 1] * ubar[2 * k + 1];
    }
    double L = p->wheelbase, h = p->wheelbase / 2.0, T = p->max_time_2_obs, sl = safe_lane(p);
    double C[NROW][5] = {{0, 1, 0, 0, 0}, {0, -1, 0, 0, 0}, {0, 1, h, 0, 0},  {0, -1, -h, 0, 0},
                         {0, 1, L, 0, 0}, {0, -1, -L, 0, 0}, {-1, 0, 0, 0, 0}, {-1, 0, 0, 0, -T},
                         {0, 0, 0, 0, 1}};
    memcpy(Q->C, C, sizeof(C));
    for (int j = 0; j < NROW; ++j) Q->on[j] = 1;
    if (!Q->has_obs) Q->on[6] = Q->on[7] = 0;
    for (int k = 1; k <= N; ++k) {
        const double* x = Q->Xbar[k];
        double pv0 = x[1], pv1 = x[1] + h * x[2], pv2 = x[1] + L * x[2];
        Q->b[k][0] = -sl - pv0;  Q->b[k][1] = -(sl - pv0);
        Q->b[k][2] = -sl - pv1;  Q->b[k][3] = -(sl - pv1);
        Q->b[k][4] = -sl - pv2;  Q->b[k][5] = -(sl - pv2);
        if (Q->has_obs) {
            double shat = INFINITY;
            for (int i = 0; i < nobs; ++i) {
                double sp = obs[2 * i] + obs[2 * i + 1] * (k * dt);
                if (sp < shat) shat = sp;
            }
            Q->b[k][6] = -(shat - p->obstacle_safety_distance - x[0]);
            Q->b[k][7] = -(shat - x[0] - T * x[4]);
        }
        Q->b[k][8] = -x[4];
    }
    for (int k = 0; k < N; ++k) {
        Q->bb[k][0] = p->u_min[0] - ubar[2 * k];
        Q->bb[k][1] = -(p->u_max[0] - ubar[2 * k]);
        Q->bb[k][2] = p->u_min[1] - ubar[2 * k + 1];
        Q->bb[k][3] = -(p->u_max[1] - ubar[2 * k + 1]);
    }
}

/* x_{k+1} = A_k x_k (+ B u) */
static inline void apply_A(const qpdat* Q, int k, const double x[5], double y[5]) {
    y[0] = x[0] + Q->dt * x[4];
    y[1] = x[1] + Q->a12[k] * x[2] + Q->a14[k] * x[4];
    y[2] = x[2] + Q->a20[k] * x[0] + Q->a23[k] * x[3] + Q->a24[k] * x[4];
    y[3] = x[3];
    y[4] = x[4];
}

static inline void apply_AT(const qpdat* Q, int k, const double m[5], double y[5]) {
    y[0] = m[0] + Q->a20[k] * m[2];
    y[1] = m[1];
    y[2] = m[2] + Q->a12[k] * m[1];
    y[3] = m[3] + Q->a23[k] * m[2];
    y[4] = m[4] + Q->dt * m[0] + Q->a14[k] * m[1] + Q->a24[k] * m[2];
}

static void rollout_lin(const qpdat* Q, const double* du, double X[][5]) {
    memset(X[0], 0, 5 * sizeof(double));
    for (int k = 0; k < Q->N; ++k) {
        apply_A(Q, k, X[k], X[k + 1]);
        X[k + 1][3] += Q->dt * du[2 * k];
        X[k + 1][4] += Q->dt * du[2 * k + 1];
    }
}

/* g[t] = z[t] + B' mu_{t+1},  mu_N = y_N, mu_k = A_k' mu_{k+1} + y_k */
static void adjoint(const qpdat* Q, double y[][5], double z[][2], double* g) {
    double mu[5] = {0, 0, 0, 0, 0};
    for (int k = Q->N; k >= 1; --k) {
        for (int a = 0; a < 5; ++a) mu[a] += y[k][a];
        g[2 * (k - 1)] = z[k - 1][0] + Q->dt * mu[3];
        g[2 * (k - 1) + 1] = z[k - 1][1] + Q->dt * mu[4];
        double m2[5];
        apply_AT(Q, k - 1, mu, m2);
        memcpy(mu, m2, sizeof(mu));
    }
}

static inline double dot5(const double a[5], const double b[5]) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4];
}

typedef struct {
    double du[2 * MAXN];
    double s[MAXN + 1][NROW], lam[MAXN + 1][NROW], xi[MAXN + 1][NROW], nu[MAXN + 1][NROW];
    double sb[MAXN][NBOX], lb[MAXN][NBOX];
} ipm_state;

typedef struct {
    double K[MAXN][2][5], Sinv[MAXN][3];
    double Qt[MAXN + 1][5][5], Rt[MAXN][2];
    double d[MAXN + 1][NROW], db[MAXN][NBOX];
} ipm_fact;

typedef struct {
    double du[2 * MAXN], dX[MAXN + 1][5];
    double dl[MAXN + 1][NROW], ds[MAXN + 1][NROW], dxi[MAXN + 1][NROW], dnu[MAXN + 1][NROW];
    double dlb[MAXN][NBOX], dsb[MAXN][NBOX];
} ipm_dir;

static const double box_sign[NBOX] = {1.0, -1.0, 1.0, -1.0};
static const int box_comp[NBOX] = {0, 0, 1, 1};

static int riccati_factor(const qpdat* Q, ipm_fact* F);

/* barrier weights and augmented stage Hessians, then the Riccati factorisation */
static int factor(const qpdat* Q, const ipm_state* S, ipm_fact* F) {
    int N = Q->N;
    for (int k = 1; k <= N; ++k) {
        memcpy(F->Qt[k], Q->Q[k], sizeof(F->Qt[k]));
        for (int j = 0; j < NROW; ++j) {
            if (!Q->on[j]) continue;
            double d = S->s[k][j] / S->lam[k][j] + S->xi[k][j] / S->nu[k][j];
            F->d[k][j] = d;
            double w = 1.0 / d;
            const double* c = Q->C[j];
            for (int a = 0; a < 5; ++a)
                for (int bq = 0; bq < 5; ++bq) F->Qt[k][a][bq] += w * c[a] * c[bq];
        }
    }
    for (int t = 0; t < N; ++t) {
        F->Rt[t][0] = Q->R[0];
        F->Rt[t][1] = Q->R[1];
        for (int j = 0; j < NBOX; ++j) {
            double d = S->sb[t][j] / S->lb[t][j];
            F->db[t][j] = d;
            F->Rt[t][box_comp[j]] += 1.0 / d;
        }
    }
    return riccati_factor(Q, F);
}

/* Riccati factorisation of  min sum 0.5 x_k'Qt_k x_k + 0.5 u_k'Rt_k u_k  s.t. x_{k+1} = A_k x_k + B u_k */
static int riccati_factor(const qpdat* Q, ipm_fact* F) {
    int N = Q->N;
    double dt = Q->dt;
    double P[5][5];
    memcpy(P, F->Qt[N], sizeof(P));
    int bad = 0;
    for (int k = N - 1; k >= 0; --k) {
        double M[5][5];
        for (int i = 0; i < 5; ++i) {
            M[i][0] = P[i][0] + P[i][2] * Q->a20[k];
            M[i][1] = P[i][1];
            M[i][2] = P[i][2] + P[i][1] * Q->a12[k];
            M[i][3] = P[i][3] + P[i][2] * Q->a23[k];
            M[i][4] = P[i][4] + P[i][0] * dt + P[i][1] * Q->a14[k] + P[i][2] * Q->a24[k];
        }
        double s00 = F->Rt[k][0] + dt * dt * P[3][3];
        double s01 = dt * dt * P[3][4];
        double s11 = F->Rt[k][1] + dt * dt * P[4][4];
        /* S = Ls Ls' (2x2 Cholesky); W = Ls^-1 L; L'S^-1 L = W'W; K = -Ls^-T W */
        if (!(s00 > 0.0)) { s00 = 1e-300 + fabs(s00); bad = 1; }
        double l00 = sqrt(s00), l10 = s01 / l00, r11 = s11 - l10 * l10;
        if (!(r11 > 1e-14 * s11)) { r11 = 1e-14 * fabs(s11) + 1e-300; bad = 1; }
        double l11 = sqrt(r11);
        F->Sinv[k][0] = l00; F->Sinv[k][1] = l10; F->Sinv[k][2] = l11;   /* Cholesky factor of S */
        double W0[5], W1[5];
        for (int j = 0; j < 5; ++j) {
            W0[j] = dt * M[3][j] / l00;
            W1[j] = (dt * M[4][j] - l10 * W0[j]) / l11;
            double z1 = W1[j] / l11;
            double z0 = (W0[j] - l10 * z1) / l00;
            F->K[k][0][j] = -z0;
            F->K[k][1][j] = -z1;
        }
        if (k >= 1) {
            double Pn[5][5];
            for (int j = 0; j < 5; ++j) {
                Pn[0][j] = M[0][j] + Q->a20[k] * M[2][j];
                Pn[1][j] = M[1][j];
                Pn[2][j] = M[2][j] + Q->a12[k] * M[1][j];
                Pn[3][j] = M[3][j] + Q->a23[k] * M[2][j];
                Pn[4][j] = M[4][j] + dt * M[0][j] + Q->a14[k] * M[1][j] + Q->a24[k] * M[2][j];
            }
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j)
                    Pn[i][j] += F->Qt[k][i][j] - (W0[i] * W0[j] + W1[i] * W1[j]);
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) P[i][j] = 0.5 * (Pn[i][j] + Pn[j][i]);
        }
    }
    return bad;
}

static void riccati_solve(const qpdat* Q, const ipm_fact* F, double qh[][5], double gh[][2], ipm_dir* D);

/* Solve the Newton system for complementarity targets r4 (s*lam rows), r5 (xi*nu rows),
 * given residuals rp/rpb/rx and the dual residual pieces y (stage) / z (control). */
static void newton(const qpdat* Q, const ipm_state* S, const ipm_fact* F, double rp[][NROW],
                   double rpb[][NBOX], double rx[][NROW], double y[][5], double z[][2],
                   double r4[][NROW], double r5[][NROW], double r4b[][NBOX], ipm_dir* D) {
    int N = Q->N;
    double dt = Q->dt;
    double qh[MAXN + 1][5], gh[MAXN][2];
    double rhs[MAXN + 1][NROW], rhsb[MAXN][NBOX];
    for (int k = 1; k <= N; ++k) {
        for (int a = 0; a < 5; ++a) qh[k][a] = -y[k][a];
        for (int j = 0; j < NROW; ++j) {
            if (!Q->on[j]) continue;
            double l = S->lam[k][j], nu = S->nu[k][j], xi = S->xi[k][j];
            double rh = -rp[k][j] - r4[k][j] / l + (r5[k][j] + xi * rx[k][j]) / nu;
            rhs[k][j] = rh;
            double w = rh / F->d[k][j];
            for (int a = 0; a < 5; ++a) qh[k][a] += Q->C[j][a] * w;
        }
    }
    for (int t = 0; t < N; ++t) {
        gh[t][0] = -z[t][0];
        gh[t][1] = -z[t][1];
        for (int j = 0; j < NBOX; ++j) {
            double rh = -rpb[t][j] - r4b[t][j] / S->lb[t][j];
            rhsb[t][j] = rh;
            gh[t][box_comp[j]] += box_sign[j] * rh / F->db[t][j];
        }
    }
    riccati_solve(Q, F, qh, gh, D);
    for (int k = 1; k <= N; ++k) {
        for (int j = 0; j < NROW; ++j) {
            if (!Q->on[j]) continue;
            double dl = (rhs[k][j] - dot5(Q->C[j], D->dX[k])) / F->d[k][j];
            D->dl[k][j] = dl;
            D->ds[k][j] = -(r4[k][j] + S->s[k][j] * dl) / S->lam[k][j];
            double dn = rx[k][j] - dl;
            D->dnu[k][j] = dn;
            D->dxi[k][j] = -(r5[k][j] + S->xi[k][j] * dn) / S->nu[k][j];
        }
    }
    for (int t = 0; t < N; ++t) {
        for (int j = 0; j < NBOX; ++j) {
            double dl = (rhsb[t][j] - box_sign[j] * D->du[2 * t + box_comp[j]]) / F->db[t][j];
            D->dlb[t][j] = dl;
            D->dsb[t][j] = -(r4b[t][j] + S->sb[t][j] * dl) / S->lb[t][j];
        }
    }
}

/* LQR solve with the factorisation F: linear terms -qh (state, k=1..N), -gh (control);
 * writes D->du and D->dX (x_0 = 0). */
static void riccati_solve(const qpdat* Q, const ipm_fact* F, double qh[][5], double gh[][2], ipm_dir* D) {
    int N = Q->N;
    double dt = Q->dt;
    double p[5], kk[MAXN][2];
    memcpy(p, qh[N], sizeof(p));
    for (int k = N - 1; k >= 0; --k) {
        double h0 = gh[k][0] + dt * p[3], h1 = gh[k][1] + dt * p[4];
        const double* Lc = F->Sinv[k];          /* Cholesky factor (l00, l10, l11) of S */
        double w0 = h0 / Lc[0], w1 = (h1 - Lc[1] * w0) / Lc[2];
        kk[k][1] = w1 / Lc[2];
        kk[k][0] = (w0 - Lc[1] * kk[k][1]) / Lc[0];
        if (k >= 1) {
            double pa[5];
            apply_AT(Q, k, p, pa);
            for (int a = 0; a < 5; ++a) p[a] = qh[k][a] + pa[a] + F->K[k][0][a] * h0 + F->K[k][1][a] * h1;
        }
    }
    /* forward */
    memset(D->dX[0], 0, 5 * sizeof(double));
    for (int k = 0; k < N; ++k) {
        double* x = D->dX[k];
        double u0 = kk[k][0] + dot5(F->K[k][0], x);
        double u1 = kk[k][1] + dot5(F->K[k][1], x);
        D->du[2 * k] = u0;
        D->du[2 * k + 1] = u1;
        apply_A(Q, k, x, D->dX[k + 1]);
        D->dX[k + 1][3] += dt * u0;
        D->dX[k + 1][4] += dt * u1;
    }
}

static inline double ratio(double v, double dv, double a) {
    return (dv < 0.0 && -v / dv < a) ? -v / dv : a;
}

static double max_step(const qpdat* Q, const ipm_state* S, const ipm_dir* D) {
    double a = 1.0;
    for (int k = 1; k <= Q->N; ++k)
        for (int j = 0; j < NROW; ++j) {
            if (!Q->on[j]) continue;
            a = ratio(S->s[k][j], D->ds[k][j], a);
            a = ratio(S->lam[k][j], D->dl[k][j], a);
            a = ratio(S->xi[k][j], D->dxi[k][j], a);
            a = ratio(S->nu[k][j], D->dnu[k][j], a);
        }
    for (int t = 0; t < Q->N; ++t)
        for (int j = 0; j < NBOX; ++j) {
            a = ratio(S->sb[t][j], D->dsb[t][j], a);
            a = ratio(S->lb[t][j], D->dlb[t][j], a);
        }
    return a;
}

/* Active-set polish of the interior-point result.
 * Rows are classified from the final iterate: violated (soft, xi > nu: multiplier fixed at rho),
 * active (lam > s: equality), inactive.  The equality-constrained QP
 *     min 0.5 x'Hx + f'x - rho sum_V a_i'x   s.t.  a_i'x = b_i (i in A)
 * is solved by the same stage-wise Riccati machinery with penalty weights 1/delta on the active
 * rows and iterative refinement on its exact KKT residual.  The result is accepted only if it is
 * KKT-consistent (multiplier signs/caps, inactive rows satisfied, violated rows still violated);
 * otherwise the interior-point iterate stands.  Returns 1 if accepted (S->du replaced). */
#define POLISH_DELTA 1e-11
#define POLISH_REFINE 2
#define POLISH_ROUNDS 6
#define XO_ROUNDS 1         /* rounds of the crossover attempt before the interior point */
#define MU_CHECK 1e-4       /* interior-point checkpoint: a polish is tried once mu is below this ... */
#define CHECK_SEP 100.0     /* ... and every row's slack and multiplier differ by this factor (no near-tie) */
#define CHECK_ROUNDS 2      /* polish rounds at the checkpoint (the interior point continues if they fail) */
/* MPC_CHECKPOINT=0 in the environment switches the checkpoint off (A/B against the round-4 interior point;
 * the product's libmpcqp reads the same variable) */
static int check_on(void) {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("MPC_CHECKPOINT");
        on = !(e && e[0] == '0');
    }
    return on;
}
/* Classification left by the last polish_from call of this thread (the accepted one, or the one the last
 * rejected round flipped to): the SQP's next re-linearisation starts its crossover from it (given = 2). */
static __thread unsigned char last_cls[MAXN + 1][NROW], last_clb[MAXN][NBOX];
/* given = 1: start from the all-inactive classification (crossover) instead of classifying S;
 * given = 2: start from the previous QP's classification (last_cls / last_clb) */
/* du of the last crossover's solve from the all-inactive classification (given = 1): the unconstrained optimum
 * of QP(ubar), which the interior point's start then reuses instead of a second factorisation and solve */
static __thread double xo_du[2 * MAXN];
static int polish_from(const qpdat* Q, ipm_state* S, int* infeasible, int given, int rounds) {
    int N = Q->N;
    double rho = Q->rho;
    static __thread ipm_fact F;
    static __thread ipm_dir D;
    static __thread ipm_state T;       /* working copy: du, lam (A rows) */
    static __thread unsigned char cls[MAXN + 1][NROW], clb[MAXN][NBOX];   /* 0 inactive, 1 active, 2 violated */
    static __thread unsigned char flip[MAXN + 1][NROW], flipb[MAXN][NBOX];
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < NROW; ++j) {
            cls[k][j] = 0;
            if (!Q->on[j] || given == 1) continue;
            if (given == 2) cls[k][j] = last_cls[k][j];
            else if (S->xi[k][j] > S->nu[k][j]) cls[k][j] = 2;
            else if (S->lam[k][j] > S->s[k][j]) cls[k][j] = 1;
        }
    for (int t = 0; t < N; ++t)
        for (int j = 0; j < NBOX; ++j)
            clb[t][j] = given == 1 ? 0 : (given == 2 ? last_clb[t][j] : S->lb[t][j] > S->sb[t][j]);
    int accepted = 0;
    for (int round = 0; round < rounds; ++round) {
        memcpy(&T, S, sizeof(T));
        for (int k = 1; k <= N; ++k) {
            memcpy(F.Qt[k], Q->Q[k], sizeof(F.Qt[k]));
            for (int j = 0; j < NROW; ++j)
                if (Q->on[j] && cls[k][j] == 1) {
                    const double* c = Q->C[j];
                    for (int a = 0; a < 5; ++a)
                        for (int b = 0; b < 5; ++b) F.Qt[k][a][b] += c[a] * c[b] / POLISH_DELTA;
                    if (!(S->lam[k][j] > 0.0)) T.lam[k][j] = 0.0;
                }
        }
        for (int t = 0; t < N; ++t) {
            F.Rt[t][0] = Q->R[0];
            F.Rt[t][1] = Q->R[1];
            for (int j = 0; j < NBOX; ++j)
                if (clb[t][j]) F.Rt[t][box_comp[j]] += 1.0 / POLISH_DELTA;
        }
        riccati_factor(Q, &F);
        double X[MAXN + 1][5];
        /* the crossover from the all-inactive classification (given = 1) solves the unconstrained LQR: one solve
         * is its exact optimum, nothing to refine (the kernel's MODE_XO runs one solve too) */
        const int nref = given == 1 ? 1 : POLISH_REFINE;
        for (int r = 0; r <= nref; ++r) {
            rollout_lin(Q, T.du, X);
            /* exact KKT residual of the equality QP; LQR right-hand side */
            double qh[MAXN + 1][5], gh[MAXN][2], r2[MAXN + 1][NROW], r2b[MAXN][NBOX];
            for (int k = 1; k <= N; ++k) {
                for (int a = 0; a < 5; ++a) {
                    double acc = Q->q[k][a];
                    for (int b = 0; b < 5; ++b) acc += Q->Q[k][a][b] * X[k][b];
                    qh[k][a] = -acc;
                }
                for (int j = 0; j < NROW; ++j) {
                    if (!Q->on[j] || cls[k][j] == 0) continue;
                    const double* c = Q->C[j];
                    double lam = cls[k][j] == 2 ? rho : T.lam[k][j];
                    for (int a = 0; a < 5; ++a) qh[k][a] += lam * c[a];
                    if (cls[k][j] == 1) {
                        r2[k][j] = Q->b[k][j] - dot5(c, X[k]);
                        for (int a = 0; a < 5; ++a) qh[k][a] += c[a] * r2[k][j] / POLISH_DELTA;
                    }
                }
            }
            for (int t = 0; t < N; ++t) {
                gh[t][0] = -(Q->R[0] * T.du[2 * t] + Q->r[t][0]);
                gh[t][1] = -(Q->R[1] * T.du[2 * t + 1] + Q->r[t][1]);
                for (int j = 0; j < NBOX; ++j) {
                    if (!clb[t][j]) continue;
                    double sg = box_sign[j];
                    gh[t][box_comp[j]] += sg * T.lb[t][j];
                    r2b[t][j] = Q->bb[t][j] - sg * T.du[2 * t + box_comp[j]];
                    gh[t][box_comp[j]] += sg * r2b[t][j] / POLISH_DELTA;
                }
            }
            if (r == nref) break;
            riccati_solve(Q, &F, qh, gh, &D);
            for (int i = 0; i < 2 * N; ++i) T.du[i] += D.du[i];
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < NROW; ++j)
                    if (Q->on[j] && cls[k][j] == 1)
                        T.lam[k][j] += (r2[k][j] - dot5(Q->C[j], D.dX[k])) / POLISH_DELTA;
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < NBOX; ++j)
                    if (clb[t][j])
                        T.lb[t][j] += (r2b[t][j] - box_sign[j] * D.du[2 * t + box_comp[j]]) / POLISH_DELTA;
        }
        /* the crossover's solve is the unconstrained optimum of QP(ubar): kept for the interior-point start */
        if (given == 1 && round == 0) memcpy(xo_du, T.du, sizeof(double) * 2 * N);
        /* acceptance: KKT consistency of the polished point; otherwise fix the worst row and retry */
        double lmax = 1.0;
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j)
                if (Q->on[j] && cls[k][j] == 1 && fabs(T.lam[k][j]) > lmax) lmax = fabs(T.lam[k][j]);
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < NBOX; ++j)
                if (clb[t][j] && fabs(T.lb[t][j]) > lmax) lmax = fabs(T.lb[t][j]);
        int nviol = 0, wk = -1, wj = -1, wbox = 0;
        double worst = 0.0;
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j) {
                if (!Q->on[j]) continue;
                double bsc = 1.0 + fabs(Q->b[k][j]);
                double r = dot5(Q->C[j], X[k]) - Q->b[k][j];
                double bad = 0.0;
                if (cls[k][j] == 1) {
                    double l = T.lam[k][j];
                    if (l < -1e-9 * lmax) bad = -l / lmax;
                    else if (l > rho * (1.0 + 1e-9)) bad = (l - rho) / lmax;
                    else if (fabs(r) > 1e-7 * bsc) bad = fabs(r) / bsc;
                } else if (cls[k][j] == 2) {
                    if (r > 1e-9 * bsc) bad = r / bsc;
                    if (r < -1e-6 * bsc) nviol++;
                } else if (r < -1e-9 * bsc) bad = -r / bsc;
                if (bad > worst) { worst = bad; wk = k; wj = j; wbox = 0; }
                flip[k][j] = bad > 0.0;
            }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < NBOX; ++j) {
                double bsc = 1.0 + fabs(Q->bb[t][j]);
                double r = box_sign[j] * T.du[2 * t + box_comp[j]] - Q->bb[t][j];
                double bad = 0.0;
                if (clb[t][j]) {
                    if (T.lb[t][j] < -1e-9 * lmax) bad = -T.lb[t][j] / lmax;
                    else if (fabs(r) > 1e-7 * bsc) bad = fabs(r) / bsc;
                } else if (r < -1e-9 * bsc) bad = -r / bsc;
                if (bad > worst) { worst = bad; wk = t; wj = j; wbox = 1; }
                flipb[t][j] = bad > 0.0;
            }
        int finite = 1;
        for (int i = 0; i < 2 * N; ++i) if (!(T.du[i] == T.du[i])) finite = 0;
        if (!finite) break;
        if (getenv("ORC_TRACE"))
            fprintf(stderr, "polish round %d worst %.3e at %s k=%d j=%d nviol=%d\n", round, worst, wbox ? "box" : "row",
                    wk, wj, nviol);
        if (wk < 0) {
            memcpy(S->du, T.du, sizeof(double) * 2 * N);
            *infeasible = nviol > 0;
            accepted = 1;
            break;
        }
        (void)wbox;
        for (int k = 1; k <= N; ++k)           /* primal-dual active-set update of every offending row */
            for (int j = 0; j < NROW; ++j)
                if (flip[k][j]) {
                    unsigned char c = cls[k][j];
                    cls[k][j] = (c == 1) ? (T.lam[k][j] > rho ? 2 : 0) : 1;
                }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < NBOX; ++j)
                if (flipb[t][j]) clb[t][j] = !clb[t][j];
    }
    memcpy(last_cls, cls, sizeof(last_cls));
    memcpy(last_clb, clb, sizeof(last_clb));
    return accepted;
}

static int polish(const qpdat* Q, ipm_state* S, int* infeasible) { return polish_from(Q, S, infeasible, 0, POLISH_ROUNDS); }

/* total complementarity after a step of length a along D */
static double comp_after(const qpdat* Q, const ipm_state* S, const ipm_dir* D, double a) {
    double c = 0.0;
    for (int k = 1; k <= Q->N; ++k)
        for (int j = 0; j < NROW; ++j) {
            if (!Q->on[j]) continue;
            c += (S->s[k][j] + a * D->ds[k][j]) * (S->lam[k][j] + a * D->dl[k][j]) +
                 (S->xi[k][j] + a * D->dxi[k][j]) * (S->nu[k][j] + a * D->dnu[k][j]);
        }
    for (int t = 0; t < Q->N; ++t)
        for (int j = 0; j < NBOX; ++j) c += (S->sb[t][j] + a * D->dsb[t][j]) * (S->lb[t][j] + a * D->dlb[t][j]);
    return c;
}

/* Mehrotra predictor-corrector PDIP for QP(ubar); returns status, du in S->du */
static int pdip(const qpdat* Q, const mpc_params* p, ipm_state* S, int* iters, int warm) {
    int N = Q->N;
    double rho = Q->rho;
    static __thread ipm_fact F;
    static __thread ipm_dir D, Da;
    memset(S, 0, sizeof(*S));
    int nsoft = 0;
    for (int j = 0; j < NROW; ++j) nsoft += Q->on[j];
    double Mtot = (double)(2 * nsoft * N + NBOX * N);
    if (p->polish >= 2) {
        /* Crossover first: the active-set solve started from the unconstrained optimum (all rows
         * inactive, du = 0, multipliers 0), XO_ROUNDS rounds.  When it certifies (KKT-consistent), it is
         * the exact optimum and no interior-point iteration is needed (70% of the C2 batch). */
        static __thread ipm_state Z;
        memset(&Z, 0, sizeof(Z));
        int inf = 0;
        if (polish_from(Q, &Z, &inf, warm ? 2 : 1, XO_ROUNDS)) {
            memcpy(S->du, Z.du, sizeof(double) * 2 * N);
            *iters = 0;
            return inf ? MPC_INFEASIBLE : MPC_OK;
        }
    }

    double X[MAXN + 1][5];
    double bscale = 0.0, rowc = 0.0;
    {
    /* Interior-point start (round 3): centred at the unconstrained optimum of QP(ubar) (one Riccati
     * factorisation and solve without rows), or at du = 0 when the soft rows are less violated there.  Each soft row with value r = C x - b there gets slack
     * max(r, 0) + START_SHIFT and elastic slack max(-r, 0) + START_SHIFT, and the multiplier pair on the
     * pair's central path with lambda + nu = rho (lambda s = nu xi): primal and dual row residuals are zero
     * and every pair equally centred.  Box rows start on the rows' central path (sb lb = the mean soft-row
     * complementarity, sb >= 1).  With tol_mu 1e-10 (round 2: the start at du = 0 with s lam = 1000,
     * lam <= rho/2, and 1e-9), maximum iterations C2 22 -> 20, C3 24 -> 22, C4 27 -> 25, C5 29 -> 27, and
     * every feasible C5 instance polish-certified. */
    if (p->polish >= 2 && !warm) {
        /* the crossover above solved exactly this system (all rows inactive: the stage Hessians and the
         * right-hand side -q, -r of the start); its solution is the start's, bit for bit */
        memcpy(S->du, xo_du, sizeof(double) * 2 * N);
    } else {
        static __thread ipm_fact F0;
        static __thread ipm_dir D0;
        double qh[MAXN + 1][5], gh[MAXN][2];
        for (int k = 1; k <= N; ++k) {
            memcpy(F0.Qt[k], Q->Q[k], sizeof(F0.Qt[k]));
            for (int a = 0; a < 5; ++a) qh[k][a] = -Q->q[k][a];
        }
        for (int t = 0; t < N; ++t) {
            F0.Rt[t][0] = Q->R[0];
            F0.Rt[t][1] = Q->R[1];
            gh[t][0] = -Q->r[t][0];
            gh[t][1] = -Q->r[t][1];
        }
        riccati_factor(Q, &F0);
        riccati_solve(Q, &F0, qh, gh, &D0);
        memcpy(S->du, D0.du, sizeof(double) * 2 * N);
    }
    rollout_lin(Q, S->du, X);
    {
        /* the start's primal point: the unconstrained optimum, or du = 0 (the warm start ubar, which already
         * brakes for obstacles ahead) when the soft rows are less violated there (sum of max(-r, 0)) */
        double v_unc = 0.0, v_bar = 0.0;
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j) {
                if (!Q->on[j]) continue;
                const double r = dot5(Q->C[j], X[k]) - Q->b[k][j];
                v_unc += r < 0.0 ? -r : 0.0;
                v_bar += Q->b[k][j] > 0.0 ? Q->b[k][j] : 0.0;
            }
        if (v_bar < v_unc) {
            memset(S->du, 0, sizeof(double) * 2 * N);
            rollout_lin(Q, S->du, X);
        }
    }
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < NROW; ++j) {
            if (!Q->on[j]) continue;
            const double r = dot5(Q->C[j], X[k]) - Q->b[k][j];
            const double sv = (r > 0.0 ? r : 0.0) + START_SHIFT, xi = (r < 0.0 ? -r : 0.0) + START_SHIFT;
            S->s[k][j] = sv;
            S->xi[k][j] = xi;
            S->lam[k][j] = rho * xi / (sv + xi);
            S->nu[k][j] = rho * sv / (sv + xi);
            rowc += sv * S->lam[k][j];
            if (fabs(Q->b[k][j]) > bscale) bscale = fabs(Q->b[k][j]);
        }
    const double mrow = rowc / (double)(nsoft * N);
    for (int t = 0; t < N; ++t)
        for (int j = 0; j < NBOX; ++j) {
            const double v = box_sign[j] * S->du[2 * t + box_comp[j]] - Q->bb[t][j];
            S->sb[t][j] = v > 1.0 ? v : 1.0;
            S->lb[t][j] = mrow / S->sb[t][j];
            if (fabs(Q->bb[t][j]) > bscale) bscale = fabs(Q->bb[t][j]);
        }
    }
    double y[MAXN + 1][5], yc[MAXN + 1][5], ya[MAXN + 1][5], z[MAXN][2], zc[MAXN][2], za[MAXN][2];
    double rp[MAXN + 1][NROW], rx[MAXN + 1][NROW], rpb[MAXN][NBOX];
    double r4[MAXN + 1][NROW], r5[MAXN + 1][NROW], r4b[MAXN][NBOX];
    double gd[2 * MAXN], gc[2 * MAXN], ga[2 * MAXN];
    int status = MPC_MAX_ITER, it;
    int stall = 0, checked = 0;
    for (it = 0; it < p->max_iter; ++it) {
        rollout_lin(Q, S->du, X);
        memset(yc, 0, sizeof(yc));
        memset(ya, 0, sizeof(ya));
        double rpmax = 0.0, rxmax = 0.0, comp = 0.0;
        for (int k = 1; k <= N; ++k) {
            for (int a = 0; a < 5; ++a) {
                double acc = Q->q[k][a];
                for (int bq = 0; bq < 5; ++bq) acc += Q->Q[k][a][bq] * X[k][bq];
                yc[k][a] = acc;
            }
            for (int j = 0; j < NROW; ++j) {
                if (!Q->on[j]) continue;
                const double* c = Q->C[j];
                for (int a = 0; a < 5; ++a) ya[k][a] -= S->lam[k][j] * c[a];
                double r = dot5(c, X[k]) + S->xi[k][j] - S->s[k][j] - Q->b[k][j];
                rp[k][j] = r;
                if (fabs(r) > rpmax) rpmax = fabs(r);
                double rr = rho - S->lam[k][j] - S->nu[k][j];
                rx[k][j] = rr;
                if (fabs(rr) > rxmax) rxmax = fabs(rr);
                comp += S->s[k][j] * S->lam[k][j] + S->xi[k][j] * S->nu[k][j];
            }
            for (int a = 0; a < 5; ++a) y[k][a] = yc[k][a] + ya[k][a];
        }
        for (int t = 0; t < N; ++t) {
            zc[t][0] = Q->R[0] * S->du[2 * t] + Q->r[t][0];
            zc[t][1] = Q->R[1] * S->du[2 * t + 1] + Q->r[t][1];
            za[t][0] = -S->lb[t][0] + S->lb[t][1];
            za[t][1] = -S->lb[t][2] + S->lb[t][3];
            z[t][0] = zc[t][0] + za[t][0];
            z[t][1] = zc[t][1] + za[t][1];
            for (int j = 0; j < NBOX; ++j) {
                double r = box_sign[j] * S->du[2 * t + box_comp[j]] - S->sb[t][j] - Q->bb[t][j];
                rpb[t][j] = r;
                if (fabs(r) > rpmax) rpmax = fabs(r);
                comp += S->sb[t][j] * S->lb[t][j];
            }
        }
        adjoint(Q, y, z, gd);
        adjoint(Q, yc, zc, gc);
        adjoint(Q, ya, za, ga);
        double rdmax = 0.0, sd = 0.0;
        for (int i = 0; i < 2 * N; ++i) {
            if (fabs(gd[i]) > rdmax) rdmax = fabs(gd[i]);
            if (fabs(gc[i]) > sd) sd = fabs(gc[i]);
            if (fabs(ga[i]) > sd) sd = fabs(ga[i]);
        }
        double mu = comp / Mtot;
        if (getenv("ORC_TRACE"))
        {
            double lm = 0, lbm = 0;
            for (int k = 1; k <= N; ++k) for (int j = 0; j < NROW; ++j) if (Q->on[j] && S->lam[k][j] > lm) lm = S->lam[k][j];
            for (int t = 0; t < N; ++t) for (int j = 0; j < NBOX; ++j) if (S->lb[t][j] > lbm) lbm = S->lb[t][j];
            fprintf(stderr, "it %2d mu %.3e rd %.3e (abs %.3e sd %.2e) rp %.3e lam %.6e lb %.6e u0 %.12e\n", it, mu,
                    rdmax / (1.0 + sd), rdmax, sd, rpmax / (1.0 + bscale), lm, lbm, S->du[0]);
        }
        if (!(mu == mu) || !(rdmax == rdmax)) { status = MPC_NUMERICAL; break; }
        /* Converged once complementarity and the primal residual are small: the interior point only has
         * to identify the active set to ~1e-10; the active-set polish then makes the solution exact.
         * The dual residual carries O(eps/mu) noise of the active multipliers (barrier weights ~1/mu):
         * it is required to 1e4*tol, otherwise the iterate is flagged NUMERICAL (polish may still accept it). */
        if (mu <= p->tol_mu && rpmax <= 10.0 * p->tol * (1.0 + bscale) && rxmax <= p->tol * rho) {
            status = rdmax <= 1e4 * p->tol * (1.0 + sd) ? MPC_OK : MPC_NUMERICAL;
            break;
        }
        /* Interior-point checkpoint (once per QP): once mu <= MU_CHECK and every row's
         * slack and multiplier (s, lambda; xi, nu; box s, lambda) are CHECK_SEP apart, the iterate's
         * classification is tried by CHECK_ROUNDS polish rounds; a certified point is the QP's exact optimum
         * (the QP is strictly convex), otherwise the interior point continues from the unchanged iterate. */
        if (p->polish && !checked && mu <= MU_CHECK && check_on()) {
            int tie = 0;
            for (int k = 1; k <= N && !tie; ++k)
                for (int j = 0; j < NROW; ++j) {
                    if (!Q->on[j]) continue;
                    const double s = S->s[k][j], l = S->lam[k][j], x = S->xi[k][j], n = S->nu[k][j];
                    if (!(s > CHECK_SEP * l || l > CHECK_SEP * s) || !(x > CHECK_SEP * n || n > CHECK_SEP * x)) tie = 1;
                }
            for (int t = 0; t < N && !tie; ++t)
                for (int j = 0; j < NBOX; ++j)
                    if (!(S->sb[t][j] > CHECK_SEP * S->lb[t][j] || S->lb[t][j] > CHECK_SEP * S->sb[t][j])) tie = 1;
            if (!tie) {
                static __thread ipm_state C;
                int inf = 0;
                checked = 1;
                memcpy(&C, S, sizeof(C));
                if (polish_from(Q, &C, &inf, 0, CHECK_ROUNDS)) {
                    memcpy(S->du, C.du, sizeof(double) * 2 * N);
                    *iters = it;
                    return inf ? MPC_INFEASIBLE : MPC_OK;
                }
            }
        }
        factor(Q, S, &F);
        /* predictor */
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j) {
                r4[k][j] = S->s[k][j] * S->lam[k][j];
                r5[k][j] = S->xi[k][j] * S->nu[k][j];
            }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < NBOX; ++j) r4b[t][j] = S->sb[t][j] * S->lb[t][j];
        newton(Q, S, &F, rp, rpb, rx, y, z, r4, r5, r4b, &Da);
        double aa = max_step(Q, S, &Da);
        double ca = 0.0;
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j) {
                if (!Q->on[j]) continue;
                ca += (S->s[k][j] + aa * Da.ds[k][j]) * (S->lam[k][j] + aa * Da.dl[k][j]) +
                      (S->xi[k][j] + aa * Da.dxi[k][j]) * (S->nu[k][j] + aa * Da.dnu[k][j]);
            }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < NBOX; ++j)
                ca += (S->sb[t][j] + aa * Da.dsb[t][j]) * (S->lb[t][j] + aa * Da.dlb[t][j]);
        double mua = ca / Mtot;
        double sig = mua / mu;
        sig = sig * sig * sig;
        /* corrector */
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j) {
                r4[k][j] = S->s[k][j] * S->lam[k][j] + Da.ds[k][j] * Da.dl[k][j] - sig * mu;
                r5[k][j] = S->xi[k][j] * S->nu[k][j] + Da.dxi[k][j] * Da.dnu[k][j] - sig * mu;
            }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < NBOX; ++j)
                r4b[t][j] = S->sb[t][j] * S->lb[t][j] + Da.dsb[t][j] * Da.dlb[t][j] - sig * mu;
        newton(Q, S, &F, rp, rpb, rx, y, z, r4, r5, r4b, &D);
        double a = TAU * max_step(Q, S, &D);
        if (a > 1.0) a = 1.0;
        double cnew = comp_after(Q, S, &D, a);
        if (cnew > comp) {
            /* safeguard: the second-order term made things worse (happens after a poor affine step);
             * take the plain centred Newton direction instead */
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < NROW; ++j) {
                    r4[k][j] = S->s[k][j] * S->lam[k][j] - sig * mu;
                    r5[k][j] = S->xi[k][j] * S->nu[k][j] - sig * mu;
                }
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < NBOX; ++j) r4b[t][j] = S->sb[t][j] * S->lb[t][j] - sig * mu;
            newton(Q, S, &F, rp, rpb, rx, y, z, r4, r5, r4b, &D);
            a = TAU * max_step(Q, S, &D);
            if (a > 1.0) a = 1.0;
            cnew = comp_after(Q, S, &D, a);
        }
        if (getenv("ORC_TRACE")) fprintf(stderr, "      aff %.3e sig %.3e alpha %.3e\n", aa, sig, a);
        {
            /* breakdown guard: a step whose complementarity or control direction is not finite is not
             * taken; the current iterate goes to the polish instead (NUMERICAL unless it certifies) */
            int fin = cnew == cnew && cnew < INFINITY;
            for (int i = 0; i < 2 * N && fin; ++i) fin = D.du[i] == D.du[i] && fabs(D.du[i]) < INFINITY;
            if (!fin) { status = MPC_NUMERICAL; ++it; break; }
        }
        stall = (mu < 1e-6 && cnew > 0.9 * comp) ? stall + 1 : 0;   /* late-phase no-progress counter */
        for (int i = 0; i < 2 * N; ++i) S->du[i] += a * D.du[i];
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j) {
                if (!Q->on[j]) continue;
                S->s[k][j] += a * D.ds[k][j];
                S->lam[k][j] += a * D.dl[k][j];
                S->xi[k][j] += a * D.dxi[k][j];
                S->nu[k][j] += a * D.dnu[k][j];
            }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < NBOX; ++j) {
                S->sb[t][j] += a * D.dsb[t][j];
                S->lb[t][j] += a * D.dlb[t][j];
            }
        if (stall >= 5) { status = MPC_NUMERICAL; ++it; break; }
    }
    *iters = it;
    int bad = 0;
    for (int i = 0; i < 2 * N; ++i) if (!(S->du[i] == S->du[i])) bad = 1;
    if (bad) {
        memset(S->du, 0, sizeof(double) * 2 * N);
        return MPC_NUMERICAL;
    }
    if (status == MPC_OK) {
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < NROW; ++j)
                if (Q->on[j] && S->xi[k][j] > 1e-6 * (1.0 + fabs(Q->b[k][j]))) status = MPC_INFEASIBLE;
    }
    if (p->polish) {
        int inf = 0;
        if (polish(Q, S, &inf)) status = inf ? MPC_INFEASIBLE : MPC_OK;
    }
    return status;
}

int orc_build_qp(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs,
                 int nobs, const double* ubar, double* H, double* f, double* c0, double* A, double* lo,
                 double* hi, double* blo, double* bhi) {
    static __thread qpdat Q;
    build_stage_qp(t, p, x0, obs, nobs, ubar, &Q);
    int N = p->N, n = 2 * N;
    double* G = (double*)calloc((size_t)(N + 1) * 5 * n, sizeof(double));
#define GG(k, a, j) G[((size_t)(k) * 5 + (a)) * n + (j)]
    for (int k = 0; k < N; ++k) {
        for (int j = 0; j < n; ++j) {
            double x[5] = {GG(k, 0, j), GG(k, 1, j), GG(k, 2, j), GG(k, 3, j), GG(k, 4, j)}, yv[5];
            apply_A(&Q, k, x, yv);
            for (int a = 0; a < 5; ++a) GG(k + 1, a, j) = yv[a];
        }
        GG(k + 1, 3, 2 * k) += Q.dt;
        GG(k + 1, 4, 2 * k + 1) += Q.dt;
    }
    memset(H, 0, sizeof(double) * n * n);
    memset(f, 0, sizeof(double) * n);
    for (int k = 1; k <= N; ++k)
        for (int i = 0; i < n; ++i) {
            double qg[5];
            for (int a = 0; a < 5; ++a) {
                double acc = 0;
                for (int bq = 0; bq < 5; ++bq) acc += Q.Q[k][a][bq] * GG(k, bq, i);
                qg[a] = acc;
            }
            for (int j = 0; j < n; ++j) {
                double acc = 0;
                for (int a = 0; a < 5; ++a) acc += GG(k, a, j) * qg[a];
                H[i * n + j] += acc;
            }
            double acc = 0;
            for (int a = 0; a < 5; ++a) acc += GG(k, a, i) * Q.q[k][a];
            f[i] += acc;
        }
    for (int k = 0; k < N; ++k) {
        H[(2 * k) * n + 2 * k] += Q.R[0];
        H[(2 * k + 1) * n + 2 * k + 1] += Q.R[1];
        f[2 * k] += Q.r[k][0];
        f[2 * k + 1] += Q.r[k][1];
    }
    *c0 = Q.c0;
    /* rows: d, d+h o, d+L o, [s, s+T v], v  as lo <= c.x <= hi */
    int m = 0;
    for (int k = 1; k <= N; ++k) {
        int rowsj[6][3] = {{0, 0, 1}, {2, 2, 3}, {4, 4, 5}, {6, -1, 6}, {7, -1, 7}, {8, 8, -1}};
        /* {coefficient row (positive form index), lo-row index, hi-row index}; C[hi] = -C */
        for (int rr = 0; rr < 6; ++rr) {
            if ((rr == 3 || rr == 4) && !Q.has_obs) continue;
            const double* c = Q.C[rowsj[rr][0]];
            double sgn = (rr == 3 || rr == 4) ? -1.0 : 1.0;   /* obstacle rows stored as -c >= -hi */
            for (int j = 0; j < n; ++j) {
                double acc = 0;
                for (int a = 0; a < 5; ++a) acc += sgn * c[a] * GG(k, a, j);
                A[(size_t)m * n + j] = acc;
            }
            lo[m] = rowsj[rr][1] >= 0 ? Q.b[k][rowsj[rr][1]] : -INFINITY;
            hi[m] = rowsj[rr][2] >= 0 ? -Q.b[k][rowsj[rr][2]] : INFINITY;
            ++m;
        }
    }
    for (int k = 0; k < N; ++k) {
        blo[2 * k] = Q.bb[k][0];
        bhi[2 * k] = -Q.bb[k][1];
        blo[2 * k + 1] = Q.bb[k][2];
        bhi[2 * k + 1] = -Q.bb[k][3];
    }
#undef GG
    free(G);
    return m;
}

/* SQP stopping rules besides convergence (max |dU| <= sqp_tol), DESIGN.md section "SQP": a 2-cycle (the QP
 * returns the point of two QPs back while moving far from the last one: the Gauss-Newton model jumping
 * across a kink of the piecewise-linear reference), and SQP_INF_STREAK consecutive elastic (infeasible) QPs,
 * whose iterates wander without converging.  Mirrored by the kernel's SQP loop (mpcqp.hip). */
#define SQP_CYCLE_REL 1e-6
#define SQP_INF_STREAK 5
int orc_solve(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs, int nobs,
              const double* ubar, double* u0, double* U, double* Xpred, int* iters) {
    static __thread qpdat Q;
    static __thread ipm_state S;
    int N = p->N;
    double ub[2 * MAXN], Uo[2 * MAXN];
    if (ubar) memcpy(ub, ubar, sizeof(double) * 2 * N);
    else orc_warm_start(t, p, x0, obs, nobs, ub);
    int status = MPC_OK, total = 0;
    int nsqp = p->sqp_iters < 0 ? 0 : p->sqp_iters;   /* 0: U = ubar */
    double u2[2 * MAXN];                              /* U two QPs back (for the cycle test) */
    memcpy(u2, ub, sizeof(double) * 2 * N);
    int ninf = 0, conv = 0;
    memcpy(Uo, ub, sizeof(double) * 2 * N);
    for (int it = 0; it < nsqp; ++it) {
        build_stage_qp(t, p, x0, obs, nobs, ub, &Q);
        int ni = 0;
        status = pdip(&Q, p, &S, &ni, it > 0);
        total += ni;
        double step = 0.0, back2 = 0.0;
        for (int i = 0; i < 2 * N; ++i) {
            Uo[i] = ub[i] + S.du[i];
            step = fabs(S.du[i]) > step ? fabs(S.du[i]) : step;
            const double b2 = fabs(Uo[i] - u2[i]);
            back2 = b2 > back2 ? b2 : back2;
        }
        memcpy(u2, ub, sizeof(double) * 2 * N);
        memcpy(ub, Uo, sizeof(double) * 2 * N);
        ninf = status == MPC_INFEASIBLE ? ninf + 1 : 0;
        if (nsqp > 1) {
            if (step <= p->sqp_tol) { conv = 1; break; }                 /* converged re-linearisation */
            if (p->sqp_tol > 0.0) {                                      /* sqp_tol 0: all sqp_iters QPs */
                if (it >= 2 && back2 <= SQP_CYCLE_REL * step) break;     /* 2-cycle: back where it was */
                if (ninf >= SQP_INF_STREAK) break;                       /* elastic QPs in a row */
            }
        }
    }
    if (U) memcpy(U, Uo, sizeof(double) * 2 * N);
    if (u0) { u0[0] = Uo[0]; u0[1] = Uo[1]; }
    if (Xpred) orc_predict(t, p, x0, Uo, Xpred);                 /* :261 */
    if (iters) *iters = total;
    if (nsqp > 1 && p->sqp_tol > 0.0 && !conv) status |= MPC_SQP_UNCONVERGED;
    return status;
}

int orc_solve_batch(const orc_table* t, const mpc_params* p, int B, const double* x0, const double* obs,
                    const int* n_obs, const double* ubar, double* u0, double* U, double* Xpred, int* status,
                    int* iters, int num_threads) {
    if (!t || !p || B < 0 || p->N < 1 || p->N > MAXN) return MPC_E_ARG;
    int N = p->N, mo = p->max_obs;
#ifdef _OPENMP
    if (num_threads <= 0) num_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(num_threads)
#endif
    for (int b = 0; b < B; ++b) {
        int no = n_obs ? n_obs[b] : 0;
        if (no > mo) no = mo;
        int it = 0;
        int st = orc_solve(t, p, x0 + 5 * (size_t)b, obs ? obs + (size_t)b * mo * 2 : NULL, no,
                           ubar ? ubar + (size_t)b * 2 * N : NULL, u0 ? u0 + 2 * (size_t)b : NULL,
                           U ? U + (size_t)b * 2 * N : NULL, Xpred ? Xpred + (size_t)b * 5 * (N + 1) : NULL, &it);
        if (status) status[b] = st;
        if (iters) iters[b] = it;
    }
    (void)num_threads;
    return MPC_SUCCESS;
}

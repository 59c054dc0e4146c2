// plan.hip — MI355X batched offline planner: libmpcplan.so (C ABI: include/mpcplan.h).
//
// The chunk NLP of the reference's offline planner (TrajectoryOptimizer, trajectory_planning.py:8-391,
// driven by optimize_full_trajectory :419-559) solved for B independent chunks per launch, FP64, one chunk
// per lane.  The algorithm is the one DESIGN.md ("Offline planner") describes and oracle/plan_oracle.c
// restates on the CPU (the test's checker; nothing here includes, links or calls it):
//   Gauss-Newton / exact-Hessian SQP over z = [X, U, S] from the reference's initial guess (:357-376), a
//   non-monotone L1-merit line search, speed limits frozen after a 2-cycle at a limit change; each QP by an
//   active-set crossover from the previous QP's active rows, else a Mehrotra interior point on the
//   stage-wise Riccati recursion followed by the same equality-constrained solve ("polish").
//
// Mapping: one lane = one chunk.  The chunk's stage data (A, B, Hessians, rows, factors, iterates) lives in
// a per-wave block of global scratch, element e of lane l at block[e * 64 + l]: every access of a wave to
// one logical element is one contiguous 512-byte line, and a wave's whole working set is one contiguous
// block (L2 / MALL locality).  The recursions run per lane in registers (P, the 8x8 stage Hessian).  The
// batch is HBM / L2-bandwidth bound, not MFMA work: there is no GEMM shape in a 5-state Riccati.
// Lanes of a wave diverge in iteration counts; a finished lane idles until its wave's slowest chunk ends.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mpcplan.h"

namespace {

constexpr int WAVE = 64;
constexpr int NZ = 8;             // stage variables: x (s, d, o, k, v), w (u1, u2, S)
constexpr int NR = 11;            // rows per stage at most
constexpr double RHO = 1e8;       // penalty of the active rows in the equality-constrained solve
constexpr int AL_STEPS = 4;
constexpr int POLISH_ROUNDS = 6;
constexpr double SHIFT0 = 1.0;
constexpr double TAU = 0.995;
constexpr double CYCLE_REL = 1e-6;
constexpr double DELTA0 = 1e-6;
constexpr double DELTA_MAX = 1e4;
constexpr double EXACT_STEP = 0.1;
constexpr double LS_ARMIJO = 1e-4;
constexpr int LS_STEPS = 12;
constexpr double LS_FULL = 1e-3;
constexpr int LS_MEMORY = 4;

enum { ROW_VMIN, ROW_VMAX, ROW_LATP, ROW_LATM, ROW_KMIN, ROW_KMAX, ROW_U1MIN, ROW_U1MAX, ROW_U2MIN, ROW_U2MAX,
       ROW_S, ROW_STERM };

struct DevRoute {
    const double *s, *cx, *cy, *vmax;
    int M;
    double s_total;
};

// per-lane scratch layout (in doubles, per stage counts times NP = Nmax + 1)
struct Layout {
    int NP;
    int oA, oB, oC, oD1, oH, oGQ, oG, oK, oL, oEZ, oZ, oS, oLAM, oY, oGL, oDZ, oDSA, oDLA, oRP, oDS, oDL, oTZ, oTLAM,
        oMY, oMLAT, oZB, oZ2, oZN, oDZV, oVLIM, oVL, oACT, oTACT, total;
};

__host__ __device__ Layout make_layout(int Nmax) {
    Layout y;
    y.NP = Nmax + 1;
    int o = 0;
    auto take = [&](int per) { const int r = o; o += per * y.NP; return r; };  // NOLINT
    y.oA = take(25); y.oB = take(15); y.oC = take(5); y.oD1 = take(25); y.oH = take(64); y.oGQ = take(NZ);
    y.oG = take(NR); y.oK = take(15); y.oL = take(6); y.oEZ = take(2 * NZ); y.oZ = take(NZ); y.oS = take(NR);
    y.oLAM = take(NR); y.oY = take(NR); y.oGL = take(NZ); y.oDZ = take(NZ); y.oDSA = take(NR); y.oDLA = take(NR);
    y.oRP = take(NR); y.oDS = take(NR); y.oDL = take(NR); y.oTZ = take(NZ); y.oTLAM = take(NR); y.oMY = take(5);
    y.oMLAT = take(2); y.oZB = take(NZ); y.oZ2 = take(NZ); y.oZN = take(NZ); y.oDZV = take(NZ); y.oVLIM = take(1);
    y.oVL = take(1); y.oACT = take(NR); y.oTACT = take(NR);
    y.total = o;
    return y;
}

// one lane's view of its scratch: element e at b[e * 64]
struct Ln {
    double* b;
    __device__ double& operator[](int e) const { return b[(size_t)e * WAVE]; }
};

// ------------------------------------------------------------------------------------------------------
// route: k_ref_fun (:445-459) and v_max_fun (:470-473)
// ------------------------------------------------------------------------------------------------------
__device__ int lower_bound_d(const double* x, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (x[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

__device__ int upper_bound_d(const double* x, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (x[m] <= v) lo = m + 1; else hi = m;
    }
    return lo;
}

// kappa(s) with d/ds and d2/ds2 (k2 may be null): s_to_t linear (searchsorted left, clipped to [1, M-1]),
// spline piece floor(t) clipped to [0, M-2]
__device__ double route_kappa(const DevRoute& R, double s, double* k1, double* k2) {
    const int M = R.M;
    int i = lower_bound_d(R.s, M, s);
    i = i < 1 ? 1 : (i > M - 1 ? M - 1 : i);
    const double slope = 1.0 / (R.s[i] - R.s[i - 1]);
    const double t = slope * (s - R.s[i - 1]) + (double)(i - 1);
    int j = (int)floor(t);
    j = j < 0 ? 0 : (j > M - 2 ? M - 2 : j);
    const double tau = t - (double)j;
    const double* a = R.cx + 4 * j;
    const double* b = R.cy + 4 * j;
    const double x1 = (3.0 * a[0] * tau + 2.0 * a[1]) * tau + a[2], x2 = 6.0 * a[0] * tau + 2.0 * a[1], x3 = 6.0 * a[0];
    const double y1 = (3.0 * b[0] * tau + 2.0 * b[1]) * tau + b[2], y2 = 6.0 * b[0] * tau + 2.0 * b[1], y3 = 6.0 * b[0];
    const double num = x1 * y2 - y1 * x2;
    const double q = x1 * x1 + y1 * y1;
    const double sq = sqrt(q);
    double den = q * sq + 1e-9;
    const bool clamp = den < 1e-8;
    if (clamp) den = 1e-8;
    const double k = num / den;
    if (k1) {
        const double dnum = x1 * y3 - y1 * x3;
        const double dden = clamp ? 0.0 : 3.0 * sq * (x1 * x2 + y1 * y2);
        const double kt = (dnum - k * dden) / den;
        *k1 = kt * slope;
        if (k2) {
            const double d2num = x2 * y3 - y2 * x3;
            const double qd = 2.0 * (x1 * x2 + y1 * y2), qdd = 2.0 * (x2 * x2 + x1 * x3 + y2 * y2 + y1 * y3);
            const double d2den = (clamp || sq == 0.0) ? 0.0 : 0.75 * qd * qd / sq + 1.5 * sq * qdd;
            *k2 = (d2num - 2.0 * kt * dden - k * d2den) / den * slope * slope;
        }
    }
    return k;
}

__device__ double route_vmax(const DevRoute& R, double s) {
    const int i = upper_bound_d(R.s, R.M, s);
    return R.vmax[i > 0 ? i - 1 : 0];
}

// ------------------------------------------------------------------------------------------------------
// the NLP's functions (trajectory_planning.py:50-89, :128-170, :181-210) and derivatives
// ------------------------------------------------------------------------------------------------------
__device__ double guard_den(double den) {
    if (fabs(den) < 1e-4) den = den > 0.0 ? 1e-4 : (den < 0.0 ? -1e-4 : 1e-4);
    return den;
}

__device__ void dyn(const double x[5], double u1, double u2, double kr, double f[5]) {
    const double den = guard_den(1.0 - x[1] * kr);
    const double sd = (x[4] * cos(x[2])) / den;
    f[0] = sd;
    f[1] = x[4] * sin(x[2]);
    f[2] = x[4] * x[3] - sd * kr;
    f[3] = u1;
    f[4] = u2;
}

__device__ void dyn_jac(const double x[5], double kr, double dk, double F[25]) {
    const double d = x[1], o = x[2], k = x[3], v = x[4];
    const double raw = 1.0 - d * kr;
    const bool g = fabs(raw) < 1e-4;
    const double den = guard_den(raw);
    const double c = cos(o), sn = sin(o);
    const double sd = v * c / den;
    double ds[5];
    ds[0] = g ? 0.0 : v * c * d * dk / (den * den);
    ds[1] = g ? 0.0 : v * c * kr / (den * den);
    ds[2] = -v * sn / den;
    ds[3] = 0.0;
    ds[4] = c / den;
#pragma unroll
    for (int i = 0; i < 25; ++i) F[i] = 0.0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        F[j] = ds[j];
        F[10 + j] = -kr * ds[j];
    }
    F[7] = v * c;
    F[9] = sn;
    F[10] += -dk * sd;
    F[13] += v;
    F[14] += k;
}

__device__ void hess_f(const double x[5], double kr, double k1, double k2, const double y[5], double W[25]) {
    const double d = x[1], o = x[2], v = x[4];
    const double raw = 1.0 - d * kr;
    const bool gu = fabs(raw) < 1e-4;
    const double g = 1.0 / guard_den(raw);
    const double c = cos(o), sn = sin(o);
    const double gs = gu ? 0.0 : d * k1 * g * g, gd = gu ? 0.0 : kr * g * g;
    const double gss = gu ? 0.0 : d * k2 * g * g + 2.0 * d * d * k1 * k1 * g * g * g;
    const double gsd = gu ? 0.0 : k1 * g * g + 2.0 * d * k1 * kr * g * g * g;
    const double gdd = gu ? 0.0 : 2.0 * kr * kr * g * g * g;
    const double ds[5] = {v * c * gs, v * c * gd, -v * sn * g, 0.0, c * g};
    const double sd = v * c * g;
    const double cs = y[0] - y[2] * kr;
#pragma unroll
    for (int i = 0; i < 25; ++i) W[i] = 0.0;
    W[0] = cs * v * c * gss;
    W[1] = W[5] = cs * v * c * gsd;
    W[6] = cs * v * c * gdd;
    W[2] = W[10] = cs * -v * sn * gs;
    W[7] = W[11] = cs * -v * sn * gd;
    W[12] = cs * -v * c * g;
    W[4] = W[20] = cs * c * gs;
    W[9] = W[21] = cs * c * gd;
    W[14] = W[22] = cs * -sn * g;
    W[12] += -y[1] * v * sn;
    W[14] += y[1] * c;
    W[22] += y[1] * c;
    W[19] += y[2];
    W[23] += y[2];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        W[j] += -y[2] * k1 * ds[j];
        W[5 * j] += -y[2] * k1 * ds[j];
    }
    W[0] += -y[2] * sd * k2;
}

__device__ void defect(const DevRoute& R, const plan_params& P, const double xa[5], const double xb[5], double u1,
                       double u2, double def[5]) {
    const double h = P.dt;
    double fa[5], fb[5], fm[5], xm[5];
    dyn(xa, u1, u2, route_kappa(R, xa[0], nullptr, nullptr), fa);
    dyn(xb, u1, u2, route_kappa(R, xb[0], nullptr, nullptr), fb);
#pragma unroll
    for (int i = 0; i < 5; ++i) xm[i] = 0.5 * (xa[i] + xb[i]) + (h / 8.0) * (fa[i] - fb[i]);
    dyn(xm, u1, u2, route_kappa(R, xm[0], nullptr, nullptr), fm);
#pragma unroll
    for (int i = 0; i < 5; ++i) def[i] = xb[i] - (xa[i] + P.defect_sign * (h / 6.0) * (fa[i] + 4.0 * fm[i] + fb[i]));
}

// ------------------------------------------------------------------------------------------------------
// per-chunk state held in registers
// ------------------------------------------------------------------------------------------------------
struct Chunk {
    int N, fin;
    double x0[5], st, den;
    double delta;
    double xi0[5], e[2], nu[2];
};

// the rows of stage k (kinds in order) — the structure of build_qp in the oracle
__device__ int stage_rows(int k, int N, int fin, int kinds[NR]) {
    int n = 0;
    if (!(fin && k == N)) {
        kinds[n++] = ROW_VMIN;
        kinds[n++] = ROW_VMAX;
        if (k > 0) {
            kinds[n++] = ROW_LATP;
            kinds[n++] = ROW_LATM;
        }
    }
    if (k > 0) {
        kinds[n++] = ROW_KMIN;
        kinds[n++] = ROW_KMAX;
    }
    if (k < N) {
        kinds[n++] = ROW_U1MIN;
        kinds[n++] = ROW_U1MAX;
        kinds[n++] = ROW_U2MIN;
        kinds[n++] = ROW_U2MAX;
        kinds[n++] = ROW_S;
    }
    if (k == N && !fin) kinds[n++] = ROW_STERM;
    return n;
}

// coefficients of a row over (x_k, w_k), at the SQP iterate's (k, v) of stage k
__device__ void row_coef(int kind, bool has_w, double kb, double vb, double a[NZ]) {
#pragma unroll
    for (int u = 0; u < NZ; ++u) a[u] = 0.0;
    switch (kind) {
        case ROW_VMIN: a[4] = 1.0; a[7] = has_w ? 1.0 : 0.0; break;
        case ROW_VMAX: a[4] = -1.0; a[7] = has_w ? -1.0 : 0.0; break;
        case ROW_LATP: a[3] = -vb * vb; a[4] = -2.0 * kb * vb; break;
        case ROW_LATM: a[3] = vb * vb; a[4] = 2.0 * kb * vb; break;
        case ROW_KMIN: a[3] = 1.0; break;
        case ROW_KMAX: a[3] = -1.0; break;
        case ROW_U1MIN: a[5] = 1.0; break;
        case ROW_U1MAX: a[5] = -1.0; break;
        case ROW_U2MIN: a[6] = 1.0; break;
        case ROW_U2MAX: a[6] = -1.0; break;
        case ROW_S: a[7] = 1.0; break;
        default: a[0] = 1.0; break;                              // ROW_STERM
    }
}

struct Ctx {
    DevRoute R;
    plan_params P;
    Layout Y;
    Ln S;
    Chunk C;
};

// row j of stage k: coefficients (from the SQP iterate in ZB)
__device__ inline void coef_of(const Ctx& X, int k, int kind, double a[NZ]) {
    row_coef(kind, k < X.C.N, X.S[X.Y.oZB + NZ * k + 3], X.S[X.Y.oZB + NZ * k + 4], a);
}

__device__ inline double row_val(const Ctx& X, int k, int j, const double a[NZ], int oz) {
    double v = X.S[X.Y.oG + NR * k + j];
#pragma unroll
    for (int u = 0; u < NZ; ++u) v += a[u] * X.S[oz + NZ * k + u];
    return v;
}

// Gaussian elimination with partial pivoting on a 5x5 system with ncol right-hand sides (registers)
template <int NC>
__device__ bool solve5(double M[25], double R[5 * NC]) {
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        int pr = c;
        for (int i = c + 1; i < 5; ++i)
            if (fabs(M[5 * i + c]) > fabs(M[5 * pr + c])) pr = i;
        if (M[5 * pr + c] == 0.0) return false;
        if (pr != c) {
            for (int j = 0; j < 5; ++j) { const double t = M[5 * c + j]; M[5 * c + j] = M[5 * pr + j]; M[5 * pr + j] = t; }
            for (int j = 0; j < NC; ++j) { const double t = R[NC * c + j]; R[NC * c + j] = R[NC * pr + j]; R[NC * pr + j] = t; }
        }
        for (int i = c + 1; i < 5; ++i) {
            const double f = M[5 * i + c] / M[5 * c + c];
            for (int j = c; j < 5; ++j) M[5 * i + j] -= f * M[5 * c + j];
            for (int j = 0; j < NC; ++j) R[NC * i + j] -= f * R[NC * c + j];
        }
    }
    for (int c = 4; c >= 0; --c)
        for (int j = 0; j < NC; ++j) {
            double v = R[NC * c + j];
            for (int k = c + 1; k < 5; ++k) v -= M[5 * c + k] * R[NC * k + j];
            R[NC * c + j] = v / M[5 * c + c];
        }
    return true;
}

// interval k's linearisation at the iterate (xa, xb, u): A, B, c, D1 into scratch
__device__ bool interval_lin(Ctx& X, int k, const double xa[5], const double xb[5], double u1, double u2) {
    const double h = X.P.dt, sg = X.P.defect_sign;
    double dka, dkb, dkm, fa[5], fb[5], fm[5], xm[5], Fa[25], Fb[25], Fm[25];
    const double ka = route_kappa(X.R, xa[0], &dka, nullptr);
    const double kb = route_kappa(X.R, xb[0], &dkb, nullptr);
    dyn(xa, u1, u2, ka, fa);
    dyn(xb, u1, u2, kb, fb);
#pragma unroll
    for (int i = 0; i < 5; ++i) xm[i] = 0.5 * (xa[i] + xb[i]) + (h / 8.0) * (fa[i] - fb[i]);
    const double km = route_kappa(X.R, xm[0], &dkm, nullptr);
    dyn(xm, u1, u2, km, fm);
    double def[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) def[i] = xb[i] - (xa[i] + sg * (h / 6.0) * (fa[i] + 4.0 * fm[i] + fb[i]));
    dyn_jac(xa, ka, dka, Fa);
    dyn_jac(xb, kb, dkb, Fb);
    dyn_jac(xm, km, dkm, Fm);
    double D1[25], R[5 * 8];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            double m0 = 0.0, m1 = 0.0;
#pragma unroll
            for (int l = 0; l < 5; ++l) {
                const double ia = (l == j ? 0.5 : 0.0) + (h / 8.0) * Fa[5 * l + j];
                const double ib = (l == j ? 0.5 : 0.0) - (h / 8.0) * Fb[5 * l + j];
                m0 += Fm[5 * i + l] * ia;
                m1 += Fm[5 * i + l] * ib;
            }
            R[8 * i + j] = -((i == j ? -1.0 : 0.0) - sg * (h / 6.0) * (Fa[5 * i + j] + 4.0 * m0));
            D1[5 * i + j] = (i == j ? 1.0 : 0.0) - sg * (h / 6.0) * (4.0 * m1 + Fb[5 * i + j]);
        }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        R[8 * i + 5] = i == 3 ? sg * h : 0.0;
        R[8 * i + 6] = i == 4 ? sg * h : 0.0;
        R[8 * i + 7] = -def[i];
    }
#pragma unroll
    for (int i = 0; i < 25; ++i) X.S[X.Y.oD1 + 25 * k + i] = D1[i];
    if (!solve5<8>(D1, R)) return false;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
#pragma unroll
        for (int j = 0; j < 5; ++j) X.S[X.Y.oA + 25 * k + 5 * i + j] = R[8 * i + j];
        X.S[X.Y.oB + 15 * k + 3 * i + 0] = R[8 * i + 5];
        X.S[X.Y.oB + 15 * k + 3 * i + 1] = R[8 * i + 6];
        X.S[X.Y.oB + 15 * k + 3 * i + 2] = 0.0;
        X.S[X.Y.oC + 5 * k + i] = R[8 * i + 7];
    }
    return true;
}

// interval k's share of the Lagrangian Hessian (-y . def_k over (x_a, x_b)) folded into stage k's Hessian
// and gradient along x_{k+1} = A x_k + B w_k + c
__device__ void interval_hess_fold(Ctx& X, int k, const double xa[5], const double xb[5], double u1, double u2,
                                   const double y[5]) {
    const double h = X.P.dt, f6 = X.P.defect_sign * h / 6.0;
    double k1a, k2a, k1b, k2b, k1m, k2m, fa[5], fb[5], fm[5], xm[5], Fa[25], Fb[25], Fm[25];
    const double ka = route_kappa(X.R, xa[0], &k1a, &k2a);
    const double kb = route_kappa(X.R, xb[0], &k1b, &k2b);
    dyn(xa, u1, u2, ka, fa);
    dyn(xb, u1, u2, kb, fb);
#pragma unroll
    for (int i = 0; i < 5; ++i) xm[i] = 0.5 * (xa[i] + xb[i]) + (h / 8.0) * (fa[i] - fb[i]);
    const double km = route_kappa(X.R, xm[0], &k1m, &k2m);
    dyn(xm, u1, u2, km, fm);
    dyn_jac(xa, ka, k1a, Fa);
    dyn_jac(xb, kb, k1b, Fb);
    dyn_jac(xm, km, k1m, Fm);
    double yb[5], Wm[25], Haa[25], Hab[25], Hbb[25];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < 5; ++i) v += Fm[5 * i + j] * y[i];
        yb[j] = v;
    }
    hess_f(xm, km, k1m, k2m, y, Wm);
    {
        // Ma' Wm Ma, Ma' Wm Mb, Mb' Wm Mb with Ma = I/2 + h/8 Fa, Mb = I/2 - h/8 Fb
        double WMa[25], WMb[25];
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                double va = 0.0, vb = 0.0;
#pragma unroll
                for (int l = 0; l < 5; ++l) {
                    va += Wm[5 * i + l] * ((l == j ? 0.5 : 0.0) + (h / 8.0) * Fa[5 * l + j]);
                    vb += Wm[5 * i + l] * ((l == j ? 0.5 : 0.0) - (h / 8.0) * Fb[5 * l + j]);
                }
                WMa[5 * i + j] = va;
                WMb[5 * i + j] = vb;
            }
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                double aa = 0.0, ab = 0.0, bb = 0.0;
#pragma unroll
                for (int l = 0; l < 5; ++l) {
                    const double mai = (l == i ? 0.5 : 0.0) + (h / 8.0) * Fa[5 * l + i];
                    const double mbi = (l == i ? 0.5 : 0.0) - (h / 8.0) * Fb[5 * l + i];
                    aa += mai * WMa[5 * l + j];
                    ab += mai * WMb[5 * l + j];
                    bb += mbi * WMb[5 * l + j];
                }
                Haa[5 * i + j] = 4.0 * aa;
                Hab[5 * i + j] = f6 * 4.0 * ab;
                Hbb[5 * i + j] = 4.0 * bb;
            }
    }
    {
        double W[25];
        hess_f(xa, ka, k1a, k2a, y, W);
#pragma unroll
        for (int i = 0; i < 25; ++i) Haa[i] += W[i];
        hess_f(xa, ka, k1a, k2a, yb, W);
#pragma unroll
        for (int i = 0; i < 25; ++i) Haa[i] = f6 * (Haa[i] + 4.0 * (h / 8.0) * W[i]);
        hess_f(xb, kb, k1b, k2b, y, W);
#pragma unroll
        for (int i = 0; i < 25; ++i) Hbb[i] += W[i];
        hess_f(xb, kb, k1b, k2b, yb, W);
#pragma unroll
        for (int i = 0; i < 25; ++i) Hbb[i] = f6 * (Hbb[i] - 4.0 * (h / 8.0) * W[i]);
    }
    // fold: T = [I 0; A B]
    double T[5][NZ], c[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
#pragma unroll
        for (int j = 0; j < 5; ++j) T[i][j] = X.S[X.Y.oA + 25 * k + 5 * i + j];
#pragma unroll
        for (int j = 0; j < 3; ++j) T[i][5 + j] = X.S[X.Y.oB + 15 * k + 3 * i + j];
        c[i] = X.S[X.Y.oC + 5 * k + i];
    }
    double HbT[5][NZ], HabT[5][NZ];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < NZ; ++j) {
            double vb = 0.0, va = 0.0;
#pragma unroll
            for (int l = 0; l < 5; ++l) { vb += Hbb[5 * i + l] * T[l][j]; va += Hab[5 * i + l] * T[l][j]; }
            HbT[i][j] = vb;
            HabT[i][j] = va;
        }
#pragma unroll
    for (int i = 0; i < NZ; ++i)
#pragma unroll
        for (int j = 0; j < NZ; ++j) {
            double v = 0.0;
#pragma unroll
            for (int l = 0; l < 5; ++l) v += T[l][i] * HbT[l][j];
            if (i < 5) v += HabT[i][j];
            if (j < 5) v += HabT[j][i];
            if (i < 5 && j < 5) v += Haa[5 * i + j];
            X.S[X.Y.oH + 64 * k + 8 * i + j] += v;
        }
    double hbc[5];
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        double v = 0.0;
#pragma unroll
        for (int m = 0; m < 5; ++m) v += Hbb[5 * l + m] * c[m];
        hbc[l] = v;
    }
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
        double v = 0.0;
#pragma unroll
        for (int l = 0; l < 5; ++l) v += T[l][i] * hbc[l];
        if (i < 5)
#pragma unroll
            for (int m = 0; m < 5; ++m) v += Hab[5 * i + m] * c[m];
        X.S[X.Y.oGQ + NZ * k + i] += v;
    }
}

// the QP at the SQP iterate in ZB (frozen: speed limits from VLIM; exact: multipliers MY / MLAT)
__device__ bool build_qp(Ctx& X, bool frozen, bool exact) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    const plan_params& P = X.P;
    const double den = X.C.den;
    X.C.delta = 0.0;
    for (int k = 0; k <= N; ++k) {
        double x[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = S[Y.oZB + NZ * k + i];
#pragma unroll
        for (int i = 0; i < 64; ++i) S[Y.oH + 64 * k + i] = 0.0;
#pragma unroll
        for (int i = 0; i < NZ; ++i) S[Y.oGQ + NZ * k + i] = 0.0;
        const double u1 = k < N ? S[Y.oZB + NZ * k + 5] : 0.0, u2 = k < N ? S[Y.oZB + NZ * k + 6] : 0.0;
        const double sl = k < N ? S[Y.oZB + NZ * k + 7] : 0.0;
        if (k < N) {
            S[Y.oH + 64 * k + 0] = 2.0 * P.w_s / (den * den);
            S[Y.oH + 64 * k + 9] = 2.0 * P.w_y;
            S[Y.oH + 64 * k + 18] = 2.0 * P.w_y;
            S[Y.oH + 64 * k + 45] = 2.0 * P.w_u;
            S[Y.oH + 64 * k + 54] = 2.0 * P.w_u;
            S[Y.oH + 64 * k + 63] = 2.0 * P.w_slack;
            S[Y.oGQ + NZ * k + 0] = -2.0 * P.w_s * (X.R.s_total - x[0]) / (den * den);
            S[Y.oGQ + NZ * k + 1] = 2.0 * P.w_y * x[1];
            S[Y.oGQ + NZ * k + 2] = 2.0 * P.w_y * x[2];
            S[Y.oGQ + NZ * k + 5] = 2.0 * P.w_u * u1;
            S[Y.oGQ + NZ * k + 6] = 2.0 * P.w_u * u2;
            S[Y.oGQ + NZ * k + 7] = 2.0 * P.w_slack * sl;
            double xb[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) xb[i] = S[Y.oZB + NZ * (k + 1) + i];
            if (!interval_lin(X, k, x, xb, u1, u2)) return false;
            if (exact) {
                double y[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) y[i] = S[Y.oMY + 5 * k + i];
                interval_hess_fold(X, k, x, xb, u1, u2, y);
            }
        }
        int kinds[NR];
        const int nr = stage_rows(k, N, X.C.fin, kinds);
        const double kk = x[3], v = x[4];
        for (int j = 0; j < nr; ++j) {
            double gv = 0.0;
            switch (kinds[j]) {
                case ROW_VMIN: gv = v + sl - P.v_min; break;
                case ROW_VMAX: gv = (frozen ? S[Y.oVLIM + k] : route_vmax(X.R, x[0])) - (v + sl); break;
                case ROW_LATP: gv = P.a_max - kk * v * v; break;
                case ROW_LATM: gv = P.a_max + kk * v * v; break;
                case ROW_KMIN: gv = kk - P.k_min; break;
                case ROW_KMAX: gv = P.k_max - kk; break;
                case ROW_U1MIN: gv = u1 - P.u_min[0]; break;
                case ROW_U1MAX: gv = P.u_max[0] - u1; break;
                case ROW_U2MIN: gv = u2 - P.u_min[1]; break;
                case ROW_U2MAX: gv = P.u_max[1] - u2; break;
                case ROW_S: gv = sl; break;
                default: gv = x[0] - X.C.st / 2.0; break;
            }
            S[Y.oG + NR * k + j] = gv;
        }
        if (exact && k > 0 && !(X.C.fin && k == N)) {
            const double lp = S[Y.oMLAT + 2 * k], lm = S[Y.oMLAT + 2 * k + 1];
            S[Y.oH + 64 * k + 8 * 3 + 4] += 2.0 * v * (lp - lm);
            S[Y.oH + 64 * k + 8 * 4 + 3] += 2.0 * v * (lp - lm);
            S[Y.oH + 64 * k + 8 * 4 + 4] += 2.0 * kk * (lp - lm);
        }
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) X.C.xi0[i] = X.C.x0[i] - S[Y.oZB + i];
    X.C.e[0] = X.C.st - S[Y.oZB + NZ * N + 0];
    X.C.e[1] = -S[Y.oZB + NZ * N + 4];
    return true;
}

// row weights of the factorisation: mode 0 = lam / s (interior point), 1 = RHO on TACT rows (polish)
__device__ inline double row_weight(const Ctx& X, int k, int j, int mode) {
    if (mode == 0) return X.S[X.Y.oLAM + NR * k + j] / X.S[X.Y.oS + NR * k + j];
    return X.S[X.Y.oTACT + NR * k + j] != 0.0 ? RHO : 0.0;
}

__device__ void stage_hess(const Ctx& X, int k, int mode, double H[NZ][NZ]) {
    const int N = X.C.N;
#pragma unroll
    for (int i = 0; i < NZ; ++i)
#pragma unroll
        for (int j = 0; j < NZ; ++j) H[i][j] = X.S[X.Y.oH + 64 * k + 8 * i + j];
    const int nv = k < N ? NZ : 5;
#pragma unroll
    for (int i = 0; i < NZ; ++i)
        if (i < nv) H[i][i] += X.C.delta;
    int kinds[NR];
    const int nr = stage_rows(k, N, X.C.fin, kinds);
    for (int j = 0; j < nr; ++j) {
        const double w = row_weight(X, k, j, mode);
        if (w == 0.0) continue;
        double a[NZ];
        coef_of(X, k, kinds[j], a);
#pragma unroll
        for (int u = 0; u < NZ; ++u)
#pragma unroll
            for (int v = 0; v < NZ; ++v) H[u][v] += w * a[u] * a[v];
    }
}

__device__ bool chol3(const double H[3][3], double L[6]) {
    if (!(H[0][0] > 0.0)) return false;
    L[0] = sqrt(H[0][0]);
    L[1] = H[1][0] / L[0];
    const double d1 = H[1][1] - L[1] * L[1];
    if (!(d1 > 0.0)) return false;
    L[2] = sqrt(d1);
    L[3] = H[2][0] / L[0];
    L[4] = (H[2][1] - L[3] * L[1]) / L[2];
    const double d2 = H[2][2] - L[3] * L[3] - L[4] * L[4];
    if (!(d2 > 0.0)) return false;
    L[5] = sqrt(d2);
    return true;
}

__device__ inline void chol3_solve(const double L[6], double b[3]) {
    const double y0 = b[0] / L[0];
    const double y1 = (b[1] - L[1] * y0) / L[2];
    const double y2 = (b[2] - L[3] * y0 - L[4] * y1) / L[5];
    b[2] = y2 / L[5];
    b[1] = (y1 - L[4] * b[2]) / L[2];
    b[0] = (y0 - L[1] * b[1] - L[3] * b[2]) / L[0];
}

// LQ solve with zero initial state and homogeneous dynamics: stage linear terms at ogl, result at odz
__device__ void solve_core(const Ctx& X, int ogl, int odz) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    double p[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) p[i] = S[ogl + NZ * N + i];
    // backward: kk_k into odz's w slots (scratch until the forward pass overwrites them in order)
    for (int k = N - 1; k >= 0; --k) {
        double Bm[15], h[3], L[6];
#pragma unroll
        for (int i = 0; i < 15; ++i) Bm[i] = S[Y.oB + 15 * k + i];
#pragma unroll
        for (int i = 0; i < 6; ++i) L[i] = S[Y.oL + 6 * k + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            double v = S[ogl + NZ * k + 5 + i];
#pragma unroll
            for (int l = 0; l < 5; ++l) v += Bm[3 * l + i] * p[l];
            h[i] = v;
        }
        double t[3] = {-h[0], -h[1], -h[2]};
        chol3_solve(L, t);
#pragma unroll
        for (int i = 0; i < 3; ++i) S[odz + NZ * k + 5 + i] = t[i];
        if (k > 0) {
            double pn[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                double v = S[ogl + NZ * k + i];
#pragma unroll
                for (int l = 0; l < 5; ++l) v += S[Y.oA + 25 * k + 5 * l + i] * p[l];
#pragma unroll
                for (int l = 0; l < 3; ++l) v += S[Y.oK + 15 * k + 5 * l + i] * h[l];
                pn[i] = v;
            }
#pragma unroll
            for (int i = 0; i < 5; ++i) p[i] = pn[i];
        }
    }
    double x[5] = {0, 0, 0, 0, 0};
    for (int k = 0; k < N; ++k) {
        double w[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            double v = S[odz + NZ * k + 5 + i];
#pragma unroll
            for (int l = 0; l < 5; ++l) v += S[Y.oK + 15 * k + 5 * i + l] * x[l];
            w[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) S[odz + NZ * k + i] = x[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) S[odz + NZ * k + 5 + i] = w[i];
        double xn[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            double v = 0.0;
#pragma unroll
            for (int l = 0; l < 5; ++l) v += S[Y.oA + 25 * k + 5 * i + l] * x[l];
#pragma unroll
            for (int l = 0; l < 2; ++l) v += S[Y.oB + 15 * k + 3 * i + l] * w[l];
            xn[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = xn[i];
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) S[odz + NZ * N + i] = x[i];
#pragma unroll
    for (int i = 5; i < NZ; ++i) S[odz + NZ * N + i] = 0.0;
}

// Riccati factorisation with row weights of `mode`; false when a control pivot is not positive
__device__ bool factor(Ctx& X, int mode, double Em[4]) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    double H[NZ][NZ], P[25];
    stage_hess(X, N, mode, H);
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) P[5 * i + j] = H[i][j];
    for (int k = N - 1; k >= 0; --k) {
        stage_hess(X, k, mode, H);
        double A[25], Bm[10], PA[25], PB[10], Hww[3][3], Hwx[15], L[6];
#pragma unroll
        for (int i = 0; i < 25; ++i) A[i] = S[Y.oA + 25 * k + i];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            Bm[2 * i] = S[Y.oB + 15 * k + 3 * i];
            Bm[2 * i + 1] = S[Y.oB + 15 * k + 3 * i + 1];
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) {
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                double v = 0.0;
#pragma unroll
                for (int l = 0; l < 5; ++l) v += P[5 * i + l] * A[5 * l + j];
                PA[5 * i + j] = v;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                double v = 0.0;
#pragma unroll
                for (int l = 0; l < 5; ++l) v += P[5 * i + l] * Bm[2 * l + j];
                PB[2 * i + j] = v;
            }
        }
        // B's S column is zero: its rows / columns of Hww and Hwx are the stage Hessian's alone
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                double v = H[5 + i][5 + j];
                if (i < 2 && j < 2)
#pragma unroll
                    for (int l = 0; l < 5; ++l) v += Bm[2 * l + i] * PB[2 * l + j];
                Hww[i][j] = v;
            }
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                double v = H[5 + i][j];
                if (i < 2)
#pragma unroll
                    for (int l = 0; l < 5; ++l) v += Bm[2 * l + i] * PA[5 * l + j];
                Hwx[5 * i + j] = v;
            }
        }
        if (!chol3(Hww, L)) return false;
        double K[15];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            double col[3] = {-Hwx[j], -Hwx[5 + j], -Hwx[10 + j]};
            chol3_solve(L, col);
            K[j] = col[0];
            K[5 + j] = col[1];
            K[10 + j] = col[2];
        }
#pragma unroll
        for (int i = 0; i < 15; ++i) S[Y.oK + 15 * k + i] = K[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) S[Y.oL + 6 * k + i] = L[i];
        if (k > 0) {
            double Pn[25];
#pragma unroll
            for (int i = 0; i < 5; ++i)
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    double v = H[i][j];
#pragma unroll
                    for (int l = 0; l < 5; ++l) v += A[5 * l + i] * PA[5 * l + j];
#pragma unroll
                    for (int l = 0; l < 3; ++l) v += Hwx[5 * l + i] * K[5 * l + j];
                    Pn[5 * i + j] = v;
                }
#pragma unroll
            for (int i = 0; i < 5; ++i)
#pragma unroll
                for (int j = 0; j < 5; ++j) P[5 * i + j] = 0.5 * (Pn[5 * i + j] + Pn[5 * j + i]);
        }
    }
    if (X.C.fin) {
        for (int c = 0; c < 2; ++c) {
            const int og = Y.oGL, oe = Y.oEZ;
            for (int k = 0; k <= N; ++k)
#pragma unroll
                for (int i = 0; i < NZ; ++i) S[og + NZ * k + i] = 0.0;
            S[og + NZ * N + (c == 0 ? 0 : 4)] = 1.0;
            solve_core(X, og, Y.oDZ);
            for (int k = 0; k <= N; ++k)
#pragma unroll
                for (int i = 0; i < NZ; ++i) S[oe + 2 * NZ * k + NZ * c + i] = S[Y.oDZ + NZ * k + i];
        }
        Em[0] = S[Y.oEZ + 2 * NZ * N + 0];           // E row s, force 0
        Em[1] = S[Y.oEZ + 2 * NZ * N + NZ + 0];      // E row s, force 1
        Em[2] = S[Y.oEZ + 2 * NZ * N + 4];           // E row v, force 0
        Em[3] = S[Y.oEZ + 2 * NZ * N + NZ + 4];
        const double det = Em[0] * Em[3] - Em[1] * Em[2];
        if (!(fabs(det) > 0.0) || !isfinite(det)) return false;
    }
    return true;
}

__device__ bool factor_reg(Ctx& X, int mode, double Em[4]) {
    while (!factor(X, mode, Em)) {
        if (X.C.delta >= DELTA_MAX) return false;
        X.C.delta = X.C.delta > 0.0 ? 10.0 * X.C.delta : DELTA0;
    }
    return true;
}

// full solve: gl at oGL, result at oDZ; meets E dz_N = rE exactly (final chunk), nu = terminal forces
__device__ void solve(Ctx& X, const double Em[4], const double rE[2], double nu[2]) {
    solve_core(X, X.Y.oGL, X.Y.oDZ);
    nu[0] = nu[1] = 0.0;
    if (!X.C.fin) return;
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    const double b0 = rE[0] - S[Y.oDZ + NZ * N + 0], b1 = rE[1] - S[Y.oDZ + NZ * N + 4];
    const double det = Em[0] * Em[3] - Em[1] * Em[2];
    const double n0 = (b0 * Em[3] - Em[1] * b1) / det;
    const double n1 = (Em[0] * b1 - Em[2] * b0) / det;
    for (int k = 0; k <= N; ++k)
#pragma unroll
        for (int i = 0; i < NZ; ++i)
            S[Y.oDZ + NZ * k + i] += n0 * S[Y.oEZ + 2 * NZ * k + i] + n1 * S[Y.oEZ + 2 * NZ * k + NZ + i];
    nu[0] = n0;
    nu[1] = n1;
}

// dynamics-feasible start at oz: dx_0 = xi0, dw = 0
__device__ void rollout(const Ctx& X, int oz) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    double x[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) x[i] = X.C.xi0[i];
    for (int k = 0; k <= N; ++k) {
#pragma unroll
        for (int i = 0; i < 5; ++i) S[oz + NZ * k + i] = x[i];
#pragma unroll
        for (int i = 5; i < NZ; ++i) S[oz + NZ * k + i] = 0.0;
        if (k == N) break;
        double xn[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            double v = S[Y.oC + 5 * k + i];
#pragma unroll
            for (int l = 0; l < 5; ++l) v += S[Y.oA + 25 * k + 5 * i + l] * x[l];
            xn[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = xn[i];
    }
}

// gradient of the QP objective at the stage-k variables in oz
__device__ void grad_f(const Ctx& X, int k, int oz, double g[NZ]) {
    const int nv = k < X.C.N ? NZ : 5;
    double z[NZ];
#pragma unroll
    for (int i = 0; i < NZ; ++i) z[i] = X.S[oz + NZ * k + i];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
        double v = X.S[X.Y.oGQ + NZ * k + i] + (i < nv ? X.C.delta * z[i] : 0.0);
#pragma unroll
        for (int j = 0; j < NZ; ++j) v += X.S[X.Y.oH + 64 * k + 8 * i + j] * z[j];
        g[i] = i < nv ? v : 0.0;
    }
}

// equality-constrained QP on the TACT rows (estimates TLAM), solution into TZ / TLAM; 0 = KKT-consistent,
// > 0 = offending rows (flipped in TACT), -1 = breakdown
__device__ int eqp(Ctx& X, double scale, double nu[2]) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    double Em[4];
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < NR; ++j)
            S[Y.oY + NR * k + j] = S[Y.oTACT + NR * k + j] != 0.0 ? S[Y.oTLAM + NR * k + j] : 0.0;
    if (!factor_reg(X, 1, Em)) return -1;
    rollout(X, Y.oTZ);
    for (int it = 0; it < AL_STEPS; ++it) {
        for (int k = 0; k <= N; ++k) {
            double g[NZ];
            grad_f(X, k, Y.oTZ, g);
            int kinds[NR];
            const int nr = stage_rows(k, N, X.C.fin, kinds);
            for (int j = 0; j < nr; ++j) {
                if (S[Y.oTACT + NR * k + j] == 0.0) continue;
                double a[NZ];
                coef_of(X, k, kinds[j], a);
                const double f = RHO * row_val(X, k, j, a, Y.oTZ) - S[Y.oY + NR * k + j];
#pragma unroll
                for (int u = 0; u < NZ; ++u) g[u] += f * a[u];
            }
#pragma unroll
            for (int u = 0; u < NZ; ++u) S[Y.oGL + NZ * k + u] = g[u];
        }
        const double rE[2] = {X.C.e[0] - S[Y.oTZ + NZ * N + 0], X.C.e[1] - S[Y.oTZ + NZ * N + 4]};
        solve(X, Em, rE, nu);
        for (int k = 0; k <= N; ++k) {
#pragma unroll
            for (int u = 0; u < NZ; ++u) S[Y.oTZ + NZ * k + u] += S[Y.oDZ + NZ * k + u];
            int kinds[NR];
            const int nr = stage_rows(k, N, X.C.fin, kinds);
            for (int j = 0; j < nr; ++j)
                if (S[Y.oTACT + NR * k + j] != 0.0) {
                    double a[NZ];
                    coef_of(X, k, kinds[j], a);
                    S[Y.oY + NR * k + j] -= RHO * row_val(X, k, j, a, Y.oTZ);
                }
        }
    }
    bool finite = true;
    for (int k = 0; k <= N; ++k)
#pragma unroll
        for (int u = 0; u < NZ; ++u) finite &= (bool)isfinite(S[Y.oTZ + NZ * k + u]);
    if (!finite) return -1;
    int bad = 0;
    const double tr = 1e-9 * scale, tl = 1e-9 * scale;
    for (int k = 0; k <= N; ++k) {
        int kinds[NR];
        const int nr = stage_rows(k, N, X.C.fin, kinds);
        for (int j = 0; j < nr; ++j) {
            double a[NZ];
            coef_of(X, k, kinds[j], a);
            const double rv = row_val(X, k, j, a, Y.oTZ);
            if (S[Y.oTACT + NR * k + j] != 0.0) {
                const double y = S[Y.oY + NR * k + j];
                S[Y.oTLAM + NR * k + j] = y;
                if (y < -tl || fabs(rv) > tr) { S[Y.oTACT + NR * k + j] = 0.0; ++bad; }
            } else {
                S[Y.oTLAM + NR * k + j] = 0.0;
                if (rv < -tr) { S[Y.oTACT + NR * k + j] = 1.0; ++bad; }
            }
        }
    }
    return bad;
}

// Mehrotra predictor-corrector interior point; solution in Z, S, LAM; 0 converged, 1 cap, -1 breakdown
__device__ int ipm(Ctx& X, int* iters) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    rollout(X, Y.oZ);
    int m = 0;
    for (int k = 0; k <= N; ++k) {
        int kinds[NR];
        const int nr = stage_rows(k, N, X.C.fin, kinds);
        for (int j = 0; j < nr; ++j) {
            double a[NZ];
            coef_of(X, k, kinds[j], a);
            const double rv = row_val(X, k, j, a, Y.oZ);
            S[Y.oS + NR * k + j] = (rv > 0.0 ? rv : 0.0) + SHIFT0;
            S[Y.oLAM + NR * k + j] = 1.0;
            ++m;
        }
    }
    double phi = 1.0, Em[4];
    int it = 0, rc = 1;
    for (; it < X.P.max_iter; ++it) {
        double mu = 0.0;
        for (int k = 0; k <= N; ++k) {
            int kinds[NR];
            const int nr = stage_rows(k, N, X.C.fin, kinds);
            for (int j = 0; j < nr; ++j) {
                double a[NZ];
                coef_of(X, k, kinds[j], a);
                S[Y.oRP + NR * k + j] = row_val(X, k, j, a, Y.oZ) - S[Y.oS + NR * k + j];
                mu += S[Y.oS + NR * k + j] * S[Y.oLAM + NR * k + j];
            }
        }
        mu /= m;
        if (!isfinite(mu)) { rc = -1; break; }
        if (mu <= X.P.tol && phi <= 1e-12) { rc = 0; break; }
        if (!factor_reg(X, 0, Em)) { rc = -1; break; }
        const double rE[2] = {X.C.e[0] - S[Y.oZ + NZ * N + 0], X.C.e[1] - S[Y.oZ + NZ * N + 4]};
        for (int pass = 0; pass < 2; ++pass) {
            double sigma_mu = 0.0;
            if (pass == 1) {
                double am = 1.0;
                for (int k = 0; k <= N; ++k) {
                    int kinds[NR];
                    const int nr = stage_rows(k, N, X.C.fin, kinds);
                    for (int j = 0; j < nr; ++j) {
                        const double dsa = S[Y.oDSA + NR * k + j], dla = S[Y.oDLA + NR * k + j];
                        if (dsa < 0.0) am = fmin(am, -S[Y.oS + NR * k + j] / dsa);
                        if (dla < 0.0) am = fmin(am, -S[Y.oLAM + NR * k + j] / dla);
                    }
                }
                double mua = 0.0;
                for (int k = 0; k <= N; ++k) {
                    int kinds[NR];
                    const int nr = stage_rows(k, N, X.C.fin, kinds);
                    for (int j = 0; j < nr; ++j)
                        mua += (S[Y.oS + NR * k + j] + am * S[Y.oDSA + NR * k + j]) *
                               (S[Y.oLAM + NR * k + j] + am * S[Y.oDLA + NR * k + j]);
                }
                mua /= m;
                const double ratio = mua / mu;
                sigma_mu = ratio * ratio * ratio * mu;
            }
            for (int k = 0; k <= N; ++k) {
                double g[NZ];
                grad_f(X, k, Y.oZ, g);
                int kinds[NR];
                const int nr = stage_rows(k, N, X.C.fin, kinds);
                for (int j = 0; j < nr; ++j) {
                    double a[NZ];
                    coef_of(X, k, kinds[j], a);
                    const double s = S[Y.oS + NR * k + j], l = S[Y.oLAM + NR * k + j];
                    double rs = -s * l;
                    if (pass == 1) rs += sigma_mu - S[Y.oDSA + NR * k + j] * S[Y.oDLA + NR * k + j];
                    const double f = l + (rs - l * S[Y.oRP + NR * k + j]) / s;
#pragma unroll
                    for (int u = 0; u < NZ; ++u) g[u] -= f * a[u];
                }
#pragma unroll
                for (int u = 0; u < NZ; ++u) S[Y.oGL + NZ * k + u] = g[u];
            }
            solve(X, Em, rE, X.C.nu);
            const int ods = pass == 0 ? Y.oDSA : Y.oDS, odl = pass == 0 ? Y.oDLA : Y.oDL;
            for (int k = 0; k <= N; ++k) {
                int kinds[NR];
                const int nr = stage_rows(k, N, X.C.fin, kinds);
                for (int j = 0; j < nr; ++j) {
                    double a[NZ];
                    coef_of(X, k, kinds[j], a);
                    const double s = S[Y.oS + NR * k + j], l = S[Y.oLAM + NR * k + j];
                    double rs = -s * l;
                    if (pass == 1) rs += sigma_mu - S[Y.oDSA + NR * k + j] * S[Y.oDLA + NR * k + j];
                    double v = S[Y.oRP + NR * k + j];
#pragma unroll
                    for (int u = 0; u < NZ; ++u) v += a[u] * S[Y.oDZ + NZ * k + u];
                    S[ods + NR * k + j] = v;
                    S[odl + NR * k + j] = (rs - l * v) / s;
                }
            }
        }
        double amax = 1.0 / TAU;
        bool finite = true;
        for (int k = 0; k <= N; ++k) {
            int kinds[NR];
            const int nr = stage_rows(k, N, X.C.fin, kinds);
            for (int j = 0; j < nr; ++j) {
                const double ds = S[Y.oDS + NR * k + j], dl = S[Y.oDL + NR * k + j];
                if (ds < 0.0) amax = fmin(amax, -S[Y.oS + NR * k + j] / ds);
                if (dl < 0.0) amax = fmin(amax, -S[Y.oLAM + NR * k + j] / dl);
            }
#pragma unroll
            for (int u = 0; u < NZ; ++u) finite &= (bool)isfinite(S[Y.oDZ + NZ * k + u]);
        }
        const double alpha = fmin(1.0, TAU * amax);
        if (!isfinite(alpha) || !finite) { rc = -1; break; }
        for (int k = 0; k <= N; ++k) {
#pragma unroll
            for (int u = 0; u < NZ; ++u) S[Y.oZ + NZ * k + u] += alpha * S[Y.oDZ + NZ * k + u];
            int kinds[NR];
            const int nr = stage_rows(k, N, X.C.fin, kinds);
            for (int j = 0; j < nr; ++j) {
                S[Y.oS + NR * k + j] += alpha * S[Y.oDS + NR * k + j];
                S[Y.oLAM + NR * k + j] += alpha * S[Y.oDL + NR * k + j];
            }
        }
        phi *= 1.0 - alpha;
    }
    *iters = it;
    return rc;
}

// copy the polish result (TZ, TLAM, TACT) to the solution (Z, LAM, ACT)
__device__ void accept_polish(const Ctx& X, bool with_act) {
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    for (int k = 0; k <= X.C.N; ++k) {
#pragma unroll
        for (int u = 0; u < NZ; ++u) S[Y.oZ + NZ * k + u] = S[Y.oTZ + NZ * k + u];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            S[Y.oLAM + NR * k + j] = S[Y.oTLAM + NR * k + j];
            if (with_act) S[Y.oACT + NR * k + j] = S[Y.oTACT + NR * k + j];
        }
    }
}

// one QP: 0 solved (KKT point), 1 interior-point answer without a certified polish, -1 failure
__device__ int qp_solve(Ctx& X, bool have_cls, int* iters) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    double scale = 1.0, nu[2];
    for (int k = 0; k <= N; ++k) {
        int kinds[NR];
        const int nr = stage_rows(k, N, X.C.fin, kinds);
        for (int j = 0; j < nr; ++j) scale = fmax(scale, fabs(S[Y.oG + NR * k + j]));
    }
    *iters = 0;
    if (have_cls) {
        for (int k = 0; k <= N; ++k)
#pragma unroll
            for (int j = 0; j < NR; ++j) {
                S[Y.oTACT + NR * k + j] = S[Y.oACT + NR * k + j];
                S[Y.oTLAM + NR * k + j] = S[Y.oLAM + NR * k + j];
            }
        if (eqp(X, scale, nu) == 0) {
            accept_polish(X, false);
            X.C.nu[0] = nu[0];
            X.C.nu[1] = nu[1];
            return 0;
        }
    }
    const int rc = ipm(X, iters);
    if (rc < 0) return -1;
    for (int k = 0; k <= N; ++k)
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            S[Y.oTACT + NR * k + j] = S[Y.oS + NR * k + j] < S[Y.oLAM + NR * k + j] ? 1.0 : 0.0;
            S[Y.oTLAM + NR * k + j] = S[Y.oLAM + NR * k + j];
        }
    for (int round = 0; round < POLISH_ROUNDS; ++round) {
        const int bad = eqp(X, scale, nu);
        if (bad < 0) break;
        if (bad == 0) {
            accept_polish(X, true);
            X.C.nu[0] = nu[0];
            X.C.nu[1] = nu[1];
            return 0;
        }
    }
    for (int k = 0; k <= N; ++k)
#pragma unroll
        for (int j = 0; j < NR; ++j)
            S[Y.oACT + NR * k + j] = S[Y.oS + NR * k + j] < S[Y.oLAM + NR * k + j] ? 1.0 : 0.0;
    return rc == 0 ? 1 : -1;
}

// NLP multipliers from the QP solution (oracle multipliers()): MY, MLAT
__device__ void multipliers(const Ctx& X) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    double pi[5];
    for (int k = N; k >= 0; --k) {
        double g[NZ];
        grad_f(X, k, Y.oZ, g);
        int kinds[NR];
        const int nr = stage_rows(k, N, X.C.fin, kinds);
        S[Y.oMLAT + 2 * k] = 0.0;
        S[Y.oMLAT + 2 * k + 1] = 0.0;
        for (int j = 0; j < nr; ++j) {
            double a[NZ];
            coef_of(X, k, kinds[j], a);
            const double l = S[Y.oLAM + NR * k + j];
#pragma unroll
            for (int u = 0; u < NZ; ++u) g[u] -= l * a[u];
            if (kinds[j] == ROW_LATP) S[Y.oMLAT + 2 * k] = l;
            if (kinds[j] == ROW_LATM) S[Y.oMLAT + 2 * k + 1] = l;
        }
        if (k == N) {
#pragma unroll
            for (int i = 0; i < 5; ++i) pi[i] = g[i];
            if (X.C.fin) {
                pi[0] += X.C.nu[0];
                pi[4] += X.C.nu[1];
            }
            continue;
        }
        double D1t[25], y[5];
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) D1t[5 * i + j] = S[Y.oD1 + 25 * k + 5 * j + i];
#pragma unroll
        for (int i = 0; i < 5; ++i) y[i] = pi[i];
        if (solve5<1>(D1t, y)) {
#pragma unroll
            for (int i = 0; i < 5; ++i) S[Y.oMY + 5 * k + i] = y[i];
        } else {
#pragma unroll
            for (int i = 0; i < 5; ++i) S[Y.oMY + 5 * k + i] = 0.0;
        }
        if (k > 0) {
            double pn[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                double v = g[i];
#pragma unroll
                for (int l = 0; l < 5; ++l) v += S[Y.oA + 25 * k + 5 * l + i] * pi[l];
                pn[i] = v;
            }
#pragma unroll
            for (int i = 0; i < 5; ++i) pi[i] = pn[i];
        }
    }
}

// the NLP's cost (:128-170) and L1 violation at the iterate in oz (+ alpha * DZV when alpha != 0)
__device__ void cost_viol(const Ctx& X, int oz, double alpha, double* f, double* viol) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    const plan_params& P = X.P;
    auto zv = [&](int k, int i) { return S[oz + NZ * k + i] + (alpha != 0.0 ? alpha * S[Y.oDZV + NZ * k + i] : 0.0); };
    double c = 0.0, v = 0.0;
    for (int i = 0; i < 5; ++i) v += fabs(zv(0, i) - X.C.x0[i]);
    for (int k = 0; k <= N; ++k) {
        double x[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = zv(k, i);
        const double u1 = k < N ? zv(k, 5) : 0.0, u2 = k < N ? zv(k, 6) : 0.0, sl = k < N ? zv(k, 7) : 0.0;
        if (k < N) {
            const double e = (X.R.s_total - x[0]) / X.C.den;
            c += P.w_y * (x[1] * x[1] + x[2] * x[2]) + P.w_s * e * e + P.w_u * (u1 * u1 + u2 * u2) + P.w_slack * (sl * sl);
            double xb[5], def[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) xb[i] = zv(k + 1, i);
            defect(X.R, P, x, xb, u1, u2, def);
#pragma unroll
            for (int i = 0; i < 5; ++i) v += fabs(def[i]);
        }
        const double kk = x[3], vv = x[4];
        double g[12];
        int n = 0;
        if (!(X.C.fin && k == N)) {
            g[n++] = vv + sl - P.v_min;
            g[n++] = S[Y.oVL + k] - (vv + sl);
            if (k > 0) {
                g[n++] = P.a_max - kk * vv * vv;
                g[n++] = P.a_max + kk * vv * vv;
            }
        }
        if (k > 0) {
            g[n++] = kk - P.k_min;
            g[n++] = P.k_max - kk;
        }
        if (k < N) {
            g[n++] = u1 - P.u_min[0];
            g[n++] = P.u_max[0] - u1;
            g[n++] = u2 - P.u_min[1];
            g[n++] = P.u_max[1] - u2;
            g[n++] = sl;
        }
        if (k == N && !X.C.fin) g[n++] = x[0] - X.C.st / 2.0;
        for (int j = 0; j < n; ++j) v += g[j] < 0.0 ? -g[j] : 0.0;
    }
    if (X.C.fin) v += fabs(zv(N, 0) - X.C.st) + fabs(zv(N, 4));
    *f = c;
    *viol = v;
}

__device__ double cost_dir(const Ctx& X) {
    const int N = X.C.N;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    const plan_params& P = X.P;
    double v = 0.0;
    for (int k = 0; k < N; ++k) {
            v += 2.0 * P.w_y * (S[Y.oZB + NZ * k + 1] * S[Y.oDZV + NZ * k + 1] + S[Y.oZB + NZ * k + 2] * S[Y.oDZV + NZ * k + 2]);
        v += -2.0 * P.w_s * (X.R.s_total - S[Y.oZB + NZ * k]) / (X.C.den * X.C.den) * S[Y.oDZV + NZ * k];
        v += 2.0 * P.w_u * (S[Y.oZB + NZ * k + 5] * S[Y.oDZV + NZ * k + 5] + S[Y.oZB + NZ * k + 6] * S[Y.oDZV + NZ * k + 6]);
        v += 2.0 * P.w_slack * S[Y.oZB + NZ * k + 7] * S[Y.oDZV + NZ * k + 7];
    }
    return v;
}

struct KArgs {
    DevRoute R;
    plan_params P;
    int B, Nmax, Nfixed;
    const int* N;
    const double *x0, *st;
    const int* fin;
    double *X, *U, *S;
    int *status, *iters, *sqp;
    double* scratch;
    int per_lane;        // Layout.total
};

__global__ void __launch_bounds__(WAVE) plan_chunk_kernel(KArgs a) {
    const int lane = threadIdx.x;
    const int b = blockIdx.x * WAVE + lane;
    if (b >= a.B) return;
    Ctx X;
    X.R = a.R;
    X.P = a.P;
    X.Y = make_layout(a.Nmax);
    X.S.b = a.scratch + (size_t)blockIdx.x * a.per_lane * WAVE + lane;
    Chunk& C = X.C;
    C.N = a.N ? a.N[b] : a.Nfixed;
    const int N = C.N;
    C.fin = a.fin ? (a.fin[b] != 0) : 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) C.x0[i] = a.x0[5 * (size_t)b + i];
    C.st = a.st[b];
    C.den = fmax(1.0, a.R.s_total - C.x0[0]);
    C.nu[0] = C.nu[1] = 0.0;
    const Ln& S = X.S;
    const Layout& Y = X.Y;
    // initial guess (:357-376)
    const double dss = (C.st - C.x0[0]) / N;
    for (int k = 0; k <= N; ++k) {
#pragma unroll
        for (int i = 0; i < NZ; ++i) S[Y.oZB + NZ * k + i] = 0.0;
        S[Y.oZB + NZ * k + 0] = k == N ? C.st : C.x0[0] + k * dss;
        S[Y.oZB + NZ * k + 4] = C.fin ? (k == N ? 0.0 : C.x0[4] + k * ((0.0 - C.x0[4]) / N)) : C.x0[4];
#pragma unroll
        for (int i = 0; i < NZ; ++i) S[Y.oZ2 + NZ * k + i] = S[Y.oZB + NZ * k + i];
    }
    int status = PLAN_NOT_CONVERGED, total = 0, nq = 0, since = 0;
    bool have_cls = false, frozen = false;
    double last = INFINITY, mu_m = 0.0, hf[LS_MEMORY], hv[LS_MEMORY];
    int nh = 0;
    for (int it = 0; it < a.P.sqp_iters; ++it, ++since) {
        bool exact = last <= EXACT_STEP;
        int rc = -1;
        for (;;) {
            if (!build_qp(X, frozen, exact)) { rc = -2; break; }
            int ni = 0;
            rc = qp_solve(X, have_cls, &ni);
            total += ni;
            if (rc >= 0 || !exact) break;
            exact = false;
        }
        ++nq;
        if (rc == -2) { status = PLAN_NUMERICAL; break; }
        if (rc < 0) { status = PLAN_QP_FAILED; break; }
        have_cls = true;
        multipliers(X);
        double full = 0.0;
        for (int k = 0; k <= N; ++k)
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                const double d = (k < N || i < 5) ? S[Y.oZ + NZ * k + i] : 0.0;
                S[Y.oDZV + NZ * k + i] = d;
                full = fmax(full, fabs(d));
            }
        for (int k = 0; k <= N; ++k) {
            if (k < N)
#pragma unroll
                for (int i = 0; i < 5; ++i) mu_m = fmax(mu_m, 2.0 * fabs(S[Y.oMY + 5 * k + i]));
            int kinds[NR];
            const int nr = stage_rows(k, N, C.fin, kinds);
            for (int j = 0; j < nr; ++j) mu_m = fmax(mu_m, 2.0 * fabs(S[Y.oLAM + NR * k + j]));
        }
        if (C.fin) mu_m = fmax(mu_m, 2.0 * fmax(fabs(C.nu[0]), fabs(C.nu[1])));
        double alpha = 1.0;
        if (full > LS_FULL) {
            for (int k = 0; k <= N; ++k) S[Y.oVL + k] = frozen ? S[Y.oVLIM + k] : route_vmax(X.R, S[Y.oZB + NZ * k]);
            double f0, v0;
            cost_viol(X, Y.oZB, 0.0, &f0, &v0);
            const double dd = cost_dir(X) - mu_m * v0;
            hf[nh % LS_MEMORY] = f0;
            hv[nh % LS_MEMORY] = v0;
            ++nh;
            double m0 = -INFINITY;
            for (int i = 0; i < (nh < LS_MEMORY ? nh : LS_MEMORY); ++i) m0 = fmax(m0, hf[i] + mu_m * hv[i]);
            for (int ls = 0; ls < LS_STEPS; ++ls) {
                double f1, v1;
                cost_viol(X, Y.oZB, alpha, &f1, &v1);
                if (f1 + mu_m * v1 <= m0 + LS_ARMIJO * alpha * dd || ls == LS_STEPS - 1) break;
                alpha *= 0.5;
            }
        }
        double step = 0.0, back2 = 0.0;
        bool fin = true;
        for (int k = 0; k <= N; ++k)
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                if (k == N && i >= 5) continue;
                const double zo = S[Y.oZB + NZ * k + i];
                const double zn = zo + alpha * S[Y.oDZV + NZ * k + i];
                S[Y.oZN + NZ * k + i] = zn;
                step = fmax(step, fabs(zn - zo));
                back2 = fmax(back2, fabs(zn - S[Y.oZ2 + NZ * k + i]));
                fin &= (bool)isfinite(zn);
            }
        if (!fin) { status = PLAN_NUMERICAL; break; }
        for (int k = 0; k <= N; ++k)
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                if (k == N && i >= 5) continue;
                S[Y.oZ2 + NZ * k + i] = S[Y.oZB + NZ * k + i];
                S[Y.oZB + NZ * k + i] = S[Y.oZN + NZ * k + i];
            }
        last = step;
        if (step <= a.P.sqp_tol) { status = frozen ? PLAN_FROZEN_LIMITS : PLAN_OK; break; }
        if (since >= 2 && back2 <= CYCLE_REL * step) {
            if (frozen) break;
            for (int k = 0; k <= N; ++k)
                S[Y.oVLIM + k] = fmin(route_vmax(X.R, S[Y.oZB + NZ * k]), route_vmax(X.R, S[Y.oZ2 + NZ * k]));
            frozen = true;
            since = -1;
            for (int k = 0; k <= N; ++k)
#pragma unroll
                for (int i = 0; i < NZ; ++i) S[Y.oZ2 + NZ * k + i] = S[Y.oZB + NZ * k + i];
        }
    }
    if (status == PLAN_FROZEN_LIMITS) {
        for (int k = 0; k <= N; ++k)
            if (S[Y.oZB + NZ * k + 4] + (k < N ? S[Y.oZB + NZ * k + 7] : 0.0) > route_vmax(X.R, S[Y.oZB + NZ * k]) + 1e-9)
                status = PLAN_NOT_CONVERGED;
    }
    // outputs: rows past this chunk's N are zero
    const int Nm = a.Nmax;
    if (a.X)
        for (int k = 0; k <= Nm; ++k)
#pragma unroll
            for (int i = 0; i < 5; ++i) a.X[((size_t)b * (Nm + 1) + k) * 5 + i] = k <= N ? S[Y.oZB + NZ * k + i] : 0.0;
    if (a.U)
        for (int k = 0; k < Nm; ++k) {
            a.U[((size_t)b * Nm + k) * 2 + 0] = k < N ? S[Y.oZB + NZ * k + 5] : 0.0;
            a.U[((size_t)b * Nm + k) * 2 + 1] = k < N ? S[Y.oZB + NZ * k + 6] : 0.0;
        }
    if (a.S)
        for (int k = 0; k < Nm; ++k) a.S[(size_t)b * Nm + k] = k < N ? S[Y.oZB + NZ * k + 7] : 0.0;
    if (a.status) a.status[b] = status;
    if (a.iters) a.iters[b] = total;
    if (a.sqp) a.sqp[b] = nq;
}

__global__ void route_eval_kernel(DevRoute R, int n, const double* s, double* k, double* dk, double* vm) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double d1 = 0.0;
    const double kv = route_kappa(R, s[i], &d1, nullptr);
    k[i] = kv;
    dk[i] = d1;
    vm[i] = route_vmax(R, s[i]);
}

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace

struct plan_ctx {
    int device;
    plan_params p;
    DevRoute R;
    double* d_route;          // s | cx | cy | vmax
    double* scratch;
    size_t scratch_doubles;
    // host-entry staging
    void* io;
    size_t io_bytes;
};

static int check_params(const plan_params* p) {
    if (!p) return fail(PLAN_E_ARG, "params is NULL");
    if (!(p->dt > 0.0)) return fail(PLAN_E_ARG, "dt must be > 0");
    if (p->N < 1 || p->N > PLAN_MAX_N) return fail(PLAN_E_ARG, "N out of range [1, PLAN_MAX_N]");
    if (p->sqp_iters < 1 || p->max_iter < 1) return fail(PLAN_E_ARG, "sqp_iters and max_iter must be >= 1");
    if (!(p->sqp_tol >= 0.0) || !(p->tol > 0.0)) return fail(PLAN_E_ARG, "tolerances must be positive");
    if (!(p->defect_sign == 1.0 || p->defect_sign == -1.0)) return fail(PLAN_E_ARG, "defect_sign must be +1 or -1");
    if (!(p->u_min[0] < p->u_max[0]) || !(p->u_min[1] < p->u_max[1]) || !(p->k_min < p->k_max))
        return fail(PLAN_E_ARG, "bounds must satisfy min < max");
    return PLAN_SUCCESS;
}

extern "C" {

void plan_default_params(plan_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->N = 20;
    p->dt = 0.3;
    p->w_y = 10.0; p->w_s = 10.0; p->w_u = 0.1; p->w_slack = 100.0;
    p->u_min[0] = -0.6; p->u_min[1] = -5.0;
    p->u_max[0] = 0.6; p->u_max[1] = 4.0;
    p->k_min = -0.8; p->k_max = 0.8;
    p->a_max = 6.0;
    p->v_min = 0.0;
    p->defect_sign = 1.0;
    p->sqp_iters = 100;
    p->sqp_tol = 1e-9;
    p->max_iter = 100;
    p->tol = 1e-10;
}

const char* plan_last_error(void) { return g_err.c_str(); }
int plan_version(void) { return MPCPLAN_VERSION; }

int plan_create(const double* s, int M, const double* cx, const double* cy, const double* vmax, const plan_params* p,
                int device, plan_ctx** out) {
    if (!out) return fail(PLAN_E_ARG, "out is NULL");
    *out = nullptr;
    if (!s || !cx || !cy || !vmax) return fail(PLAN_E_ARG, "route arrays must not be NULL");
    if (M < 3) return fail(PLAN_E_ARG, "a route needs at least 3 way-points");
    for (int i = 1; i < M; ++i)
        if (!(s[i] > s[i - 1])) return fail(PLAN_E_ARG, "route s must be strictly increasing");
    for (int i = 0; i < 4 * (M - 1); ++i)
        if (!std::isfinite(cx[i]) || !std::isfinite(cy[i])) return fail(PLAN_E_ARG, "spline coefficients must be finite");
    for (int i = 0; i < M; ++i)
        if (!std::isfinite(vmax[i])) return fail(PLAN_E_ARG, "speed limits must be finite");
    if (int rc = check_params(p)) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PLAN_E_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(PLAN_E_DEVICE, "device index out of range (there is no host backend)");
    if (hipSetDevice(device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    plan_ctx* c = new plan_ctx();
    c->device = device;
    c->p = *p;
    const size_t n = (size_t)M + 8 * (size_t)(M - 1) + M;
    if (hipMalloc(&c->d_route, n * sizeof(double)) != hipSuccess) {
        delete c;
        return fail(PLAN_E_ALLOC, "route allocation failed");
    }
    std::vector<double> h(n);
    std::memcpy(h.data(), s, sizeof(double) * M);
    std::memcpy(h.data() + M, cx, sizeof(double) * 4 * (M - 1));
    std::memcpy(h.data() + M + 4 * (M - 1), cy, sizeof(double) * 4 * (M - 1));
    std::memcpy(h.data() + M + 8 * (M - 1), vmax, sizeof(double) * M);
    if (hipMemcpy(c->d_route, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(c->d_route);
        delete c;
        return fail(PLAN_E_DEVICE, "route upload failed");
    }
    c->R.s = c->d_route;
    c->R.cx = c->d_route + M;
    c->R.cy = c->d_route + M + 4 * (M - 1);
    c->R.vmax = c->d_route + M + 8 * (M - 1);
    c->R.M = M;
    c->R.s_total = s[M - 1];
    *out = c;
    return PLAN_SUCCESS;
}

int plan_set_params(plan_ctx* c, const plan_params* p) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (int rc = check_params(p)) return rc;
    c->p = *p;
    return PLAN_SUCCESS;
}

void plan_destroy(plan_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    if (c->d_route) (void)hipFree(c->d_route);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->io) (void)hipFree(c->io);
    delete c;
}

int plan_solve_chunks_device(plan_ctx* c, int B, int Nmax, const int* N, const double* x0, const double* s_target,
                             const int* is_final, double* X, double* U, double* S, int* status, int* iters, int* sqp,
                             void* stream) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (B < 0) return fail(PLAN_E_ARG, "B must be >= 0");
    if (B == 0) return PLAN_SUCCESS;
    if (!x0 || !s_target) return fail(PLAN_E_ARG, "x0 and s_target are required");
    if (!N) Nmax = c->p.N;
    if (Nmax < 1 || Nmax > PLAN_MAX_N) return fail(PLAN_E_ARG, "Nmax out of range [1, PLAN_MAX_N]");
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    hipStream_t st = (hipStream_t)stream;
    const Layout Y = make_layout(Nmax);
    const int waves = (B + WAVE - 1) / WAVE;
    const size_t need = (size_t)waves * WAVE * Y.total;
    if (need > c->scratch_doubles) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
            return fail(PLAN_E_ALLOC, "scratch too small while the stream is being captured: run one eager call first");
        (void)hipStreamSynchronize(st);
        if (c->scratch) (void)hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_doubles = 0;
        if (hipMalloc(&c->scratch, need * sizeof(double)) != hipSuccess) return fail(PLAN_E_ALLOC, "scratch allocation failed");
        c->scratch_doubles = need;
    }
    KArgs a;
    a.R = c->R;
    a.P = c->p;
    a.B = B;
    a.Nmax = Nmax;
    a.Nfixed = c->p.N;
    a.N = N;
    a.x0 = x0;
    a.st = s_target;
    a.fin = is_final;
    a.X = X;
    a.U = U;
    a.S = S;
    a.status = status;
    a.iters = iters;
    a.sqp = sqp;
    a.scratch = c->scratch;
    a.per_lane = Y.total;
    hipLaunchKernelGGL(plan_chunk_kernel, dim3(waves), dim3(WAVE), 0, st, a);
    if (hipGetLastError() != hipSuccess) return fail(PLAN_E_LAUNCH, "plan kernel launch failed");
    return PLAN_SUCCESS;
}

int plan_solve_chunks(plan_ctx* c, int B, const int* N, const double* x0, const double* s_target, const int* is_final,
                      double* X, double* U, double* S, int* status, int* iters, int* sqp) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (B < 0) return fail(PLAN_E_ARG, "B must be >= 0");
    if (B == 0) return PLAN_SUCCESS;
    if (!x0 || !s_target) return fail(PLAN_E_ARG, "x0 and s_target are required");
    int Nmax = c->p.N;
    if (N) {
        Nmax = 0;
        for (int b = 0; b < B; ++b) {
            if (N[b] < 1 || N[b] > PLAN_MAX_N) return fail(PLAN_E_ARG, "N[b] out of range [1, PLAN_MAX_N]");
            Nmax = std::max(Nmax, N[b]);
        }
    }
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    // one staging block: inputs, then outputs
    const size_t nX = (size_t)B * (Nmax + 1) * 5, nU = (size_t)B * Nmax * 2, nS = (size_t)B * Nmax;
    const size_t bytes = sizeof(double) * (5 * (size_t)B + B + nX + nU + nS) + sizeof(int) * (5 * (size_t)B);
    if (bytes > c->io_bytes) {
        if (c->io) (void)hipFree(c->io);
        c->io = nullptr;
        c->io_bytes = 0;
        if (hipMalloc(&c->io, bytes) != hipSuccess) return fail(PLAN_E_ALLOC, "staging allocation failed");
        c->io_bytes = bytes;
    }
    double* d_x0 = (double*)c->io;
    double* d_st = d_x0 + 5 * (size_t)B;
    double* d_X = d_st + B;
    double* d_U = d_X + nX;
    double* d_S = d_U + nU;
    int* d_N = (int*)(d_S + nS);
    int* d_fin = d_N + B;
    int* d_status = d_fin + B;
    int* d_iters = d_status + B;
    int* d_sqp = d_iters + B;
    bool ok = hipMemcpy(d_x0, x0, sizeof(double) * 5 * B, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_st, s_target, sizeof(double) * B, hipMemcpyHostToDevice) == hipSuccess;
    if (ok && N) ok = hipMemcpy(d_N, N, sizeof(int) * B, hipMemcpyHostToDevice) == hipSuccess;
    if (ok && is_final) ok = hipMemcpy(d_fin, is_final, sizeof(int) * B, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) return fail(PLAN_E_DEVICE, "input upload failed");
    int rc = plan_solve_chunks_device(c, B, Nmax, N ? d_N : nullptr, d_x0, d_st, is_final ? d_fin : nullptr, d_X, d_U,
                                      d_S, d_status, d_iters, d_sqp, nullptr);
    if (rc != PLAN_SUCCESS) return rc;
    if (hipDeviceSynchronize() != hipSuccess) return fail(PLAN_E_DEVICE, "plan kernel failed");
    ok = (!X || hipMemcpy(X, d_X, sizeof(double) * nX, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!U || hipMemcpy(U, d_U, sizeof(double) * nU, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!S || hipMemcpy(S, d_S, sizeof(double) * nS, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!status || hipMemcpy(status, d_status, sizeof(int) * B, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!iters || hipMemcpy(iters, d_iters, sizeof(int) * B, hipMemcpyDeviceToHost) == hipSuccess) &&
         (!sqp || hipMemcpy(sqp, d_sqp, sizeof(int) * B, hipMemcpyDeviceToHost) == hipSuccess);
    if (!ok) return fail(PLAN_E_DEVICE, "output download failed");
    return PLAN_SUCCESS;
}

int plan_route_eval(plan_ctx* c, int n, const double* s, double* kappa, double* dkappa, double* vmax) {
    if (!c) return fail(PLAN_E_ARG, "ctx is NULL");
    if (n < 0 || (n > 0 && (!s || !kappa || !dkappa || !vmax))) return fail(PLAN_E_ARG, "bad arguments");
    if (n == 0) return PLAN_SUCCESS;
    if (hipSetDevice(c->device) != hipSuccess) return fail(PLAN_E_DEVICE, "hipSetDevice failed");
    double* d = nullptr;
    if (hipMalloc(&d, sizeof(double) * 4 * (size_t)n) != hipSuccess) return fail(PLAN_E_ALLOC, "allocation failed");
    int rc = PLAN_SUCCESS;
    if (hipMemcpy(d, s, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(PLAN_E_DEVICE, "upload failed");
    if (rc == PLAN_SUCCESS) {
        hipLaunchKernelGGL(route_eval_kernel, dim3((n + 255) / 256), dim3(256), 0, nullptr, c->R, n, d, d + n, d + 2 * n,
                           d + 3 * n);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = fail(PLAN_E_LAUNCH, "route kernel failed");
    }
    if (rc == PLAN_SUCCESS &&
        (hipMemcpy(kappa, d + n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(dkappa, d + 2 * n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(vmax, d + 3 * n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess))
        rc = fail(PLAN_E_DEVICE, "download failed");
    (void)hipFree(d);
    return rc;
}

}  // extern "C"

// mpcqp.hip — MI355X (gfx950) batched tracking-MPC solver + its C ABI (include/mpcqp.h).
//
// Hot path replaced: TrajectoryTracker.solve(x0, obstacles)
//   medinammartin3/Safe-Autonomous-Driving-MPC trajectory_tracking.py:213-263
// with TrajectoryLoader.get_state/get_control (trajectory_loader.py:86-102) on a device table.
//
// One 64-lane wavefront (= one workgroup) per MPC instance:
//   K1  warm start (trajectory_tracking.py:224-246), lane j = control step j
//   K1  nominal rollout == predict(x0, ubar) (:87-114), lookups lane-parallel, bit-exact
//   K2  Gauss-Newton QP(ubar) stage data, lane k = stage k
//   K4  Mehrotra primal-dual interior point: row/stage-parallel residuals, barrier weights,
//       step lengths on lanes; the Newton systems solved by a stage-wise (Riccati) recursion
//       executed wave-uniformly from LDS (FP64; the dense condensed Cholesky loses ~5 digits
//       on these problems)
//   K5  predict(x0, U*) (:261) and outputs
// Compiled with -ffp-contract=off: the interp / rollout / warm-start arithmetic is bit-exact to
// the reference's numpy arithmetic; the solver uses explicit fma() where it wants fusion.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mpcqp.h"

#define WAVE 64
#define NROW 9
#define NBOX 4
#define XI0 1e-4
#define TAU 0.995

// ------------------------------------------------------------------------------------------
// device table + kernel parameters
// ------------------------------------------------------------------------------------------
struct DevTable {
    const double* s;   // [T]  (strict-monotone fixed, trajectory_loader.py:26-30)
    const double* d;
    const double* o;
    const double* k;
    const double* v;
    const double* u1;  // [Tu]
    const double* u2;
    int T, Tu;
    double smax;
    double last[5];    // X_ref[-1] verbatim (trajectory_loader.py:90-91)
};

struct KParams {
    int N, max_obs, linearization, sqp_iters, max_iter, polish;
    double dt, u_min0, u_min1, u_max0, u_max1;
    double w_d, w_o, w_v, w_u1, w_u2;
    double osd, tgap, L, sl, brake_distance, brake_accel;
    double tol, tol_mu, rho;
};

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmin(v, __shfl_xor(v, m, WAVE));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, WAVE));
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
    return v;
}
__device__ __forceinline__ void wave_sync() { __syncthreads(); }

// ------------------------------------------------------------------------------------------
// reference signal: scipy interp1d 'linear' + extrapolate (scipy _interpolate.py:457-483)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int seg(const double* __restrict__ x, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (x[mid] < v) lo = mid + 1; else hi = mid;
    }
    lo = lo < 1 ? 1 : lo;
    lo = lo > n - 1 ? n - 1 : lo;
    return lo;
}
__device__ __forceinline__ double lin(const double* x, const double* y, int i, double v) {
    double slope = (y[i] - y[i - 1]) / (x[i] - x[i - 1]);
    return slope * (v - x[i - 1]) + y[i - 1];
}
__device__ __forceinline__ double slope_at(const double* x, const double* y, int i) {
    return (y[i] - y[i - 1]) / (x[i] - x[i - 1]);
}
// get_state (trajectory_loader.py:86-93): out[5]; slopes (d,o,k,v) for Gauss-Newton (0 past s_max)
__device__ void get_state(const DevTable& t, double s, double* out, double* sl) {
    if (s >= t.smax) {
        for (int j = 0; j < 5; ++j) out[j] = t.last[j];
        if (sl) sl[0] = sl[1] = sl[2] = sl[3] = 0.0;
        return;
    }
    int i = seg(t.s, t.T, s);
    out[0] = s;
    out[1] = lin(t.s, t.d, i, s);
    out[2] = lin(t.s, t.o, i, s);
    out[3] = lin(t.s, t.k, i, s);
    out[4] = lin(t.s, t.v, i, s);
    if (sl) {
        sl[0] = slope_at(t.s, t.d, i);
        sl[1] = slope_at(t.s, t.o, i);
        sl[2] = slope_at(t.s, t.k, i);
        sl[3] = slope_at(t.s, t.v, i);
    }
}
// get_control (trajectory_loader.py:95-102)
__device__ void get_control(const DevTable& t, double s, double* out) {
    if (s >= t.smax) { out[0] = 0.0; out[1] = 0.0; return; }
    int i = seg(t.s, t.Tu, s);
    out[0] = lin(t.s, t.u1, i, s);
    out[1] = lin(t.s, t.u2, i, s);
}

// ------------------------------------------------------------------------------------------
// per-instance LDS layout (doubles); stage arrays indexed by stage k = 0..N
// ------------------------------------------------------------------------------------------
struct Lds {
    double* A5;    // [N][5]    a12,a14,a20,a23,a24 of A_k = I + J'_k  (a04 = dt)
    double* cst;   // [N+1][6]  cost data of stage k: (-d_ref', -o_ref', -v_ref') and the residuals r_d, r_o, r_v
    double* Qt;    // [N+1][10] Riccati stage Hessians on (s,d,o,v) (barrier / penalty augmented), packed
    double* Rt;    // [N][2]
    double* Kf;    // [N][10]   Riccati gains K_t (2x5)
    double* Si;    // [N][3]    (1/l00, l10, 1/l11) of S_t = Ls Ls'
    double* qh;    // [N+1][4]  LQR stage linear terms (state)
    double* gh;    // [N][2]    LQR stage linear terms (control)
    double* kk;    // [N][2]
    double* Xr;    // [N+1][5]  rollout of the current iterate
    double* dX;    // [N+1][5]  rollout of the direction
    double* du;    // [N][2]    current iterate dU
    double* dud;   // [N][2]    direction dU
    double* dub;   // [N][2]    interior-point iterate kept during the polish
    double* yc;    // [N+1][4]  dual-residual stage terms: cost part
    double* ya;    // [N+1][4]  dual-residual stage terms: multiplier part
    double* zc;    // [N][2]
    double* za;    // [N][2]
    double* ub;    // [N][2]    linearisation point
    double* xb;    // [N+1][5]  nominal rollout / predict output
    double* kap;   // [N+1]     k_ref(xbar_k); then shat_k (min obstacle prediction)
};

__host__ __device__ inline int lds_doubles(int N) {
    int NP = N + 1;
    return N * 5 + NP * 6 + NP * 10 + N * 2 + N * 10 + N * 3 + NP * 4 + N * 2 + N * 2 + NP * 5 + NP * 5 + N * 2 +
           N * 2 + N * 2 + NP * 4 + NP * 4 + N * 2 + N * 2 + N * 2 + NP * 5 + NP;
}

__device__ inline Lds carve(double* p, int N) {
    Lds L;
    int NP = N + 1;
    L.A5 = p; p += N * 5;
    L.cst = p; p += NP * 6;
    L.Qt = p; p += NP * 10;
    L.Rt = p; p += N * 2;
    L.Kf = p; p += N * 10;
    L.Si = p; p += N * 3;
    L.qh = p; p += NP * 4;
    L.gh = p; p += N * 2;
    L.kk = p; p += N * 2;
    L.Xr = p; p += NP * 5;
    L.dX = p; p += NP * 5;
    L.du = p; p += N * 2;
    L.dud = p; p += N * 2;
    L.dub = p; p += N * 2;
    L.yc = p; p += NP * 4;
    L.ya = p; p += NP * 4;
    L.zc = p; p += N * 2;
    L.za = p; p += N * 2;
    L.ub = p; p += N * 2;
    L.xb = p; p += NP * 5;
    L.kap = p; p += NP;
    return L;
}

// packed symmetric 4x4 on (s,d,o,v): index of (a,b)
__host__ __device__ __forceinline__ int p4(int a, int b) {
    if (a > b) { int t = a; a = b; b = t; }
    return a == 0 ? b : (a == 1 ? 3 + b : (a == 2 ? 5 + b : 9));
}
// state index (0..4: s,d,o,k,v) of reduced index (0..3: s,d,o,v)
__device__ __forceinline__ int st4(int a) { return a == 3 ? 4 : a; }

// soft row coefficient vectors over (s,d,o,v) (the oracle's C[][] without the k entry)
__device__ __forceinline__ void row_coef(int j, double h, double L, double T, double c[4]) {
    c[0] = c[1] = c[2] = c[3] = 0.0;
    switch (j) {
        case 0: c[1] = 1.0; break;
        case 1: c[1] = -1.0; break;
        case 2: c[1] = 1.0; c[2] = h; break;
        case 3: c[1] = -1.0; c[2] = -h; break;
        case 4: c[1] = 1.0; c[2] = L; break;
        case 5: c[1] = -1.0; c[2] = -L; break;
        case 6: c[0] = -1.0; break;
        case 7: c[0] = -1.0; c[3] = -T; break;
        default: c[3] = 1.0; break;
    }
}
__device__ __forceinline__ double bsign(int j) { return (j & 1) ? -1.0 : 1.0; }   // box rows +u1,-u1,+u2,-u2
__device__ __forceinline__ double dot4(const double c[4], const double x[4]) {
    return fma(c[0], x[0], fma(c[1], x[1], fma(c[2], x[2], c[3] * x[3])));
}
// 1/x to full double precision: v_rcp_f64 + two Newton steps (no IEEE division sequence)
__device__ __forceinline__ double frcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// ------------------------------------------------------------------------------------------
// lane groups: IPW instances per 64-lane wavefront, GL = 64 / IPW lanes each
// ------------------------------------------------------------------------------------------
template <int GL>
struct Grp {
    int base;   // first lane of the group
    __device__ __forceinline__ double sum(double v) const {
#pragma unroll
        for (int m = GL / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
        return v;
    }
    __device__ __forceinline__ double max(double v) const {
#pragma unroll
        for (int m = GL / 2; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, WAVE));
        return v;
    }
    __device__ __forceinline__ double min(double v) const {
#pragma unroll
        for (int m = GL / 2; m >= 1; m >>= 1) v = fmin(v, __shfl_xor(v, m, WAVE));
        return v;
    }
    __device__ __forceinline__ double get(double v, int rel) const { return __shfl(v, base + rel, WAVE); }
};

// nonlinear rollout (predict, trajectory_tracking.py:87-114), bit-exact.  s, v, k do not depend on
// the k_ref lookups, so they are rolled first; lane j then looks up k_ref(s_j); then d, o.
__device__ void predict_grp(const DevTable& tab, int N, double dt, const double* x0, const double* uU, double* xout,
                            double* kap, int ln) {
    if (ln == 0) {
        double s = x0[0], k = x0[3], v = x0[4];
        for (int a = 0; a < 5; ++a) xout[a] = x0[a];
        for (int j = 0; j < N; ++j) {
            double s1 = s + dt * v;
            double k1 = k + dt * uU[2 * j];
            double v1 = v + dt * uU[2 * j + 1];
            s = s1; k = k1; v = v1;
            xout[5 * (j + 1) + 0] = s;
            xout[5 * (j + 1) + 3] = k;
            xout[5 * (j + 1) + 4] = v;
        }
    }
    wave_sync();
    if (ln < N) {
        double st[5];
        get_state(tab, xout[5 * ln], st, nullptr);
        kap[ln] = st[3];
    }
    wave_sync();
    if (ln == 0) {
        double d = x0[1], o = x0[2];
        for (int j = 0; j < N; ++j) {
            double v = xout[5 * j + 4], k = xout[5 * j + 3];
            double xd1 = v * o, xd2 = v * (k - kap[j]);
            double d1 = d + dt * xd1;
            double o1 = o + dt * xd2;
            d = d1; o = o1;
            xout[5 * (j + 1) + 1] = d;
            xout[5 * (j + 1) + 2] = o;
        }
    }
    wave_sync();
}

// A_k x with A_k = I + J'_k (sparse)
__device__ __forceinline__ void applyA(const double* a, double dt, const double x[5], double y[5]) {
    y[0] = fma(dt, x[4], x[0]);
    y[1] = fma(a[0], x[2], fma(a[1], x[4], x[1]));
    y[2] = fma(a[2], x[0], fma(a[3], x[3], fma(a[4], x[4], x[2])));
    y[3] = x[3];
    y[4] = x[4];
}
__device__ __forceinline__ void applyAT(const double* a, double dt, const double m[5], double y[5]) {
    y[0] = fma(a[2], m[2], m[0]);
    y[1] = m[1];
    y[2] = fma(a[0], m[1], m[2]);
    y[3] = fma(a[3], m[2], m[3]);
    y[4] = fma(dt, m[0], fma(a[1], m[1], fma(a[4], m[2], m[4])));
}

// X = G u : rollout of the linear model from x_0 = 0 (group-uniform; lane 0 of the group writes)
__device__ void rollout_lin(const Lds& S, int N, double dt, const double* u, double* X, int ln) {
    if (ln == 0) {
        double x[5] = {0, 0, 0, 0, 0};
        for (int a = 0; a < 5; ++a) X[a] = 0.0;
        for (int j = 0; j < N; ++j) {
            double y[5];
            applyA(S.A5 + 5 * j, dt, x, y);
            y[3] = fma(dt, u[2 * j], y[3]);
            y[4] = fma(dt, u[2 * j + 1], y[4]);
            for (int a = 0; a < 5; ++a) { x[a] = y[a]; X[5 * (j + 1) + a] = y[a]; }
        }
    }
    wave_sync();
}

// Riccati factorisation of  min sum 0.5 x'Qt x + 0.5 u'Rt u,  x_{t+1} = A_t x_t + B u_t,  x_0 = 0,
// spread over 25 lanes of the group: lane (i, j) = ln / 5, ln % 5 holds P[i][j].  Per stage:
// M = P A (gather row i of P), S = Rt + B'P B = Ls Ls' (uniform), W = Ls^-1 B'M, K = -Ls^-T W,
// P <- Qt + A'M - W'W (gather column j of M), symmetrised.  The Cholesky form keeps ~2 more digits
// than an explicit S^-1 once barrier weights reach 1e12.
template <int GL>
__device__ void riccati_factor(const Lds& S, const Grp<GL>& G, int N, double dt, int ln) {
    const int i = ln / 5, j = ln - 5 * (ln / 5);
    const bool act = ln < 25;
    const int ri = i == 4 ? 3 : i, rj = j == 4 ? 3 : j;
    const bool qv = act && i != 3 && j != 3;
    const int qo = qv ? p4(ri, rj) : 0;
    double P = qv ? S.Qt[10 * N + qo] : 0.0;
    const double dt2 = dt * dt;
    for (int t = N - 1; t >= 0; --t) {
        const double* a = S.A5 + 5 * t;
        const double a12 = a[0], a14 = a[1], a20 = a[2], a23 = a[3], a24 = a[4];
        const double r0 = S.Rt[2 * t], r1 = S.Rt[2 * t + 1];
        const double qt = (qv && t >= 1) ? S.Qt[10 * t + qo] : 0.0;
        // M[i][j] = P[i][j] + sum_l P[i][l] J'[l][j]
        const double p0 = G.get(P, 5 * i + 0), p1 = G.get(P, 5 * i + 1), p2 = G.get(P, 5 * i + 2);
        double M = P;
        if (j == 0) M = fma(p2, a20, M);
        else if (j == 2) M = fma(p1, a12, M);
        else if (j == 3) M = fma(p2, a23, M);
        else if (j == 4) M = fma(p0, dt, fma(p1, a14, fma(p2, a24, M)));
        // S = Rt + dt^2 P[{3,4},{3,4}]  (uniform)
        const double P33 = G.get(P, 18), P34 = G.get(P, 19), P44 = G.get(P, 24);
        double s00 = fma(dt2, P33, r0), s01 = dt2 * P34, s11 = fma(dt2, P44, r1);
        if (!(s00 > 0.0)) s00 = 1e-300 + fabs(s00);
        const double l00 = sqrt(s00), il00 = frcp(l00), l10 = s01 * il00;
        double r11 = s11 - l10 * l10;
        if (!(r11 > 1e-14 * s11)) r11 = 1e-14 * fabs(s11) + 1e-300;
        const double l11 = sqrt(r11), il11 = frcp(l11);
        // column j of M, and M[3][i], M[4][i]
        const double m0 = G.get(M, j), m1 = G.get(M, 5 + j), m2 = G.get(M, 10 + j);
        const double m3 = G.get(M, 15 + j), m4 = G.get(M, 20 + j);
        const double mi3 = G.get(M, 15 + i), mi4 = G.get(M, 20 + i);
        const double W0j = dt * m3 * il00, W1j = (dt * m4 - l10 * W0j) * il11;
        const double W0i = dt * mi3 * il00, W1i = (dt * mi4 - l10 * W0i) * il11;
        if (act && i == 0) {
            const double K1 = -W1j * il11;
            const double K0 = -(W0j + l10 * K1) * il00;
            S.Kf[10 * t + j] = K0;
            S.Kf[10 * t + 5 + j] = K1;
        }
        if (ln == 0) { S.Si[3 * t] = il00; S.Si[3 * t + 1] = l10; S.Si[3 * t + 2] = il11; }
        // (A'M)[i][j] = M[i][j] + sum_l J'[l][i] M[l][j]
        double Nij = M;
        if (i == 0) Nij = fma(a20, m2, Nij);
        else if (i == 2) Nij = fma(a12, m1, Nij);
        else if (i == 3) Nij = fma(a23, m2, Nij);
        else if (i == 4) Nij = fma(dt, m0, fma(a14, m1, fma(a24, m2, Nij)));
        const double Pn = Nij - fma(W0i, W0j, W1i * W1j);
        const double Pt = G.get(Pn, 5 * j + i);
        P = act ? 0.5 * (Pn + Pt) + qt : 0.0;
    }
    wave_sync();
}

// LQR solve with the factorisation: linear terms -qh (stages 1..N), -gh (controls).
// Writes dud (controls) and dX (states, x_0 = 0).  Group-uniform; lane 0 of the group writes.
__device__ void riccati_solve(const Lds& S, int N, double dt, int ln) {
    double p5[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < 4; ++a) p5[st4(a)] = S.qh[4 * N + a];
    for (int t = N - 1; t >= 0; --t) {
        double h0 = fma(dt, p5[3], S.gh[2 * t]);
        double h1 = fma(dt, p5[4], S.gh[2 * t + 1]);
        const double* si = S.Si + 3 * t;
        double w0 = h0 * si[0];
        double w1 = (h1 - si[1] * w0) * si[2];
        double k1 = w1 * si[2];
        double k0 = (w0 - si[1] * k1) * si[0];
        if (ln == 0) { S.kk[2 * t] = k0; S.kk[2 * t + 1] = k1; }
        if (t >= 1) {
            double pa[5];
            applyAT(S.A5 + 5 * t, dt, p5, pa);
            const double* K = S.Kf + 10 * t;
#pragma unroll
            for (int a = 0; a < 5; ++a) p5[a] = fma(K[a], h0, fma(K[5 + a], h1, pa[a]));
#pragma unroll
            for (int a = 0; a < 4; ++a) p5[st4(a)] += S.qh[4 * t + a];
        }
    }
    wave_sync();
    if (ln == 0) {
        double x[5] = {0, 0, 0, 0, 0};
        for (int a = 0; a < 5; ++a) S.dX[a] = 0.0;
        for (int t = 0; t < N; ++t) {
            const double* K = S.Kf + 10 * t;
            double v0 = S.kk[2 * t], v1 = S.kk[2 * t + 1];
#pragma unroll
            for (int a = 0; a < 5; ++a) { v0 = fma(K[a], x[a], v0); v1 = fma(K[5 + a], x[a], v1); }
            S.dud[2 * t] = v0;
            S.dud[2 * t + 1] = v1;
            double y[5];
            applyA(S.A5 + 5 * t, dt, x, y);
            y[3] = fma(dt, v0, y[3]);
            y[4] = fma(dt, v1, y[4]);
#pragma unroll
            for (int a = 0; a < 5; ++a) { x[a] = y[a]; S.dX[5 * (t + 1) + a] = y[a]; }
        }
    }
    wave_sync();
}

// max |g| and the scale max(|g_cost|, |g_mult|) of the dual residual g = G'y + z (adjoint recursion)
__device__ void dual_norms(const Lds& S, int N, double dt, double& rdmax, double& sd) {
    double mc[5] = {0, 0, 0, 0, 0}, ma[5] = {0, 0, 0, 0, 0};
    rdmax = 0.0;
    sd = 0.0;
    for (int k = N; k >= 1; --k) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            mc[st4(a)] += S.yc[4 * k + a];
            ma[st4(a)] += S.ya[4 * k + a];
        }
        const int t = k - 1;
        double gc0 = fma(dt, mc[3], S.zc[2 * t]), gc1 = fma(dt, mc[4], S.zc[2 * t + 1]);
        double ga0 = fma(dt, ma[3], S.za[2 * t]), ga1 = fma(dt, ma[4], S.za[2 * t + 1]);
        rdmax = fmax(rdmax, fmax(fabs(gc0 + ga0), fabs(gc1 + ga1)));
        sd = fmax(sd, fmax(fmax(fabs(gc0), fabs(gc1)), fmax(fabs(ga0), fabs(ga1))));
        double y[5];
        applyAT(S.A5 + 5 * t, dt, mc, y);
#pragma unroll
        for (int a = 0; a < 5; ++a) mc[a] = y[a];
        applyAT(S.A5 + 5 * t, dt, ma, y);
#pragma unroll
        for (int a = 0; a < 5; ++a) ma[a] = y[a];
    }
}

// cost Hessian (packed 4x4 on s,d,o,v) and gradient of stage k from cst = (-d', -o', -v', r_d, r_o, r_v):
// Q = 2 sum_j w_j m_j m_j',  q = 2 sum_j w_j r_j m_j,  m_j = e_j + (-ref_j') e_s   
__device__ __forceinline__ void stage_cost(const double* cst, double wd, double wo, double wv, double Q[10],
                                           double q[4]) {
    const double w[3] = {2.0 * wd, 2.0 * wo, 2.0 * wv};
#pragma unroll
    for (int a = 0; a < 10; ++a) Q[a] = 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a) q[a] = 0.0;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
        const double m0 = cst[jj];        // s entry; the own entry (index jj+1) is 1
        const double r = cst[3 + jj];
        Q[p4(0, 0)] = fma(w[jj] * m0, m0, Q[p4(0, 0)]);
        Q[p4(0, jj + 1)] += w[jj] * m0;
        Q[p4(jj + 1, jj + 1)] += w[jj];
        q[0] = fma(w[jj] * r, m0, q[0]);
        q[jj + 1] += w[jj] * r;
    }
}

#define POLISH_DELTA 1e-11
#define POLISH_REFINE 4
#define POLISH_ROUNDS 6
#define MU0 1.0

// Row slots: the 9 soft rows and 4 box rows of a stage are spread over P lanes (part = lane % P):
// lane slot s holds soft row j = part * R + s (if < 9) and box row part * RB + s (if < 4).
template <int P>
struct Parts {
    static constexpr int R = (NROW + P - 1) / P;
    static constexpr int RB = (NBOX + P - 1) / P;
};

// ------------------------------------------------------------------------------------------
// the solver kernel: one wavefront per MPC instance; stage k = 1..N is owned by the P lanes
// (k-1)*P .. (k-1)*P+P-1 (control t = k-1 with it); 25 lanes run the Riccati factorisation;
// the vector recursions run wave-uniformly from LDS.
// ------------------------------------------------------------------------------------------
template <int P>
__global__ void __launch_bounds__(WAVE)
mpc_solve_kernel(DevTable tab, KParams Pr, int B, const double* __restrict__ x0g, const double* __restrict__ obsg,
                 const int* __restrict__ nobsg, const double* __restrict__ ubarg, double* __restrict__ u0g,
                 double* __restrict__ Ug, double* __restrict__ Xg, int* __restrict__ statusg,
                 int* __restrict__ itersg) {
    constexpr int R = Parts<P>::R, RB = Parts<P>::RB;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int b = blockIdx.x;
    if (b >= B) return;
    const int ln = threadIdx.x;
    const Grp<WAVE> G{0};
    const int N = Pr.N;
    const int NP = N + 1;
    const double dt = Pr.dt;
    const double rho = Pr.rho;
    const double hL = Pr.L / 2.0;
    Lds S = carve(smem, N);

    double x0[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) x0[j] = x0g[5 * (size_t)b + j];
    int nobs = nobsg ? nobsg[b] : 0;
    nobs = nobs < 0 ? 0 : (nobs > Pr.max_obs ? Pr.max_obs : nobs);
    const double* obs = obsg ? obsg + (size_t)b * Pr.max_obs * 2 : nullptr;
    const bool has_obs = nobs > 0;

    // stage ownership
    const int part = ln % P;
    const int k = ln / P + 1;                 // stage of this lane
    const bool live = k <= N;                 // lane owns rows of stage k (and boxes of control k-1)
    const int sbase = ln - part;              // first lane of this stage
    const bool lead = live && part == 0;      // writes the stage sums

    // row slots of this lane
    int rj[R];
    bool ron[R];
    double cf[R][4];
#pragma unroll
    for (int s = 0; s < R; ++s) {
        rj[s] = part * R + s;
        ron[s] = live && rj[s] < NROW && ((rj[s] != 6 && rj[s] != 7) || has_obs);
        row_coef(rj[s] < NROW ? rj[s] : 0, hL, Pr.L, Pr.tgap, cf[s]);
    }
    int bj[RB];
    bool bon[RB];
#pragma unroll
    for (int s = 0; s < RB; ++s) {
        bj[s] = part * RB + s;
        bon[s] = live && bj[s] < NBOX;
    }
    // sum of a per-lane partial over the P lanes of the stage (valid on the stage's part-0 lane)
    auto stage_sum = [&](double v) {
        double r = v;
#pragma unroll
        for (int q = 1; q < P; ++q) r += G.get(v, sbase + q);
        return r;
    };

    // ---- K1: linearisation point ---------------------------------------------------------
    if (ln < N) {
        if (ubarg) {
            S.ub[2 * ln] = ubarg[(size_t)b * 2 * N + 2 * ln];
            S.ub[2 * ln + 1] = ubarg[(size_t)b * 2 * N + 2 * ln + 1];
        } else {
            // warm start, trajectory_tracking.py:224-246: s_curr advanced by repeated addition,
            // sticky brake flag over steps 0..ln
            double s_curr = x0[0], v_curr = x0[4];
            bool brake = false;
            for (int j = 0; j <= ln; ++j) {
                if (j > 0) s_curr += v_curr * dt;
                for (int i = 0; i < nobs; ++i)
                    if ((obs[2 * i] - s_curr) < Pr.brake_distance) brake = true;
            }
            double ur[2];
            get_control(tab, s_curr, ur);
            S.ub[2 * ln] = ur[0];
            S.ub[2 * ln + 1] = brake ? Pr.brake_accel : ur[1];
        }
    }
    wave_sync();

    int nsoft = 0;
    for (int j = 0; j < NROW; ++j) nsoft += ((j != 6 && j != 7) || has_obs) ? 1 : 0;
    const double Mtot = (double)(2 * nsoft * N + NBOX * N);
    const double R0 = 2.0 * Pr.w_u1, R1 = 2.0 * Pr.w_u2;

    const int nsqp = Pr.sqp_iters < 0 ? 0 : Pr.sqp_iters;   // 0: return ubar and predict(x0, ubar)
    int status = MPC_OK, total_it = 0;
    for (int sqp = 0; sqp < nsqp; ++sqp) {
        // ---- K1: nominal rollout == predict(x0, ubar), into Xr ------------------------------
        predict_grp(tab, N, dt, x0, S.ub, S.Xr, S.kap, ln);
        // ---- K2: stage data of QP(ubar) ----------------------------------------------------
        const bool gn = Pr.linearization != 0;
        double refk[5], slk[4];
        if (ln <= N) get_state(tab, S.Xr[5 * ln], refk, slk);
        if (ln < N) {
            const double* x = S.Xr + 5 * ln;
            double dk = gn ? slk[2] : 0.0;
            S.A5[5 * ln + 0] = dt * x[4];
            S.A5[5 * ln + 1] = dt * x[2];
            S.A5[5 * ln + 2] = dt * (-x[4] * dk);
            S.A5[5 * ln + 3] = dt * x[4];
            S.A5[5 * ln + 4] = dt * (x[3] - refk[3]);
        }
        // cost data of stage k (lookups done by lane k)
        {
            const double rk1 = G.get(refk[1], k), rk2 = G.get(refk[2], k), rk4 = G.get(refk[4], k);
            const double sk0 = G.get(slk[0], k), sk1 = G.get(slk[1], k), sk3 = G.get(slk[3], k);
            if (lead) {
                const double* x = S.Xr + 5 * k;
                S.cst[6 * k + 0] = gn ? -sk0 : 0.0;
                S.cst[6 * k + 1] = gn ? -sk1 : 0.0;
                S.cst[6 * k + 2] = gn ? -sk3 : 0.0;
                S.cst[6 * k + 3] = x[1] - rk1;
                S.cst[6 * k + 4] = x[2] - rk2;
                S.cst[6 * k + 5] = x[4] - rk4;
            }
        }
        // row bounds of this lane's rows, box bounds of its boxes
        double bk[R], bb[RB];
        double bscale_l = 0.0;
        {
            double shat = INFINITY;
            if (live && has_obs)
                for (int i = 0; i < nobs; ++i) {
                    double sp = obs[2 * i] + obs[2 * i + 1] * (k * dt);
                    shat = sp < shat ? sp : shat;
                }
            const double* x = S.Xr + 5 * (live ? k : 0);
            const double sl = Pr.sl;
            const double pv0 = x[1], pv1 = x[1] + hL * x[2], pv2 = x[1] + Pr.L * x[2];
#pragma unroll
            for (int s = 0; s < R; ++s) {
                const int j = rj[s];
                double v = 0.0;
                switch (j) {
                    case 0: v = -sl - pv0; break;
                    case 1: v = -(sl - pv0); break;
                    case 2: v = -sl - pv1; break;
                    case 3: v = -(sl - pv1); break;
                    case 4: v = -sl - pv2; break;
                    case 5: v = -(sl - pv2); break;
                    case 6: v = has_obs ? -(shat - Pr.osd - x[0]) : 0.0; break;
                    case 7: v = has_obs ? -(shat - x[0] - Pr.tgap * x[4]) : 0.0; break;
                    case 8: v = -x[4]; break;
                    default: v = 0.0; break;
                }
                bk[s] = ron[s] ? v : 0.0;
                bscale_l = fmax(bscale_l, fabs(bk[s]));
            }
            const double ub0 = live ? S.ub[2 * (k - 1)] : 0.0, ub1 = live ? S.ub[2 * (k - 1) + 1] : 0.0;
#pragma unroll
            for (int s = 0; s < RB; ++s) {
                double v = 0.0;
                switch (bj[s]) {
                    case 0: v = Pr.u_min0 - ub0; break;
                    case 1: v = -(Pr.u_max0 - ub0); break;
                    case 2: v = Pr.u_min1 - ub1; break;
                    case 3: v = -(Pr.u_max1 - ub1); break;
                    default: v = 0.0; break;
                }
                bb[s] = bon[s] ? v : 0.0;
                bscale_l = fmax(bscale_l, fabs(bb[s]));
            }
        }
        const double bscale = G.max(bscale_l);
        wave_sync();

        // ---- K4: PDIP; interior-point state of this lane's rows in registers ---------------------
        double rs[R], rl[R], rxi[R], rnu[R], sb[RB], lb[RB];
#pragma unroll
        for (int s = 0; s < R; ++s) {
            // centred start: xi covers the violation, s*lam = MU0 with lam <= rho/2, nu = rho - lam
            const double r0 = -bk[s];
            const double xi = (r0 < 0 ? -r0 : 0.0) + XI0;
            const double sv = r0 + xi;
            const double lam = fmin(MU0 * frcp(sv), 0.5 * rho);
            rxi[s] = xi; rs[s] = sv; rl[s] = lam; rnu[s] = rho - lam;
        }
#pragma unroll
        for (int s = 0; s < RB; ++s) {
            const double r0 = -bb[s];
            sb[s] = r0 > 1.0 ? r0 : 1.0;
            lb[s] = 1.0;
        }
        if (ln < N) { S.du[2 * ln] = 0.0; S.du[2 * ln + 1] = 0.0; }
        wave_sync();

        int it = 0, st_here = MPC_MAX_ITER, stall = 0;
        bool done = false;
        double mu = 0.0;
        for (int iter = 0; iter < Pr.max_iter; ++iter) {
            rollout_lin(S, N, dt, S.du, S.dX, ln);
            // -- stage-parallel residuals ------------------------------------------------------
            double x4[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) x4[a] = live ? S.dX[5 * k + st4(a)] : 0.0;
            const double du0 = live ? S.du[2 * (k - 1)] : 0.0, du1 = live ? S.du[2 * (k - 1) + 1] : 0.0;
            double rpmax = 0.0, rxmax = 0.0, comp = 0.0;
            double ya[4] = {0, 0, 0, 0}, za0 = 0.0, za1 = 0.0;
#pragma unroll
            for (int s = 0; s < R; ++s) {
                if (!ron[s]) continue;
                const double rp = dot4(cf[s], x4) + rxi[s] - rs[s] - bk[s];
                const double rx = rho - rl[s] - rnu[s];
#pragma unroll
                for (int a = 0; a < 4; ++a) ya[a] = fma(-rl[s], cf[s][a], ya[a]);
                rpmax = fmax(rpmax, fabs(rp));
                rxmax = fmax(rxmax, fabs(rx));
                comp = fma(rs[s], rl[s], fma(rxi[s], rnu[s], comp));
            }
#pragma unroll
            for (int s = 0; s < RB; ++s) {
                if (!bon[s]) continue;
                const double rp = bsign(bj[s]) * ((bj[s] < 2) ? du0 : du1) - sb[s] - bb[s];
                rpmax = fmax(rpmax, fabs(rp));
                comp = fma(sb[s], lb[s], comp);
                if (bj[s] < 2) za0 += -bsign(bj[s]) * lb[s]; else za1 += -bsign(bj[s]) * lb[s];
            }
#pragma unroll
            for (int a = 0; a < 4; ++a) ya[a] = stage_sum(ya[a]);
            za0 = stage_sum(za0);
            za1 = stage_sum(za1);
            if (lead) {
                double Qs[10], qs[4], yc[4];
                stage_cost(S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    double acc = qs[a];
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc = fma(Qs[p4(a, c)], x4[c], acc);
                    yc[a] = acc;
                }
#pragma unroll
                for (int a = 0; a < 4; ++a) { S.yc[4 * k + a] = yc[a]; S.ya[4 * k + a] = ya[a]; }
                S.zc[2 * (k - 1)] = fma(R0, du0, R0 * S.ub[2 * (k - 1)]);
                S.zc[2 * (k - 1) + 1] = fma(R1, du1, R1 * S.ub[2 * (k - 1) + 1]);
                S.za[2 * (k - 1)] = za0;
                S.za[2 * (k - 1) + 1] = za1;
            }
            rpmax = G.max(rpmax);
            rxmax = G.max(rxmax);
            comp = G.sum(comp);
            wave_sync();
            double rdmax, sd;
            dual_norms(S, N, dt, rdmax, sd);
            mu = comp / Mtot;
            if (!(mu == mu) || !(rdmax == rdmax)) { st_here = MPC_NUMERICAL; it = iter; done = true; break; }
            if (mu <= Pr.tol_mu && rpmax <= 10.0 * Pr.tol * (1.0 + bscale) && rxmax <= Pr.tol * rho) {
                // converged: the polish then makes the active set exact;
                // the dual residual carries O(eps/mu) multiplier noise, required to 1e4*tol
                st_here = rdmax <= 1e4 * Pr.tol * (1.0 + sd) ? MPC_OK : MPC_NUMERICAL;
                it = iter;
                done = true;
                break;
            }
            // -- barrier weights, augmented stage Hessians ---------------------------------------
            double il[R], inu[R], wv[R], ilb[RB], wb[RB];
            {
                double Qp[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int s = 0; s < R; ++s) {
                    il[s] = frcp(rl[s]);
                    inu[s] = frcp(rnu[s]);
                    wv[s] = ron[s] ? frcp(fma(rs[s], il[s], rxi[s] * inu[s])) : 0.0;   // 1/d
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int c = a; c < 4; ++c) Qp[p4(a, c)] = fma(wv[s] * cf[s][a], cf[s][c], Qp[p4(a, c)]);
                }
                double r0 = 0.0, r1 = 0.0;
#pragma unroll
                for (int s = 0; s < RB; ++s) {
                    ilb[s] = frcp(lb[s]);
                    wb[s] = bon[s] ? lb[s] * frcp(sb[s]) : 0.0;
                    if (bj[s] < 2) r0 += wb[s]; else r1 += wb[s];
                }
#pragma unroll
                for (int a = 0; a < 10; ++a) Qp[a] = stage_sum(Qp[a]);
                r0 = stage_sum(r0);
                r1 = stage_sum(r1);
                if (lead) {
                    double Qs[10], qs[4];
                    stage_cost(S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                    for (int a = 0; a < 10; ++a) S.Qt[10 * k + a] = Qp[a] + Qs[a];
                    S.Rt[2 * (k - 1)] = R0 + r0;
                    S.Rt[2 * (k - 1) + 1] = R1 + r1;
                }
            }
            wave_sync();
            riccati_factor(S, G, N, dt, ln);
            // -- predictor, corrector (and, if needed, centred) solves ---------------------------------
            double p4v[R], p5v[R], pbv[RB];
            double sig = 0.0;
            bool applied = false;
#pragma unroll 1
            for (int pass = 0; pass < 3; ++pass) {
                // pass 0: affine predictor; 1: Mehrotra corrector; 2: plain centred direction, taken when
                // the corrector would not reduce complementarity (oracle: comp_after > comp)
                const double smu = (pass >= 1) ? sig * mu : 0.0;
                double r4[R], r5[R], r4b[RB], rh[R], rhb[RB];
                {
                    double q4[4] = {0, 0, 0, 0}, g0 = 0.0, g1 = 0.0;
#pragma unroll
                    for (int s = 0; s < R; ++s) {
                        r4[s] = rs[s] * rl[s] - smu;
                        r5[s] = rxi[s] * rnu[s] - smu;
                        if (pass == 1) { r4[s] += p4v[s]; r5[s] += p5v[s]; }
                        const double rp = dot4(cf[s], x4) + rxi[s] - rs[s] - bk[s];
                        const double rx = rho - rl[s] - rnu[s];
                        rh[s] = -rp - r4[s] * il[s] + fma(rxi[s], rx, r5[s]) * inu[s];
                        const double w = ron[s] ? rh[s] * wv[s] : 0.0;
#pragma unroll
                        for (int a = 0; a < 4; ++a) q4[a] = fma(cf[s][a], w, q4[a]);
                    }
#pragma unroll
                    for (int s = 0; s < RB; ++s) {
                        r4b[s] = sb[s] * lb[s] - smu;
                        if (pass == 1) r4b[s] += pbv[s];
                        const double rp = bsign(bj[s]) * ((bj[s] < 2) ? du0 : du1) - sb[s] - bb[s];
                        rhb[s] = -rp - r4b[s] * ilb[s];
                        const double v = bsign(bj[s]) * rhb[s] * wb[s];
                        if (bj[s] < 2) g0 += v; else g1 += v;
                    }
#pragma unroll
                    for (int a = 0; a < 4; ++a) q4[a] = stage_sum(q4[a]);
                    g0 = stage_sum(g0);
                    g1 = stage_sum(g1);
                    if (lead) {
#pragma unroll
                        for (int a = 0; a < 4; ++a) S.qh[4 * k + a] = q4[a] - (S.yc[4 * k + a] + S.ya[4 * k + a]);
                        S.gh[2 * (k - 1)] = g0 - (S.zc[2 * (k - 1)] + S.za[2 * (k - 1)]);
                        S.gh[2 * (k - 1) + 1] = g1 - (S.zc[2 * (k - 1) + 1] + S.za[2 * (k - 1) + 1]);
                    }
                }
                wave_sync();
                riccati_solve(S, N, dt, ln);
                // row directions and the step length
                double dsv[R], dlv[R], dxv[R], dnv[R], dsb[RB], dlb[RB];
                double amax = 1.0;
                {
                    double dx4[4];
#pragma unroll
                    for (int a = 0; a < 4; ++a) dx4[a] = live ? S.dX[5 * k + st4(a)] : 0.0;
#pragma unroll
                    for (int s = 0; s < R; ++s) {
                        const double rx = rho - rl[s] - rnu[s];
                        const double dl = (rh[s] - dot4(cf[s], dx4)) * wv[s];
                        const double ds = -fma(rs[s], dl, r4[s]) * il[s];
                        const double dn = rx - dl;
                        const double dxi = -fma(rxi[s], dn, r5[s]) * inu[s];
                        dsv[s] = ds; dlv[s] = dl; dxv[s] = dxi; dnv[s] = dn;
                        if (!ron[s]) continue;
                        if (ds < 0.0) amax = fmin(amax, -rs[s] / ds);
                        if (dl < 0.0) amax = fmin(amax, -rl[s] / dl);
                        if (dxi < 0.0) amax = fmin(amax, -rxi[s] / dxi);
                        if (dn < 0.0) amax = fmin(amax, -rnu[s] / dn);
                    }
                    const double dd0 = live ? S.dud[2 * (k - 1)] : 0.0, dd1 = live ? S.dud[2 * (k - 1) + 1] : 0.0;
#pragma unroll
                    for (int s = 0; s < RB; ++s) {
                        const double duu = (bj[s] < 2) ? dd0 : dd1;
                        const double dl = (rhb[s] - bsign(bj[s]) * duu) * wb[s];
                        const double ds = -fma(sb[s], dl, r4b[s]) * ilb[s];
                        dsb[s] = ds; dlb[s] = dl;
                        if (!bon[s]) continue;
                        if (ds < 0.0) amax = fmin(amax, -sb[s] / ds);
                        if (dl < 0.0) amax = fmin(amax, -lb[s] / dl);
                    }
                }
                amax = G.min(amax);
                // complementarity after the step (pass 0: at the full affine step length)
                const double a_try = (pass == 0) ? amax : fmin(1.0, TAU * amax);
                double ca = 0.0;
#pragma unroll
                for (int s = 0; s < R; ++s)
                    if (ron[s])
                        ca += fma(a_try, dsv[s], rs[s]) * fma(a_try, dlv[s], rl[s]) +
                              fma(a_try, dxv[s], rxi[s]) * fma(a_try, dnv[s], rnu[s]);
#pragma unroll
                for (int s = 0; s < RB; ++s)
                    if (bon[s]) ca += fma(a_try, dsb[s], sb[s]) * fma(a_try, dlb[s], lb[s]);
                ca = G.sum(ca);
                if (pass == 0) {
                    const double r = ca / comp;
                    sig = r * r * r;
#pragma unroll
                    for (int s = 0; s < R; ++s) { p4v[s] = dsv[s] * dlv[s]; p5v[s] = dxv[s] * dnv[s]; }
#pragma unroll
                    for (int s = 0; s < RB; ++s) pbv[s] = dsb[s] * dlb[s];
                    continue;
                }
                if (pass == 1 && ca > comp) continue;     // safeguard: take the centred direction
                const double alpha = a_try;
                applied = true;
                stall = (mu < 1e-6 && ca > 0.9 * comp) ? stall + 1 : 0;
#pragma unroll
                for (int s = 0; s < R; ++s) {
                    if (!ron[s]) continue;
                    rs[s] = fma(alpha, dsv[s], rs[s]);
                    rl[s] = fma(alpha, dlv[s], rl[s]);
                    rxi[s] = fma(alpha, dxv[s], rxi[s]);
                    rnu[s] = fma(alpha, dnv[s], rnu[s]);
                }
#pragma unroll
                for (int s = 0; s < RB; ++s) {
                    if (!bon[s]) continue;
                    sb[s] = fma(alpha, dsb[s], sb[s]);
                    lb[s] = fma(alpha, dlb[s], lb[s]);
                }
                if (ln < N) {
                    S.du[2 * ln] = fma(alpha, S.dud[2 * ln], S.du[2 * ln]);
                    S.du[2 * ln + 1] = fma(alpha, S.dud[2 * ln + 1], S.du[2 * ln + 1]);
                }
                break;
            }
            (void)applied;
            wave_sync();
            it = iter + 1;
            if (stall >= 5) { st_here = MPC_NUMERICAL; done = true; break; }
        }
        (void)done;
        total_it += it;
        // NaN guard and the infeasibility flag
        double bad = 0.0;
        if (ln < N) bad = (S.du[2 * ln] == S.du[2 * ln] && S.du[2 * ln + 1] == S.du[2 * ln + 1]) ? 0.0 : 1.0;
        bad = G.max(bad);
        if (bad > 0.0) {
            st_here = MPC_NUMERICAL;
            if (ln < N) { S.du[2 * ln] = 0.0; S.du[2 * ln + 1] = 0.0; }
        } else if (st_here == MPC_OK) {
            double inf = 0.0;
#pragma unroll
            for (int s = 0; s < R; ++s)
                if (ron[s] && rxi[s] > 1e-6 * (1.0 + fabs(bk[s]))) inf = 1.0;
            if (G.max(inf) > 0.0) st_here = MPC_INFEASIBLE;
        }
        wave_sync();

        // ---- active-set polish (oracle polish()) --------------------------
        if (Pr.polish && bad == 0.0) {
            // class per row: 0 inactive, 1 active (equality), 2 violated (multiplier fixed at rho)
            int cls[R], clb[RB];
#pragma unroll
            for (int s = 0; s < R; ++s) cls[s] = !ron[s] ? 0 : (rxi[s] > rnu[s] ? 2 : (rl[s] > rs[s] ? 1 : 0));
#pragma unroll
            for (int s = 0; s < RB; ++s) clb[s] = (bon[s] && lb[s] > sb[s]) ? 1 : 0;
            if (ln < N) { S.dub[2 * ln] = S.du[2 * ln]; S.dub[2 * ln + 1] = S.du[2 * ln + 1]; }
            wave_sync();
            bool accepted = false;
            double nviol_acc = 0.0;
            for (int round = 0; round < POLISH_ROUNDS; ++round) {
                double tl[R], tlb[RB];
                {
                    if (ln < N) { S.du[2 * ln] = S.dub[2 * ln]; S.du[2 * ln + 1] = S.dub[2 * ln + 1]; }
                    double Qp[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                    for (int s = 0; s < R; ++s) {
                        tl[s] = rl[s];
                        const double w = cls[s] == 1 ? 1.0 / POLISH_DELTA : 0.0;
#pragma unroll
                        for (int a = 0; a < 4; ++a)
#pragma unroll
                            for (int c = a; c < 4; ++c) Qp[p4(a, c)] = fma(w * cf[s][a], cf[s][c], Qp[p4(a, c)]);
                    }
                    double r0 = 0.0, r1 = 0.0;
#pragma unroll
                    for (int s = 0; s < RB; ++s) {
                        tlb[s] = lb[s];
                        if (clb[s] == 1) { if (bj[s] < 2) r0 += 1.0 / POLISH_DELTA; else r1 += 1.0 / POLISH_DELTA; }
                    }
#pragma unroll
                    for (int a = 0; a < 10; ++a) Qp[a] = stage_sum(Qp[a]);
                    r0 = stage_sum(r0);
                    r1 = stage_sum(r1);
                    if (lead) {
                        double Qs[10], qs[4];
                        stage_cost(S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                        for (int a = 0; a < 10; ++a) S.Qt[10 * k + a] = Qp[a] + Qs[a];
                        S.Rt[2 * (k - 1)] = R0 + r0;
                        S.Rt[2 * (k - 1) + 1] = R1 + r1;
                    }
                }
                wave_sync();
                riccati_factor(S, G, N, dt, ln);
                double x4[4];
#pragma unroll 1
                for (int r = 0; r <= POLISH_REFINE; ++r) {
                    rollout_lin(S, N, dt, S.du, S.dX, ln);
#pragma unroll
                    for (int a = 0; a < 4; ++a) x4[a] = live ? S.dX[5 * k + st4(a)] : 0.0;
                    if (r == POLISH_REFINE) break;
                    // exact KKT residual of the equality QP -> LQR right-hand side
                    double r2[R], r2b[RB];
                    const double du0 = live ? S.du[2 * (k - 1)] : 0.0, du1 = live ? S.du[2 * (k - 1) + 1] : 0.0;
                    {
                        double q4[4] = {0, 0, 0, 0}, g0 = 0.0, g1 = 0.0;
#pragma unroll
                        for (int s = 0; s < R; ++s) {
                            r2[s] = (cls[s] == 1) ? bk[s] - dot4(cf[s], x4) : 0.0;
                            const double wgt = (cls[s] == 2) ? rho : (cls[s] == 1 ? tl[s] + r2[s] * (1.0 / POLISH_DELTA) : 0.0);
#pragma unroll
                            for (int a = 0; a < 4; ++a) q4[a] = fma(cf[s][a], wgt, q4[a]);
                        }
#pragma unroll
                        for (int s = 0; s < RB; ++s) {
                            const double uu = (bj[s] < 2) ? du0 : du1;
                            r2b[s] = (clb[s] == 1) ? bb[s] - bsign(bj[s]) * uu : 0.0;
                            const double v = (clb[s] == 1) ? bsign(bj[s]) * (tlb[s] + r2b[s] * (1.0 / POLISH_DELTA)) : 0.0;
                            if (bj[s] < 2) g0 += v; else g1 += v;
                        }
#pragma unroll
                        for (int a = 0; a < 4; ++a) q4[a] = stage_sum(q4[a]);
                        g0 = stage_sum(g0);
                        g1 = stage_sum(g1);
                        if (lead) {
                            double Qs[10], qs[4];
                            stage_cost(S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                            for (int a = 0; a < 4; ++a) {
                                double acc = qs[a];
#pragma unroll
                                for (int c = 0; c < 4; ++c) acc = fma(Qs[p4(a, c)], x4[c], acc);
                                S.qh[4 * k + a] = q4[a] - acc;
                            }
                            S.gh[2 * (k - 1)] = g0 - fma(R0, du0, R0 * S.ub[2 * (k - 1)]);
                            S.gh[2 * (k - 1) + 1] = g1 - fma(R1, du1, R1 * S.ub[2 * (k - 1) + 1]);
                        }
                    }
                    wave_sync();
                    riccati_solve(S, N, dt, ln);
                    {
                        double dx4[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) dx4[a] = live ? S.dX[5 * k + st4(a)] : 0.0;
#pragma unroll
                        for (int s = 0; s < R; ++s)
                            if (cls[s] == 1) tl[s] += (r2[s] - dot4(cf[s], dx4)) * (1.0 / POLISH_DELTA);
                        const double dd0 = live ? S.dud[2 * (k - 1)] : 0.0, dd1 = live ? S.dud[2 * (k - 1) + 1] : 0.0;
#pragma unroll
                        for (int s = 0; s < RB; ++s)
                            if (clb[s] == 1)
                                tlb[s] += (r2b[s] - bsign(bj[s]) * ((bj[s] < 2) ? dd0 : dd1)) * (1.0 / POLISH_DELTA);
                    }
                    wave_sync();
                    if (ln < N) { S.du[2 * ln] += S.dud[2 * ln]; S.du[2 * ln + 1] += S.dud[2 * ln + 1]; }
                    wave_sync();
                }
                // acceptance: KKT consistency; otherwise flip every offending row and retry
                double lmax = 1.0;
#pragma unroll
                for (int s = 0; s < R; ++s)
                    if (cls[s] == 1) lmax = fmax(lmax, fabs(tl[s]));
#pragma unroll
                for (int s = 0; s < RB; ++s)
                    if (clb[s] == 1) lmax = fmax(lmax, fabs(tlb[s]));
                lmax = G.max(lmax);
                double worst = 0.0, nviol = 0.0, finite = 1.0;
                bool flip[R], flipb[RB];
                {
                    const double du0 = live ? S.du[2 * (k - 1)] : 0.0, du1 = live ? S.du[2 * (k - 1) + 1] : 0.0;
                    if (!(du0 == du0) || !(du1 == du1)) finite = 0.0;
#pragma unroll
                    for (int s = 0; s < R; ++s) {
                        flip[s] = false;
                        if (!ron[s]) continue;
                        const double bsc = 1.0 + fabs(bk[s]);
                        const double r = dot4(cf[s], x4) - bk[s];
                        double badv = 0.0;
                        if (cls[s] == 1) {
                            if (tl[s] < -1e-9 * lmax) badv = -tl[s] / lmax;
                            else if (tl[s] > rho * (1.0 + 1e-9)) badv = (tl[s] - rho) / lmax;
                            else if (fabs(r) > 1e-7 * bsc) badv = fabs(r) / bsc;
                        } else if (cls[s] == 2) {
                            if (r > 1e-9 * bsc) badv = r / bsc;
                            if (r < -1e-6 * bsc) nviol += 1.0;
                        } else if (r < -1e-9 * bsc) badv = -r / bsc;
                        worst = fmax(worst, badv);
                        flip[s] = badv > 0.0;
                    }
#pragma unroll
                    for (int s = 0; s < RB; ++s) {
                        flipb[s] = false;
                        if (!bon[s]) continue;
                        const double bsc = 1.0 + fabs(bb[s]);
                        const double r = bsign(bj[s]) * ((bj[s] < 2) ? du0 : du1) - bb[s];
                        double badv = 0.0;
                        if (clb[s] == 1) {
                            if (tlb[s] < -1e-9 * lmax) badv = -tlb[s] / lmax;
                            else if (fabs(r) > 1e-7 * bsc) badv = fabs(r) / bsc;
                        } else if (r < -1e-9 * bsc) badv = -r / bsc;
                        worst = fmax(worst, badv);
                        flipb[s] = badv > 0.0;
                    }
                }
                worst = G.max(worst);
                nviol = G.sum(nviol);
                finite = G.min(finite);
                if (finite == 0.0) break;
                if (worst == 0.0) {
                    accepted = true;
                    nviol_acc = nviol;
                    if (ln < N) { S.dub[2 * ln] = S.du[2 * ln]; S.dub[2 * ln + 1] = S.du[2 * ln + 1]; }
                    wave_sync();
                    break;
                }
#pragma unroll
                for (int s = 0; s < R; ++s)
                    if (flip[s]) cls[s] = (cls[s] == 1) ? (tl[s] > rho ? 2 : 0) : 1;
#pragma unroll
                for (int s = 0; s < RB; ++s)
                    if (flipb[s]) clb[s] = 1 - clb[s];
                wave_sync();
            }
            // the accepted polish (or, if none, the interior-point iterate) is in dub
            if (ln < N) { S.du[2 * ln] = S.dub[2 * ln]; S.du[2 * ln + 1] = S.dub[2 * ln + 1]; }
            if (accepted) st_here = nviol_acc > 0.0 ? MPC_INFEASIBLE : MPC_OK;
            wave_sync();
        }
        status = st_here;
        if (ln < N) {
            S.ub[2 * ln] += S.du[2 * ln];
            S.ub[2 * ln + 1] += S.du[2 * ln + 1];
        }
        wave_sync();
    }

    // ---- K5: outputs: U*, u0, predict(x0, U*) ----------------------------------------------
    predict_grp(tab, N, dt, x0, S.ub, S.Xr, S.kap, ln);
    if (ln < N && Ug) {
        Ug[(size_t)b * 2 * N + 2 * ln] = S.ub[2 * ln];
        Ug[(size_t)b * 2 * N + 2 * ln + 1] = S.ub[2 * ln + 1];
    }
    if (Xg)
        for (int i = ln; i < 5 * NP; i += WAVE) Xg[(size_t)b * 5 * NP + i] = S.Xr[i];
    if (ln == 0) {
        if (u0g) { u0g[2 * (size_t)b] = S.ub[0]; u0g[2 * (size_t)b + 1] = S.ub[1]; }
        if (statusg) statusg[b] = status;
        if (itersg) itersg[b] = total_it;
    }
}

__global__ void mpc_lookup_kernel(DevTable tab, int n, const double* __restrict__ s, double* __restrict__ st,
                                  double* __restrict__ ct) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double o[5], c[2];
    get_state(tab, s[i], o, nullptr);
    get_control(tab, s[i], c);
    if (st)
        for (int j = 0; j < 5; ++j) st[5 * (size_t)i + j] = o[j];
    if (ct) { ct[2 * (size_t)i] = c[0]; ct[2 * (size_t)i + 1] = c[1]; }
}

// ------------------------------------------------------------------------------------------
// host side: C ABI
// ------------------------------------------------------------------------------------------
static thread_local std::string g_err = "";

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr, code)                                                                           \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) return fail(code, std::string(#expr ": ") + hipGetErrorString(e_));    \
    } while (0)

struct mpc_ctx {
    int device;
    mpc_params p;
    DevTable tab;
    double* table_buf;
    // host-API staging buffers
    size_t cap_B;
    int cap_N, cap_obs;
    double *x0, *obs, *ub, *u0, *U, *X;
    int *nobs, *status, *iters;
    double *ls, *lst, *lct;
    size_t cap_lookup;
    hipStream_t stream;
};

extern "C" void mpc_default_params(mpc_params* p) {
    std::memset(p, 0, sizeof(*p));
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
    p->polish = 1;
}

extern "C" const char* mpc_last_error(void) { return g_err.c_str(); }
extern "C" int mpc_version(void) { return MPCQP_VERSION; }

static int check_params(const mpc_params* p) {
    if (!p) return fail(MPC_E_ARG, "params is NULL");
    if (p->N < 1 || p->N > MPC_MAX_N) return fail(MPC_E_ARG, "N out of range [1, 63]");
    if (p->max_obs < 0 || p->max_obs > MPC_MAX_OBS) return fail(MPC_E_ARG, "max_obs out of range [0, 64]");
    if (!(p->dt > 0)) return fail(MPC_E_ARG, "dt must be > 0");
    if (p->max_iter < 1) return fail(MPC_E_ARG, "max_iter must be >= 1");
    if (p->sqp_iters < 0 || p->sqp_iters > 100) return fail(MPC_E_ARG, "sqp_iters out of range [0, 100]");
    if (!(p->elastic_rho > 1.0)) return fail(MPC_E_ARG, "elastic_rho must be > 1");
    return MPC_SUCCESS;
}

static KParams kparams(const mpc_params* p) {
    KParams k;
    k.N = p->N;
    k.max_obs = p->max_obs;
    k.linearization = p->linearization;
    k.sqp_iters = p->sqp_iters;
    k.max_iter = p->max_iter;
    k.dt = p->dt;
    k.u_min0 = p->u_min[0]; k.u_min1 = p->u_min[1];
    k.u_max0 = p->u_max[0]; k.u_max1 = p->u_max[1];
    k.w_d = p->w_d; k.w_o = p->w_o; k.w_v = p->w_v; k.w_u1 = p->w_u1; k.w_u2 = p->w_u2;
    k.osd = p->obstacle_safety_distance;
    k.tgap = p->max_time_2_obs;
    k.L = p->wheelbase;
    k.sl = p->lane_width / 2.0 - p->vehicle_radius - p->safe_lane_margin;   // trajectory_tracking.py:169
    k.brake_distance = p->brake_distance;
    k.brake_accel = p->brake_accel;
    k.tol = p->tol;
    k.tol_mu = p->tol_mu;
    k.rho = p->elastic_rho;
    k.polish = p->polish;
    return k;
}

extern "C" int mpc_create(const double* X, int T, const double* U, int Tu, const mpc_params* p, int device,
                          mpc_ctx** out) {
    if (!out) return fail(MPC_E_ARG, "out is NULL");
    *out = nullptr;
    if (!X || !U || T < 2 || Tu < 2) return fail(MPC_E_ARG, "trajectory table needs T >= 2, Tu >= 2");
    int rc = check_params(p);
    if (rc) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(MPC_E_DEVICE, "no HIP device available (libmpcqp has no CPU backend)");
    if (device < 0 || device >= ndev) return fail(MPC_E_DEVICE, "device index out of range");
    HIPCHK(hipSetDevice(device), MPC_E_DEVICE);
    int tu = Tu < T ? Tu : T;   // limit = min(len(s), len(U))   trajectory_loader.py:73-75
    std::vector<double> h((size_t)5 * T + 2 * tu);
    double* s = h.data();
    for (int i = 0; i < T; ++i) {
        double si = X[5 * i];
        if (i > 0 && si <= s[i - 1]) si = s[i - 1] + 1e-5;   // trajectory_loader.py:28-30
        s[i] = si;
        h[T + i] = X[5 * i + 1];
        h[2 * T + i] = X[5 * i + 2];
        h[3 * T + i] = X[5 * i + 3];
        h[4 * T + i] = X[5 * i + 4];
    }
    for (int i = 0; i < tu; ++i) { h[5 * T + i] = U[2 * i]; h[5 * T + tu + i] = U[2 * i + 1]; }
    mpc_ctx* c = (mpc_ctx*)std::calloc(1, sizeof(mpc_ctx));
    if (!c) return fail(MPC_E_ALLOC, "calloc");
    c->device = device;
    c->p = *p;
    if (hipMalloc(&c->table_buf, h.size() * sizeof(double)) != hipSuccess) {
        std::free(c);
        return fail(MPC_E_ALLOC, "hipMalloc table");
    }
    if (hipMemcpy(c->table_buf, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(c->table_buf);
        std::free(c);
        return fail(MPC_E_DEVICE, "hipMemcpy table");
    }
    c->tab.s = c->table_buf;
    c->tab.d = c->table_buf + T;
    c->tab.o = c->table_buf + 2 * T;
    c->tab.k = c->table_buf + 3 * T;
    c->tab.v = c->table_buf + 4 * T;
    c->tab.u1 = c->table_buf + 5 * T;
    c->tab.u2 = c->table_buf + 5 * T + tu;
    c->tab.T = T;
    c->tab.Tu = tu;
    c->tab.smax = s[T - 1];
    for (int j = 0; j < 5; ++j) c->tab.last[j] = X[5 * (T - 1) + j];
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        hipFree(c->table_buf);
        std::free(c);
        return fail(MPC_E_DEVICE, "hipStreamCreate");
    }
    *out = c;
    return MPC_SUCCESS;
}

extern "C" int mpc_set_params(mpc_ctx* c, const mpc_params* p) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    int rc = check_params(p);
    if (rc) return rc;
    c->p = *p;
    return MPC_SUCCESS;
}

extern "C" int mpc_get_params(const mpc_ctx* c, mpc_params* p) {
    if (!c || !p) return fail(MPC_E_ARG, "NULL argument");
    *p = c->p;
    return MPC_SUCCESS;
}

static void free_staging(mpc_ctx* c) {
    hipFree(c->x0); hipFree(c->obs); hipFree(c->ub); hipFree(c->u0); hipFree(c->U); hipFree(c->X);
    hipFree(c->nobs); hipFree(c->status); hipFree(c->iters);
    c->x0 = c->obs = c->ub = c->u0 = c->U = c->X = nullptr;
    c->nobs = c->status = c->iters = nullptr;
    c->cap_B = 0;
}

extern "C" void mpc_destroy(mpc_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    free_staging(c);
    hipFree(c->ls); hipFree(c->lst); hipFree(c->lct);
    hipFree(c->table_buf);
    hipStreamDestroy(c->stream);
    std::free(c);
}

extern "C" int mpc_solve_batch_device(mpc_ctx* c, int B, const double* x0, const double* obs, const int* n_obs,
                                      const double* ubar, double* u0, double* U, double* Xpred, int* status,
                                      int* iters, void* stream) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    if (B < 0) return fail(MPC_E_ARG, "B < 0");
    if (B == 0) return MPC_SUCCESS;
    if (!x0) return fail(MPC_E_ARG, "x0 is NULL");
    if (c->p.max_obs > 0 && n_obs && !obs) return fail(MPC_E_ARG, "n_obs given but obs is NULL");
    int rc = check_params(&c->p);
    if (rc) return rc;
    KParams kp = kparams(&c->p);
    if (!obs) kp.max_obs = 0;
    size_t lds = sizeof(double) * (size_t)lds_doubles(kp.N);
    if (lds > 160 * 1024) return fail(MPC_E_ARG, "horizon too long for LDS");
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    // rows of a stage spread over P lanes: all 64 lanes carry row state when N is short
    const int* nob = obs ? n_obs : nullptr;
    hipStream_t st = (hipStream_t)stream;
    if (3 * kp.N <= WAVE)
        hipLaunchKernelGGL(mpc_solve_kernel<3>, dim3(B), dim3(WAVE), lds, st, c->tab, kp, B, x0, obs, nob, ubar, u0,
                           U, Xpred, status, iters);
    else if (2 * kp.N <= WAVE)
        hipLaunchKernelGGL(mpc_solve_kernel<2>, dim3(B), dim3(WAVE), lds, st, c->tab, kp, B, x0, obs, nob, ubar, u0,
                           U, Xpred, status, iters);
    else
        hipLaunchKernelGGL(mpc_solve_kernel<1>, dim3(B), dim3(WAVE), lds, st, c->tab, kp, B, x0, obs, nob, ubar, u0,
                           U, Xpred, status, iters);
    HIPCHK(hipGetLastError(), MPC_E_LAUNCH);
    return MPC_SUCCESS;
}

template <typename T>
static int grow(T** ptr, size_t n) {
    hipFree(*ptr);
    *ptr = nullptr;
    if (n == 0) return 0;
    return hipMalloc(ptr, n * sizeof(T)) == hipSuccess ? 0 : -1;
}

extern "C" int mpc_solve_batch(mpc_ctx* c, int B, const double* x0, const double* obs, const int* n_obs,
                               const double* ubar, double* u0, double* U, double* Xpred, int* status, int* iters) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    if (B < 0) return fail(MPC_E_ARG, "B < 0");
    if (B == 0) return MPC_SUCCESS;
    if (!x0) return fail(MPC_E_ARG, "x0 is NULL");
    int rc = check_params(&c->p);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    const int N = c->p.N, mo = c->p.max_obs;
    if ((size_t)B > c->cap_B || N > c->cap_N || mo > c->cap_obs) {
        size_t nb = (size_t)B > c->cap_B ? (size_t)B : c->cap_B;
        int nn = N > c->cap_N ? N : c->cap_N;
        int no = mo > c->cap_obs ? mo : c->cap_obs;
        free_staging(c);
        if (grow(&c->x0, nb * 5) || grow(&c->obs, nb * (no > 0 ? no : 1) * 2) || grow(&c->ub, nb * 2 * nn) ||
            grow(&c->u0, nb * 2) || grow(&c->U, nb * 2 * nn) || grow(&c->X, nb * 5 * (nn + 1)) ||
            grow(&c->nobs, nb) || grow(&c->status, nb) || grow(&c->iters, nb))
            return fail(MPC_E_ALLOC, "hipMalloc staging");
        c->cap_B = nb;
        c->cap_N = nn;
        c->cap_obs = no;
    }
    hipStream_t s = c->stream;
    HIPCHK(hipMemcpyAsync(c->x0, x0, sizeof(double) * 5 * B, hipMemcpyHostToDevice, s), MPC_E_DEVICE);
    const bool use_obs = mo > 0 && obs;
    if (use_obs) {
        HIPCHK(hipMemcpyAsync(c->obs, obs, sizeof(double) * 2 * mo * B, hipMemcpyHostToDevice, s), MPC_E_DEVICE);
        if (n_obs) {
            HIPCHK(hipMemcpyAsync(c->nobs, n_obs, sizeof(int) * B, hipMemcpyHostToDevice, s), MPC_E_DEVICE);
        } else {
            std::vector<int> full(B, mo);
            HIPCHK(hipMemcpyAsync(c->nobs, full.data(), sizeof(int) * B, hipMemcpyHostToDevice, s), MPC_E_DEVICE);
            HIPCHK(hipStreamSynchronize(s), MPC_E_DEVICE);
        }
    }
    if (ubar) HIPCHK(hipMemcpyAsync(c->ub, ubar, sizeof(double) * 2 * N * B, hipMemcpyHostToDevice, s), MPC_E_DEVICE);
    rc = mpc_solve_batch_device(c, B, c->x0, use_obs ? c->obs : nullptr, use_obs ? c->nobs : nullptr,
                                ubar ? c->ub : nullptr, c->u0, c->U, c->X, c->status, c->iters, (void*)s);
    if (rc) return rc;
    if (u0) HIPCHK(hipMemcpyAsync(u0, c->u0, sizeof(double) * 2 * B, hipMemcpyDeviceToHost, s), MPC_E_DEVICE);
    if (U) HIPCHK(hipMemcpyAsync(U, c->U, sizeof(double) * 2 * N * B, hipMemcpyDeviceToHost, s), MPC_E_DEVICE);
    if (Xpred)
        HIPCHK(hipMemcpyAsync(Xpred, c->X, sizeof(double) * 5 * (N + 1) * B, hipMemcpyDeviceToHost, s), MPC_E_DEVICE);
    if (status) HIPCHK(hipMemcpyAsync(status, c->status, sizeof(int) * B, hipMemcpyDeviceToHost, s), MPC_E_DEVICE);
    if (iters) HIPCHK(hipMemcpyAsync(iters, c->iters, sizeof(int) * B, hipMemcpyDeviceToHost, s), MPC_E_DEVICE);
    HIPCHK(hipStreamSynchronize(s), MPC_E_DEVICE);
    return MPC_SUCCESS;
}

extern "C" int mpc_lookup(mpc_ctx* c, int n, const double* s, double* out_state, double* out_control) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    if (n < 0 || (n > 0 && !s)) return fail(MPC_E_ARG, "bad lookup arguments");
    if (n == 0) return MPC_SUCCESS;
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    if ((size_t)n > c->cap_lookup) {
        if (grow(&c->ls, n) || grow(&c->lst, (size_t)n * 5) || grow(&c->lct, (size_t)n * 2))
            return fail(MPC_E_ALLOC, "hipMalloc lookup");
        c->cap_lookup = n;
    }
    hipStream_t st = c->stream;
    HIPCHK(hipMemcpyAsync(c->ls, s, sizeof(double) * n, hipMemcpyHostToDevice, st), MPC_E_DEVICE);
    hipLaunchKernelGGL(mpc_lookup_kernel, dim3((n + 255) / 256), dim3(256), 0, st, c->tab, n, c->ls, c->lst, c->lct);
    HIPCHK(hipGetLastError(), MPC_E_LAUNCH);
    if (out_state)
        HIPCHK(hipMemcpyAsync(out_state, c->lst, sizeof(double) * 5 * n, hipMemcpyDeviceToHost, st), MPC_E_DEVICE);
    if (out_control)
        HIPCHK(hipMemcpyAsync(out_control, c->lct, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, st), MPC_E_DEVICE);
    HIPCHK(hipStreamSynchronize(st), MPC_E_DEVICE);
    return MPC_SUCCESS;
}

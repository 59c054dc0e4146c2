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
// per-instance LDS layout (doubles); stage arrays indexed k = 0..N, row arrays [j][k]
// ------------------------------------------------------------------------------------------
struct Lds {
    double* A5;    // [N][5]    a12,a14,a20,a23,a24 of A_k = I + J'_k  (a04 = dt)
    double* Qs;    // [N+1][10] cost Hessian on (s,d,o,v), packed upper
    double* qs;    // [N+1][4]
    double* bs;    // [N+1][9]  soft row bounds
    double* bb;    // [N][4]    box row bounds
    double* rr;    // [N][2]    R * ubar
    double* Qt;    // [N+1][10] Riccati stage Hessians (barrier / penalty augmented)
    double* Rt;    // [N][2]
    double* Kf;    // [N][10]   Riccati gains K_k (2x5)
    double* Si;    // [N][3]    (1/l00, l10, 1/l11) of S_k = Ls Ls'
    double* qh;    // [N+1][4]  LQR stage linear terms
    double* gh;    // [N][2]
    double* kk;    // [N][2]
    double* Xr;    // [N+1][5]  rollout of the current iterate
    double* dX;    // [N+1][5]  rollout of the direction
    double* du;    // [N][2]    current iterate dU
    double* dud;   // [N][2]    direction dU
    double* dub;   // [N][2]    backup (interior-point iterate during the polish)
    double* ys;    // [N+1][4]  dual residual stage terms: cost part
    double* ya;    // [N+1][4]  dual residual stage terms: multiplier part
    double* zs;    // [N][2]
    double* za;    // [N][2]
    double* ub;    // [N][2]    linearisation point
    double* xb;    // [N+1][5]  nominal rollout / predict output
    double* kap;   // [N+1]
    // interior-point row state (soft rows [9][N+1], box rows [4][N])
    double *rs, *rl, *rxi, *rnu, *pa4, *pa5, *tl;
    double *bsv, *blv, *pab, *tlb;
    double* cls;   // [9][N+1] polish row class, [4][N] box class after it
};

__host__ __device__ inline int lds_doubles(int N) {
    int NP = N + 1;
    return N * 5 + NP * 10 + NP * 4 + NP * 9 + N * 4 + N * 2 + NP * 10 + N * 2 + N * 10 + N * 3 + NP * 4 + N * 2 +
           N * 2 + NP * 5 + NP * 5 + N * 2 + N * 2 + N * 2 + NP * 4 + NP * 4 + N * 2 + N * 2 + N * 2 + NP * 5 + NP +
           7 * 9 * NP + 4 * 4 * N + 9 * NP + 4 * N;
}

__device__ inline Lds carve(double* p, int N) {
    Lds L;
    int NP = N + 1;
    L.A5 = p; p += N * 5;
    L.Qs = p; p += NP * 10;
    L.qs = p; p += NP * 4;
    L.bs = p; p += NP * 9;
    L.bb = p; p += N * 4;
    L.rr = p; p += N * 2;
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
    L.ys = p; p += NP * 4;
    L.ya = p; p += NP * 4;
    L.zs = p; p += N * 2;
    L.za = p; p += N * 2;
    L.ub = p; p += N * 2;
    L.xb = p; p += NP * 5;
    L.kap = p; p += NP;
    L.rs = p; p += 9 * NP;
    L.rl = p; p += 9 * NP;
    L.rxi = p; p += 9 * NP;
    L.rnu = p; p += 9 * NP;
    L.pa4 = p; p += 9 * NP;
    L.pa5 = p; p += 9 * NP;
    L.tl = p; p += 9 * NP;
    L.bsv = p; p += 4 * N;
    L.blv = p; p += 4 * N;
    L.pab = p; p += 4 * N;
    L.tlb = p; p += 4 * N;
    L.cls = p; p += 9 * NP + 4 * N;
    return L;
}

// packed symmetric 4x4 on (s,d,o,v): index of (a,b)
__device__ __forceinline__ int p4(int a, int b) {
    if (a > b) { int t = a; a = b; b = t; }
    return a == 0 ? b : (a == 1 ? 3 + b : (a == 2 ? 5 + b : 9));
}
// state index (0..4: s,d,o,k,v) of reduced index (0..3: s,d,o,v)
__device__ __forceinline__ int st4(int a) { return a == 3 ? 4 : a; }

// soft row coefficient vectors over (s,d,o,v) (oracle C[][] with the k entry dropped)
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

// nonlinear rollout (predict, trajectory_tracking.py:87-114), bit-exact.  s, v, k do not depend on
// the k_ref lookups, so they are rolled first; lane j then looks up k_ref(s_j); then d, o.
__device__ void predict_wave(const DevTable& tab, const KParams& P, const double* x0, const double* uU,
                             double* xout, double* kap, int lane) {
    const int N = P.N;
    const double dt = P.dt;
    if (lane == 0) {
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
    if (lane < N) {
        double st[5];
        get_state(tab, xout[5 * lane], st, nullptr);
        kap[lane] = st[3];
    }
    wave_sync();
    if (lane == 0) {
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

// X = G u : rollout of the linear model from x_0 = 0 (uniform; lane 0 writes)
__device__ void rollout_lin(const Lds& S, int N, double dt, const double* u, double* X, int lane) {
    if (lane == 0) {
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

// Riccati factorisation of  min sum 0.5 x'Qt x + 0.5 u'Rt u,  x_{k+1} = A_k x_k + B u_k,  x_0 = 0.
// S_k = Rt_k + B'P B = Ls Ls' (2x2 Cholesky), W = Ls^-1 B'P A, K = -Ls^-T W, P <- Qt + A'PA - W'W.
// The Cholesky form keeps ~2 more digits than an explicit S^-1 when the barrier weights reach
// 1e12+.  Wave-uniform; lane 0 writes Kf, Si.
__device__ void riccati_factor(const Lds& S, int N, double dt, int lane) {
    double Pm[5][5];
#pragma unroll
    for (int a = 0; a < 5; ++a)
#pragma unroll
        for (int c = 0; c < 5; ++c) Pm[a][c] = 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) Pm[st4(a)][st4(c)] = S.Qt[10 * N + p4(a, c)];
    const double dt2 = dt * dt;
    for (int t = N - 1; t >= 0; --t) {
        const double* a = S.A5 + 5 * t;
        const double a12 = a[0], a14 = a[1], a20 = a[2], a23 = a[3], a24 = a[4];
        double M[5][5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            M[i][0] = fma(Pm[i][2], a20, Pm[i][0]);
            M[i][1] = Pm[i][1];
            M[i][2] = fma(Pm[i][1], a12, Pm[i][2]);
            M[i][3] = fma(Pm[i][2], a23, Pm[i][3]);
            M[i][4] = fma(Pm[i][0], dt, fma(Pm[i][1], a14, fma(Pm[i][2], a24, Pm[i][4])));
        }
        double s00 = fma(dt2, Pm[3][3], S.Rt[2 * t]);
        double s01 = dt2 * Pm[3][4];
        double s11 = fma(dt2, Pm[4][4], S.Rt[2 * t + 1]);
        if (!(s00 > 0.0)) s00 = 1e-300 + fabs(s00);
        double l00 = sqrt(s00), l10 = s01 / l00, r11 = s11 - l10 * l10;
        if (!(r11 > 1e-14 * s11)) r11 = 1e-14 * fabs(s11) + 1e-300;
        double l11 = sqrt(r11);
        double il00 = 1.0 / l00, il11 = 1.0 / l11;
        double W0[5], W1[5], K0[5], K1[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            W0[j] = dt * M[3][j] * il00;
            W1[j] = (dt * M[4][j] - l10 * W0[j]) * il11;
            K1[j] = -W1[j] * il11;
            K0[j] = -(W0[j] + l10 * K1[j]) * il00;
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < 5; ++j) { S.Kf[10 * t + j] = K0[j]; S.Kf[10 * t + 5 + j] = K1[j]; }
            S.Si[3 * t] = il00; S.Si[3 * t + 1] = l10; S.Si[3 * t + 2] = il11;
        }
        if (t >= 1) {
            double Pn[5][5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                Pn[0][j] = fma(a20, M[2][j], M[0][j]);
                Pn[1][j] = M[1][j];
                Pn[2][j] = fma(a12, M[1][j], M[2][j]);
                Pn[3][j] = fma(a23, M[2][j], M[3][j]);
                Pn[4][j] = fma(dt, M[0][j], fma(a14, M[1][j], fma(a24, M[2][j], M[4][j])));
            }
            const double* qt = S.Qt + 10 * t;
#pragma unroll
            for (int i = 0; i < 5; ++i)
#pragma unroll
                for (int j = i; j < 5; ++j) {
                    double ww = fma(W0[i], W0[j], W1[i] * W1[j]);
                    double q = (i != 3 && j != 3) ? qt[p4(i == 4 ? 3 : i, j == 4 ? 3 : j)] : 0.0;
                    double val = 0.5 * ((Pn[i][j] - ww) + (Pn[j][i] - ww)) + q;
                    Pm[i][j] = val;
                    Pm[j][i] = val;
                }
        }
    }
    wave_sync();
}

// LQR solve with the factorisation: linear terms -qh (stages 1..N), -gh (controls).
// Writes dud (controls) and dX (states, x_0 = 0).  Wave-uniform; lane 0 writes.
__device__ void riccati_solve(const Lds& S, int N, double dt, int lane) {
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
        if (lane == 0) { S.kk[2 * t] = k0; S.kk[2 * t + 1] = k1; }
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
    if (lane == 0) {
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

// max |g_d| and the scale max(|g_cost|, |g_mult|) of the dual residual g = G'(y) + z, by the
// adjoint recursion over the stage terms ys (cost) and ya (multipliers).  Wave-uniform.
__device__ void dual_norms(const Lds& S, int N, double dt, double& rdmax, double& sd) {
    double mc[5] = {0, 0, 0, 0, 0}, ma[5] = {0, 0, 0, 0, 0};
    rdmax = 0.0;
    sd = 0.0;
    for (int k = N; k >= 1; --k) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            mc[st4(a)] += S.ys[4 * k + a];
            ma[st4(a)] += S.ya[4 * k + a];
        }
        const int t = k - 1;
        double gc0 = fma(dt, mc[3], S.zs[2 * t]), gc1 = fma(dt, mc[4], S.zs[2 * t + 1]);
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

#define POLISH_DELTA 1e-11
#define POLISH_REFINE 4
#define POLISH_ROUNDS 6

// ------------------------------------------------------------------------------------------
// the solver kernel: one wavefront per MPC instance
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(WAVE)
mpc_solve_kernel(DevTable tab, KParams P, int B, const double* __restrict__ x0g, const double* __restrict__ obsg,
                 const int* __restrict__ nobsg, const double* __restrict__ ubarg, double* __restrict__ u0g,
                 double* __restrict__ Ug, double* __restrict__ Xg, int* __restrict__ statusg,
                 int* __restrict__ itersg) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int b = blockIdx.x;
    if (b >= B) return;
    const int lane = threadIdx.x;
    const int N = P.N;
    const int NP = N + 1;
    const double dt = P.dt;
    const double rho = P.rho;
    const double hL = P.L / 2.0;
    Lds S = carve(smem, N);

    double x0[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) x0[j] = x0g[5 * (size_t)b + j];
    int nobs = nobsg ? nobsg[b] : 0;
    nobs = nobs < 0 ? 0 : (nobs > P.max_obs ? P.max_obs : nobs);
    const double* obs = obsg ? obsg + (size_t)b * P.max_obs * 2 : nullptr;
    const bool has_obs = nobs > 0;
    const bool live = lane < N;     // lane owns soft rows of stage k = lane+1 and box rows of control t = lane
    const int k = lane + 1;

    // ---- K1: linearisation point ---------------------------------------------------------
    if (live) {
        if (ubarg) {
            S.ub[2 * lane] = ubarg[(size_t)b * 2 * N + 2 * lane];
            S.ub[2 * lane + 1] = ubarg[(size_t)b * 2 * N + 2 * lane + 1];
        } else {
            // warm start, trajectory_tracking.py:224-246: s_curr advanced by repeated addition,
            // sticky brake flag over steps 0..lane
            double s_curr = x0[0], v_curr = x0[4];
            bool brake = false;
            for (int j = 0; j <= lane; ++j) {
                if (j > 0) s_curr += v_curr * dt;
                for (int i = 0; i < nobs; ++i)
                    if ((obs[2 * i] - s_curr) < P.brake_distance) brake = true;
            }
            double ur[2];
            get_control(tab, s_curr, ur);
            S.ub[2 * lane] = ur[0];
            S.ub[2 * lane + 1] = brake ? P.brake_accel : ur[1];
        }
    }
    wave_sync();

    int nsoft = 0;
    for (int j = 0; j < NROW; ++j) nsoft += ((j != 6 && j != 7) || has_obs) ? 1 : 0;
    const double Mtot = (double)(2 * nsoft * N + NBOX * N);
    const double R0 = 2.0 * P.w_u1, R1 = 2.0 * P.w_u2;

    const int nsqp = P.sqp_iters < 0 ? 0 : P.sqp_iters;   // 0: return ubar and predict(x0, ubar)
    int status = MPC_OK, total_it = 0;
    for (int sqp = 0; sqp < nsqp; ++sqp) {
        // ---- K1: nominal rollout == predict(x0, ubar) ------------------------------------
        predict_wave(tab, P, x0, S.ub, S.xb, S.kap, lane);
        // ---- K2: stage data of QP(ubar) ----------------------------------------------------
        const bool gn = P.linearization != 0;
        double refk[5], slk[4];
        if (lane <= N) get_state(tab, S.xb[5 * lane], refk, slk);
        if (live) {
            const double* x = S.xb + 5 * lane;
            double dk = gn ? slk[2] : 0.0;
            S.A5[5 * lane + 0] = dt * x[4];
            S.A5[5 * lane + 1] = dt * x[2];
            S.A5[5 * lane + 2] = dt * (-x[4] * dk);
            S.A5[5 * lane + 3] = dt * x[4];
            S.A5[5 * lane + 4] = dt * (x[3] - refk[3]);
        }
        double bscale_l = 0.0;
        if (lane >= 1 && lane <= N) {
            const int kk = lane;
            const double* x = S.xb + 5 * kk;
            double ref[3] = {refk[1], refk[2], refk[4]};
            double dref[3] = {gn ? slk[0] : 0.0, gn ? slk[1] : 0.0, gn ? slk[3] : 0.0};
            double w[3] = {P.w_d, P.w_o, P.w_v};
            int idx[3] = {1, 2, 4};
            double Qp[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, q4[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                double m[4] = {-dref[j], 0.0, 0.0, 0.0};
                m[j + 1] = 1.0;
                double r0 = x[idx[j]] - ref[j];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    q4[a] += 2.0 * w[j] * r0 * m[a];
#pragma unroll
                    for (int c = a; c < 4; ++c) Qp[p4(a, c)] += 2.0 * w[j] * m[a] * m[c];
                }
            }
            for (int a = 0; a < 10; ++a) S.Qs[10 * kk + a] = Qp[a];
            for (int a = 0; a < 4; ++a) S.qs[4 * kk + a] = q4[a];
            const double Lw = P.L, sl = P.sl;
            double pv0 = x[1], pv1 = x[1] + hL * x[2], pv2 = x[1] + Lw * x[2];
            double bk[NROW];
            bk[0] = -sl - pv0; bk[1] = -(sl - pv0);
            bk[2] = -sl - pv1; bk[3] = -(sl - pv1);
            bk[4] = -sl - pv2; bk[5] = -(sl - pv2);
            bk[6] = 0.0; bk[7] = 0.0;
            if (has_obs) {
                double shat = INFINITY;
                for (int i = 0; i < nobs; ++i) {
                    double sp = obs[2 * i] + obs[2 * i + 1] * (kk * dt);
                    shat = sp < shat ? sp : shat;
                }
                bk[6] = -(shat - P.osd - x[0]);
                bk[7] = -(shat - x[0] - P.tgap * x[4]);
            }
            bk[8] = -x[4];
#pragma unroll
            for (int j = 0; j < NROW; ++j) {
                S.bs[NROW * kk + j] = bk[j];
                if ((j != 6 && j != 7) || has_obs) bscale_l = fmax(bscale_l, fabs(bk[j]));
            }
        }
        if (live) {
            double ub0 = S.ub[2 * lane], ub1 = S.ub[2 * lane + 1];
            S.bb[4 * lane + 0] = P.u_min0 - ub0;
            S.bb[4 * lane + 1] = -(P.u_max0 - ub0);
            S.bb[4 * lane + 2] = P.u_min1 - ub1;
            S.bb[4 * lane + 3] = -(P.u_max1 - ub1);
            S.rr[2 * lane] = R0 * ub0;
            S.rr[2 * lane + 1] = R1 * ub1;
#pragma unroll
            for (int j = 0; j < NBOX; ++j) bscale_l = fmax(bscale_l, fabs(S.bb[4 * lane + j]));
        }
        const double bscale = wave_max(bscale_l);
        wave_sync();

        // ---- K4: PDIP ------------------------------------------------------------------------
        if (live) {
#pragma unroll
            for (int j = 0; j < NROW; ++j) {
                const bool on = (j != 6 && j != 7) || has_obs;
                double r0 = -S.bs[NROW * k + j];
                double xi = (r0 < 0 ? -r0 : 0.0) + XI0;
                S.rxi[j * NP + k] = on ? xi : 1.0;
                S.rs[j * NP + k] = on ? r0 + xi : 1.0;
                S.rl[j * NP + k] = on ? 1.0 : 0.0;
                S.rnu[j * NP + k] = on ? rho - 1.0 : 0.0;
            }
#pragma unroll
            for (int j = 0; j < NBOX; ++j) {
                double r0 = -S.bb[4 * lane + j];
                S.bsv[j * N + lane] = r0 > 1.0 ? r0 : 1.0;
                S.blv[j * N + lane] = 1.0;
            }
            S.du[2 * lane] = 0.0;
            S.du[2 * lane + 1] = 0.0;
        }
        wave_sync();

        int it;
        int st_here = MPC_MAX_ITER;
        int stall = 0;
        bool have_acc = false, inf_acc = false;
        double acc0 = 0.0, acc1 = 0.0, mu = 0.0;
        for (it = 0; it < P.max_iter; ++it) {
            rollout_lin(S, N, dt, S.du, S.Xr, lane);
            // -- stage-parallel residuals -------------------------------------------------------
            double rpmax = 0.0, rxmax = 0.0, comp = 0.0;
            if (live) {
                double x4[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) x4[a] = S.Xr[5 * k + st4(a)];
                double yc[4], ya[4] = {0, 0, 0, 0};
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    double acc = S.qs[4 * k + a];
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc = fma(S.Qs[10 * k + p4(a, c)], x4[c], acc);
                    yc[a] = acc;
                }
#pragma unroll
                for (int j = 0; j < NROW; ++j) {
                    if ((j == 6 || j == 7) && !has_obs) continue;
                    double c[4];
                    row_coef(j, hL, P.L, P.tgap, c);
                    const double sv = S.rs[j * NP + k], lv = S.rl[j * NP + k];
                    const double xv = S.rxi[j * NP + k], nv = S.rnu[j * NP + k];
                    double cx = c[0] * x4[0] + c[1] * x4[1] + c[2] * x4[2] + c[3] * x4[3];
                    double r = cx + xv - sv - S.bs[NROW * k + j];
                    double rx = rho - lv - nv;
#pragma unroll
                    for (int a = 0; a < 4; ++a) ya[a] = fma(-lv, c[a], ya[a]);
                    rpmax = fmax(rpmax, fabs(r));
                    rxmax = fmax(rxmax, fabs(rx));
                    comp += sv * lv + xv * nv;
                }
#pragma unroll
                for (int a = 0; a < 4; ++a) { S.ys[4 * k + a] = yc[a]; S.ya[4 * k + a] = ya[a]; }
                const double du0 = S.du[2 * lane], du1 = S.du[2 * lane + 1];
                S.zs[2 * lane] = fma(R0, du0, S.rr[2 * lane]);
                S.zs[2 * lane + 1] = fma(R1, du1, S.rr[2 * lane + 1]);
                S.za[2 * lane] = -S.blv[0 * N + lane] + S.blv[1 * N + lane];
                S.za[2 * lane + 1] = -S.blv[2 * N + lane] + S.blv[3 * N + lane];
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    double uu = (j < 2) ? du0 : du1;
                    double r = bsign(j) * uu - S.bsv[j * N + lane] - S.bb[4 * lane + j];
                    rpmax = fmax(rpmax, fabs(r));
                    comp += S.bsv[j * N + lane] * S.blv[j * N + lane];
                }
            }
            rpmax = wave_max(rpmax);
            rxmax = wave_max(rxmax);
            comp = wave_sum(comp);
            wave_sync();
            double rdmax, sd;
            dual_norms(S, N, dt, rdmax, sd);
            mu = comp / Mtot;
            if (!(mu == mu) || !(rdmax == rdmax)) { st_here = MPC_NUMERICAL; break; }
            // the dual residual carries the O(eps/mu) noise of the active multipliers: tolerance 1e3*tol
            if (rdmax <= 1e3 * P.tol * (1.0 + sd) && rpmax <= P.tol * (1.0 + bscale) && rxmax <= P.tol * rho &&
                mu <= P.tol_mu) {
                st_here = MPC_OK;
                break;
            }
            // acceptable iterate, returned if the iteration later breaks down
            if (rdmax <= 1e4 * P.tol * (1.0 + sd) && rpmax <= 10.0 * P.tol * (1.0 + bscale) && mu <= 1e2 * P.tol_mu) {
                double inf = 0.0;
                if (live) {
#pragma unroll
                    for (int j = 0; j < NROW; ++j) {
                        if ((j == 6 || j == 7) && !has_obs) continue;
                        if (S.rxi[j * NP + k] > 1e-6 * (1.0 + fabs(S.bs[NROW * k + j]))) inf = 1.0;
                    }
                    acc0 = S.du[2 * lane];
                    acc1 = S.du[2 * lane + 1];
                }
                inf_acc = wave_max(inf) > 0.0;
                have_acc = true;
            }
            if (mu < 1e-3 * P.tol_mu) { st_here = MPC_NUMERICAL; ++it; break; }
            // -- barrier weights, augmented stage Hessians ---------------------------------------
            if (live) {
                double Qp[10];
#pragma unroll
                for (int a = 0; a < 10; ++a) Qp[a] = S.Qs[10 * k + a];
#pragma unroll
                for (int j = 0; j < NROW; ++j) {
                    if ((j == 6 || j == 7) && !has_obs) continue;
                    double c[4];
                    row_coef(j, hL, P.L, P.tgap, c);
                    double d = S.rs[j * NP + k] / S.rl[j * NP + k] + S.rxi[j * NP + k] / S.rnu[j * NP + k];
                    double w = 1.0 / d;
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int cc = a; cc < 4; ++cc)
                            if (c[a] != 0.0 && c[cc] != 0.0) Qp[p4(a, cc)] = fma(w * c[a], c[cc], Qp[p4(a, cc)]);
                }
#pragma unroll
                for (int a = 0; a < 10; ++a) S.Qt[10 * k + a] = Qp[a];
                double r0 = R0, r1 = R1;
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    double w = S.blv[j * N + lane] / S.bsv[j * N + lane];
                    if (j < 2) r0 += w; else r1 += w;
                }
                S.Rt[2 * lane] = r0;
                S.Rt[2 * lane + 1] = r1;
            }
            wave_sync();
            riccati_factor(S, N, dt, lane);
            // -- predictor and corrector solves ----------------------------------------------------
            double sig = 0.0, alpha = 0.0;
            for (int pass = 0; pass < 2; ++pass) {
                const double smu = (pass == 1) ? sig * mu : 0.0;
                if (live) {
                    double x4[4];
#pragma unroll
                    for (int a = 0; a < 4; ++a) x4[a] = S.Xr[5 * k + st4(a)];
                    double q4[4];
#pragma unroll
                    for (int a = 0; a < 4; ++a) q4[a] = -(S.ys[4 * k + a] + S.ya[4 * k + a]);
#pragma unroll
                    for (int j = 0; j < NROW; ++j) {
                        if ((j == 6 || j == 7) && !has_obs) continue;
                        double c[4];
                        row_coef(j, hL, P.L, P.tgap, c);
                        const double sv = S.rs[j * NP + k], lv = S.rl[j * NP + k];
                        const double xv = S.rxi[j * NP + k], nv = S.rnu[j * NP + k];
                        double r4 = sv * lv, r5 = xv * nv;
                        if (pass == 1) { r4 += S.pa4[j * NP + k] - smu; r5 += S.pa5[j * NP + k] - smu; }
                        double rp = c[0] * x4[0] + c[1] * x4[1] + c[2] * x4[2] + c[3] * x4[3] + xv - sv -
                                    S.bs[NROW * k + j];
                        double rx = rho - lv - nv;
                        double d = sv / lv + xv / nv;
                        double rh = -rp - r4 / lv + (r5 + xv * rx) / nv;
                        double w = rh / d;
#pragma unroll
                        for (int a = 0; a < 4; ++a) q4[a] = fma(c[a], w, q4[a]);
                    }
#pragma unroll
                    for (int a = 0; a < 4; ++a) S.qh[4 * k + a] = q4[a];
                    const double du0 = S.du[2 * lane], du1 = S.du[2 * lane + 1];
                    double g0 = -(S.zs[2 * lane] + S.za[2 * lane]);
                    double g1 = -(S.zs[2 * lane + 1] + S.za[2 * lane + 1]);
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) {
                        const double sb = S.bsv[j * N + lane], lb = S.blv[j * N + lane];
                        double r4 = sb * lb;
                        if (pass == 1) r4 += S.pab[j * N + lane] - smu;
                        double uu = (j < 2) ? du0 : du1;
                        double rp = bsign(j) * uu - sb - S.bb[4 * lane + j];
                        double rh = -rp - r4 / lb;
                        double v = bsign(j) * rh * lb / sb;
                        if (j < 2) g0 += v; else g1 += v;
                    }
                    S.gh[2 * lane] = g0;
                    S.gh[2 * lane + 1] = g1;
                }
                wave_sync();
                riccati_solve(S, N, dt, lane);
                // row directions and step length
                double amax = 1.0;
                if (live) {
                    double x4[4], dx4[4];
#pragma unroll
                    for (int a = 0; a < 4; ++a) { x4[a] = S.Xr[5 * k + st4(a)]; dx4[a] = S.dX[5 * k + st4(a)]; }
#pragma unroll
                    for (int j = 0; j < NROW; ++j) {
                        if ((j == 6 || j == 7) && !has_obs) continue;
                        double c[4];
                        row_coef(j, hL, P.L, P.tgap, c);
                        const double sv = S.rs[j * NP + k], lv = S.rl[j * NP + k];
                        const double xv = S.rxi[j * NP + k], nv = S.rnu[j * NP + k];
                        double r4 = sv * lv, r5 = xv * nv;
                        if (pass == 1) { r4 += S.pa4[j * NP + k] - smu; r5 += S.pa5[j * NP + k] - smu; }
                        double rp = c[0] * x4[0] + c[1] * x4[1] + c[2] * x4[2] + c[3] * x4[3] + xv - sv -
                                    S.bs[NROW * k + j];
                        double rx = rho - lv - nv;
                        double d = sv / lv + xv / nv;
                        double rh = -rp - r4 / lv + (r5 + xv * rx) / nv;
                        double cdx = c[0] * dx4[0] + c[1] * dx4[1] + c[2] * dx4[2] + c[3] * dx4[3];
                        double dl = (rh - cdx) / d;
                        double ds = -(r4 + sv * dl) / lv;
                        double dn = rx - dl;
                        double dxi = -(r5 + xv * dn) / nv;
                        if (pass == 0) {
                            // affine step: remember the second-order products for the corrector
                            S.pa4[j * NP + k] = ds * dl;
                            S.pa5[j * NP + k] = dxi * dn;
                            S.tl[j * NP + k] = ds;     // scratch: affine directions for mu_aff
                            S.cls[j * NP + k] = dl;
                        } else {
                            // stash the corrector direction in pa4/pa5/tl/cls until alpha is known
                            S.pa4[j * NP + k] = ds;
                            S.pa5[j * NP + k] = dl;
                            S.tl[j * NP + k] = dxi;
                            S.cls[j * NP + k] = dn;
                        }
                        if (ds < 0.0) amax = fmin(amax, -sv / ds);
                        if (dl < 0.0) amax = fmin(amax, -lv / dl);
                        if (dxi < 0.0) amax = fmin(amax, -xv / dxi);
                        if (dn < 0.0) amax = fmin(amax, -nv / dn);
                        if (pass == 0) {
                            // keep dxi, dn for mu_aff in registers-free form: recomputed below
                        }
                    }
                    const double du0 = S.du[2 * lane], du1 = S.du[2 * lane + 1];
                    const double dd0 = S.dud[2 * lane], dd1 = S.dud[2 * lane + 1];
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) {
                        const double sb = S.bsv[j * N + lane], lb = S.blv[j * N + lane];
                        double r4 = sb * lb;
                        if (pass == 1) r4 += S.pab[j * N + lane] - smu;
                        double uu = (j < 2) ? du0 : du1;
                        double duu = (j < 2) ? dd0 : dd1;
                        double rp = bsign(j) * uu - sb - S.bb[4 * lane + j];
                        double rh = -rp - r4 / lb;
                        double dl = (rh - bsign(j) * duu) * lb / sb;
                        double ds = -(r4 + sb * dl) / lb;
                        if (pass == 0) S.pab[j * N + lane] = ds * dl;
                        else { S.tlb[j * N + lane] = ds; S.cls[9 * NP + j * N + lane] = dl; }
                        if (pass == 0) { S.tlb[j * N + lane] = ds; S.cls[9 * NP + j * N + lane] = dl; }
                        if (ds < 0.0) amax = fmin(amax, -sb / ds);
                        if (dl < 0.0) amax = fmin(amax, -lb / dl);
                    }
                }
                amax = wave_min(amax);
                if (pass == 0) {
                    // mu after the affine step (needs dxi, dn: recomputed from the stored products)
                    double ca = 0.0;
                    if (live) {
                        double x4[4], dx4[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) { x4[a] = S.Xr[5 * k + st4(a)]; dx4[a] = S.dX[5 * k + st4(a)]; }
#pragma unroll
                        for (int j = 0; j < NROW; ++j) {
                            if ((j == 6 || j == 7) && !has_obs) continue;
                            const double sv = S.rs[j * NP + k], lv = S.rl[j * NP + k];
                            const double xv = S.rxi[j * NP + k], nv = S.rnu[j * NP + k];
                            const double ds = S.tl[j * NP + k], dl = S.cls[j * NP + k];
                            double dn = (rho - lv - nv) - dl;
                            double dxi = -(xv * nv + xv * dn) / nv;
                            ca += fma(amax, ds, sv) * fma(amax, dl, lv) + fma(amax, dxi, xv) * fma(amax, dn, nv);
                        }
#pragma unroll
                        for (int j = 0; j < NBOX; ++j)
                            ca += fma(amax, S.tlb[j * N + lane], S.bsv[j * N + lane]) *
                                  fma(amax, S.cls[9 * NP + j * N + lane], S.blv[j * N + lane]);
                    }
                    ca = wave_sum(ca);
                    double mua = ca / Mtot;
                    sig = mua / mu;
                    sig = sig * sig * sig;
                } else {
                    alpha = fmin(1.0, TAU * amax);
                    if (live) {
#pragma unroll
                        for (int j = 0; j < NROW; ++j) {
                            if ((j == 6 || j == 7) && !has_obs) continue;
                            const int o = j * NP + k;
                            S.rs[o] = fma(alpha, S.pa4[o], S.rs[o]);
                            S.rl[o] = fma(alpha, S.pa5[o], S.rl[o]);
                            S.rxi[o] = fma(alpha, S.tl[o], S.rxi[o]);
                            S.rnu[o] = fma(alpha, S.cls[o], S.rnu[o]);
                        }
#pragma unroll
                        for (int j = 0; j < NBOX; ++j) {
                            const int o = j * N + lane;
                            S.bsv[o] = fma(alpha, S.tlb[o], S.bsv[o]);
                            S.blv[o] = fma(alpha, S.cls[9 * NP + o], S.blv[o]);
                        }
                        S.du[2 * lane] = fma(alpha, S.dud[2 * lane], S.du[2 * lane]);
                        S.du[2 * lane + 1] = fma(alpha, S.dud[2 * lane + 1], S.du[2 * lane + 1]);
                    }
                }
                wave_sync();
            }
            stall = (alpha < 1e-10) ? stall + 1 : 0;
            if (stall >= 3) { st_here = MPC_NUMERICAL; ++it; break; }
        }
        total_it += it;
        const bool use_acc = (st_here != MPC_OK) && have_acc;
        if (use_acc && live) { S.du[2 * lane] = acc0; S.du[2 * lane + 1] = acc1; }
        wave_sync();
        double bad = 0.0;
        if (live) bad = (S.du[2 * lane] == S.du[2 * lane] && S.du[2 * lane + 1] == S.du[2 * lane + 1]) ? 0.0 : 1.0;
        bad = wave_max(bad);
        if (bad > 0.0) {
            st_here = MPC_NUMERICAL;
            if (live) { S.du[2 * lane] = 0.0; S.du[2 * lane + 1] = 0.0; }
        } else if (use_acc) {
            st_here = inf_acc ? MPC_INFEASIBLE : MPC_OK;
        } else if (st_here == MPC_OK) {
            double inf = 0.0;
            if (live) {
#pragma unroll
                for (int j = 0; j < NROW; ++j) {
                    if ((j == 6 || j == 7) && !has_obs) continue;
                    if (S.rxi[j * NP + k] > 1e-6 * (1.0 + fabs(S.bs[NROW * k + j]))) inf = 1.0;
                }
            }
            if (wave_max(inf) > 0.0) st_here = MPC_INFEASIBLE;
        }
        wave_sync();

        // ---- active-set polish (oracle polish()) --------------------------
        if (P.polish && bad == 0.0) {
            // classification from the interior-point iterate: 0 inactive, 1 active, 2 violated
            if (live) {
#pragma unroll
                for (int j = 0; j < NROW; ++j) {
                    const int o = j * NP + k;
                    double c = 0.0;
                    if ((j != 6 && j != 7) || has_obs) {
                        if (S.rxi[o] > S.rnu[o]) c = 2.0;
                        else if (S.rl[o] > S.rs[o]) c = 1.0;
                    }
                    S.cls[o] = c;
                }
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    const int o = j * N + lane;
                    S.cls[9 * NP + o] = S.blv[o] > S.bsv[o] ? 1.0 : 0.0;
                }
                S.dub[2 * lane] = S.du[2 * lane];
                S.dub[2 * lane + 1] = S.du[2 * lane + 1];
            }
            wave_sync();
            bool accepted = false;
            double nviol_acc = 0.0;
            for (int round = 0; round < POLISH_ROUNDS && !accepted; ++round) {
                if (live) {
                    S.du[2 * lane] = S.dub[2 * lane];
                    S.du[2 * lane + 1] = S.dub[2 * lane + 1];
                    double Qp[10];
#pragma unroll
                    for (int a = 0; a < 10; ++a) Qp[a] = S.Qs[10 * k + a];
#pragma unroll
                    for (int j = 0; j < NROW; ++j) {
                        const int o = j * NP + k;
                        S.tl[o] = S.rl[o];
                        if (S.cls[o] == 1.0) {
                            double c[4];
                            row_coef(j, hL, P.L, P.tgap, c);
#pragma unroll
                            for (int a = 0; a < 4; ++a)
#pragma unroll
                                for (int cc = a; cc < 4; ++cc)
                                    if (c[a] != 0.0 && c[cc] != 0.0)
                                        Qp[p4(a, cc)] = fma(c[a] / POLISH_DELTA, c[cc], Qp[p4(a, cc)]);
                        }
                    }
#pragma unroll
                    for (int a = 0; a < 10; ++a) S.Qt[10 * k + a] = Qp[a];
                    double r0 = R0, r1 = R1;
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) {
                        const int o = j * N + lane;
                        S.tlb[o] = S.blv[o];
                        if (S.cls[9 * NP + o] == 1.0) { if (j < 2) r0 += 1.0 / POLISH_DELTA; else r1 += 1.0 / POLISH_DELTA; }
                    }
                    S.Rt[2 * lane] = r0;
                    S.Rt[2 * lane + 1] = r1;
                }
                wave_sync();
                riccati_factor(S, N, dt, lane);
                for (int r = 0; r <= POLISH_REFINE; ++r) {
                    rollout_lin(S, N, dt, S.du, S.Xr, lane);
                    if (r == POLISH_REFINE) break;
                    // exact KKT residual of the equality QP -> LQR right-hand side
                    if (live) {
                        double x4[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) x4[a] = S.Xr[5 * k + st4(a)];
                        double q4[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) {
                            double acc = S.qs[4 * k + a];
#pragma unroll
                            for (int c = 0; c < 4; ++c) acc = fma(S.Qs[10 * k + p4(a, c)], x4[c], acc);
                            q4[a] = -acc;
                        }
#pragma unroll
                        for (int j = 0; j < NROW; ++j) {
                            const int o = j * NP + k;
                            const double cl = S.cls[o];
                            if (cl == 0.0) continue;
                            double c[4];
                            row_coef(j, hL, P.L, P.tgap, c);
                            double lam = (cl == 2.0) ? rho : S.tl[o];
                            double r2 = 0.0;
                            if (cl == 1.0) r2 = S.bs[NROW * k + j] - (c[0] * x4[0] + c[1] * x4[1] + c[2] * x4[2] + c[3] * x4[3]);
#pragma unroll
                            for (int a = 0; a < 4; ++a) q4[a] = fma(c[a], lam + r2 / POLISH_DELTA, q4[a]);
                            S.pa4[o] = r2;
                        }
#pragma unroll
                        for (int a = 0; a < 4; ++a) S.qh[4 * k + a] = q4[a];
                        const double du0 = S.du[2 * lane], du1 = S.du[2 * lane + 1];
                        double g0 = -fma(R0, du0, S.rr[2 * lane]);
                        double g1 = -fma(R1, du1, S.rr[2 * lane + 1]);
#pragma unroll
                        for (int j = 0; j < NBOX; ++j) {
                            const int o = j * N + lane;
                            if (S.cls[9 * NP + o] != 1.0) continue;
                            double uu = (j < 2) ? du0 : du1;
                            double r2 = S.bb[4 * lane + j] - bsign(j) * uu;
                            double v = bsign(j) * (S.tlb[o] + r2 / POLISH_DELTA);
                            if (j < 2) g0 += v; else g1 += v;
                            S.pab[o] = r2;
                        }
                        S.gh[2 * lane] = g0;
                        S.gh[2 * lane + 1] = g1;
                    }
                    wave_sync();
                    riccati_solve(S, N, dt, lane);
                    if (live) {
                        double dx4[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) dx4[a] = S.dX[5 * k + st4(a)];
#pragma unroll
                        for (int j = 0; j < NROW; ++j) {
                            const int o = j * NP + k;
                            if (S.cls[o] != 1.0) continue;
                            double c[4];
                            row_coef(j, hL, P.L, P.tgap, c);
                            double cdx = c[0] * dx4[0] + c[1] * dx4[1] + c[2] * dx4[2] + c[3] * dx4[3];
                            S.tl[o] += (S.pa4[o] - cdx) / POLISH_DELTA;
                        }
                        const double dd0 = S.dud[2 * lane], dd1 = S.dud[2 * lane + 1];
#pragma unroll
                        for (int j = 0; j < NBOX; ++j) {
                            const int o = j * N + lane;
                            if (S.cls[9 * NP + o] != 1.0) continue;
                            double duu = (j < 2) ? dd0 : dd1;
                            S.tlb[o] += (S.pab[o] - bsign(j) * duu) / POLISH_DELTA;
                        }
                        S.du[2 * lane] += dd0;
                        S.du[2 * lane + 1] += dd1;
                    }
                    wave_sync();
                }
                // acceptance: KKT consistency; otherwise flip every offending row and retry
                double lmax = 1.0;
                if (live) {
#pragma unroll
                    for (int j = 0; j < NROW; ++j)
                        if (S.cls[j * NP + k] == 1.0) lmax = fmax(lmax, fabs(S.tl[j * NP + k]));
#pragma unroll
                    for (int j = 0; j < NBOX; ++j)
                        if (S.cls[9 * NP + j * N + lane] == 1.0) lmax = fmax(lmax, fabs(S.tlb[j * N + lane]));
                }
                lmax = wave_max(lmax);
                double worst = 0.0, nviol = 0.0, finite = 1.0;
                if (live) {
                    double x4[4];
#pragma unroll
                    for (int a = 0; a < 4; ++a) x4[a] = S.Xr[5 * k + st4(a)];
#pragma unroll
                    for (int j = 0; j < NROW; ++j) {
                        if ((j == 6 || j == 7) && !has_obs) continue;
                        const int o = j * NP + k;
                        double c[4];
                        row_coef(j, hL, P.L, P.tgap, c);
                        const double bj = S.bs[NROW * k + j];
                        const double bsc = 1.0 + fabs(bj);
                        const double r = (c[0] * x4[0] + c[1] * x4[1] + c[2] * x4[2] + c[3] * x4[3]) - bj;
                        const double cl = S.cls[o];
                        double badv = 0.0;
                        if (cl == 1.0) {
                            const double l = S.tl[o];
                            if (l < -1e-9 * lmax) badv = -l / lmax;
                            else if (l > rho * (1.0 + 1e-9)) badv = (l - rho) / lmax;
                            else if (fabs(r) > 1e-7 * bsc) badv = fabs(r) / bsc;
                        } else if (cl == 2.0) {
                            if (r > 1e-9 * bsc) badv = r / bsc;
                            if (r < -1e-6 * bsc) nviol += 1.0;
                        } else if (r < -1e-9 * bsc) badv = -r / bsc;
                        worst = fmax(worst, badv);
                        S.pa5[o] = badv;        // offending-row flag for the flip below
                    }
                    const double du0 = S.du[2 * lane], du1 = S.du[2 * lane + 1];
                    if (!(du0 == du0) || !(du1 == du1)) finite = 0.0;
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) {
                        const int o = j * N + lane;
                        const double bj = S.bb[4 * lane + j];
                        const double bsc = 1.0 + fabs(bj);
                        const double r = bsign(j) * ((j < 2) ? du0 : du1) - bj;
                        double badv = 0.0;
                        if (S.cls[9 * NP + o] == 1.0) {
                            if (S.tlb[o] < -1e-9 * lmax) badv = -S.tlb[o] / lmax;
                            else if (fabs(r) > 1e-7 * bsc) badv = fabs(r) / bsc;
                        } else if (r < -1e-9 * bsc) badv = -r / bsc;
                        worst = fmax(worst, badv);
                        S.pab[o] = badv;
                    }
                }
                worst = wave_max(worst);
                nviol = wave_sum(nviol);
                finite = wave_min(finite);
                if (finite == 0.0) break;
                if (worst == 0.0) {
                    accepted = true;
                    nviol_acc = nviol;
                } else if (live) {
#pragma unroll
                    for (int j = 0; j < NROW; ++j) {
                        if ((j == 6 || j == 7) && !has_obs) continue;
                        const int o = j * NP + k;
                        if (S.pa5[o] > 0.0) {
                            const double cl = S.cls[o];
                            S.cls[o] = (cl == 1.0) ? (S.tl[o] > rho ? 2.0 : 0.0) : 1.0;
                        }
                    }
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) {
                        const int o = j * N + lane;
                        if (S.pab[o] > 0.0) S.cls[9 * NP + o] = (S.cls[9 * NP + o] == 1.0) ? 0.0 : 1.0;
                    }
                }
                wave_sync();
            }
            if (accepted) {
                st_here = nviol_acc > 0.0 ? MPC_INFEASIBLE : MPC_OK;
            } else if (live) {
                S.du[2 * lane] = S.dub[2 * lane];
                S.du[2 * lane + 1] = S.dub[2 * lane + 1];
            }
            wave_sync();
        }
        status = st_here;
        if (live) {
            S.ub[2 * lane] += S.du[2 * lane];
            S.ub[2 * lane + 1] += S.du[2 * lane + 1];
        }
        wave_sync();
    }

    // ---- K5: outputs: U*, u0, predict(x0, U*) ----------------------------------------------
    predict_wave(tab, P, x0, S.ub, S.xb, S.kap, lane);
    if (live && Ug) {
        Ug[(size_t)b * 2 * N + 2 * lane] = S.ub[2 * lane];
        Ug[(size_t)b * 2 * N + 2 * lane + 1] = S.ub[2 * lane + 1];
    }
    if (Xg)
        for (int i = lane; i < 5 * NP; i += WAVE) Xg[(size_t)b * 5 * NP + i] = S.xb[i];
    if (lane == 0) {
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
    p->tol_mu = 1e-12;
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
    k.polish = p->polish;
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
    hipLaunchKernelGGL(mpc_solve_kernel, dim3(B), dim3(WAVE), lds, (hipStream_t)stream, c->tab, kp, B, x0,
                       obs, obs ? n_obs : nullptr, ubar, u0, U, Xpred, status, iters);
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

// cpu_backend.h -- the host (CPU) backend of libmpcqp: mpc_create(..., device = -1, ...).
//
// BASELINE config 1 ("trajectory1.json, N=10, single ego, CPU path") runs the reference's tracker without a
// GPU.  This backend serves that case behind the same C ABI: the same QP(ubar), the same
// solver (crossover first, Mehrotra PDIP on the stage-wise Riccati recursion, active-set polish, the
// Gauss-Newton SQP with warm crossovers and its stopping rules) and the same outputs
// and status codes as the HIP kernels, computed per instance in IEEE double on host threads (batch split
// over std::thread workers, each with its own scratch).  It is product code: it shares the trajectory table
// builder (host_table.h) with the device path and nothing with the test oracle.
//
// Reference functions restated here (medinammartin3/Safe-Autonomous-Driving-MPC):
//   warm start  trajectory_tracking.py:224-246      predict     :87-114 (dynamics :50-67)
//   cost        :116-152 (Gauss-Newton model)        constraints :155-211 (6 row types, min over obstacles)
//   solve       :213-263 (SLSQP replaced)            get_state / get_control  trajectory_loader.py:86-102
//   get_global_pose  trajectory_loader.py:104-116    ObstaclesFSM.update :330-374, run_simulation :377-443
#ifndef MPCQP_CPU_BACKEND_H
#define MPCQP_CPU_BACKEND_H

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "host_table.h"

namespace mpcqp_cpu {

using mpcqp_host::HostTable;

constexpr int kMaxN = MPC_MAX_N;
constexpr int kRows = 9;          // soft rows per stage: lane +-d, +-(d + L/2 o), +-(d + L o), 2 obstacle, v >= 0
constexpr int kBox = 4;           // box rows per control: +u1, -u1, +u2, -u2
constexpr double kTau = 0.995;    // the device constants (mpcqp.hip: TAU, START_SHIFT, POLISH_*, SQP_*)
constexpr double kStartShift = 3.0;
constexpr double kMuCheck = 1e-4;     // interior-point checkpoint (mpcqp.hip: MU_CHECK, CHECK_SEP, CHECK_ROUNDS)
constexpr double kCheckSep = 100.0;
constexpr int kCheckRounds = 2;
// MPC_CHECKPOINT=0 in the environment switches the checkpoint off (A/B; the device kernels read the same flag)
inline bool checkpoint_on() {
    static const bool on = [] {
        const char* e = std::getenv("MPC_CHECKPOINT");
        return !(e && e[0] == '0');
    }();
    return on;
}
constexpr double kDelta = 1e-11;
constexpr int kRefine = 2;
constexpr int kPolishRounds = 6;
constexpr int kXoRounds = 1;
constexpr double kCycleRel = 1e-6;
constexpr int kInfStreak = 5;
constexpr double kBoxSign[kBox] = {1.0, -1.0, 1.0, -1.0};
constexpr int kBoxComp[kBox] = {0, 0, 1, 1};

// ---------------------------------------------------------------------------------------------
// reference signal on the host table (the device lookups' arithmetic: scipy interp1d linear, extrapolate)
// ---------------------------------------------------------------------------------------------
struct Ref {
    const HostTable* h;
    const double *s, *d, *o, *k, *v, *u1, *u2, *gx, *gy, *gpsi;
    explicit Ref(const HostTable& t) : h(&t) {
        const double* b = t.buf.data();
        const size_t T = (size_t)t.T, tu = (size_t)t.tu;
        s = b; d = b + T; o = b + 2 * T; k = b + 3 * T; v = b + 4 * T;
        u1 = b + 5 * T; u2 = u1 + tu;
        gx = b + 5 * T + 2 * tu; gy = gx + T; gpsi = gy + T;
    }
    double lin(const double* y, int i, double x) const {
        const double slope = (y[i] - y[i - 1]) / (s[i] - s[i - 1]);
        return slope * (x - s[i - 1]) + y[i - 1];
    }
    double slope(const double* y, int i) const { return (y[i] - y[i - 1]) / (s[i] - s[i - 1]); }
    // get_state (trajectory_loader.py:86-93); slopes of (d, o, k, v) for the Gauss-Newton model, 0 past s_max
    void state(double x, double out[5], double sl[4] = nullptr) const {
        if (x >= h->smax) {
            for (int j = 0; j < 5; ++j) out[j] = h->last[j];
            if (sl) sl[0] = sl[1] = sl[2] = sl[3] = 0.0;
            return;
        }
        const int i = mpcqp_host::seg_host(*h, h->T, x);
        out[0] = x;
        out[1] = lin(d, i, x);
        out[2] = lin(o, i, x);
        out[3] = lin(k, i, x);
        out[4] = lin(v, i, x);
        if (sl) {
            sl[0] = slope(d, i);
            sl[1] = slope(o, i);
            sl[2] = slope(k, i);
            sl[3] = slope(v, i);
        }
    }
    // get_control (trajectory_loader.py:95-102)
    void control(double x, double out[2]) const {
        if (x >= h->smax) { out[0] = out[1] = 0.0; return; }
        const int i = mpcqp_host::seg_host(*h, h->tu, x);
        out[0] = lin(u1, i, x);
        out[1] = lin(u2, i, x);
    }
    // get_global_pose (trajectory_loader.py:104-116)
    void pose(double x, double dd, double out[3]) const {
        if (x > h->smax) x = h->smax;
        const int j = mpcqp_host::seg_host(*h, h->T, x);
        const double xr = lin(gx, j, x), yr = lin(gy, j, x), psi = lin(gpsi, j, x);
        out[0] = xr - dd * std::sin(psi);
        out[1] = yr + dd * std::cos(psi);
        out[2] = psi;
    }
};

// ---------------------------------------------------------------------------------------------
// one instance: QP(ubar) stage data, interior-point state, Riccati factors, directions
// ---------------------------------------------------------------------------------------------
struct StageQp {
    int N = 0;
    bool obs = false;
    double dt = 0.0, rho = 0.0;
    double Xb[kMaxN + 1][5];                                   // nominal rollout predict(x0, ubar)
    double a12[kMaxN], a14[kMaxN], a20[kMaxN], a23[kMaxN], a24[kMaxN];   // A_k = I + J'_k (J'(0,4) = dt)
    double Q[kMaxN + 1][5][5], q[kMaxN + 1][5];                // Gauss-Newton state cost, stages 1..N
    double R[2], r[kMaxN][2];                                  // control cost
    double C[kRows][5];                                        // soft-row coefficients (C x + xi >= b + s)
    bool on[kRows];
    double b[kMaxN + 1][kRows];
    double bb[kMaxN][kBox];                                    // box rows (hard)
};
struct IpState {
    double du[2 * kMaxN];
    double s[kMaxN + 1][kRows], l[kMaxN + 1][kRows], xi[kMaxN + 1][kRows], nu[kMaxN + 1][kRows];
    double sb[kMaxN][kBox], lb[kMaxN][kBox];
};
struct Factors {
    double K[kMaxN][2][5], Lc[kMaxN][3];                        // feedback, Cholesky factor (l00, l10, l11) of S
    double Qt[kMaxN + 1][5][5], Rt[kMaxN][2];                  // augmented stage Hessians
    double d[kMaxN + 1][kRows], db[kMaxN][kBox];               // barrier diagonals
};
struct Direction {
    double du[2 * kMaxN], dX[kMaxN + 1][5];
    double dl[kMaxN + 1][kRows], ds[kMaxN + 1][kRows], dxi[kMaxN + 1][kRows], dnu[kMaxN + 1][kRows];
    double dlb[kMaxN][kBox], dsb[kMaxN][kBox];
};

static inline double dot5(const double a[5], const double b[5]) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4];
}

class Worker {
public:
    Worker(const Ref& ref, const mpc_params& p) : R_(ref), p_(p) {}

    // TrajectoryTracker.solve (trajectory_tracking.py:213-263) for one instance; returns the status code
    int solve(const double x0[5], const double* obs, int nobs, const double* ubar, double* u0, double* U,
              double* Xpred, int* iters) {
        const int N = p_.N;
        double ub[2 * kMaxN], uo[2 * kMaxN], u2[2 * kMaxN];
        if (ubar) std::memcpy(ub, ubar, sizeof(double) * 2 * N);
        else warm_start(x0, obs, nobs, ub);
        std::memcpy(uo, ub, sizeof(double) * 2 * N);
        std::memcpy(u2, ub, sizeof(double) * 2 * N);
        const int nsqp = p_.sqp_iters < 0 ? 0 : p_.sqp_iters;
        int status = MPC_OK, total = 0, ninf = 0;
        bool conv = false;
        for (int it = 0; it < nsqp; ++it) {
            build(x0, obs, nobs, ub);
            int ni = 0;
            status = pdip(ni, it > 0);
            total += ni;
            double step = 0.0, back2 = 0.0;
            for (int i = 0; i < 2 * N; ++i) {
                uo[i] = ub[i] + S_.du[i];
                step = std::max(step, std::fabs(S_.du[i]));
                back2 = std::max(back2, std::fabs(uo[i] - u2[i]));
            }
            std::memcpy(u2, ub, sizeof(double) * 2 * N);
            std::memcpy(ub, uo, sizeof(double) * 2 * N);
            ninf = status == MPC_INFEASIBLE ? ninf + 1 : 0;
            if (nsqp > 1) {
                if (step <= p_.sqp_tol) { conv = true; break; }                  // re-linearisation converged
                if (p_.sqp_tol > 0.0 && ((it >= 2 && back2 <= kCycleRel * step) || ninf >= kInfStreak)) break;
            }
        }
        if (U) std::memcpy(U, uo, sizeof(double) * 2 * N);
        if (u0) { u0[0] = uo[0]; u0[1] = uo[1]; }
        if (Xpred) predict(x0, uo, reinterpret_cast<double(*)[5]>(Xpred));    // :261
        if (iters) *iters = total;
        if (nsqp > 1 && p_.sqp_tol > 0.0 && !conv) status |= MPC_SQP_UNCONVERGED;
        return status;
    }

    // warm start ubar (trajectory_tracking.py:224-246): reference controls along s advanced at the current
    // speed; a sticky brake once an obstacle is within brake_distance
    void warm_start(const double x0[5], const double* obs, int nobs, double* ub) const {
        double s = x0[0];
        bool brake = false;
        for (int j = 0; j < p_.N; ++j) {
            for (int i = 0; i < nobs; ++i)
                if ((obs[2 * i] - s) < p_.brake_distance) brake = true;
            double ur[2];
            R_.control(s, ur);
            ub[2 * j] = ur[0];
            ub[2 * j + 1] = brake ? p_.brake_accel : ur[1];
            s += x0[4] * p_.dt;
        }
    }

    // explicit-Euler rollout (trajectory_tracking.py:87-114), k_ref looked up at the predicted s
    void predict(const double x0[5], const double* U, double (*X)[5]) const {
        const double dt = p_.dt;
        double x[5];
        std::memcpy(x, x0, sizeof(x));
        std::memcpy(X[0], x0, sizeof(x));
        for (int k = 0; k < p_.N; ++k) {
            double st[5];
            R_.state(x[0], st);
            const double xd[5] = {x[4], x[4] * x[2], x[4] * (x[3] - st[3]), U[2 * k], U[2 * k + 1]};
            for (int j = 0; j < 5; ++j) x[j] = x[j] + dt * xd[j];
            std::memcpy(X[k + 1], x, sizeof(x));
        }
    }

private:
    const Ref& R_;
    const mpc_params& p_;
    StageQp q_;
    IpState S_, Z_, T_, C_;
    Factors F_;
    Direction D_, Da_;
    unsigned char cls_[kMaxN + 1][kRows], clb_[kMaxN][kBox];      // 0 inactive, 1 active, 2 violated
    unsigned char flip_[kMaxN + 1][kRows], flipb_[kMaxN][kBox];
    unsigned char last_cls_[kMaxN + 1][kRows], last_clb_[kMaxN][kBox];   // the SQP's warm crossover
    double xo_du_[2 * kMaxN];   // du of the last cold crossover solve: the unconstrained optimum (interior-point start)

    // ---- QP(ubar): Gauss-Newton model of cost/constraints around the nominal rollout
    void build(const double x0[5], const double* obs, int nobs, const double* ub) {
        StageQp& Q = q_;
        const int N = p_.N;
        const double dt = p_.dt;
        const bool gn = p_.linearization != 0;
        Q.N = N;
        Q.dt = dt;
        Q.rho = p_.elastic_rho;
        Q.obs = nobs > 0;
        predict(x0, ub, Q.Xb);
        for (int k = 0; k < N; ++k) {
            const double* x = Q.Xb[k];
            double st[5], sl[4];
            R_.state(x[0], st, sl);
            const double dk = gn ? sl[2] : 0.0;
            Q.a12[k] = dt * x[4];
            Q.a14[k] = dt * x[2];
            Q.a20[k] = dt * (-x[4] * dk);
            Q.a23[k] = dt * x[4];
            Q.a24[k] = dt * (x[3] - st[3]);
        }
        const double w[3] = {p_.w_d, p_.w_o, p_.w_v};
        const int comp[3] = {1, 2, 4};
        std::memset(Q.Q, 0, sizeof(Q.Q));
        std::memset(Q.q, 0, sizeof(Q.q));
        for (int k = 1; k <= N; ++k) {
            const double* x = Q.Xb[k];
            double st[5], sl[4];
            R_.state(x[0], st, sl);
            const double ref[3] = {st[1], st[2], st[4]};
            const double dref[3] = {gn ? sl[0] : 0.0, gn ? sl[1] : 0.0, gn ? sl[3] : 0.0};
            for (int j = 0; j < 3; ++j) {
                // residual x_c - ref_c(s): gradient e_c - ref_c'(s) e_s
                double m[5] = {0, 0, 0, 0, 0};
                m[comp[j]] = 1.0;
                m[0] = -dref[j];
                const double r0 = x[comp[j]] - ref[j];
                for (int a = 0; a < 5; ++a) {
                    Q.q[k][a] += 2.0 * w[j] * r0 * m[a];
                    for (int c = 0; c < 5; ++c) Q.Q[k][a][c] += 2.0 * w[j] * m[a] * m[c];
                }
            }
        }
        Q.R[0] = 2.0 * p_.w_u1;
        Q.R[1] = 2.0 * p_.w_u2;
        for (int k = 0; k < N; ++k) {
            Q.r[k][0] = Q.R[0] * ub[2 * k];
            Q.r[k][1] = Q.R[1] * ub[2 * k + 1];
        }
        const double L = p_.wheelbase, h = p_.wheelbase / 2.0, tg = p_.max_time_2_obs;
        const double sl = p_.lane_width / 2.0 - p_.vehicle_radius - p_.safe_lane_margin;   // :169
        const double C[kRows][5] = {{0, 1, 0, 0, 0}, {0, -1, 0, 0, 0}, {0, 1, h, 0, 0},   {0, -1, -h, 0, 0},
                                    {0, 1, L, 0, 0}, {0, -1, -L, 0, 0}, {-1, 0, 0, 0, 0}, {-1, 0, 0, 0, -tg},
                                    {0, 0, 0, 0, 1}};
        std::memcpy(Q.C, C, sizeof(C));
        for (int j = 0; j < kRows; ++j) Q.on[j] = (j != 6 && j != 7) || Q.obs;
        for (int k = 1; k <= N; ++k) {
            const double* x = Q.Xb[k];
            const double pv0 = x[1], pv1 = x[1] + h * x[2], pv2 = x[1] + L * x[2];
            Q.b[k][0] = -sl - pv0;
            Q.b[k][1] = -(sl - pv0);
            Q.b[k][2] = -sl - pv1;
            Q.b[k][3] = -(sl - pv1);
            Q.b[k][4] = -sl - pv2;
            Q.b[k][5] = -(sl - pv2);
            Q.b[k][6] = Q.b[k][7] = 0.0;
            if (Q.obs) {
                // the obstacle rows of :194-204 for every obstacle collapse to the nearest predicted one
                double shat = INFINITY;
                for (int i = 0; i < nobs; ++i) shat = std::min(shat, obs[2 * i] + obs[2 * i + 1] * (k * dt));
                Q.b[k][6] = -(shat - p_.obstacle_safety_distance - x[0]);
                Q.b[k][7] = -(shat - x[0] - tg * x[4]);
            }
            Q.b[k][8] = -x[4];
        }
        for (int k = 0; k < N; ++k) {
            Q.bb[k][0] = p_.u_min[0] - ub[2 * k];
            Q.bb[k][1] = -(p_.u_max[0] - ub[2 * k]);
            Q.bb[k][2] = p_.u_min[1] - ub[2 * k + 1];
            Q.bb[k][3] = -(p_.u_max[1] - ub[2 * k + 1]);
        }
    }

    // ---- linear model pieces: x_{k+1} = A_k x_k + B u_k, B = dt e3 e1' + dt e4 e2'
    void apply_A(int k, const double x[5], double y[5]) const {
        const StageQp& Q = q_;
        y[0] = x[0] + Q.dt * x[4];
        y[1] = x[1] + Q.a12[k] * x[2] + Q.a14[k] * x[4];
        y[2] = x[2] + Q.a20[k] * x[0] + Q.a23[k] * x[3] + Q.a24[k] * x[4];
        y[3] = x[3];
        y[4] = x[4];
    }
    void apply_AT(int k, const double m[5], double y[5]) const {
        const StageQp& Q = q_;
        y[0] = m[0] + Q.a20[k] * m[2];
        y[1] = m[1];
        y[2] = m[2] + Q.a12[k] * m[1];
        y[3] = m[3] + Q.a23[k] * m[2];
        y[4] = m[4] + Q.dt * m[0] + Q.a14[k] * m[1] + Q.a24[k] * m[2];
    }
    void rollout(const double* du, double (*X)[5]) const {
        std::memset(X[0], 0, sizeof(double) * 5);
        for (int k = 0; k < q_.N; ++k) {
            apply_A(k, X[k], X[k + 1]);
            X[k + 1][3] += q_.dt * du[2 * k];
            X[k + 1][4] += q_.dt * du[2 * k + 1];
        }
    }
    // g_t = z_t + B' mu_{t+1} with mu_N = y_N, mu_k = A_k' mu_{k+1} + y_k: the dual residual in control space
    void adjoint(const double (*y)[5], const double (*z)[2], double* g) const {
        double mu[5] = {0, 0, 0, 0, 0};
        for (int k = q_.N; k >= 1; --k) {
            for (int a = 0; a < 5; ++a) mu[a] += y[k][a];
            g[2 * (k - 1)] = z[k - 1][0] + q_.dt * mu[3];
            g[2 * (k - 1) + 1] = z[k - 1][1] + q_.dt * mu[4];
            double m2[5];
            apply_AT(k - 1, mu, m2);
            std::memcpy(mu, m2, sizeof(mu));
        }
    }

    // ---- Riccati factorisation of  min sum 0.5 x'Qt x + 0.5 u'Rt u  (Cholesky form of S)
    void riccati_factor() {
        const StageQp& Q = q_;
        Factors& F = F_;
        const int N = Q.N;
        const double dt = Q.dt;
        double P[5][5];
        std::memcpy(P, F.Qt[N], sizeof(P));
        for (int k = N - 1; k >= 0; --k) {
            double M[5][5];                                    // P A_k
            for (int i = 0; i < 5; ++i) {
                M[i][0] = P[i][0] + P[i][2] * Q.a20[k];
                M[i][1] = P[i][1];
                M[i][2] = P[i][2] + P[i][1] * Q.a12[k];
                M[i][3] = P[i][3] + P[i][2] * Q.a23[k];
                M[i][4] = P[i][4] + P[i][0] * dt + P[i][1] * Q.a14[k] + P[i][2] * Q.a24[k];
            }
            double s00 = F.Rt[k][0] + dt * dt * P[3][3];
            const double s01 = dt * dt * P[3][4];
            const double s11 = F.Rt[k][1] + dt * dt * P[4][4];
            if (!(s00 > 0.0)) s00 = 1e-300 + std::fabs(s00);
            const double l00 = std::sqrt(s00), l10 = s01 / l00;
            double r11 = s11 - l10 * l10;
            if (!(r11 > 1e-14 * s11)) r11 = 1e-14 * std::fabs(s11) + 1e-300;
            const double l11 = std::sqrt(r11);
            F.Lc[k][0] = l00;
            F.Lc[k][1] = l10;
            F.Lc[k][2] = l11;
            double W0[5], W1[5];
            for (int j = 0; j < 5; ++j) {
                W0[j] = dt * M[3][j] / l00;
                W1[j] = (dt * M[4][j] - l10 * W0[j]) / l11;
                const double z1 = W1[j] / l11;
                F.K[k][1][j] = -z1;
                F.K[k][0][j] = -(W0[j] - l10 * z1) / l00;
            }
            if (k == 0) break;
            double Pn[5][5];
            for (int j = 0; j < 5; ++j) {
                double col[5] = {M[0][j], M[1][j], M[2][j], M[3][j], M[4][j]}, at[5];
                apply_AT(k, col, at);
                for (int i = 0; i < 5; ++i) Pn[i][j] = at[i];
            }
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) Pn[i][j] += F.Qt[k][i][j] - (W0[i] * W0[j] + W1[i] * W1[j]);
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) P[i][j] = 0.5 * (Pn[i][j] + Pn[j][i]);
        }
    }
    // LQR solve for the linear terms -qh (states 1..N) and -gh (controls); writes D.du, D.dX (x_0 = 0)
    void riccati_solve(const double (*qh)[5], const double (*gh)[2], Direction& D) const {
        const StageQp& Q = q_;
        const Factors& F = F_;
        const int N = Q.N;
        const double dt = Q.dt;
        double p[5], kk[kMaxN][2];
        std::memcpy(p, qh[N], sizeof(p));
        for (int k = N - 1; k >= 0; --k) {
            const double h0 = gh[k][0] + dt * p[3], h1 = gh[k][1] + dt * p[4];
            const double* Lc = F.Lc[k];
            const double w0 = h0 / Lc[0], w1 = (h1 - Lc[1] * w0) / Lc[2];
            kk[k][1] = w1 / Lc[2];
            kk[k][0] = (w0 - Lc[1] * kk[k][1]) / Lc[0];
            if (k >= 1) {
                double pa[5];
                apply_AT(k, p, pa);
                for (int a = 0; a < 5; ++a) p[a] = qh[k][a] + pa[a] + F.K[k][0][a] * h0 + F.K[k][1][a] * h1;
            }
        }
        std::memset(D.dX[0], 0, sizeof(double) * 5);
        for (int k = 0; k < N; ++k) {
            const double* x = D.dX[k];
            const double v0 = kk[k][0] + dot5(F.K[k][0], x), v1 = kk[k][1] + dot5(F.K[k][1], x);
            D.du[2 * k] = v0;
            D.du[2 * k + 1] = v1;
            apply_A(k, x, D.dX[k + 1]);
            D.dX[k + 1][3] += dt * v0;
            D.dX[k + 1][4] += dt * v1;
        }
    }

    // barrier diagonals, augmented Hessians and the factorisation at the current iterate
    void factor() {
        const StageQp& Q = q_;
        for (int k = 1; k <= Q.N; ++k) {
            std::memcpy(F_.Qt[k], Q.Q[k], sizeof(F_.Qt[k]));
            for (int j = 0; j < kRows; ++j) {
                if (!Q.on[j]) continue;
                const double d = S_.s[k][j] / S_.l[k][j] + S_.xi[k][j] / S_.nu[k][j];
                F_.d[k][j] = d;
                const double w = 1.0 / d;
                for (int a = 0; a < 5; ++a)
                    for (int c = 0; c < 5; ++c) F_.Qt[k][a][c] += w * Q.C[j][a] * Q.C[j][c];
            }
        }
        for (int t = 0; t < Q.N; ++t) {
            F_.Rt[t][0] = Q.R[0];
            F_.Rt[t][1] = Q.R[1];
            for (int j = 0; j < kBox; ++j) {
                const double d = S_.sb[t][j] / S_.lb[t][j];
                F_.db[t][j] = d;
                F_.Rt[t][kBoxComp[j]] += 1.0 / d;
            }
        }
        riccati_factor();
    }

    // Newton direction for complementarity targets r4 (s lam), r5 (xi nu), r4b (box), residuals rp/rpb/rx and
    // the dual residual pieces y (stages) / z (controls), eliminated row-wise onto the Riccati system
    void newton(const double (*rp)[kRows], const double (*rpb)[kBox], const double (*rx)[kRows],
                const double (*y)[5], const double (*z)[2], const double (*r4)[kRows], const double (*r5)[kRows],
                const double (*r4b)[kBox], Direction& D) {
        const StageQp& Q = q_;
        const int N = Q.N;
        double qh[kMaxN + 1][5], gh[kMaxN][2], rh[kMaxN + 1][kRows], rhb[kMaxN][kBox];
        for (int k = 1; k <= N; ++k) {
            for (int a = 0; a < 5; ++a) qh[k][a] = -y[k][a];
            for (int j = 0; j < kRows; ++j) {
                if (!Q.on[j]) continue;
                const double v = -rp[k][j] - r4[k][j] / S_.l[k][j] + (r5[k][j] + S_.xi[k][j] * rx[k][j]) / S_.nu[k][j];
                rh[k][j] = v;
                const double w = v / F_.d[k][j];
                for (int a = 0; a < 5; ++a) qh[k][a] += Q.C[j][a] * w;
            }
        }
        for (int t = 0; t < N; ++t) {
            gh[t][0] = -z[t][0];
            gh[t][1] = -z[t][1];
            for (int j = 0; j < kBox; ++j) {
                const double v = -rpb[t][j] - r4b[t][j] / S_.lb[t][j];
                rhb[t][j] = v;
                gh[t][kBoxComp[j]] += kBoxSign[j] * v / F_.db[t][j];
            }
        }
        riccati_solve(qh, gh, D);
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < kRows; ++j) {
                if (!Q.on[j]) continue;
                const double dl = (rh[k][j] - dot5(Q.C[j], D.dX[k])) / F_.d[k][j];
                D.dl[k][j] = dl;
                D.ds[k][j] = -(r4[k][j] + S_.s[k][j] * dl) / S_.l[k][j];
                const double dn = rx[k][j] - dl;
                D.dnu[k][j] = dn;
                D.dxi[k][j] = -(r5[k][j] + S_.xi[k][j] * dn) / S_.nu[k][j];
            }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < kBox; ++j) {
                const double dl = (rhb[t][j] - kBoxSign[j] * D.du[2 * t + kBoxComp[j]]) / F_.db[t][j];
                D.dlb[t][j] = dl;
                D.dsb[t][j] = -(r4b[t][j] + S_.sb[t][j] * dl) / S_.lb[t][j];
            }
    }

    // largest step in (0, 1] keeping every slack and multiplier positive
    double max_step(const Direction& D) const {
        double a = 1.0;
        auto ratio = [&a](double v, double dv) { if (dv < 0.0 && -v / dv < a) a = -v / dv; };
        for (int k = 1; k <= q_.N; ++k)
            for (int j = 0; j < kRows; ++j) {
                if (!q_.on[j]) continue;
                ratio(S_.s[k][j], D.ds[k][j]);
                ratio(S_.l[k][j], D.dl[k][j]);
                ratio(S_.xi[k][j], D.dxi[k][j]);
                ratio(S_.nu[k][j], D.dnu[k][j]);
            }
        for (int t = 0; t < q_.N; ++t)
            for (int j = 0; j < kBox; ++j) {
                ratio(S_.sb[t][j], D.dsb[t][j]);
                ratio(S_.lb[t][j], D.dlb[t][j]);
            }
        return a;
    }
    // total complementarity after a step of length a along D
    double comp_after(const Direction& D, double a) const {
        double c = 0.0;
        for (int k = 1; k <= q_.N; ++k)
            for (int j = 0; j < kRows; ++j) {
                if (!q_.on[j]) continue;
                c += (S_.s[k][j] + a * D.ds[k][j]) * (S_.l[k][j] + a * D.dl[k][j]) +
                     (S_.xi[k][j] + a * D.dxi[k][j]) * (S_.nu[k][j] + a * D.dnu[k][j]);
            }
        for (int t = 0; t < q_.N; ++t)
            for (int j = 0; j < kBox; ++j) c += (S_.sb[t][j] + a * D.dsb[t][j]) * (S_.lb[t][j] + a * D.dlb[t][j]);
        return c;
    }

    // ---- active-set solve (crossover / polish).  Rows classified active (equality, penalty 1/delta plus
    // iterative refinement on the exact KKT residual), violated (multiplier fixed at rho) or inactive; the
    // result is accepted when KKT-consistent, otherwise every offending row changes class and the round
    // repeats.  from: 0 = classify the iterate X, 1 = all inactive (crossover), 2 = the previous QP's final
    // classification (the SQP's warm crossover).  Returns true when accepted (X.du replaced).
    bool active_set(IpState& X, int from, int rounds, bool& infeasible) {
        const StageQp& Q = q_;
        const int N = Q.N;
        const double rho = Q.rho;
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < kRows; ++j) {
                unsigned char c = 0;
                if (Q.on[j] && from != 1) {
                    if (from == 2) c = last_cls_[k][j];
                    else if (X.xi[k][j] > X.nu[k][j]) c = 2;
                    else if (X.l[k][j] > X.s[k][j]) c = 1;
                }
                cls_[k][j] = c;
            }
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < kBox; ++j)
                clb_[t][j] = from == 1 ? 0 : (from == 2 ? last_clb_[t][j] : (X.lb[t][j] > X.sb[t][j]));
        bool accepted = false;
        double Xs[kMaxN + 1][5];
        for (int round = 0; round < rounds && !accepted; ++round) {
            IpState& W = T_;
            std::memcpy(&W, &X, sizeof(W));
            for (int k = 1; k <= N; ++k) {
                std::memcpy(F_.Qt[k], Q.Q[k], sizeof(F_.Qt[k]));
                for (int j = 0; j < kRows; ++j)
                    if (Q.on[j] && cls_[k][j] == 1) {
                        for (int a = 0; a < 5; ++a)
                            for (int c = 0; c < 5; ++c) F_.Qt[k][a][c] += Q.C[j][a] * Q.C[j][c] / kDelta;
                        if (!(X.l[k][j] > 0.0)) W.l[k][j] = 0.0;
                    }
            }
            for (int t = 0; t < N; ++t) {
                F_.Rt[t][0] = Q.R[0];
                F_.Rt[t][1] = Q.R[1];
                for (int j = 0; j < kBox; ++j)
                    if (clb_[t][j]) F_.Rt[t][kBoxComp[j]] += 1.0 / kDelta;
            }
            riccati_factor();
            // from the all-inactive classification (the crossover) the first solve is the unconstrained LQR's exact
            // optimum: one solve, nothing to refine (oracle polish_from, kernel MODE_XO)
            const int nref = from == 1 ? 1 : kRefine;
            for (int r = 0; r <= nref; ++r) {
                rollout(W.du, Xs);
                double qh[kMaxN + 1][5], gh[kMaxN][2], r2[kMaxN + 1][kRows], r2b[kMaxN][kBox];
                for (int k = 1; k <= N; ++k) {
                    for (int a = 0; a < 5; ++a) {
                        double acc = Q.q[k][a];
                        for (int c = 0; c < 5; ++c) acc += Q.Q[k][a][c] * Xs[k][c];
                        qh[k][a] = -acc;
                    }
                    for (int j = 0; j < kRows; ++j) {
                        if (!Q.on[j] || cls_[k][j] == 0) continue;
                        const double lam = cls_[k][j] == 2 ? rho : W.l[k][j];
                        for (int a = 0; a < 5; ++a) qh[k][a] += lam * Q.C[j][a];
                        if (cls_[k][j] == 1) {
                            r2[k][j] = Q.b[k][j] - dot5(Q.C[j], Xs[k]);
                            for (int a = 0; a < 5; ++a) qh[k][a] += Q.C[j][a] * r2[k][j] / kDelta;
                        }
                    }
                }
                for (int t = 0; t < N; ++t) {
                    gh[t][0] = -(Q.R[0] * W.du[2 * t] + Q.r[t][0]);
                    gh[t][1] = -(Q.R[1] * W.du[2 * t + 1] + Q.r[t][1]);
                    for (int j = 0; j < kBox; ++j) {
                        if (!clb_[t][j]) continue;
                        const double sg = kBoxSign[j];
                        gh[t][kBoxComp[j]] += sg * W.lb[t][j];
                        r2b[t][j] = Q.bb[t][j] - sg * W.du[2 * t + kBoxComp[j]];
                        gh[t][kBoxComp[j]] += sg * r2b[t][j] / kDelta;
                    }
                }
                if (r == nref) break;
                riccati_solve(qh, gh, D_);
                for (int i = 0; i < 2 * N; ++i) W.du[i] += D_.du[i];
                for (int k = 1; k <= N; ++k)
                    for (int j = 0; j < kRows; ++j)
                        if (Q.on[j] && cls_[k][j] == 1) W.l[k][j] += (r2[k][j] - dot5(Q.C[j], D_.dX[k])) / kDelta;
                for (int t = 0; t < N; ++t)
                    for (int j = 0; j < kBox; ++j)
                        if (clb_[t][j]) W.lb[t][j] += (r2b[t][j] - kBoxSign[j] * D_.du[2 * t + kBoxComp[j]]) / kDelta;
            }
            // the crossover's solve is the unconstrained optimum of QP(ubar): kept for the interior-point start
            if (from == 1 && round == 0) std::memcpy(xo_du_, W.du, sizeof(double) * 2 * N);
            // KKT consistency of the solved point
            double lmax = 1.0;
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j)
                    if (Q.on[j] && cls_[k][j] == 1) lmax = std::max(lmax, std::fabs(W.l[k][j]));
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < kBox; ++j)
                    if (clb_[t][j]) lmax = std::max(lmax, std::fabs(W.lb[t][j]));
            int nviol = 0;
            bool offending = false;
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j) {
                    flip_[k][j] = 0;
                    if (!Q.on[j]) continue;
                    const double bsc = 1.0 + std::fabs(Q.b[k][j]);
                    const double r = dot5(Q.C[j], Xs[k]) - Q.b[k][j];
                    bool bad = false;
                    if (cls_[k][j] == 1) {
                        const double l = W.l[k][j];
                        bad = l < -1e-9 * lmax || l > rho * (1.0 + 1e-9) || std::fabs(r) > 1e-7 * bsc;
                    } else if (cls_[k][j] == 2) {
                        bad = r > 1e-9 * bsc;
                        if (r < -1e-6 * bsc) ++nviol;
                    } else {
                        bad = r < -1e-9 * bsc;
                    }
                    flip_[k][j] = bad;
                    offending = offending || bad;
                }
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < kBox; ++j) {
                    const double bsc = 1.0 + std::fabs(Q.bb[t][j]);
                    const double r = kBoxSign[j] * W.du[2 * t + kBoxComp[j]] - Q.bb[t][j];
                    const bool bad = clb_[t][j] ? (W.lb[t][j] < -1e-9 * lmax || std::fabs(r) > 1e-7 * bsc)
                                                : r < -1e-9 * bsc;
                    flipb_[t][j] = bad;
                    offending = offending || bad;
                }
            bool finite = true;
            for (int i = 0; i < 2 * N; ++i) finite = finite && W.du[i] == W.du[i];
            if (!finite) break;
            if (!offending) {
                std::memcpy(X.du, W.du, sizeof(double) * 2 * N);
                infeasible = nviol > 0;
                accepted = true;
                break;
            }
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j)
                    if (flip_[k][j]) cls_[k][j] = cls_[k][j] == 1 ? (W.l[k][j] > rho ? 2 : 0) : 1;
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < kBox; ++j)
                    if (flipb_[t][j]) clb_[t][j] = !clb_[t][j];
        }
        std::memcpy(last_cls_, cls_, sizeof(last_cls_));
        std::memcpy(last_clb_, clb_, sizeof(last_clb_));
        return accepted;
    }

    // ---- crossover, then (if it does not certify) Mehrotra predictor-corrector PDIP and the polish
    int pdip(int& iters, bool warm) {
        const StageQp& Q = q_;
        const int N = Q.N;
        const double rho = Q.rho;
        std::memset(&S_, 0, sizeof(S_));
        iters = 0;
        if (p_.polish >= 2) {
            std::memset(&Z_, 0, sizeof(Z_));
            bool inf = false;
            if (active_set(Z_, warm ? 2 : 1, kXoRounds, inf)) {
                std::memcpy(S_.du, Z_.du, sizeof(double) * 2 * N);
                return inf ? MPC_INFEASIBLE : MPC_OK;
            }
        }
        int nsoft = 0;
        for (int j = 0; j < kRows; ++j) nsoft += Q.on[j];
        const double Mtot = (double)(2 * nsoft * N + kBox * N);
        // start centred at the unconstrained optimum of QP(ubar) (one factorisation and solve without rows), or
        // at du = 0 when the soft rows are less violated there:
        // slack max(r, 0) + shift, elastic slack max(-r, 0) + shift for the row value r there, the multiplier
        // pair on the pair's central path with lambda + nu = rho; box rows at the mean row complementarity
        double X[kMaxN + 1][5];
        if (p_.polish >= 2 && !warm) {
            // the crossover solved exactly this system (all rows inactive): its solution is the start's
            std::memcpy(S_.du, xo_du_, sizeof(double) * 2 * N);
        } else {
            double qh[kMaxN + 1][5], gh[kMaxN][2];
            for (int k = 1; k <= N; ++k) {
                std::memcpy(F_.Qt[k], Q.Q[k], sizeof(F_.Qt[k]));
                for (int a = 0; a < 5; ++a) qh[k][a] = -Q.q[k][a];
            }
            for (int t = 0; t < N; ++t) {
                F_.Rt[t][0] = Q.R[0];
                F_.Rt[t][1] = Q.R[1];
                gh[t][0] = -Q.r[t][0];
                gh[t][1] = -Q.r[t][1];
            }
            riccati_factor();
            riccati_solve(qh, gh, D_);
            std::memcpy(S_.du, D_.du, sizeof(double) * 2 * N);
        }
        rollout(S_.du, X);
        {
            // primal point: the unconstrained optimum, or du = 0 (ubar) when the soft rows are less violated there
            double v_unc = 0.0, v_bar = 0.0;
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j) {
                    if (!Q.on[j]) continue;
                    const double r = dot5(Q.C[j], X[k]) - Q.b[k][j];
                    v_unc += r < 0.0 ? -r : 0.0;
                    v_bar += Q.b[k][j] > 0.0 ? Q.b[k][j] : 0.0;
                }
            if (v_bar < v_unc) {
                std::memset(S_.du, 0, sizeof(double) * 2 * N);
                rollout(S_.du, X);
            }
        }
        double bscale = 0.0, rowc = 0.0;
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < kRows; ++j) {
                if (!Q.on[j]) continue;
                const double r = dot5(Q.C[j], X[k]) - Q.b[k][j];
                const double sv = (r > 0.0 ? r : 0.0) + kStartShift, xi = (r < 0.0 ? -r : 0.0) + kStartShift;
                S_.s[k][j] = sv;
                S_.xi[k][j] = xi;
                S_.l[k][j] = rho * xi / (sv + xi);
                S_.nu[k][j] = rho * sv / (sv + xi);
                rowc += sv * S_.l[k][j];
                bscale = std::max(bscale, std::fabs(Q.b[k][j]));
            }
        const double mrow = rowc / (double)(nsoft * N);
        for (int t = 0; t < N; ++t)
            for (int j = 0; j < kBox; ++j) {
                const double v = kBoxSign[j] * S_.du[2 * t + kBoxComp[j]] - Q.bb[t][j];
                S_.sb[t][j] = v > 1.0 ? v : 1.0;
                S_.lb[t][j] = mrow / S_.sb[t][j];
                bscale = std::max(bscale, std::fabs(Q.bb[t][j]));
            }
        double y[kMaxN + 1][5], yc[kMaxN + 1][5], ya[kMaxN + 1][5];
        double z[kMaxN][2], zc[kMaxN][2], za[kMaxN][2];
        double rp[kMaxN + 1][kRows], rx[kMaxN + 1][kRows], rpb[kMaxN][kBox];
        double r4[kMaxN + 1][kRows], r5[kMaxN + 1][kRows], r4b[kMaxN][kBox];
        int status = MPC_MAX_ITER, it = 0, stall = 0;
        bool checked = false;
        for (it = 0; it < p_.max_iter; ++it) {
            rollout(S_.du, X);
            double rpmax = 0.0, rxmax = 0.0, comp = 0.0;
            for (int k = 1; k <= N; ++k) {
                for (int a = 0; a < 5; ++a) {
                    double acc = Q.q[k][a];
                    for (int c = 0; c < 5; ++c) acc += Q.Q[k][a][c] * X[k][c];
                    yc[k][a] = acc;
                    ya[k][a] = 0.0;
                }
                for (int j = 0; j < kRows; ++j) {
                    if (!Q.on[j]) continue;
                    for (int a = 0; a < 5; ++a) ya[k][a] -= S_.l[k][j] * Q.C[j][a];
                    rp[k][j] = dot5(Q.C[j], X[k]) + S_.xi[k][j] - S_.s[k][j] - Q.b[k][j];
                    rx[k][j] = rho - S_.l[k][j] - S_.nu[k][j];
                    rpmax = std::max(rpmax, std::fabs(rp[k][j]));
                    rxmax = std::max(rxmax, std::fabs(rx[k][j]));
                    comp += S_.s[k][j] * S_.l[k][j] + S_.xi[k][j] * S_.nu[k][j];
                }
                for (int a = 0; a < 5; ++a) y[k][a] = yc[k][a] + ya[k][a];
            }
            for (int t = 0; t < N; ++t) {
                zc[t][0] = Q.R[0] * S_.du[2 * t] + Q.r[t][0];
                zc[t][1] = Q.R[1] * S_.du[2 * t + 1] + Q.r[t][1];
                za[t][0] = -S_.lb[t][0] + S_.lb[t][1];
                za[t][1] = -S_.lb[t][2] + S_.lb[t][3];
                z[t][0] = zc[t][0] + za[t][0];
                z[t][1] = zc[t][1] + za[t][1];
                for (int j = 0; j < kBox; ++j) {
                    rpb[t][j] = kBoxSign[j] * S_.du[2 * t + kBoxComp[j]] - S_.sb[t][j] - Q.bb[t][j];
                    rpmax = std::max(rpmax, std::fabs(rpb[t][j]));
                    comp += S_.sb[t][j] * S_.lb[t][j];
                }
            }
            const double mu = comp / Mtot;
            if (!(mu == mu)) { status = MPC_NUMERICAL; break; }
            if (mu <= p_.tol_mu && rpmax <= 10.0 * p_.tol * (1.0 + bscale) && rxmax <= p_.tol * rho) {
                // converged: the dual residual (an adjoint recursion, once per solve) carries O(eps/mu)
                // multiplier noise and is required to 1e4 tol; the polish then makes the active set exact
                double gd[2 * kMaxN], gc[2 * kMaxN], ga[2 * kMaxN];
                adjoint(y, z, gd);
                adjoint(yc, zc, gc);
                adjoint(ya, za, ga);
                double rdmax = 0.0, sd = 0.0;
                for (int i = 0; i < 2 * N; ++i) {
                    rdmax = std::max(rdmax, std::fabs(gd[i]));
                    sd = std::max(sd, std::max(std::fabs(gc[i]), std::fabs(ga[i])));
                }
                status = rdmax <= 1e4 * p_.tol * (1.0 + sd) ? MPC_OK : MPC_NUMERICAL;
                break;
            }
            // checkpoint (once per QP): no near-tie between any row's slack and multiplier at mu <= kMuCheck ->
            // kCheckRounds polish rounds from the iterate's classification; certified = the exact optimum, else
            // the interior point continues from the unchanged iterate
            if (p_.polish && !checked && mu <= kMuCheck && checkpoint_on()) {
                bool tie = false;
                for (int k = 1; k <= N && !tie; ++k)
                    for (int j = 0; j < kRows; ++j) {
                        if (!Q.on[j]) continue;
                        const double s = S_.s[k][j], l = S_.l[k][j], x = S_.xi[k][j], n = S_.nu[k][j];
                        if (!(s > kCheckSep * l || l > kCheckSep * s) || !(x > kCheckSep * n || n > kCheckSep * x)) tie = true;
                    }
                for (int t = 0; t < N && !tie; ++t)
                    for (int j = 0; j < kBox; ++j)
                        if (!(S_.sb[t][j] > kCheckSep * S_.lb[t][j] || S_.lb[t][j] > kCheckSep * S_.sb[t][j])) tie = true;
                if (!tie) {
                    checked = true;
                    std::memcpy(&C_, &S_, sizeof(C_));
                    bool inf = false;
                    if (active_set(C_, 0, kCheckRounds, inf)) {
                        std::memcpy(S_.du, C_.du, sizeof(double) * 2 * N);
                        iters = it;
                        return inf ? MPC_INFEASIBLE : MPC_OK;
                    }
                }
            }
            factor();
            // predictor (affine scaling)
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j) {
                    r4[k][j] = S_.s[k][j] * S_.l[k][j];
                    r5[k][j] = S_.xi[k][j] * S_.nu[k][j];
                }
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < kBox; ++j) r4b[t][j] = S_.sb[t][j] * S_.lb[t][j];
            newton(rp, rpb, rx, y, z, r4, r5, r4b, Da_);
            const double aa = max_step(Da_);
            double sig = comp_after(Da_, aa) / Mtot / mu;
            sig = sig * sig * sig;
            // Mehrotra corrector
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j) {
                    r4[k][j] = S_.s[k][j] * S_.l[k][j] + Da_.ds[k][j] * Da_.dl[k][j] - sig * mu;
                    r5[k][j] = S_.xi[k][j] * S_.nu[k][j] + Da_.dxi[k][j] * Da_.dnu[k][j] - sig * mu;
                }
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < kBox; ++j)
                    r4b[t][j] = S_.sb[t][j] * S_.lb[t][j] + Da_.dsb[t][j] * Da_.dlb[t][j] - sig * mu;
            newton(rp, rpb, rx, y, z, r4, r5, r4b, D_);
            double a = std::min(1.0, kTau * max_step(D_));
            double cnew = comp_after(D_, a);
            if (cnew > comp) {
                // safeguard: the second-order term made it worse; take the plain centred direction
                for (int k = 1; k <= N; ++k)
                    for (int j = 0; j < kRows; ++j) {
                        r4[k][j] = S_.s[k][j] * S_.l[k][j] - sig * mu;
                        r5[k][j] = S_.xi[k][j] * S_.nu[k][j] - sig * mu;
                    }
                for (int t = 0; t < N; ++t)
                    for (int j = 0; j < kBox; ++j) r4b[t][j] = S_.sb[t][j] * S_.lb[t][j] - sig * mu;
                newton(rp, rpb, rx, y, z, r4, r5, r4b, D_);
                a = std::min(1.0, kTau * max_step(D_));
                cnew = comp_after(D_, a);
            }
            // breakdown guard: a step whose complementarity or control direction is not finite is not taken
            bool fin = cnew == cnew && cnew < INFINITY;
            for (int i = 0; i < 2 * N && fin; ++i) fin = D_.du[i] == D_.du[i] && std::fabs(D_.du[i]) < INFINITY;
            if (!fin) { status = MPC_NUMERICAL; ++it; break; }
            stall = (mu < 1e-6 && cnew > 0.9 * comp) ? stall + 1 : 0;     // late-phase no-progress counter
            for (int i = 0; i < 2 * N; ++i) S_.du[i] += a * D_.du[i];
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j) {
                    if (!Q.on[j]) continue;
                    S_.s[k][j] += a * D_.ds[k][j];
                    S_.l[k][j] += a * D_.dl[k][j];
                    S_.xi[k][j] += a * D_.dxi[k][j];
                    S_.nu[k][j] += a * D_.dnu[k][j];
                }
            for (int t = 0; t < N; ++t)
                for (int j = 0; j < kBox; ++j) {
                    S_.sb[t][j] += a * D_.dsb[t][j];
                    S_.lb[t][j] += a * D_.dlb[t][j];
                }
            if (stall >= 5) { status = MPC_NUMERICAL; ++it; break; }
        }
        iters = it;
        for (int i = 0; i < 2 * N; ++i)
            if (!(S_.du[i] == S_.du[i])) {
                std::memset(S_.du, 0, sizeof(double) * 2 * N);
                return MPC_NUMERICAL;
            }
        if (status == MPC_OK)
            for (int k = 1; k <= N; ++k)
                for (int j = 0; j < kRows; ++j)
                    if (Q.on[j] && S_.xi[k][j] > 1e-6 * (1.0 + std::fabs(Q.b[k][j]))) status = MPC_INFEASIBLE;
        if (p_.polish) {
            bool inf = false;
            if (active_set(S_, 0, kPolishRounds, inf)) status = inf ? MPC_INFEASIBLE : MPC_OK;
        }
        return status;
    }
};

// ---------------------------------------------------------------------------------------------
// the backend object behind a device = -1 context
// ---------------------------------------------------------------------------------------------
struct Backend {
    HostTable table;
    std::unique_ptr<Ref> ref;
    int threads = 0;

    explicit Backend(HostTable&& t) : table(std::move(t)), ref(new Ref(table)) {
        const char* e = std::getenv("MPC_CPU_THREADS");
        threads = e ? std::atoi(e) : 0;
        if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    }

    // run body(worker, i) for i in [0, n) over the worker threads (dynamic chunks of 8 instances)
    template <typename Body>
    void parallel(const mpc_params& p, int n, Body body) const {
        const int nt = std::max(1, std::min(threads, (n + 7) / 8));
        std::atomic<int> next(0);
        // a worker that cannot get its scratch leaves its share to the others; no exception leaves a thread
        auto run = [&]() {
            std::unique_ptr<Worker> w;
            try {
                w.reset(new Worker(*ref, p));
            } catch (...) {
                return;
            }
            for (;;) {
                const int i0 = next.fetch_add(8);
                if (i0 >= n) break;
                for (int i = i0; i < std::min(n, i0 + 8); ++i) body(*w, i);
            }
        };
        std::vector<std::thread> pool;
        if (nt > 1) {
            try {
                pool.reserve(nt - 1);
                for (int t = 1; t < nt; ++t) pool.emplace_back(run);
            } catch (...) {
                // fewer threads than asked: the ones that started and this one finish the work
            }
        }
        run();
        for (auto& th : pool) th.join();
        // every worker failed to start: nothing was solved
        if (next.load() < n) throw std::bad_alloc();
    }

    // mpc_solve_batch on host buffers (the device entry's argument contract)
    void solve_batch(const mpc_params& p, int B, const double* x0, const double* obs, const int* n_obs,
                     const double* ubar, double* u0, double* U, double* Xpred, int* status, int* iters) const {
        const int N = p.N, mo = obs ? p.max_obs : 0;
        parallel(p, B, [&](Worker& w, int b) {
            int no = obs ? (n_obs ? n_obs[b] : mo) : 0;
            no = no < 0 ? 0 : (no > mo ? mo : no);
            int it = 0;
            const int st = w.solve(x0 + 5 * (size_t)b, obs ? obs + (size_t)b * mo * 2 : nullptr, no,
                                   ubar ? ubar + (size_t)b * 2 * N : nullptr, u0 ? u0 + 2 * (size_t)b : nullptr,
                                   U ? U + (size_t)b * 2 * N : nullptr,
                                   Xpred ? Xpred + (size_t)b * 5 * (N + 1) : nullptr, &it);
            if (status) status[b] = st;
            if (iters) iters[b] = it;
        });
    }

    void lookup(int n, const double* s, double* st, double* ct) const {
        for (int i = 0; i < n; ++i) {
            double o[5], c[2];
            ref->state(s[i], o);
            ref->control(s[i], c);
            if (st) std::memcpy(st + 5 * (size_t)i, o, sizeof(o));
            if (ct) std::memcpy(ct + 2 * (size_t)i, c, sizeof(c));
        }
    }

    void pose(int n, const double* s, const double* d, double* out) const {
        for (int i = 0; i < n; ++i) ref->pose(s[i], d[i], out + 3 * (size_t)i);
    }

    // run_simulation (trajectory_tracking.py:377-443) for B egos, step-synchronous like the device loop: per
    // step the ObstaclesFSM of every ego in the loop, one batched solve over them, the Euler plant step
    int closed_loop(const mpc_params& p0, int B, const double* x_init, const mpc_fsm& F, bool with_fsm,
                    int max_steps, double s_stop, double* hist_x, double* hist_u, double* hist_obs_s,
                    int* hist_tl, int* hist_status, int* n_steps, double* step_ms) const {
        mpc_params p = p0;
        p.max_obs = with_fsm ? 2 : 0;
        const size_t nb = (size_t)B, ns = (size_t)max_steps;
        if (hist_x) std::fill(hist_x, hist_x + nb * (ns + 1) * 5, NAN);
        if (hist_u) std::fill(hist_u, hist_u + nb * ns * 2, NAN);
        if (hist_obs_s) std::fill(hist_obs_s, hist_obs_s + nb * ns, NAN);
        if (hist_tl) std::fill(hist_tl, hist_tl + nb * ns, -1);
        if (hist_status) std::fill(hist_status, hist_status + nb * ns, -1);
        if (step_ms) std::fill(step_ms, step_ms + ns, NAN);
        std::vector<double> x(x_init, x_init + nb * 5), car(nb, F.obs_start_s), timer(nb, 0.0);
        std::vector<int> flags(nb * 4, 0), active(nb), alist;
        std::vector<double> xa, obsa, u0a;
        std::vector<int> nobsa, sta;
        for (int b = 0; b < B; ++b) {
            n_steps[b] = 0;
            active[b] = x[5 * (size_t)b] <= s_stop;
            if (hist_x) std::memcpy(hist_x + (size_t)b * (ns + 1) * 5, x.data() + 5 * (size_t)b, 5 * sizeof(double));
        }
        for (int step = 0; step < max_steps; ++step) {
            const auto t0 = std::chrono::steady_clock::now();
            alist.clear();
            for (int b = 0; b < B; ++b)
                if (active[b]) alist.push_back(b);
            if (alist.empty()) break;
            const int nl = (int)alist.size();
            xa.assign((size_t)nl * 5, 0.0);
            obsa.assign((size_t)nl * 4, 0.0);
            nobsa.assign(nl, 0);
            u0a.assign((size_t)nl * 2, 0.0);
            sta.assign(nl, 0);
            for (int i = 0; i < nl; ++i) {
                const int b = alist[i];
                const double s = x[5 * (size_t)b], v = x[5 * (size_t)b + 4];
                int* fl = flags.data() + 4 * (size_t)b;      // car active, car triggered, light green, waiting
                double* o = obsa.data() + 4 * (size_t)i;
                int n = 0;
                double car_s = NAN;
                if (F.dynamic_obstacle) {                    // ObstaclesFSM.update, :335-349
                    if (!fl[1] && s >= F.obs_trigger_s) { fl[1] = 1; fl[0] = 1; }
                    if (fl[0]) {
                        car[b] = car[b] + F.obs_v * p.dt;
                        if (car[b] > F.obs_end_s) {
                            fl[0] = 0;
                        } else {
                            o[0] = car[b];
                            o[1] = F.obs_v;
                            n = 1;
                            car_s = car[b];
                        }
                    }
                }
                if (F.traffic_light && !fl[2]) {             // :351-372
                    const double dist = F.tl_pos - s;
                    if (0.0 < dist && dist < F.tl_trigger_s) {
                        o[2 * n] = F.tl_pos;
                        o[2 * n + 1] = 0.0;
                        ++n;
                        if (v < 0.1 && dist < 10.0) fl[3] = 1;
                    }
                    if (fl[3]) {
                        timer[b] += p.dt;
                        if (timer[b] >= F.tl_stop_duration) { fl[2] = 1; fl[3] = 0; }
                    }
                }
                nobsa[i] = n;
                std::memcpy(xa.data() + 5 * (size_t)i, x.data() + 5 * (size_t)b, 5 * sizeof(double));
                if (hist_obs_s) hist_obs_s[(size_t)b * ns + step] = car_s;
                if (hist_tl) hist_tl[(size_t)b * ns + step] = fl[2];
            }
            solve_batch(p, nl, xa.data(), with_fsm ? obsa.data() : nullptr, with_fsm ? nobsa.data() : nullptr,
                        nullptr, u0a.data(), nullptr, nullptr, sta.data(), nullptr);
            for (int i = 0; i < nl; ++i) {                   // plant step x + dt f(x, u0, k_ref(s)), :403-406
                const int b = alist[i];
                double* xb = x.data() + 5 * (size_t)b;
                double st[5];
                ref->state(xb[0], st);
                const double u1 = u0a[2 * (size_t)i], u2 = u0a[2 * (size_t)i + 1];
                const double xd[5] = {xb[4], xb[4] * xb[2], xb[4] * (xb[3] - st[3]), u1, u2};
                for (int j = 0; j < 5; ++j) xb[j] = xb[j] + p.dt * xd[j];
                if (hist_x) std::memcpy(hist_x + ((size_t)b * (ns + 1) + step + 1) * 5, xb, 5 * sizeof(double));
                if (hist_u) {
                    hist_u[((size_t)b * ns + step) * 2] = u1;
                    hist_u[((size_t)b * ns + step) * 2 + 1] = u2;
                }
                if (hist_status) hist_status[(size_t)b * ns + step] = sta[i];
                n_steps[b] = step + 1;
                if (!(xb[0] <= s_stop)) active[b] = 0;
            }
            if (step_ms)
                step_ms[step] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        return MPC_SUCCESS;
    }
};

}  // namespace mpcqp_cpu

#endif  // MPCQP_CPU_BACKEND_H

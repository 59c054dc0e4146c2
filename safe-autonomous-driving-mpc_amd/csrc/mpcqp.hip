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
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <new>
#include <string>
#include <vector>

#include "../../include/mpcqp.h"
#include "host_table.h"
#include "cpu_backend.h"

#define WAVE 64
#ifndef MPC_NO_NT20
#define MPC_NO_NT20 0
#endif
#define NROW 9
#define NBOX 4
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
    const double* gx;  // [T]  global pose of the reference line (trajectory_loader.py:32-62)
    const double* gy;
    const double* gpsi;
    int T, Tu;
    double smax;
    double last[5];    // X_ref[-1] verbatim (trajectory_loader.py:90-91)
    const int* bidx;   // [nb + 1] bucket index of s: bidx[g] = lower_bound(s, s0 + g h)
    int nb;
    double s0, ibh;    // s[0], 1 / h
};

struct KParams {
    int N, max_obs, linearization, sqp_iters, max_iter, polish;
    double dt, u_min0, u_min1, u_max0, u_max1;
    double w_d, w_o, w_v, w_u1, w_u2;
    double osd, tgap, L, sl, brake_distance, brake_accel;
    double tol, tol_mu, rho, sqp_tol;
    double mu_check;   // interior-point checkpoint threshold (MU_CHECK; -1 = off, MPC_CHECKPOINT=0)
    int dbg;           // diagnostics only (MPC_DBG, default 0): 1 = the crossover kernel defers without the
                       // work-list atomic (timing probe; the interior-point launch then sees an empty list)
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
// interval of v in the table's s column (n <= T: a prefix of it), i.e. scipy's searchsorted
// (lower bound) clamped to [1, n - 1].  v's bucket g brackets the lower bound: it lies in
// [bidx[g - 1], bidx[g + 2]] (one bucket of slack either side for the rounding of g), so a binary search
// over that window returns the full binary search's answer exactly.  With 4 buckets per table interval
// the window holds ~1 knot (~2 dependent L2 loads instead of log2 T; every instance looks up ~4 N times),
// and a table with clustered knots costs log2 of the knots in the window, never a linear walk.
// Host restatement: mpcqp_host::seg_host (host_table.h).
__device__ __forceinline__ int seg_t(const DevTable& t, int n, double v) {
    double gf = (v - t.s0) * t.ibh;
    gf = gf > 0.0 ? gf : 0.0;                       // also maps NaN to bucket 0
    const int g = gf < (double)(t.nb - 1) ? (int)gf : t.nb - 1;
    int lo = t.bidx[g > 0 ? g - 1 : 0];
    int hi = g + 2 <= t.nb ? t.bidx[g + 2] : t.T;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (t.s[mid] < v) lo = mid + 1; else hi = mid;
    }
    lo = lo < n ? lo : n;
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
    int i = seg_t(t, t.T, s);
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
    int i = seg_t(t, t.Tu, s);
    out[0] = lin(t.s, t.u1, i, s);
    out[1] = lin(t.s, t.u2, i, s);
}

// ------------------------------------------------------------------------------------------
// per-instance LDS layout (doubles); stage arrays indexed by stage k = 0..N
// ------------------------------------------------------------------------------------------
// Stage records read by the recursions are padded to an even number of doubles and every array
// starts 16-B aligned, so each pair is one ds_read_b128 (4 LDS cycles) instead of a ds_read2_b64 (8).
// The Riccati recursions are lane-distributed (section "distributed recursions" below): lane i = 0..4
// of a group holds row i of P / component i of the state, so the records they read per lane are laid
// out by row: QR (row i of the stage Hessian), QH (component i of the linear term); KR holds K by rows.
#define A5S 8          // stride of A5: a12, a14, a20, a23, a24, dt, 0, 0 (the zeros and dt serve the
                       // per-lane coefficient gathers of the distributed recursions)
#define SIS 4          // stride of Si (3 used)
#define QRS 20         // stride of QR: rows i = 0..4 (s,d,o,k,v) x columns (s,d,o,v); row 3 (k) zero
#define QHS 6          // stride of QH: (s,d,o,k,v) with k = 0, one pad
#define KRS 12         // stride of KR: rows r = 0, 1 of K_t, each (K(r,0..4), kk_r)
struct Lds {
    double* A5;    // [N][A5S]
    double* cst;   // [N+1][6]  cost data of stage k: (-d_ref', -o_ref', -v_ref') and the residuals r_d, r_o, r_v
    double* QR;    // [N+1][QRS] Riccati stage Hessians (barrier / penalty augmented), by row
    double* Rt;    // [N][2]
    double* KR;    // [N][KRS]  Riccati gains by row, K(r,0..4), with the solve's feed-forward kk_r in slot 5
    double* Si;    // [N][SIS]  (1/l00, l10, 1/l11) of S_t = Ls Ls'
    double* QH;    // [N+1][QHS] LQR stage linear terms (state)
    double* gh;    // [N][2]    LQR stage linear terms (control)
    double* Xr;    // [N+1][5]  nominal rollout (setup, outputs); aliases QH, which is dead then
    double* dX;    // [N+1][5]  rollout of the direction
    double* dud;   // [N][2]    direction dU
    double* ys;    // [N+1][4]  dual-residual stage terms yc + ya (cost part + multiplier part)
    double* zs;    // [N][2]    control terms zc + za
    double* ub;    // [N][2]    linearisation point
    double* kap;   // [N+1]     k_ref(xbar_k) (setup); aliases QH after Xr
    double* AC;    // [N][5][6] closed-loop rows (A_t + B K_t)(i,:) and (B kk_t)_i of the forward solve
                   //           (kernels with acl_on only; rows 0..2 are A's, written at setup)
};
// the forward solve reads closed-loop rows (AC) in the horizon-specialised kernels and for GL = 64; the
// runtime-horizon GL <= 32 kernels keep the K-row form (AC would cost them an occupancy step at N ~ 30)
__host__ __device__ constexpr bool acl_on(int GL, int NT) { return NT > 0 || GL == 64; }
// The crossover launch (MODE_XO) carves a lite layout: no AC (K-row forward solve), no cost data (held
// in registers: lane k-1 is its only writer and reader), no dual-residual terms (ys, zs; interior point
// only), and the direction dud aliases gh (gh is dead once kk is formed; dud is read only after the
// solve, and every solve's caller rewrites gh first).  At N = 20 that is 1251 doubles per instance, so
// 8 two-instance workgroups (20 KB each) fit the 160 KB of a CU: all 2048 crossover waves of a 4096
// batch are resident at once, two per SIMD, instead of running in two rounds.
// At convergence the separate dual-residual terms (yc, ya, zc, za) go to a scratch in QR rows 0..2
// (the factorisation is dead then; the polish rewrites those rows): yc of stage k at QR[k][0..3],
// ya at QR[k][4..7], zc / za of control t at QR[t][8..9] / QR[t][10..11].
#define DQ_YC 0
#define DQ_YA 4
#define DQ_ZC 8
#define DQ_ZA 10

// stage cache record of the split launch, per work-list slot: ub [N][2], Xr [N+1][5], then the crossover's solve
// (the unconstrained optimum of QP(ubar), the interior point's start) by lane: du of control k-1 and x4 of
// stage k, [N][6]; then, from an even offset, the trajectory lookups at each stage's nominal s (get_state's
// d, o, k, v and its slopes d', o', k', v'), [N+1][8], so MODE_IPM repeats no table search.  Even record size:
// every record and its lookup block start 16-byte aligned.
__host__ __device__ constexpr int stage_cache_xo(int N) { return 2 * N + 5 * (N + 1); }
__host__ __device__ constexpr int stage_cache_lk(int N) { return (stage_cache_xo(N) + 6 * N + 1) & ~1; }
__host__ __device__ constexpr int stage_cache_doubles(int N) { return stage_cache_lk(N) + 8 * (N + 1); }

__host__ __device__ inline int lds_doubles(int N, bool acl, bool lite = false) {
    int NP = N + 1;
    int n = (acl ? N * 30 : 0) + N * A5S + (lite ? 0 : NP * 6) + NP * QRS + N * 2 + N * KRS + N * SIS + NP * QHS + N * 2 +
            (lite ? 0 : N * 2 + NP * 4 + N * 2) + N * 2 + NP * 5;
    return (n + 1) & ~1;     // groups stay 16-B aligned
}

__device__ inline Lds carve(double* p, int N, bool acl, bool lite = false) {
    Lds L;
    int NP = N + 1;
    // even-sized arrays first (16-B aligned starts), the odd-sized ones last
    L.AC = p; p += acl ? N * 30 : 0;
    L.A5 = p; p += N * A5S;
    L.cst = lite ? nullptr : p; p += lite ? 0 : NP * 6;
    L.QR = p; p += NP * QRS;
    L.Rt = p; p += N * 2;
    L.KR = p; p += N * KRS;
    L.Si = p; p += N * SIS;
    L.QH = p;
    L.Xr = p;                 // Xr [NP][5] and kap [NP] share QH's NP * 6 doubles
    L.kap = p + NP * 5;
    p += NP * QHS;
    L.gh = p; p += N * 2;
    L.dud = lite ? L.gh : p; p += lite ? 0 : N * 2;
    L.ys = lite ? nullptr : p; p += lite ? 0 : NP * 4;
    L.zs = lite ? nullptr : p; p += lite ? 0 : N * 2;
    L.ub = p; p += N * 2;
    L.dX = p; p += NP * 5;
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
// structural nonzeros of the soft-row coefficient vectors (row_coef): (s,d,o,v) entry a of row j
__host__ __device__ constexpr bool row_nz(int j, int a) {
    return j <= 1 ? a == 1 : (j <= 5 ? (a == 1 || a == 2) : (j == 6 ? a == 0 : (j == 7 ? (a == 0 || a == 3) : a == 3)));
}
// dot4 over the structural nonzeros only, in dot4's association order (identical for finite x: the
// skipped terms are exact zeros); the multiplications by literal zeros are not folded by the compiler
__device__ __forceinline__ double rdot(int j, const double c[4], const double x[4]) {
    double acc = 0.0;
    bool first = true;
#pragma unroll
    for (int a = 3; a >= 0; --a)
        if (row_nz(j, a)) {
            acc = first ? c[a] * x[a] : fma(c[a], x[a], acc);
            first = false;
        }
    return acc;
}
// 1/sqrt(x) to full double precision: v_rsq_f64 + one third-order correction (the Cholesky pivots only
// enter as reciprocals; the IEEE sqrt sequence costs ~100 cycles of dependent latency on gfx950)
#ifndef MPC_HO_RECIP
#define MPC_HO_RECIP 1
#endif
__device__ __forceinline__ double frsqrt(double x) {
    double y = __builtin_amdgcn_rsq(x);
#if MPC_HO_RECIP
    // one third-order step: with e = 1 - x y^2 (|e| < 2^-22 from v_rsq_f64), 1/sqrt(x) =
    // y (1 + e/2 + 3e^2/8 + O(e^3)); 4 dependent levels instead of the 6 of two Newton steps
    const double e = fma(-x * y, y, 1.0);
    return fma(y * e, fma(0.375, e, 0.5), y);
#else
    const double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
#endif
}
// 1/x to full double precision: v_rcp_f64 + one third-order correction (no IEEE division sequence)
__device__ __forceinline__ double frcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
#if MPC_HO_RECIP
    // one third-order step: 1/x = r (1 + e + e^2 + O(e^3)) with e = 1 - x r
    return fma(r, fma(e, e, e), r);
#else
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
#endif
}

// v_max_f64 / v_min_f64 as single instructions.  For fmax/fmin LLVM first quiets every operand it
// cannot prove canonical (DPP and permlane results, selects, loop-carried values) with an extra
// v_max_f64 x, x, x; arithmetic here only ever makes quiet NaNs, for which the bare instruction already
// has fmax's semantics (the other operand wins), so results are unchanged.
__device__ __forceinline__ double vmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmin(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// max(a, |b|)
__device__ __forceinline__ double vmaxabs(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// ------------------------------------------------------------------------------------------
// lane groups: IPW instances per 64-lane wavefront, GL = 64 / IPW lanes each
// ------------------------------------------------------------------------------------------
// Cross-lane moves of a double for the group reductions: DPP within a row of 16 lanes (quad_perm
// xor 1 / xor 2, row_half_mirror, row_mirror; a few cycles each) and ds_swizzle xor 16 within 32 lanes,
// instead of ds_bpermute (~80 cycles per hop).  After the quad steps every lane of a quad holds the
// quad value, so the mirrors pair the right partners; a + b == b + a keeps all lanes bit-identical.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// Row pairs and wave halves: v_permlane16_swap / v_permlane32_swap with the value in both operands
// return both sides of the pair (rows 2r and 2r+1 of 16 lanes; lanes i and i+32) on every lane, in two
// VALU slots per double and no LDS round trip (ds_swizzle / ds_bpermute wait ~60-80 cycles per hop).
// tools/probes/xlane_probe.hip checks the semantics.
__device__ __forceinline__ double pack_d(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int W>
__device__ __forceinline__ void xpair_d(double v, double& a, double& b) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    if constexpr (W == 16) {
        const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        a = pack_d(l[0], h[0]);
        b = pack_d(l[1], h[1]);
    } else {
        const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        a = pack_d(l[0], h[0]);
        b = pack_d(l[1], h[1]);
    }
}
#define DPP_XOR1 0xB1          // quad_perm [1,0,3,2]
#define DPP_XOR2 0x4E          // quad_perm [2,3,0,1]
#define DPP_HMIRROR 0x141      // row_half_mirror
#define DPP_MIRROR 0x140       // row_mirror

template <int GL>
struct Grp {
    int base;   // first lane of the group
    template <typename OP>
    __device__ __forceinline__ double reduce(double v, OP op) const {
        v = op(v, dpp_d<DPP_XOR1>(v));
        v = op(v, dpp_d<DPP_XOR2>(v));
        v = op(v, dpp_d<DPP_HMIRROR>(v));
        v = op(v, dpp_d<DPP_MIRROR>(v));
        // the same (a, b) operand order on both sides of a pair: every lane ends bit-identical
        double a, b;
        if (GL >= 32) { xpair_d<16>(v, a, b); v = op(a, b); }
        if (GL >= 64) { xpair_d<32>(v, a, b); v = op(a, b); }
        return v;
    }
    __device__ __forceinline__ double sum(double v) const {
        return reduce(v, [](double a, double b) { return a + b; });
    }
    __device__ __forceinline__ double max(double v) const {
        return reduce(v, [](double a, double b) { return vmax(a, b); });
    }
    __device__ __forceinline__ double min(double v) const {
        return reduce(v, [](double a, double b) { return vmin(a, b); });
    }
    __device__ __forceinline__ double get(double v, int rel) const { return __shfl(v, base + rel, WAVE); }
};

// nonlinear rollout (predict, trajectory_tracking.py:87-114), bit-exact.  s, v, k do not depend on
// the k_ref lookups, so they are rolled first; lane j then looks up k_ref(s_j); then d, o.
// st_ln / sl_ln (optional): lane j <= N also returns its whole lookup at s_j with the slopes (get_state), which
// is the stage data's lookup of the QP at this rollout: one table search per stage instead of two.
__device__ void predict_grp(const DevTable& tab, int N, double dt, const double* x0, const double* uU, double* xout,
                            double* kap, int ln, double* st_ln = nullptr, double* sl_ln = nullptr) {
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
    if (st_ln ? ln <= N : ln < N) {
        double st[5];
        get_state(tab, xout[5 * ln], st, sl_ln);
        if (ln < N) kap[ln] = st[3];
        if (st_ln)
            for (int a = 0; a < 5; ++a) st_ln[a] = st[a];
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

// packed symmetric 5x5 on (s,d,o,k,v): index of (i,j)
__host__ __device__ constexpr int s5(int i, int j) {
    return i <= j ? i * 5 - i * (i - 1) / 2 + (j - i) : j * 5 - j * (j - 1) / 2 + (i - j);
}

// two doubles from a 16-B aligned LDS address: one ds_read_b128
__device__ __forceinline__ void ld2(const double* p, double& a, double& b) {
    const double2 v = *reinterpret_cast<const double2*>(p);
    a = v.x;
    b = v.y;
}
__device__ __forceinline__ void ld_a5(const double* p, double a[5]) {
    double pad;
    ld2(p, a[0], a[1]);
    ld2(p + 2, a[2], a[3]);
    ld2(p + 4, a[4], pad);
}
// Software pipeline of the stage recursions: every step starts with a full LDS wait (the data of
// this step, prefetched one step earlier), then issues the next step's loads, then computes.  The
// sched barriers keep the compiler from sinking the prefetch to the end of the step (where the next
// wait would expose its whole latency) or hoisting it above the wait.
__device__ __forceinline__ void lds_fence() {
    __builtin_amdgcn_s_waitcnt(0xc07f);      // lgkmcnt(0), vmcnt/expcnt untouched
    __builtin_amdgcn_sched_barrier(0);
}
#ifdef MPC_NO_SCHED_FENCE
__device__ __forceinline__ void sched_fence() {}
#else
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
#endif

// ------------------------------------------------------------------------------------------
// distributed recursions.  The Riccati factorisation and solves run on lanes i = 0..4 of each
// lane group: lane i holds row i of P (factorisation), component i of the co-state p (backward
// solve) and of the state direction x (forward solve).  Every cross-lane term is a
// v_fmac_f64_dpp with row_newbcast:l, i.e. a broadcast of lane l's register within its 16-lane row
// fused into the FMA (same issue cost as a plain v_fmac_f64 on gfx950).  Compared with running the
// whole 5x5 recursion redundantly on every lane, a stage costs ~90 instead of ~210 VALU
// instructions.  The other lanes of the group compute discarded values (their per-lane records are
// clamped to lane 4's; their stores are masked off).  Groups are aligned to 16-lane rows, so the
// broadcasts never cross groups.
// ------------------------------------------------------------------------------------------
// dst += src@L * c  (src broadcast from lane L of each 16-lane row); asm operand lists are written
// with early-clobber accumulators, so no accumulator shares a register with a source.  The leading
// s_nop 1 covers the VALU-write -> DPP-read hazard (2 wait states) of the sources.
#define DPPF(d, s, c, L) "v_fmac_f64_dpp " d ", " s ", " c " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
// dst -= src@L * c (DPP source negation modifier)
#define DPPFN(d, s, c, L) "v_fmac_f64_dpp " d ", -" s ", " c " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"


// Per-lane constants of the distributed recursions.  A_t = I + J'_t with J' nonzero in rows 0..2 only:
// J'(0,4) = dt, J'(1,2) = a12, J'(1,4) = a14, J'(2,0) = a20, J'(2,3) = a23, J'(2,4) = a24.  Lane i needs
// e_l(i) = J'(l,i) (column i; backward recursions) and f_m(i) = J'(i,m) (row i; forward solve).  Both
// are gathered per lane from the stage's A5 record (a12, a14, a20, a23, a24, dt, 0, 0): oXX is the
// record offset a lane reads (6 = a zero slot).
struct DLane {
    int i;                     // row / component of this lane (clamped to 4 for lanes >= 5)
    int oe1, oe2, of0, of2, of3, of4;
    double e0;                 // J'(0,i) = dt for i = 4 (constant)
    double bu;                 // B(i,:) u = bu * u_r: dt on lanes 3 (r = 0) and 4 (r = 1), else 0
    int kr, ur;                // K row r the lane reads in the forward solve (offset kr = 6 r in KR), r
    int ps;                    // slot of p_i in the backward solve's co-state record: (i + 2) % 5
    double k0, k1, k2, k3;     // symmetrisation: lane keeps its own P(i,j) when i <= j
    double r1, r2, r3, r4;     // lane is row 1, 2, 3, 4
};
__device__ __forceinline__ DLane dlane(int gl, double dt) {
    // opaque lane index: the constants are rebuilt at every recursion (a few VALU) instead of being
    // hoisted out of the interior-point loop and held in registers across the row phases
    asm volatile("" : "+v"(gl));
    DLane D;
    D.i = gl < 5 ? gl : 4;
    const int z = 6;
    D.oe1 = gl == 2 ? 0 : (gl == 4 ? 1 : z);
    D.oe2 = gl == 0 ? 2 : (gl == 3 ? 3 : (gl == 4 ? 4 : z));
    D.of0 = gl == 2 ? 2 : z;
    D.of2 = gl == 1 ? 0 : z;
    D.of3 = gl == 2 ? 3 : z;
    D.of4 = gl == 0 ? 5 : (gl == 1 ? 1 : (gl == 2 ? 4 : z));
    D.e0 = gl == 4 ? dt : 0.0;
    D.bu = gl >= 3 ? dt : 0.0;
    D.ur = gl >= 4 ? 1 : 0;
    D.kr = 6 * D.ur;
    D.ps = gl >= 3 ? gl - 3 : gl + 2;
    D.k0 = gl <= 0 ? 1.0 : 0.0;
    D.k1 = gl <= 1 ? 1.0 : 0.0;
    D.k2 = gl <= 2 ? 1.0 : 0.0;
    D.k3 = gl <= 3 ? 1.0 : 0.0;
    D.r1 = gl == 1 ? 1.0 : 0.0;
    D.r2 = gl == 2 ? 1.0 : 0.0;
    D.r3 = gl == 3 ? 1.0 : 0.0;
    D.r4 = gl == 4 ? 1.0 : 0.0;
    return D;
}

// Riccati factorisation of  min sum 0.5 x'Qt x + 0.5 u'Rt u,  x_{t+1} = A_t x_t + B u_t,  x_0 = 0.
// Per stage: S = Rt + B'P B = Ls Ls', M = P A, W = Ls^-1 B'M, K = -Ls^-T W, P <- A'M - W'W + Qt.  The
// Cholesky form keeps ~2 more digits than an explicit S^-1 once barrier weights reach 1e12 (DESIGN.md
// section 3); Qt is added last for the same reason (adding it before the cancellation A'M - W'W would
// round that difference at Qt's magnitude).  Lane i: row i of M locally; the W terms from M(3,i),
// M(4,i); row i of A'M and of W'W by broadcasts.  Restates riccati_factor() of oracle/mpc_oracle.c.
struct FacRec { double a[5], r0, r1, e1, e2, q[4]; };
__device__ __forceinline__ void load_fac(const Lds& S, const DLane& L, int t, FacRec& F) {
    const double* a5 = S.A5 + A5S * t;
    ld_a5(a5, F.a);
    ld2(S.Rt + 2 * t, F.r0, F.r1);
    F.e1 = a5[L.oe1];
    F.e2 = a5[L.oe2];
    ld2(S.QR + QRS * t + 4 * L.i, F.q[0], F.q[1]);
    ld2(S.QR + QRS * t + 4 * L.i + 2, F.q[2], F.q[3]);
}
// CF: the copy-free form (the A'M block reads p1, p3, p4 from its in-place accumulators, so pr[1], pr[3], pr[4]
// need no register copies, and a bare pivot floor): 4 instructions fewer per stage, bit-identical.  The obstacle
// kernels use it (C3 -0.7%); in the obstacle-free N = 20 interior-point kernel the same code measured +0.3%
// (300-launch A/B), so it keeps the plain form
template <bool CF>
__device__ __forceinline__ void fac_step(const Lds& S, const DLane& L, int t, bool upd, double dt, double dt2,
                                         const FacRec& F, double pr[5]) {
    const double a12 = F.a[0], a14 = F.a[1], a20 = F.a[2], a23 = F.a[3], a24 = F.a[4];
    // S = Rt + dt^2 P[{3,4},{3,4}]: P(3,3), P(3,4) from lane 3, P(4,4) from lane 4
    double s00 = F.r0, s01 = 0.0, s11 = F.r1;
    asm("s_nop 1\n\t" DPPF("%0", "%3", "%5", 3) DPPF("%1", "%4", "%5", 3) DPPF("%2", "%4", "%5", 4)
        : "+&v"(s00), "+&v"(s01), "+&v"(s11) : "v"(pr[3]), "v"(pr[4]), "v"(dt2));
    // pivot floors: never active in practice (s00 >= Rt >= 2 w_u1 > 0); a NaN pivot is floored too, the
    // NaN still reaches P and K through V and M
    if constexpr (CF) {
        // bare v_max_f64 (as vmax): fmax first quiets the asm result with a v_max_f64 x, x, x
        const double floor_ = 1e-300;
        asm("v_max_f64 %0, %0, %1" : "+v"(s00) : "s"(floor_));
    } else {
        s00 = fmax(s00, 1e-300);
    }
    const double il00 = frsqrt(s00), l10 = s01 * il00;
    const double r11 = fmax(s11 - l10 * l10, 1e-14 * s11);
    const double il11 = frsqrt(r11);
    const double c0 = dt * il00, c1 = dt * il11, c2 = -l10 * il11;
    // row i of M = P A (local)
    double m[5];
#ifndef MPC_FAC_NOP
    // (update stages: m[0], m[2..4] are formed inside the A'M block below, so that block needs no s_nop)
    if (!upd) {
#endif
    m[0] = fma(pr[2], a20, pr[0]);
    m[1] = pr[1];
    m[2] = fma(pr[1], a12, pr[2]);
    m[3] = fma(pr[2], a23, pr[3]);
    m[4] = fma(pr[0], dt, fma(pr[1], a14, fma(pr[2], a24, pr[4])));
#ifndef MPC_FAC_NOP
    }
#endif
    // row i of A'M = M(i,:) + sum_l J'(l,i) M(l,:), and V3 = M(3,i), V4 = M(4,i) = P(i,{3,4}) +
    // sum_l J'(l,i) P(l,{3,4}), all in place.  Source lane l only changes in the broadcast of a lane l'
    // with J'(l',l) != 0; with J' nonzero at (0,4), (1,2), (1,4), (2,0), (2,3), (2,4) the order l = 0, 2, 1
    // reads every source lane before its own update (a zero coefficient leaves a value unchanged).
    // The same register is written and then broadcast 7 instructions later (the DPP hazard needs 2).
    double v3 = pr[3], v4 = pr[4];
#ifndef MPC_FAC_NOP
    if (upd) {
        // The VALU-write -> DPP-read hazard (2 wait states) without an s_nop: the block first forms the rows of
        // M = P A it broadcasts (the same fma()s as above, in the same order), so every register a DPP reads was
        // written at least 2 instructions earlier inside the block (m[0] 5 before the first broadcast, m[4]
        // 4 before its own), and whatever the compiler wrote before the block is 6 or more instructions back.
        m[1] = pr[1];
        if constexpr (!CF) {
        asm("v_fma_f64 %0, %10, %13, %11\n\t"          // m0 = fma(p2, a20, p0)
            "v_fma_f64 %2, %12, %14, %10\n\t"          // m2 = fma(p1, a12, p2)
            "v_fma_f64 %3, %10, %15, %16\n\t"          // m3 = fma(p2, a23, p3)
            "v_fma_f64 %4, %10, %17, %18\n\t"          // t = fma(p2, a24, p4)
            "v_fma_f64 %4, %12, %19, %4\n\t"           // t = fma(p1, a14, t)
            "v_fma_f64 %4, %11, %20, %4\n\t"           // m4 = fma(p0, dt, t)
            DPPF("%0", "%0", "%7", 0) DPPF("%1", "%1", "%7", 0) DPPF("%2", "%2", "%7", 0) DPPF("%3", "%3", "%7", 0)
            DPPF("%4", "%4", "%7", 0) DPPF("%5", "%5", "%7", 0) DPPF("%6", "%6", "%7", 0)
            DPPF("%0", "%0", "%8", 2) DPPF("%1", "%1", "%8", 2) DPPF("%2", "%2", "%8", 2) DPPF("%3", "%3", "%8", 2)
            DPPF("%4", "%4", "%8", 2) DPPF("%5", "%5", "%8", 2) DPPF("%6", "%6", "%8", 2)
            DPPF("%0", "%0", "%9", 1) DPPF("%1", "%1", "%9", 1) DPPF("%2", "%2", "%9", 1) DPPF("%3", "%3", "%9", 1)
            DPPF("%4", "%4", "%9", 1) DPPF("%5", "%5", "%9", 1) DPPF("%6", "%6", "%9", 1)
            : "=&v"(m[0]), "+&v"(m[1]), "=&v"(m[2]), "=&v"(m[3]), "=&v"(m[4]), "+&v"(v3), "+&v"(v4)
            : "v"(L.e0), "v"(F.e2), "v"(F.e1), "v"(pr[2]), "v"(pr[0]), "v"(pr[1]),
              "v"(a20), "v"(a12), "v"(a23), "v"(pr[3]), "v"(a24), "v"(pr[4]), "v"(a14), "v"(dt));
        } else {
        // p1, p3, p4 are read from the in-place accumulators m1, v3, v4 themselves (they still hold them: the
        // broadcasts come after the six fma()s), so pr[1], pr[3], pr[4] need no copies of their own
        asm("v_fma_f64 %0, %10, %12, %11\n\t"          // m0 = fma(p2, a20, p0)
            "v_fma_f64 %2, %1, %13, %10\n\t"           // m2 = fma(p1, a12, p2)
            "v_fma_f64 %3, %10, %14, %5\n\t"           // m3 = fma(p2, a23, p3)
            "v_fma_f64 %4, %10, %15, %6\n\t"           // t = fma(p2, a24, p4)
            "v_fma_f64 %4, %1, %16, %4\n\t"            // t = fma(p1, a14, t)
            "v_fma_f64 %4, %11, %17, %4\n\t"           // m4 = fma(p0, dt, t)
            DPPF("%0", "%0", "%7", 0) DPPF("%1", "%1", "%7", 0) DPPF("%2", "%2", "%7", 0) DPPF("%3", "%3", "%7", 0)
            DPPF("%4", "%4", "%7", 0) DPPF("%5", "%5", "%7", 0) DPPF("%6", "%6", "%7", 0)
            DPPF("%0", "%0", "%8", 2) DPPF("%1", "%1", "%8", 2) DPPF("%2", "%2", "%8", 2) DPPF("%3", "%3", "%8", 2)
            DPPF("%4", "%4", "%8", 2) DPPF("%5", "%5", "%8", 2) DPPF("%6", "%6", "%8", 2)
            DPPF("%0", "%0", "%9", 1) DPPF("%1", "%1", "%9", 1) DPPF("%2", "%2", "%9", 1) DPPF("%3", "%3", "%9", 1)
            DPPF("%4", "%4", "%9", 1) DPPF("%5", "%5", "%9", 1) DPPF("%6", "%6", "%9", 1)
            : "=&v"(m[0]), "+&v"(m[1]), "=&v"(m[2]), "=&v"(m[3]), "=&v"(m[4]), "+&v"(v3), "+&v"(v4)
            : "v"(L.e0), "v"(F.e2), "v"(F.e1), "v"(pr[2]), "v"(pr[0]),
              "v"(a20), "v"(a12), "v"(a23), "v"(a24), "v"(a14), "v"(dt));
        }
    } else {
        asm("s_nop 1\n\t" DPPF("%0", "%0", "%2", 0) DPPF("%1", "%1", "%2", 0) "s_nop 1\n\t"
            DPPF("%0", "%0", "%3", 2) DPPF("%1", "%1", "%3", 2) "s_nop 1\n\t"
            DPPF("%0", "%0", "%4", 1) DPPF("%1", "%1", "%4", 1)
            : "+v"(v3), "+v"(v4) : "v"(L.e0), "v"(F.e2), "v"(F.e1));
    }
#else
    if (upd) {
        asm("s_nop 1\n\t"
            DPPF("%0", "%0", "%7", 0) DPPF("%1", "%1", "%7", 0) DPPF("%2", "%2", "%7", 0) DPPF("%3", "%3", "%7", 0)
            DPPF("%4", "%4", "%7", 0) DPPF("%5", "%5", "%7", 0) DPPF("%6", "%6", "%7", 0)
            DPPF("%0", "%0", "%8", 2) DPPF("%1", "%1", "%8", 2) DPPF("%2", "%2", "%8", 2) DPPF("%3", "%3", "%8", 2)
            DPPF("%4", "%4", "%8", 2) DPPF("%5", "%5", "%8", 2) DPPF("%6", "%6", "%8", 2)
            DPPF("%0", "%0", "%9", 1) DPPF("%1", "%1", "%9", 1) DPPF("%2", "%2", "%9", 1) DPPF("%3", "%3", "%9", 1)
            DPPF("%4", "%4", "%9", 1) DPPF("%5", "%5", "%9", 1) DPPF("%6", "%6", "%9", 1)
            : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]), "+v"(m[3]), "+v"(m[4]), "+v"(v3), "+v"(v4)
            : "v"(L.e0), "v"(F.e2), "v"(F.e1));
    } else {
        asm("s_nop 1\n\t" DPPF("%0", "%0", "%2", 0) DPPF("%1", "%1", "%2", 0) "s_nop 1\n\t"
            DPPF("%0", "%0", "%3", 2) DPPF("%1", "%1", "%3", 2) "s_nop 1\n\t"
            DPPF("%0", "%0", "%4", 1) DPPF("%1", "%1", "%4", 1)
            : "+v"(v3), "+v"(v4) : "v"(L.e0), "v"(F.e2), "v"(F.e1));
    }
#endif
    double* am = m;
    double w0, w1, K1, K0;
#ifndef MPC_FAC_NOP
    if (upd) {
        // W, K and then P -= W'W: the block first forms w0, w1, K1, K0 (the same operations as below, in the
        // same order, no contraction), so w1 is 4 instructions old at its first broadcast: no s_nop
        double tt;
        asm("v_mul_f64 %5, %9, %10\n\t"                // w0 = c0 * v3
            "v_mul_f64 %7, %11, %5\n\t"                // t = c2 * w0
            "v_fma_f64 %6, %12, %13, %7\n\t"           // w1 = fma(c1, v4, t)
            "v_mul_f64 %8, -%6, %14\n\t"               // K1 = -w1 * il11
            "v_mul_f64 %7, %15, %8\n\t"                // t = l10 * K1
            "v_add_f64 %7, %5, %7\n\t"                 // t = w0 + t
            "v_mul_f64 %7, -%7, %16\n\t"               // K0 = -t * il00
            DPPFN("%0", "%6", "%6", 0) DPPFN("%1", "%6", "%6", 1) DPPFN("%2", "%6", "%6", 2)
            DPPFN("%3", "%6", "%6", 3) DPPFN("%4", "%6", "%6", 4) DPPFN("%0", "%5", "%5", 0) DPPFN("%1", "%5", "%5", 1)
            DPPFN("%2", "%5", "%5", 2) DPPFN("%3", "%5", "%5", 3) DPPFN("%4", "%5", "%5", 4)
            : "+&v"(am[0]), "+&v"(am[1]), "+&v"(am[2]), "+&v"(am[3]), "+&v"(am[4]), "=&v"(w0), "=&v"(w1),
              "=&v"(tt), "=&v"(K1)
            : "v"(c0), "v"(v3), "v"(c2), "v"(c1), "v"(v4), "v"(il11), "v"(l10), "v"(il00));
        K0 = tt;
    } else
#endif
    {
        w0 = c0 * v3;
        w1 = fma(c1, v4, c2 * w0);
        K1 = -w1 * il11;
        K0 = -(w0 + l10 * K1) * il00;
    }
    // K by rows (lane i writes column i); the Cholesky factor of S is group-uniform: all five lanes write
    // the same values
    S.KR[KRS * t + L.i] = K0;
    S.KR[KRS * t + 6 + L.i] = K1;
    S.Si[SIS * t] = il00;
    S.Si[SIS * t + 1] = l10;
    S.Si[SIS * t + 2] = il11;
    if (upd) {
#ifndef MPC_FAC_NOP
        // P(i,j) = A'M(i,j) - W1_i W1_j - W0_i W0_j (done above) + Qt(i,j), then the symmetrisation below; the
        // block forms P's rows and the kept upper entries first (the same additions and products as the
        // MPC_FAC_NOP code), so each broadcast row is 5 or more instructions old: no s_nop
        double sy0, sy1, sy2, sy3, p0, p1, p2, p4;
        asm("v_add_f64 %5, %9, %13\n\t"                // p1 = am1 + q1
            "v_add_f64 %6, %10, %14\n\t"               // p2 = am2 + q2
            "v_add_f64 %7, %12, %15\n\t"               // p4 = am4 + q3
            "v_add_f64 %4, %8, %16\n\t"                // p0 = am0 + q0
            "v_mul_f64 %1, %5, %18\n\t"                // sy1 = p1 * k1
            "v_mul_f64 %2, %6, %19\n\t"                // sy2 = p2 * k2
            "v_mul_f64 %3, %11, %20\n\t"               // sy3 = am3 * k3
            "v_mul_f64 %0, %4, %17\n\t"                // sy0 = p0 * k0
            DPPF("%0", "%5", "%21", 0) DPPF("%1", "%6", "%22", 1) DPPF("%2", "%11", "%23", 2)
            DPPF("%3", "%7", "%24", 3) DPPF("%0", "%6", "%22", 0) DPPF("%1", "%11", "%23", 1) DPPF("%2", "%7", "%24", 2)
            DPPF("%0", "%11", "%23", 0) DPPF("%1", "%7", "%24", 1) DPPF("%0", "%7", "%24", 0)
            : "=&v"(sy0), "=&v"(sy1), "=&v"(sy2), "=&v"(sy3), "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p4)
            : "v"(am[0]), "v"(am[1]), "v"(am[2]), "v"(am[3]), "v"(am[4]), "v"(F.q[1]), "v"(F.q[2]), "v"(F.q[3]),
              "v"(F.q[0]), "v"(L.k0), "v"(L.k1), "v"(L.k2), "v"(L.k3), "v"(L.r1), "v"(L.r2), "v"(L.r3), "v"(L.r4));
        (void)p0;
        pr[0] = sy0;
        pr[1] = sy1;
        pr[2] = sy2;
        pr[3] = sy3;
        pr[4] = p4;
#else
        // P(i,j) = A'M(i,j) - W1_i W1_j - W0_i W0_j + Qt(i,j)
        asm("s_nop 1\n\t" DPPFN("%0", "%5", "%5", 0) DPPFN("%1", "%5", "%5", 1) DPPFN("%2", "%5", "%5", 2)
            DPPFN("%3", "%5", "%5", 3) DPPFN("%4", "%5", "%5", 4) DPPFN("%0", "%6", "%6", 0) DPPFN("%1", "%6", "%6", 1)
            DPPFN("%2", "%6", "%6", 2) DPPFN("%3", "%6", "%6", 3) DPPFN("%4", "%6", "%6", 4)
            : "+&v"(am[0]), "+&v"(am[1]), "+&v"(am[2]), "+&v"(am[3]), "+&v"(am[4])
            : "v"(w1), "v"(w0));
        pr[0] = am[0] + F.q[0];
        pr[1] = am[1] + F.q[1];
        pr[2] = am[2] + F.q[2];
        pr[3] = am[3];
        pr[4] = am[4] + F.q[3];
        // symmetrise: lane i takes P(j,i) from row j for j < i, so P is exactly symmetric (the upper
        // triangle is the reference, as in the oracle's packed recursion).  Lane-computed lower entries
        // differ by rounding, and with barrier weights near 1e12 that asymmetry costs interior-point
        // iterations on hard elastic instances.
        double sy0 = pr[0] * L.k0, sy1 = pr[1] * L.k1, sy2 = pr[2] * L.k2, sy3 = pr[3] * L.k3;
        asm("s_nop 1\n\t" DPPF("%0", "%4", "%8", 0) DPPF("%1", "%5", "%9", 1) DPPF("%2", "%6", "%10", 2)
            DPPF("%3", "%7", "%11", 3) DPPF("%0", "%5", "%9", 0) DPPF("%1", "%6", "%10", 1) DPPF("%2", "%7", "%11", 2)
            DPPF("%0", "%6", "%10", 0) DPPF("%1", "%7", "%11", 1) DPPF("%0", "%7", "%11", 0)
            : "+&v"(sy0), "+&v"(sy1), "+&v"(sy2), "+&v"(sy3)
            : "v"(pr[1]), "v"(pr[2]), "v"(pr[3]), "v"(pr[4]), "v"(L.r1), "v"(L.r2), "v"(L.r3), "v"(L.r4));
        pr[0] = sy0;
        pr[1] = sy1;
        pr[2] = sy2;
        pr[3] = sy3;
#endif
    }
}
// NT > 0: horizon fixed at compile time, stages fully unrolled (immediate LDS offsets, no loop control)
template <int NT, bool CF>
__device__ __forceinline__ void riccati_factor_lanes(const Lds& S, int Nrt, double dt, int gl) {
    const int N = NT > 0 ? NT : Nrt;
    const DLane L = dlane(gl, dt);
    const double dt2 = dt * dt;
    double pr[5];
    ld2(S.QR + QRS * N + 4 * L.i, pr[0], pr[1]);
    ld2(S.QR + QRS * N + 4 * L.i + 2, pr[2], pr[4]);
    pr[3] = 0.0;
#ifdef MPC_FAC_LOOP
    if constexpr (false) {
#else
    if constexpr (NT > 0) {
#endif
        FacRec buf[2];
        load_fac(S, L, NT - 1, buf[0]);
#pragma unroll
        for (int t = NT - 1; t >= 0; --t) {
            lds_fence();
            load_fac(S, L, t >= 1 ? t - 1 : 0, buf[(NT - t) & 1]);
            sched_fence();
            fac_step<CF>(S, L, t, t >= 1, dt, dt2, buf[(NT - 1 - t) & 1], pr);
        }
    } else {
        FacRec A, B;
        load_fac(S, L, N - 1, A);
        int t = N - 1;
        while (true) {
            lds_fence();
            load_fac(S, L, t >= 1 ? t - 1 : 0, B);      // unconditional: keeps the LDS wait counts exact
            sched_fence();
            fac_step<CF>(S, L, t, t >= 1, dt, dt2, A, pr);
            if (--t < 0) break;
            lds_fence();
            load_fac(S, L, t >= 1 ? t - 1 : 0, A);
            sched_fence();
            fac_step<CF>(S, L, t, t >= 1, dt, dt2, B, pr);
            if (--t < 0) break;
        }
    }
}
// the recursion runs on lanes 0..4 of each group only (exec narrowed): the other lanes would compute
// discarded values, and with them out of exec every store is a plain store
template <int NT, bool CF>
__device__ void riccati_factor(const Lds& S, int Nrt, double dt, int gl) {
    if (gl < 5) riccati_factor_lanes<NT, CF>(S, Nrt, dt, gl);
    wave_sync();
}

// LQR solve with the factorisation: linear terms -QH (stages 1..N), -gh (controls).  Writes dud
// (controls) and dX (states, x_0 = 0).  Three phases (restates riccati_solve() of oracle/mpc_oracle.c):
//  1. backward, lanes 0..4 (lane i holds p_i): p_t = (A_t + B K_t)' p_{t+1} + QH_t + K_t' gh_t, the
//     closed-loop form (one accumulator chain of five broadcast FMAs per stage);
//  2. stage-parallel, lane t: kk_t = S_t^-1 (gh_t + B' p_{t+1}) into slot 5 of the K rows;
//  3. forward, lanes 0..4 (lane i holds x_i): u_r = kk_r + K_t(r,:) x, x <- A_t x + B u.
// The co-states p_{t+1} pass from phase 1 to phase 2 through QR (dead between factorisations), in
// record slots (p3, p4, p0, p1, p2) so that phase 2 reads (p3, p4) with one ds_read_b128.
struct BwdRec { double g0, g1, qi, K0, K1, e1, e2; };
struct FwdRec { double K[5], kk, f0, f2, f3, f4; };
__device__ __forceinline__ void load_bwd(const Lds& S, const DLane& L, int t, BwdRec& B) {
    const double* a5 = S.A5 + A5S * t;
    ld2(S.gh + 2 * t, B.g0, B.g1);
    B.qi = S.QH[QHS * t + L.i];
    B.K0 = S.KR[KRS * t + L.i];
    B.K1 = S.KR[KRS * t + 6 + L.i];
    B.e1 = a5[L.oe1];
    B.e2 = a5[L.oe2];
}
__device__ __forceinline__ void load_fwd(const Lds& S, const DLane& L, int t, FwdRec& F) {
    const double* a5 = S.A5 + A5S * t;
    const double* kr = S.KR + KRS * t + L.kr;
    ld2(kr, F.K[0], F.K[1]);
    ld2(kr + 2, F.K[2], F.K[3]);
    ld2(kr + 4, F.K[4], F.kk);
    F.f0 = a5[L.of0];
    F.f2 = a5[L.of2];
    F.f3 = a5[L.of3];
    F.f4 = a5[L.of4];
}
// step t: p = p_{t+1} on entry (stored for phase 2), p_t on exit (t >= 1)
// The hazard-free block (dt K products first, no s_nop): C3 -2.6% (profiles/r06_ab_hazard.log); in every kernel
// since the stage lookups (C2 -0.1..-0.3%, profiles/r06_ab_bwd_all.log).  -DMPC_BWD_NOP: the s_nop form.
__device__ __forceinline__ void bwd_step(const Lds& S, const DLane& L, int t, double dt, const BwdRec& B, double& p) {
    S.QR[QRS * (t + 1) + L.ps] = p;
    if (t >= 1) {
        double acc = fma(B.K0, B.g0, fma(B.K1, B.g1, B.qi));
#ifdef MPC_BWD_NOP
        const double kd0 = B.K0 * dt, kd1 = B.K1 * dt;
        asm("s_nop 1\n\t" DPPF("%0", "%1", "%2", 3) DPPF("%0", "%1", "%3", 4) DPPF("%0", "%1", "%4", 2)
            DPPF("%0", "%1", "%5", 1) DPPF("%0", "%1", "%6", 0)
            : "+&v"(acc) : "v"(p), "v"(kd0), "v"(kd1), "v"(B.e2), "v"(B.e1), "v"(L.e0));
#else
        // the two products dt K(r, i) are the block's first two instructions: they are the two wait states the
        // VALU-write -> DPP-read hazard on p needs (p was written by the previous step), so no s_nop
        double kd0, kd1;
        asm("v_mul_f64 %1, %7, %9\n\t"
            "v_mul_f64 %2, %8, %9\n\t"
            DPPF("%0", "%3", "%1", 3) DPPF("%0", "%3", "%2", 4) DPPF("%0", "%3", "%4", 2)
            DPPF("%0", "%3", "%5", 1) DPPF("%0", "%3", "%6", 0)
            : "+&v"(acc), "=&v"(kd0), "=&v"(kd1)
            : "v"(p), "v"(B.e2), "v"(B.e1), "v"(L.e0), "v"(B.K0), "v"(B.K1), "v"(dt));
#endif
        p = acc + p;
    }
}
__device__ __forceinline__ void kk_stage(const Lds& S, int t, double dt) {
    double g0, g1, si0, si1, si2, pad, p3, p4;
    ld2(S.gh + 2 * t, g0, g1);
    ld2(S.Si + SIS * t, si0, si1);
    ld2(S.Si + SIS * t + 2, si2, pad);
    ld2(S.QR + QRS * (t + 1), p3, p4);
    const double h0 = fma(p3, dt, g0), h1 = fma(p4, dt, g1);
    const double w0 = h0 * si0;
    const double w1 = (h1 - si1 * w0) * si2;
    const double k1 = w1 * si2;
    const double k0 = (w0 - si1 * k1) * si0;
    S.KR[KRS * t + 5] = k0;
    S.KR[KRS * t + 11] = k1;
}
// closed-loop rows 3, 4 of stage t for the forward solve: e_{3+r}' + dt K_t(r,:) and dt kk_r
// Every LDS read of a stage-parallel phase is issued before its first LDS write: the compiler cannot tell the
// arrays of the layout apart, so a read after a write would wait for it (one LDS round trip per element)
__device__ __forceinline__ void ac_rows(const Lds& S, int t, double dt) {
    const double* kr = S.KR + KRS * t;
    double* ac = S.AC + 30 * t + 18;
    double k[2][6];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int m = 0; m < 6; m += 2) ld2(kr + 6 * r + m, k[r][m], k[r][m + 1]);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
        for (int m = 0; m < 5; ++m) ac[6 * r + m] = (m == 3 + r) ? fma(dt, k[r][m], 1.0) : dt * k[r][m];
        ac[6 * r + 5] = dt * k[r][5];
    }
}
// u_t = kk_t + K_t x_t after the closed-loop forward solve (stage-parallel; the accumulation order of
// the K-row forward step)
__device__ __forceinline__ void u_stage(const Lds& S, int t) {
    const double* kr = S.KR + KRS * t;
    const double* x = S.dX + 5 * t;
    double xv[5], k[2][6];
#pragma unroll
    for (int m = 0; m < 5; ++m) xv[m] = x[m];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int m = 0; m < 6; m += 2) ld2(kr + 6 * r + m, k[r][m], k[r][m + 1]);
    double u[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        u[r] = k[r][5];
#pragma unroll
        for (int m = 0; m < 5; ++m) u[r] = fma(xv[m], k[r][m], u[r]);
    }
    *reinterpret_cast<double2*>(S.dud + 2 * t) = make_double2(u[0], u[1]);
}
struct AclRec { double c[5], d; };
__device__ __forceinline__ void load_acl(const Lds& S, const DLane& L, int t, AclRec& F) {
    const double* ac = S.AC + 30 * t + 6 * L.i;
    ld2(ac, F.c[0], F.c[1]);
    ld2(ac + 2, F.c[2], F.c[3]);
    ld2(ac + 4, F.c[4], F.d);
}
// x_{t+1}(i) = sum_m Acl_t(i,m) x_m + (B kk_t)_i: one chain of five broadcast FMAs.
// NOP: the s_nop 1 covering the VALU-write -> DPP-read hazard on x.  Only the first step needs it (x = 0 was
// just materialised); in the unrolled recursions every later x is the previous chain's last FMA, followed by
// its LDS store, the next record's loads and waits (tools/dpp_hazard_check.py checks the listing)
template <bool NOP = true>
__device__ __forceinline__ void acl_step(const Lds& S, const DLane& L, int t, AclRec& F, double& x) {
#ifdef MPC_ACL_NOP
    constexpr bool P = true;
#else
    constexpr bool P = NOP;
#endif
    if constexpr (P)
        asm("s_nop 1\n\t" DPPF("%0", "%1", "%2", 0) DPPF("%0", "%1", "%3", 1) DPPF("%0", "%1", "%4", 2)
            DPPF("%0", "%1", "%5", 3) DPPF("%0", "%1", "%6", 4)
            : "+&v"(F.d) : "v"(x), "v"(F.c[0]), "v"(F.c[1]), "v"(F.c[2]), "v"(F.c[3]), "v"(F.c[4]));
    else
        asm(DPPF("%0", "%1", "%2", 0) DPPF("%0", "%1", "%3", 1) DPPF("%0", "%1", "%4", 2)
            DPPF("%0", "%1", "%5", 3) DPPF("%0", "%1", "%6", 4)
            : "+&v"(F.d) : "v"(x), "v"(F.c[0]), "v"(F.c[1]), "v"(F.c[2]), "v"(F.c[3]), "v"(F.c[4]));
    x = F.d;
    S.dX[5 * (t + 1) + L.i] = x;
}
__device__ __forceinline__ void fwd_step(const Lds& S, const DLane& L, int t, const FwdRec& F, double& x) {
    // u: lanes 0..3 accumulate row 0 of K (u0), lane 4 row 1 (u1); xa = J'_t x (row i)
    double u = F.kk, xa = 0.0;
    asm("s_nop 1\n\t" DPPF("%0", "%2", "%3", 0) DPPF("%1", "%2", "%8", 0) DPPF("%0", "%2", "%4", 1)
        DPPF("%1", "%2", "%9", 2) DPPF("%0", "%2", "%5", 2) DPPF("%1", "%2", "%10", 3) DPPF("%0", "%2", "%6", 3)
        DPPF("%1", "%2", "%11", 4) DPPF("%0", "%2", "%7", 4)
        : "+&v"(u), "+&v"(xa)
        : "v"(x), "v"(F.K[0]), "v"(F.K[1]), "v"(F.K[2]), "v"(F.K[3]), "v"(F.K[4]), "v"(F.f0), "v"(F.f2),
          "v"(F.f3), "v"(F.f4));
    x = fma(L.bu, u, x + xa);
    S.dX[5 * (t + 1) + L.i] = x;
    S.dud[2 * t + L.ur] = u;
}

// NT > 0: the horizon is a compile-time constant and the recursions are fully unrolled.
template <int NT>
__device__ __forceinline__ void solve_bwd_lanes(const Lds& S, int N, double dt, int gl) {
    const DLane L = dlane(gl, dt);
    double p = S.QH[QHS * N + L.i];
#ifdef MPC_SOLVE_LOOP
    if constexpr (false) {
#else
    if constexpr (NT > 0) {
#endif
        BwdRec buf[2];
        load_bwd(S, L, NT - 1, buf[0]);
#pragma unroll
        for (int t = NT - 1; t >= 0; --t) {
            sched_fence();
            load_bwd(S, L, t >= 1 ? t - 1 : 0, buf[(NT - t) & 1]);
            sched_fence();
            bwd_step(S, L, t, dt, buf[(NT - 1 - t) & 1], p);
        }
    } else {
        BwdRec A, B;
        load_bwd(S, L, N - 1, A);
        int t = N - 1;
        while (true) {
            sched_fence();
            load_bwd(S, L, t >= 1 ? t - 1 : 0, B);
            sched_fence();
            bwd_step(S, L, t, dt, A, p);
            if (--t < 0) break;
            sched_fence();
            load_bwd(S, L, t >= 1 ? t - 1 : 0, A);
            sched_fence();
            bwd_step(S, L, t, dt, B, p);
            if (--t < 0) break;
        }
    }
}
template <int NT>
__device__ __forceinline__ void solve_acl_lanes(const Lds& S, int N, double dt, int gl) {
    const DLane L = dlane(gl, dt);
    double x = 0.0;
    S.dX[L.i] = 0.0;
    if constexpr (NT > 0) {
        AclRec buf[2];
        load_acl(S, L, 0, buf[0]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            sched_fence();
            load_acl(S, L, t + 1 < NT ? t + 1 : t, buf[(t + 1) & 1]);
            sched_fence();
            if (t == 0) acl_step<true>(S, L, t, buf[t & 1], x);
            else acl_step<false>(S, L, t, buf[t & 1], x);
        }
    } else {
        AclRec A, B;
        load_acl(S, L, 0, A);
        int t = 0;
        while (true) {
            sched_fence();
            load_acl(S, L, t + 1 < N ? t + 1 : t, B);
            sched_fence();
            acl_step(S, L, t, A, x);
            if (++t >= N) break;
            sched_fence();
            load_acl(S, L, t + 1 < N ? t + 1 : t, A);
            sched_fence();
            acl_step(S, L, t, B, x);
            if (++t >= N) break;
        }
    }
}
template <int NT>
__device__ __forceinline__ void solve_fwd_lanes(const Lds& S, int N, double dt, int gl) {
    const DLane L = dlane(gl, dt);
    double x = 0.0;
    S.dX[L.i] = 0.0;
#ifdef MPC_SOLVE_LOOP
    if constexpr (false) {
#else
    if constexpr (NT > 0) {
#endif
        FwdRec buf[2];
        load_fwd(S, L, 0, buf[0]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            sched_fence();
            load_fwd(S, L, t + 1 < NT ? t + 1 : t, buf[(t + 1) & 1]);
            sched_fence();
            fwd_step(S, L, t, buf[t & 1], x);
        }
    } else {
        FwdRec A, B;
        load_fwd(S, L, 0, A);
        int t = 0;
        while (true) {
            sched_fence();
            load_fwd(S, L, t + 1 < N ? t + 1 : t, B);
            sched_fence();
            fwd_step(S, L, t, A, x);
            if (++t >= N) break;
            sched_fence();
            load_fwd(S, L, t + 1 < N ? t + 1 : t, A);
            sched_fence();
            fwd_step(S, L, t, B, x);
            if (++t >= N) break;
        }
    }
}
// the recursions run on lanes 0..4 of each group (exec narrowed), the stage phases on lanes 0..N-1.
// ACL: the forward solve runs on closed-loop rows (built with kk) and u follows stage-parallel.
template <int NT, bool ACL>
__device__ void riccati_solve(const Lds& S, int Nrt, double dt, int gl) {
    const int N = NT > 0 ? NT : Nrt;
    if (gl < 5) solve_bwd_lanes<NT>(S, N, dt, gl);
    wave_sync();
    if (gl < N) {
        kk_stage(S, gl, dt);
        if (ACL) ac_rows(S, gl, dt);
    }
    wave_sync();
    if (ACL) {
        if (gl < 5) solve_acl_lanes<NT>(S, N, dt, gl);
        wave_sync();
        if (gl < N) u_stage(S, gl);
    } else {
        if (gl < 5) solve_fwd_lanes<NT>(S, N, dt, gl);
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
            mc[st4(a)] += S.QR[QRS * k + DQ_YC + a];
            ma[st4(a)] += S.QR[QRS * k + DQ_YA + a];
        }
        const int t = k - 1;
        double gc0 = fma(dt, mc[3], S.QR[QRS * t + DQ_ZC]), gc1 = fma(dt, mc[4], S.QR[QRS * t + DQ_ZC + 1]);
        double ga0 = fma(dt, ma[3], S.QR[QRS * t + DQ_ZA]), ga1 = fma(dt, ma[4], S.QR[QRS * t + DQ_ZA + 1]);
        rdmax = fmax(rdmax, fmax(fabs(gc0 + ga0), fabs(gc1 + ga1)));
        sd = fmax(sd, fmax(fmax(fabs(gc0), fabs(gc1)), fmax(fabs(ga0), fabs(ga1))));
        double y[5];
        applyAT(S.A5 + A5S * t, dt, mc, y);
#pragma unroll
        for (int a = 0; a < 5; ++a) mc[a] = y[a];
        applyAT(S.A5 + A5S * t, dt, ma, y);
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

// phase-cycle instrumentation of a diagnostic build (-DMPC_PROF, tools/phase_probe.py); compiled
// out of the product library
#ifdef MPC_PROF
__device__ unsigned long long g_prof[16];
#define PROF_DECL                                \
    unsigned long long prof_acc[12];             \
    for (int i_ = 0; i_ < 12; ++i_) prof_acc[i_] = 0; \
    unsigned long long prof_t = __builtin_amdgcn_s_memtime();
#define PROF(i)                                                  \
    {                                                            \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
        prof_acc[i] += t_ - prof_t;                              \
        prof_t = t_;                                             \
    }
#define PROF_END \
    if (gl == 0 && bvalid) for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&g_prof[i_], prof_acc[i_]);
#else
#define PROF_DECL
#define PROF(i)
#define PROF_END
#endif

#define POLISH_DELTA 1e-11
#define POLISH_REFINE 2
#define POLISH_ROUNDS 6
#define XO_ROUNDS 1            // rounds of the crossover attempt before the interior point
// SQP stopping rules besides convergence (oracle orc_solve): a 2-cycle (the QP returns the point of two QPs
// back, |U_k - U_k-2| <= SQP_CYCLE_REL |U_k - U_k-1|), and SQP_INF_STREAK elastic QPs in a row
#define SQP_CYCLE_REL 1e-6
#define SQP_INF_STREAK 5
#define START_SHIFT 3.0     // interior-point start: slack and elastic slack beyond the row value (oracle pdip)
// interior-point checkpoint (oracle pdip): once mu <= MU_CHECK and every row's slack and
// multiplier are CHECK_SEP apart, CHECK_ROUNDS polish rounds try the iterate's classification; a certified point
// is the QP's exact optimum, otherwise the interior point continues from the unchanged iterate (once per QP)
#define MU_CHECK 1e-4
#define CHECK_SEP 100.0
#define CHECK_ROUNDS 2

// ------------------------------------------------------------------------------------------
// the solver kernel.  A 64-lane wavefront carries G = 64 / GL MPC instances, one per aligned group
// of GL lanes (GL = 16, 32 or 64, the smallest with N + 1 <= GL).  Within a group, lane k-1 owns
// stage k = 1..N: its 9 soft rows and the 4 box rows of control k-1, whose interior-point state
// lives in that lane's registers (row ids are compile-time, so the row coefficients fold away).
// The stage-wise recursions (Riccati factorisation and solves, rollouts) run group-uniformly
// from the group's LDS region: one instruction stream serves G instances, which is what pays for
// the inherently sequential part of the algorithm on a 64-wide SIMD.
// All branching is group-uniform, so a group that has converged simply drops out of the exec mask.
// ------------------------------------------------------------------------------------------
// soft-row id of lane slot j: without obstacles the slots hold rows 0-5 and 8
template <bool OBS>
__device__ __forceinline__ constexpr int rid(int j) { return OBS ? j : (j < 6 ? j : 8); }

// Launch modes.  MODE_FULL: crossover (polish = 2), interior point, polish, outputs -- one launch per
// batch.  The split pair MODE_XO + MODE_IPM is the same computation in two launches: MODE_XO runs the
// setup and the crossover for every instance, writes the outputs of the instances it certifies and
// appends the others to a device work list; MODE_IPM then runs the interior point (and polish) on the
// listed instances only.  Results are identical (a failed crossover leaves no state behind), but the
// expensive instances all start at once instead of queueing behind cheap ones on the same SIMD
// ("two-phase launch").  MODE_ONE is MODE_FULL for a single QP (sqp_iters = 1):
// the SQP loop is then a compile-time single pass, so no state is carried across it (the runtime loop
// costs the one-launch kernels ~400 B of scratch per lane at N = 40).
#define MODE_FULL 0
#define MODE_XO 1
#define MODE_IPM 2
#define MODE_ONE 3

// NT > 0: kernel specialised for horizon N = NT (the stage recursions are unrolled); NT = 0: any N.
template <int GL, bool OBS, int MODE, int NT>
__global__ void __launch_bounds__(WAVE, MODE == MODE_XO ? 2 : 1)   // crossover: two waves per SIMD (256 VGPRs)
mpc_solve_kernel(DevTable tab, KParams Pr, int B, const double* __restrict__ x0g, const double* __restrict__ obsg,
                 const int* __restrict__ nobsg, const double* __restrict__ ubarg, double* __restrict__ u0g,
                 double* __restrict__ Ug, double* __restrict__ Xg, int* __restrict__ statusg,
                 int* __restrict__ itersg, int* __restrict__ wlist, int* __restrict__ wcount,
                 double* __restrict__ stc, int* __restrict__ wnext) {
    constexpr int G = WAVE / GL;
    constexpr int NR = OBS ? NROW : NROW - 2;    // soft rows held per lane (6, 7: obstacle rows)
    // the Riccati solves of the horizon-specialised kernels are fully unrolled, obstacle kernels included.
    // (Round 1 kept them looped in the obstacle kernels, whose lanes hold 9 rows, for fewer spills; since
    // the split kernels carry no runtime SQP loop, unrolled is faster there too: C4 0.660 -> 0.609 ms,
    // C3 -0.8%, and C5 5.67 -> 4.16 ms together with the unrolled factorisation of NT = 40.)
    constexpr int NTR = NT;
    // row right-hand sides recomputed after the solve (WRC) instead of held live across it: obstacle
    // kernels only (measured neutral on the obstacle-free N = 20 kernel)
    constexpr bool WRC = OBS;
    // the factorisation's copy-free A'M block (fac_step): obstacle kernels only (see fac_step)
#if defined(MPC_FAC_CF_NONE)
    constexpr bool FAC_CF = false;
#elif defined(MPC_FAC_CF_ALL)
    constexpr bool FAC_CF = true;
#else
    constexpr bool FAC_CF = OBS;
#endif
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int ln = threadIdx.x;
    const int grp = ln / GL, gl = ln % GL;
    int b;
    bool bvalid;
    int cslot = 0;      // MODE_IPM: work-list slot whose record this group uses (a spare group repeats the last)
    // MODE_XO of an eager call zeroes the other of the context's two list counters for the next call
    // (launch_solve), so no memset launch separates the batches
    if (MODE == MODE_XO && wnext && blockIdx.x == 0 && threadIdx.x == 0) *wnext = 0;
    if (MODE == MODE_IPM) {
        // instances deferred by the MODE_XO launch; waves past the end of the list exit at once
        const int cnt = *wcount;
        if ((int)blockIdx.x * G >= cnt) return;
        const int slot = blockIdx.x * G + grp;
        bvalid = slot < cnt;
        cslot = bvalid ? slot : cnt - 1;
        b = wlist[cslot];
    } else {
        b = blockIdx.x * G + grp;
        bvalid = b < B;
        if (!bvalid) b = B - 1;      // a spare group repeats the last instance; its outputs are dropped
    }
    PROF_DECL
    const Grp<GL> Q{grp * GL};
    const int N = NT > 0 ? NT : Pr.N;
    const int NP = N + 1;
    const double dt = Pr.dt;
    const double rho = Pr.rho;
    const double hL = Pr.L / 2.0;
    constexpr bool LITE = MODE == MODE_XO;          // lite LDS layout (see lds_doubles)
    constexpr bool ACL = acl_on(GL, NT) && !LITE;
    Lds S = carve(smem + (size_t)grp * lds_doubles(N, ACL, LITE), N, ACL, LITE);

    double x0[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) x0[j] = x0g[5 * (size_t)b + j];
    // n_obs may be NULL with an obstacle slab: every instance then uses all max_obs rows (as the
    // host entry mpc_solve_batch does)
    int nobs = nobsg ? nobsg[b] : (obsg ? Pr.max_obs : 0);
    nobs = nobs < 0 ? 0 : (nobs > Pr.max_obs ? Pr.max_obs : nobs);
    const double* obs = obsg ? obsg + (size_t)b * Pr.max_obs * 2 : nullptr;
    const bool has_obs = nobs > 0;

    const int k = gl + 1;            // stage of this lane
    const bool live = k <= N;        // lane owns the rows of stage k and the boxes of control k-1
    // rowon: the row exists for this instance (group-uniform: the obstacle rows need obstacles);
    // ron = rowon on a live lane.  The per-iteration phases use rowon only: dead lanes (stages past N)
    // compute discarded values and are masked where lane values meet (the group reductions)
    bool ron[NR], rowon[NR];
    double cf[NR][4];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        rowon[j] = (rid<OBS>(j) != 6 && rid<OBS>(j) != 7) || has_obs;
        ron[j] = live && rowon[j];
        row_coef(rid<OBS>(j), hL, Pr.L, Pr.tgap, cf[j]);
    }

    // stage cache of the split launch (stc != nullptr): MODE_XO leaves each deferred instance's
    // linearisation point ub [N][2] and nominal rollout Xr [N+1][5] at its work-list slot, so MODE_IPM
    // loads them instead of repeating the warm start and the rollout (stage_cache_doubles)
    const bool cached = MODE == MODE_IPM && stc != nullptr;
    const double* stc_in = nullptr;
    if (cached) stc_in = stc + (size_t)cslot * stage_cache_doubles(N);
    // ---- K1: linearisation point ---------------------------------------------------------
    if (cached) {
        if (gl < N) {
            S.ub[2 * gl] = stc_in[2 * gl];
            S.ub[2 * gl + 1] = stc_in[2 * gl + 1];
        }
        for (int i = gl; i < 5 * NP; i += GL) S.Xr[i] = stc_in[2 * N + i];
    } else if (gl < N) {
        if (ubarg) {
            S.ub[2 * gl] = ubarg[(size_t)b * 2 * N + 2 * gl];
            S.ub[2 * gl + 1] = ubarg[(size_t)b * 2 * N + 2 * gl + 1];
        } else {
            // warm start, trajectory_tracking.py:224-246: s_curr advanced by repeated addition,
            // sticky brake flag over steps 0..gl
            double s_curr = x0[0], v_curr = x0[4];
            bool brake = false;
            for (int j = 0; j <= gl; ++j) {
                if (j > 0) s_curr += v_curr * dt;
                for (int i = 0; i < nobs; ++i)
                    if ((obs[2 * i] - s_curr) < Pr.brake_distance) brake = true;
            }
            double ur[2];
            get_control(tab, s_curr, ur);
            S.ub[2 * gl] = ur[0];
            S.ub[2 * gl + 1] = brake ? Pr.brake_accel : ur[1];
        }
    }
    wave_sync();

    int nsoft = 0;
    for (int jj = 0; jj < NROW; ++jj) nsoft += ((jj != 6 && jj != 7) || has_obs) ? 1 : 0;
    const double Mtot = (double)(2 * nsoft * N + NBOX * N);
    const double R0 = 2.0 * Pr.w_u1, R1 = 2.0 * Pr.w_u2;

    // 0: return ubar and predict(x0, ubar).  The split launch (MODE_XO + MODE_IPM) runs single-QP solves
    // only (launch_solve), so there the SQP loop is a compile-time single pass: nothing is carried across it
    const int nsqp = MODE != MODE_FULL ? 1 : (Pr.sqp_iters < 0 ? 0 : Pr.sqp_iters);
    static_assert(MODE == MODE_FULL || MODE == MODE_XO || MODE == MODE_IPM || MODE == MODE_ONE, "launch mode");
    int status = MPC_OK, total_it = 0;
    // SQP state carried across re-linearisations (MODE_FULL): the row / box classification the last polish
    // left (2 bits per row, then one per box row), which starts the next QP's crossover (oracle polish_from,
    // given = 2); U two QPs back at this lane's control; the count of elastic QPs in a row
    int wcls = 0, ninf = 0;
    bool sqp_conv = false;
    double pb0 = 0.0, pb1 = 0.0;
    bool xo_ok = false;                    // MODE_XO: the crossover certified this instance
    double cstr[6] = {0, 0, 0, 0, 0, 0};   // LITE: cost data of stage k (this lane's only)
    // the lookup at this lane's stage (get_state at the nominal s_gl, with slopes): MODE_XO keeps it for the
    // stage cache.  Obstacle-free kernels only (LKC): in the obstacle kernels the longer-lived lookups moved
    // the register allocation against it (C3 +0.6%, C5 +0.3%; C4 -1.2%)
    constexpr bool LKC = !OBS;
    double refk[5] = {0, 0, 0, 0, 0}, slk[4] = {0, 0, 0, 0};
    for (int sqp = 0; sqp < nsqp; ++sqp) {
        // ---- K1: nominal rollout == predict(x0, ubar), into Xr (cached: loaded above), with the stage
        // lookups; cached: the lookups come from the stage cache ---------------------------------------
        if (!LKC) {
            if (!cached) predict_grp(tab, N, dt, x0, S.ub, S.Xr, S.kap, gl);
            if (gl <= N) get_state(tab, S.Xr[5 * gl], refk, slk);
        } else if (!cached) {
            predict_grp(tab, N, dt, x0, S.ub, S.Xr, S.kap, gl, refk, slk);
        } else if (gl <= N) {
            const double2* lk = reinterpret_cast<const double2*>(stc_in + stage_cache_lk(N) + 8 * gl);
            const double2 l0 = lk[0], l1 = lk[1], l2 = lk[2], l3 = lk[3];
            refk[1] = l0.x; refk[2] = l0.y; refk[3] = l1.x; refk[4] = l1.y;
            slk[0] = l2.x; slk[1] = l2.y; slk[2] = l3.x; slk[3] = l3.y;
        }
        // ---- K2: stage data of QP(ubar) ----------------------------------------------------
        const bool gn = Pr.linearization != 0;
        if (gl < N) {
            const double* x = S.Xr + 5 * gl;
            double dk = gn ? slk[2] : 0.0;
            S.A5[A5S * gl + 0] = dt * x[4];
            S.A5[A5S * gl + 1] = dt * x[2];
            S.A5[A5S * gl + 2] = dt * (-x[4] * dk);
            S.A5[A5S * gl + 3] = dt * x[4];
            S.A5[A5S * gl + 4] = dt * (x[3] - refk[3]);
            S.A5[A5S * gl + 5] = dt;      // a04, read by the per-lane gathers (DLane)
            S.A5[A5S * gl + 6] = 0.0;     // the gathers' zero slot
            S.A5[A5S * gl + 7] = 0.0;
            if (ACL) {
                // rows 0..2 of the forward solve's closed-loop matrix are A_t's (B has rows 3, 4 only)
                double* ac = S.AC + 30 * gl;
                const double a12 = dt * x[4], a14 = dt * x[2], a20 = dt * (-x[4] * dk), a23 = dt * x[4];
                const double a24 = dt * (x[3] - refk[3]);
                ac[0] = 1.0; ac[1] = 0.0; ac[2] = 0.0; ac[3] = 0.0; ac[4] = dt; ac[5] = 0.0;
                ac[6] = 0.0; ac[7] = 1.0; ac[8] = a12; ac[9] = 0.0; ac[10] = a14; ac[11] = 0.0;
                ac[12] = a20; ac[13] = 0.0; ac[14] = 1.0; ac[15] = a23; ac[16] = a24; ac[17] = 0.0;
            }
        }
        if (gl <= N) {
            // the k row of QR is structurally zero (no cost or row touches k); the k entry of QH is
            // written as zero by every QH writer (QH shares its space with Xr, which is live here)
#pragma unroll
            for (int j = 0; j < 4; ++j) S.QR[QRS * gl + 12 + j] = 0.0;
        }
        // cost data of stage k (lookups done by lane k of the group)
        {
            const int src = k < GL ? k : GL - 1;
            const double rk1 = Q.get(refk[1], src), rk2 = Q.get(refk[2], src), rk4 = Q.get(refk[4], src);
            const double sk0 = Q.get(slk[0], src), sk1 = Q.get(slk[1], src), sk3 = Q.get(slk[3], src);
            if (live) {
                const double* x = S.Xr + 5 * k;
                double* c = LITE ? cstr : S.cst + 6 * k;
                c[0] = gn ? -sk0 : 0.0;
                c[1] = gn ? -sk1 : 0.0;
                c[2] = gn ? -sk3 : 0.0;
                c[3] = x[1] - rk1;
                c[4] = x[2] - rk2;
                c[5] = x[4] - rk4;
            }
        }
        // row bounds of stage k, box bounds of control k-1
        double bk[NR], bb[NBOX];
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
            double v[NROW];  // by row id
            v[0] = -sl - pv0;
            v[1] = -(sl - pv0);
            v[2] = -sl - pv1;
            v[3] = -(sl - pv1);
            v[4] = -sl - pv2;
            v[5] = -(sl - pv2);
            v[6] = has_obs ? -(shat - Pr.osd - x[0]) : 0.0;
            v[7] = has_obs ? -(shat - x[0] - Pr.tgap * x[4]) : 0.0;
            v[8] = -x[4];
#pragma unroll
            for (int j = 0; j < NR; ++j) {
                bk[j] = ron[j] ? v[rid<OBS>(j)] : 0.0;
                bscale_l = fmax(bscale_l, fabs(bk[j]));
            }
            const double ub0 = live ? S.ub[2 * (k - 1)] : 0.0, ub1 = live ? S.ub[2 * (k - 1) + 1] : 0.0;
            bb[0] = live ? Pr.u_min0 - ub0 : 0.0;
            bb[1] = live ? -(Pr.u_max0 - ub0) : 0.0;
            bb[2] = live ? Pr.u_min1 - ub1 : 0.0;
            bb[3] = live ? -(Pr.u_max1 - ub1) : 0.0;
#pragma unroll
            for (int j = 0; j < NBOX; ++j) bscale_l = fmax(bscale_l, fabs(bb[j]));
        }
        const double bscale = Q.max(bscale_l);
        wave_sync();

        // ---- K4: crossover, then (if it does not certify) PDIP and the polish of its iterate ------
        // Phase 0 is the active-set solve started from the unconstrained optimum: all rows inactive,
        // multipliers 0, du = 0 (oracle pdip(): XO_ROUNDS rounds).  When it certifies (KKT-consistent),
        // it is the exact optimum and no interior-point iteration runs (70% of the C2 batch).
        double rs[NR], rl[NR], rxi[NR], rnu[NR], sb[NBOX], lb[NBOX];
#pragma unroll
        for (int j = 0; j < NR; ++j) { rs[j] = 0.0; rl[j] = 0.0; rxi[j] = 0.0; rnu[j] = 0.0; }
#pragma unroll
        for (int j = 0; j < NBOX; ++j) { sb[j] = 0.0; lb[j] = 0.0; }
        int it = 0, st_here = MPC_MAX_ITER, stall = 0;
        double mu = 0.0;
        // x4: state of stage k along the current iterate, G du (du = 0 at the start); updated with the
        // state direction of every step, so the linear rollout never re-runs (it is linear in du)
        double x4[4] = {0.0, 0.0, 0.0, 0.0};
        double du0 = 0.0, du1 = 0.0;        // control k-1 of the current iterate
        // MODE_XO runs phase 0 only and MODE_IPM phase 1 only (both compile-time)
        const int phase_lo = MODE == MODE_XO ? 0 : (MODE == MODE_IPM ? 1 : (Pr.polish >= 2 ? 0 : 1));
        constexpr int phase_hi = MODE == MODE_XO ? 1 : 2;
        for (int phase = phase_lo; phase < phase_hi; ++phase) {
        bool accepted = false;
        double bad = 0.0;
        // checkpoint: chk = the interior point stopped there (segment end), checked = it was tried this QP
        bool chk = false, checked = false;
        if (phase == 1) {
            // Start centred at the unconstrained optimum of QP(ubar) (oracle pdip): one
            // factorisation and solve without rows gives du and the state x4 of stage k there (or du = 0, see
            // below); each soft row of
            // value r gets slack max(r, 0) + START_SHIFT and elastic slack max(-r, 0) + START_SHIFT, and its
            // multiplier pair the pair's central point with lambda + nu = rho; box rows the mean row
            // complementarity.  (Round 2 started at du = 0 with s lam = 1000, lam <= rho / 2 and stopped at
            // mu <= 1e-9: C2 22 -> 20 iterations at most, C5 29 -> 27)
            // The crossover (phase 0 from the all-inactive classification) solved exactly this system: the same
            // factorisation inputs and right-hand side, in the same solve form, so its solution is the start's
            // bit for bit.  MODE_FULL / MODE_ONE still hold it in dX / dud; MODE_IPM reads it from the stage
            // cache; otherwise (no crossover ran, a warm SQP crossover, or no cache) it is recomputed here, in
            // the crossover's solve form (the K-row form wherever the split launch exists, G >= 2).
            const bool xo_start = (MODE == MODE_IPM) ? cached : (phase_lo == 0 && !(MODE == MODE_FULL && sqp > 0));
            if (live && !xo_start) {
                double Qs[10], qs[4];
                stage_cost(LITE ? cstr : S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                for (int a = 0; a < 4; ++a) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) S.QR[QRS * k + 4 * st4(a) + c] = Qs[p4(a, c)];
                    S.QH[QHS * k + st4(a)] = -qs[a];
                }
                S.QH[QHS * k + 3] = 0.0;
                S.QH[QHS * k + 5] = 0.0;
                S.Rt[2 * (k - 1)] = R0;
                S.Rt[2 * (k - 1) + 1] = R1;
                S.gh[2 * (k - 1)] = -(R0 * S.ub[2 * (k - 1)]);
                S.gh[2 * (k - 1) + 1] = -(R1 * S.ub[2 * (k - 1) + 1]);
            }
            if (!xo_start) {
                wave_sync();
                riccati_factor<NT, FAC_CF>(S, N, dt, gl);
                if constexpr (ACL && GL == 64) riccati_solve<NTR, ACL>(S, N, dt, gl);
                else riccati_solve<NTR, false>(S, N, dt, gl);
            }
            if (MODE == MODE_IPM && cached) {
                const double* xo = stc_in + stage_cache_xo(N) + 6 * (live ? k - 1 : 0);
                du0 = live ? xo[0] : 0.0;
                du1 = live ? xo[1] : 0.0;
#pragma unroll
                for (int a = 0; a < 4; ++a) x4[a] = live ? xo[2 + a] : 0.0;
            } else {
#pragma unroll
                for (int a = 0; a < 4; ++a) x4[a] = live ? S.dX[5 * k + st4(a)] : 0.0;
                du0 = live ? S.dud[2 * (k - 1)] : 0.0;
                du1 = live ? S.dud[2 * (k - 1) + 1] : 0.0;
            }
            {
                // primal point: the unconstrained optimum, or du = 0 (the warm start ubar, which already brakes
                // for obstacles ahead) when the soft rows are less violated there (sum of max(-r, 0))
                double vu = 0.0, vb = 0.0;
    #pragma unroll
                for (int j = 0; j < NR; ++j)
                    if (ron[j]) {
                        const double r = rdot(rid<OBS>(j), cf[j], x4) - bk[j];
                        vu += r < 0.0 ? -r : 0.0;
                        vb += bk[j] > 0.0 ? bk[j] : 0.0;
                    }
                vu = Q.sum(vu);
                vb = Q.sum(vb);
                if (vb < vu) {
    #pragma unroll
                    for (int a = 0; a < 4; ++a) x4[a] = 0.0;
                    du0 = 0.0;
                    du1 = 0.0;
                }
            }
            double rowc = 0.0;
    #pragma unroll
            for (int j = 0; j < NR; ++j) {
                const double r = rdot(rid<OBS>(j), cf[j], x4) - bk[j];
                const double sv = (r > 0.0 ? r : 0.0) + START_SHIFT, xi = (r < 0.0 ? -r : 0.0) + START_SHIFT;
                const double iq = rho * frcp(sv + xi);
                rs[j] = sv; rxi[j] = xi; rl[j] = xi * iq; rnu[j] = sv * iq;
                if (ron[j]) rowc += sv * rl[j];
            }
            const double mrow = Q.sum(live ? rowc : 0.0) / (double)(nsoft * N);
    #pragma unroll
            for (int j = 0; j < NBOX; ++j) {
                const double v = bsign(j) * (j < 2 ? du0 : du1) - bb[j];
                sb[j] = v > 1.0 ? v : 1.0;
                lb[j] = mrow * frcp(sb[j]);
            }
            wave_sync();
        }
        for (;;) {      // segments: interior point (to convergence or the checkpoint), polish; resume if needed
        if (phase == 1) {
        PROF(0)
        for (int iter = it; iter < Pr.max_iter; ++iter) {
            PROF(1)
            // the row bounds are loop-invariant; keeping them opaque stops the compiler from hoisting
            // everything derived from them out of this loop (it would stay live in registers and spill)
#ifndef MPC_NO_BK_OPAQUE
#pragma unroll
            for (int j = 0; j < NR; ++j) asm volatile("" : "+v"(bk[j]));
#pragma unroll
            for (int j = 0; j < NBOX; ++j) asm volatile("" : "+v"(bb[j]));
#endif
            // -- stage-parallel residuals ------------------------------------------------------
            double rpmax = 0.0, rxmax = 0.0, comp = 0.0;
            double ya[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < NR; ++j) {
                if (!rowon[j]) continue;
                const double rp = rdot(rid<OBS>(j), cf[j], x4) + rxi[j] - rs[j] - bk[j];
                const double rx = rho - rl[j] - rnu[j];
#pragma unroll
                for (int a = 0; a < 4; ++a) ya[a] = fma(-rl[j], cf[j][a], ya[a]);
                rpmax = vmaxabs(rpmax, rp);
                rxmax = vmaxabs(rxmax, rx);
                comp = fma(rs[j], rl[j], fma(rxi[j], rnu[j], comp));
            }
            // dual-residual stage terms of stage k / control k-1: yc (cost), zc (control cost), za (box
            // multipliers); ya (row multipliers) accumulated above
            auto dual_terms = [&](double yc[4], double zc[2], double za[2]) {
                double Qs[10], qs[4];
                stage_cost(LITE ? cstr : S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    double acc = qs[a];
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc = fma(Qs[p4(a, c)], x4[c], acc);
                    yc[a] = acc;
                }
                zc[0] = fma(R0, du0, R0 * S.ub[2 * (k - 1)]);
                zc[1] = fma(R1, du1, R1 * S.ub[2 * (k - 1) + 1]);
                za[0] = lb[1] - lb[0];
                za[1] = lb[3] - lb[2];
            };
            if (live) {
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    const double rp = bsign(j) * (j < 2 ? du0 : du1) - sb[j] - bb[j];
                    rpmax = vmaxabs(rpmax, rp);
                    comp = fma(sb[j], lb[j], comp);
                }
                double yc[4], zc[2], za[2];
                dual_terms(yc, zc, za);
#pragma unroll
                for (int a = 0; a < 4; ++a) S.ys[4 * k + a] = yc[a] + ya[a];
                S.zs[2 * (k - 1)] = zc[0] + za[0];
                S.zs[2 * (k - 1) + 1] = zc[1] + za[1];
            }
            rpmax = Q.max(live ? rpmax : 0.0);
            rxmax = Q.max(live ? rxmax : 0.0);
            comp = Q.sum(live ? comp : 0.0);
            wave_sync();
            PROF(2)
            mu = comp / Mtot;
            if (!(mu == mu)) { st_here = MPC_NUMERICAL; it = iter; break; }
            if (mu <= Pr.tol_mu && rpmax <= 10.0 * Pr.tol * (1.0 + bscale) && rxmax <= Pr.tol * rho) {
                // converged: the polish then makes the active set exact;
                // the dual residual carries O(eps/mu) multiplier noise, required to 1e4*tol.  Its
                // adjoint recursion is only run here, once per solve.
                if (live) {
                    double yc[4], zc[2], za[2];
                    dual_terms(yc, zc, za);
#pragma unroll
                    for (int a = 0; a < 4; ++a) {
                        S.QR[QRS * k + DQ_YC + a] = yc[a];
                        S.QR[QRS * k + DQ_YA + a] = ya[a];
                    }
                    S.QR[QRS * (k - 1) + DQ_ZC] = zc[0];
                    S.QR[QRS * (k - 1) + DQ_ZC + 1] = zc[1];
                    S.QR[QRS * (k - 1) + DQ_ZA] = za[0];
                    S.QR[QRS * (k - 1) + DQ_ZA + 1] = za[1];
                }
                wave_sync();
                double rdmax, sd;
                dual_norms(S, N, dt, rdmax, sd);
                PROF(3)
                st_here = rdmax <= 1e4 * Pr.tol * (1.0 + sd) ? MPC_OK : MPC_NUMERICAL;
                it = iter;
                break;
            }
            if (Pr.polish && !checked && mu <= Pr.mu_check) {
                double tie = 0.0;
#pragma unroll
                for (int j = 0; j < NR; ++j)
                    if (rowon[j] && (!(rs[j] > CHECK_SEP * rl[j] || rl[j] > CHECK_SEP * rs[j]) ||
                                     !(rxi[j] > CHECK_SEP * rnu[j] || rnu[j] > CHECK_SEP * rxi[j])))
                        tie = 1.0;
#pragma unroll
                for (int j = 0; j < NBOX; ++j)
                    if (!(sb[j] > CHECK_SEP * lb[j] || lb[j] > CHECK_SEP * sb[j])) tie = 1.0;
                if (Q.max(live ? tie : 0.0) == 0.0) {
                    chk = true;
                    it = iter;
                    break;
                }
            }
            // -- barrier weights, augmented stage Hessians ---------------------------------------
            double il[NR], inu[NR], wv[NR], ilb[NBOX], wb[NBOX];
            {
                double Qp[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    il[j] = frcp(rl[j]);
                    inu[j] = frcp(rnu[j]);
                    wv[j] = rowon[j] ? frcp(fma(rs[j], il[j], rxi[j] * inu[j])) : 0.0;   // 1/d
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int c = a; c < 4; ++c)
                            if (row_nz(rid<OBS>(j), a) && row_nz(rid<OBS>(j), c))
                                Qp[p4(a, c)] = fma(wv[j] * cf[j][a], cf[j][c], Qp[p4(a, c)]);
                }
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    ilb[j] = frcp(lb[j]);
                    wb[j] = live ? lb[j] * frcp(sb[j]) : 0.0;
                }
                if (live) {
                    double Qs[10], qs[4];
                    stage_cost(LITE ? cstr : S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int c = 0; c < 4; ++c) S.QR[QRS * k + 4 * st4(a) + c] = Qp[p4(a, c)] + Qs[p4(a, c)];
                    S.Rt[2 * (k - 1)] = R0 + (wb[0] + wb[1]);
                    S.Rt[2 * (k - 1) + 1] = R1 + (wb[2] + wb[3]);
                }
            }
            wave_sync();
            PROF(4)
            riccati_factor<NT, FAC_CF>(S, N, dt, gl);
            PROF(5)
            // -- predictor, corrector (and, if needed, centred) solves ---------------------------------
            double p4v[NR], p5v[NR], pbv[NBOX];
#pragma unroll
            for (int j = 0; j < NR; ++j) { p4v[j] = 0.0; p5v[j] = 0.0; }
#pragma unroll
            for (int j = 0; j < NBOX; ++j) pbv[j] = 0.0;
            double sig = 0.0;
            bool breakdown = false;
            // The passes (predictor, corrector, centred direction) are unrolled in the N = 20 kernels: no
            // loop-carried copies of the predictor products at the back edge (C2 -3%).  The runtime-horizon
            // kernels keep the loop (unrolled, C4 +2%, C5 +4%): their pass count is opaque, so the full-unroll
            // request does not apply there (built with -Wno-pass-failed).
            int npass = 3;
            if constexpr (NT == 0) asm volatile("" : "+s"(npass));
#pragma unroll
            for (int pass = 0; pass < npass; ++pass) {
                // pass 0: affine predictor; 1: Mehrotra corrector; 2: plain centred direction, taken when
                // the corrector would not reduce complementarity (oracle: comp_after > comp)
                const double smu = (pass >= 1) ? sig * mu : 0.0;
                const double cw = (pass == 1) ? 1.0 : 0.0;     // weight of the second-order term
                // reduced right-hand side per row, scaled by 1/d: wr = rh / d  (newton() of the oracle).
                // Recomputed after the solve rather than held live across it (register pressure).
                auto row_wr = [&](int j) {
                    const double r4 = fma(cw, p4v[j], fma(rs[j], rl[j], -smu));
                    const double r5 = fma(cw, p5v[j], fma(rxi[j], rnu[j], -smu));
                    const double rp = rdot(rid<OBS>(j), cf[j], x4) + rxi[j] - rs[j] - bk[j];
                    const double rx = rho - rl[j] - rnu[j];
                    const double rh = -rp - r4 * il[j] + fma(rxi[j], rx, r5) * inu[j];
                    return rowon[j] ? rh * wv[j] : 0.0;
                };
                auto box_wr = [&](int j) {
                    const double r4 = fma(cw, pbv[j], fma(sb[j], lb[j], -smu));
                    const double rp = bsign(j) * (j < 2 ? du0 : du1) - sb[j] - bb[j];
                    return (-rp - r4 * ilb[j]) * wb[j];
                };
                double wr[NR], wrb[NBOX];     // kept live by the obstacle-free variant only
                {
                    double q4[4] = {0, 0, 0, 0}, g0 = 0.0, g1 = 0.0;
#pragma unroll
                    for (int j = 0; j < NR; ++j) {
                        double w;
                        if constexpr (WRC) {
                            w = row_wr(j);
                        } else {
                            const double r4 = fma(cw, p4v[j], fma(rs[j], rl[j], -smu));
                            const double r5 = fma(cw, p5v[j], fma(rxi[j], rnu[j], -smu));
                            const double rp = rdot(rid<OBS>(j), cf[j], x4) + rxi[j] - rs[j] - bk[j];
                            const double rx = rho - rl[j] - rnu[j];
                            const double rh = -rp - r4 * il[j] + fma(rxi[j], rx, r5) * inu[j];
                            wr[j] = rowon[j] ? rh * wv[j] : 0.0;
                            w = wr[j];
                        }
#pragma unroll
                        for (int a = 0; a < 4; ++a)
                            if (row_nz(rid<OBS>(j), a)) q4[a] = fma(cf[j][a], w, q4[a]);
                    }
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) {
                        double w;
                        if constexpr (WRC) {
                            w = box_wr(j);
                        } else {
                            const double r4 = fma(cw, pbv[j], fma(sb[j], lb[j], -smu));
                            const double rp = bsign(j) * (j < 2 ? du0 : du1) - sb[j] - bb[j];
                            wrb[j] = (-rp - r4 * ilb[j]) * wb[j];
                            w = wrb[j];
                        }
                        if (j < 2) g0 += bsign(j) * w; else g1 += bsign(j) * w;
                    }
                    if (live) {
                        // the dual-residual terms are read before any write (see ac_rows)
                        double ysv[4], zs0, zs1;
                        ld2(S.ys + 4 * k, ysv[0], ysv[1]);
                        ld2(S.ys + 4 * k + 2, ysv[2], ysv[3]);
                        ld2(S.zs + 2 * (k - 1), zs0, zs1);
#pragma unroll
                        for (int a = 0; a < 4; ++a) S.QH[QHS * k + st4(a)] = q4[a] - ysv[a];
                        S.QH[QHS * k + 3] = 0.0;
                        S.QH[QHS * k + 5] = 0.0;
                        *reinterpret_cast<double2*>(S.gh + 2 * (k - 1)) = make_double2(g0 - zs0, g1 - zs1);
                    }
                }
                wave_sync();
                PROF(6)
                riccati_solve<NTR, ACL>(S, N, dt, gl);
                PROF(7)
                // row directions and the largest feasible step
                double dx4[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) dx4[a] = live ? S.dX[5 * k + st4(a)] : 0.0;
                const double dd0 = live ? S.dud[2 * (k - 1)] : 0.0, dd1 = live ? S.dud[2 * (k - 1) + 1] : 0.0;
                double dsv[NR], dlv[NR], dxv[NR], dnv[NR], dsb[NBOX], dlb[NBOX];
                // ratio tests as rmax = max(1, max_j -d_j / x_j); the step to the boundary is 1 / rmax.
                // The reciprocals of lam, nu (rows) and lam (boxes) are the barrier weights' il, inu,
                // ilb; s, xi (rows) and s (boxes) take the approximate v_rcp_f64 (enough for a step
                // length).  A product and a max per term (no compare, select or NaN canonicalisation).
                double rmax = 1.0;
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    const double r4 = fma(cw, p4v[j], fma(rs[j], rl[j], -smu));
                    const double r5 = fma(cw, p5v[j], fma(rxi[j], rnu[j], -smu));
                    const double rx = rho - rl[j] - rnu[j];
                    double wj;
                    if constexpr (WRC) wj = row_wr(j); else wj = wr[j];
                    const double dl = fma(-wv[j], rdot(rid<OBS>(j), cf[j], dx4), wj);
                    const double ds = -fma(rs[j], dl, r4) * il[j];
                    const double dn = rx - dl;
                    const double dxi = -fma(rxi[j], dn, r5) * inu[j];
                    const bool on = rowon[j];
                    dsv[j] = on ? ds : 0.0;
                    dlv[j] = on ? dl : 0.0;
                    dxv[j] = on ? dxi : 0.0;
                    dnv[j] = on ? dn : 0.0;
                    rmax = vmax(rmax, -dsv[j] * __builtin_amdgcn_rcp(rs[j]));
                    rmax = vmax(rmax, -dlv[j] * il[j]);
                    rmax = vmax(rmax, -dxv[j] * __builtin_amdgcn_rcp(rxi[j]));
                    rmax = vmax(rmax, -dnv[j] * inu[j]);
                }
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    const double r4 = fma(cw, pbv[j], fma(sb[j], lb[j], -smu));
                    double wj;
                    if constexpr (WRC) wj = box_wr(j); else wj = wrb[j];
                    const double dl = fma(-wb[j] * bsign(j), (j < 2 ? dd0 : dd1), wj);
                    const double ds = -fma(sb[j], dl, r4) * ilb[j];
                    dsb[j] = ds;
                    dlb[j] = dl;
                    rmax = vmax(rmax, -dsb[j] * __builtin_amdgcn_rcp(sb[j]));
                    rmax = vmax(rmax, -dlb[j] * ilb[j]);
                }
                const double amax = __builtin_amdgcn_rcp(Q.max(live ? rmax : 1.0));
                // complementarity after the step (pass 0: at the full affine step length)
                const double a_try = (pass == 0) ? amax : fmin(1.0, TAU * amax);
                double ca = 0.0;
#pragma unroll
                for (int j = 0; j < NR; ++j)
                    if (rowon[j])
                        ca += fma(a_try, dsv[j], rs[j]) * fma(a_try, dlv[j], rl[j]) +
                              fma(a_try, dxv[j], rxi[j]) * fma(a_try, dnv[j], rnu[j]);
#pragma unroll
                for (int j = 0; j < NBOX; ++j) ca += fma(a_try, dsb[j], sb[j]) * fma(a_try, dlb[j], lb[j]);
                if (!(fabs(dd0) < INFINITY && fabs(dd1) < INFINITY)) ca = NAN;   // breakdown guard input
                ca = Q.sum(live ? ca : 0.0);
                PROF(11)
                if (pass == 0) {
                    const double r = ca / comp;
                    sig = r * r * r;
#pragma unroll
                    for (int j = 0; j < NR; ++j) { p4v[j] = dsv[j] * dlv[j]; p5v[j] = dxv[j] * dnv[j]; }
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) pbv[j] = dsb[j] * dlb[j];
                    continue;
                }
                if (pass == 1 && ca > comp) continue;     // safeguard: take the centred direction
                if (!(ca < INFINITY)) {                    // breakdown guard (oracle pdip): the step is not
                    breakdown = true;                      // taken, the current iterate goes to the polish
                    break;
                }
                const double alpha = a_try;
                stall = (mu < 1e-6 && ca > 0.9 * comp) ? stall + 1 : 0;
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    rs[j] = fma(alpha, dsv[j], rs[j]);
                    rl[j] = fma(alpha, dlv[j], rl[j]);
                    rxi[j] = fma(alpha, dxv[j], rxi[j]);
                    rnu[j] = fma(alpha, dnv[j], rnu[j]);
                }
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    sb[j] = fma(alpha, dsb[j], sb[j]);
                    lb[j] = fma(alpha, dlb[j], lb[j]);
                }
                du0 = fma(alpha, dd0, du0);
                du1 = fma(alpha, dd1, du1);
#pragma unroll
                for (int a = 0; a < 4; ++a) x4[a] = fma(alpha, dx4[a], x4[a]);
                break;
            }
            wave_sync();
            PROF(8)
            it = iter + 1;
            if (stall >= 5 || breakdown) { st_here = MPC_NUMERICAL; break; }
        }
        if (!chk) {
        total_it += it;
        // NaN guard and the infeasibility flag
        if (live) bad = (du0 == du0 && du1 == du1) ? 0.0 : 1.0;
        bad = Q.max(bad);
        if (bad > 0.0) {
            st_here = MPC_NUMERICAL;
            du0 = 0.0;
            du1 = 0.0;
        } else if (st_here == MPC_OK) {
            double inf = 0.0;
#pragma unroll
            for (int j = 0; j < NR; ++j)
                if (ron[j] && rxi[j] > 1e-6 * (1.0 + fabs(bk[j]))) inf = 1.0;
            if (Q.max(inf) > 0.0) st_here = MPC_INFEASIBLE;
        }
        }
        wave_sync();
        }   // phase 1: interior point

        // ---- active-set polish (oracle polish()) ----------------------------
        PROF(8)
        if (Pr.polish && bad == 0.0) {
            // opaque copies of the row bounds (see the interior-point loop): nothing the polish derives
            // from them is hoisted into long-lived registers
            double bkp[NR], bbp[NBOX];
#pragma unroll
            for (int j = 0; j < NR; ++j) { bkp[j] = bk[j]; asm volatile("" : "+v"(bkp[j])); }
#pragma unroll
            for (int j = 0; j < NBOX; ++j) { bbp[j] = bb[j]; asm volatile("" : "+v"(bbp[j])); }
            // class per row: 0 inactive, 1 active (equality), 2 violated (multiplier fixed at rho)
            int cls[NR], clb[NBOX];
#pragma unroll
            for (int j = 0; j < NR; ++j) cls[j] = !ron[j] ? 0 : (rxi[j] > rnu[j] ? 2 : (rl[j] > rs[j] ? 1 : 0));
#pragma unroll
            for (int j = 0; j < NBOX; ++j) clb[j] = (live && lb[j] > sb[j]) ? 1 : 0;
            if (MODE == MODE_FULL && phase == 0 && sqp > 0) {
                // re-linearisation: the crossover starts from the previous QP's classification
#pragma unroll
                for (int j = 0; j < NR; ++j) cls[j] = ron[j] ? (wcls >> (2 * j)) & 3 : 0;
#pragma unroll
                for (int j = 0; j < NBOX; ++j) clb[j] = live ? (wcls >> (2 * NR + j)) & 1 : 0;
            }
            // the interior-point iterate (du, x4) is the start of every round and the fallback
            double pu0 = du0, pu1 = du1;
            double nviol_acc = 0.0;
            const int rounds = phase == 0 ? XO_ROUNDS : (chk ? CHECK_ROUNDS : POLISH_ROUNDS);
            for (int round = 0; round < rounds; ++round) {
                double tl[NR], tlb[NBOX];
#pragma unroll
                for (int j = 0; j < NR; ++j) tl[j] = rl[j];
#pragma unroll
                for (int j = 0; j < NBOX; ++j) tlb[j] = lb[j];
                if (live) {
                    double Qp[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                    for (int j = 0; j < NR; ++j) {
                        const double w = cls[j] == 1 ? 1.0 / POLISH_DELTA : 0.0;
#pragma unroll
                        for (int a = 0; a < 4; ++a)
#pragma unroll
                            for (int c = a; c < 4; ++c)
                                if (row_nz(rid<OBS>(j), a) && row_nz(rid<OBS>(j), c))
                                    Qp[p4(a, c)] = fma(w * cf[j][a], cf[j][c], Qp[p4(a, c)]);
                    }
                    double Qs[10], qs[4];
                    stage_cost(LITE ? cstr : S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int c = 0; c < 4; ++c) S.QR[QRS * k + 4 * st4(a) + c] = Qp[p4(a, c)] + Qs[p4(a, c)];
                    S.Rt[2 * (k - 1)] = R0 + (clb[0] + clb[1]) * (1.0 / POLISH_DELTA);
                    S.Rt[2 * (k - 1) + 1] = R1 + (clb[2] + clb[3]) * (1.0 / POLISH_DELTA);
                }
                wave_sync();
                riccati_factor<NT, FAC_CF>(S, N, dt, gl);
                double xp[4] = {x4[0], x4[1], x4[2], x4[3]};
                pu0 = du0;
                pu1 = du1;
                // the crossover from the all-inactive classification solves the unconstrained LQR: the first solve
                // is its exact optimum (no active-row penalties to refine), so it runs one solve, not
                // POLISH_REFINE (oracle polish_from, host backend active_set)
                const int nref = (phase == 0 && !(MODE == MODE_FULL && sqp > 0)) ? 1 : POLISH_REFINE;
#pragma unroll 1
                for (int r = 0; r < nref; ++r) {
                    // exact KKT residual of the equality QP -> LQR right-hand side
                    double r2[NR], r2b[NBOX];
#pragma unroll
                    for (int j = 0; j < NR; ++j) r2[j] = (cls[j] == 1) ? bkp[j] - rdot(rid<OBS>(j), cf[j], xp) : 0.0;
#pragma unroll
                    for (int j = 0; j < NBOX; ++j) r2b[j] = (clb[j] == 1) ? bbp[j] - bsign(j) * (j < 2 ? pu0 : pu1) : 0.0;
                    if (live) {
                        double q4[4] = {0, 0, 0, 0}, g0 = 0.0, g1 = 0.0;
#pragma unroll
                        for (int j = 0; j < NR; ++j) {
                            const double wgt = (cls[j] == 2) ? rho : (cls[j] == 1 ? tl[j] + r2[j] * (1.0 / POLISH_DELTA) : 0.0);
#pragma unroll
                            for (int a = 0; a < 4; ++a)
                                if (row_nz(rid<OBS>(j), a)) q4[a] = fma(cf[j][a], wgt, q4[a]);
                        }
#pragma unroll
                        for (int j = 0; j < NBOX; ++j) {
                            const double v = (clb[j] == 1) ? bsign(j) * (tlb[j] + r2b[j] * (1.0 / POLISH_DELTA)) : 0.0;
                            if (j < 2) g0 += v; else g1 += v;
                        }
                        double Qs[10], qs[4], ub0, ub1;
                        stage_cost(LITE ? cstr : S.cst + 6 * k, Pr.w_d, Pr.w_o, Pr.w_v, Qs, qs);
                        ld2(S.ub + 2 * (k - 1), ub0, ub1);        // reads before the writes (see ac_rows)
#pragma unroll
                        for (int a = 0; a < 4; ++a) {
                            double acc = qs[a];
#pragma unroll
                            for (int c = 0; c < 4; ++c) acc = fma(Qs[p4(a, c)], xp[c], acc);
                            S.QH[QHS * k + st4(a)] = q4[a] - acc;
                        }
                        S.QH[QHS * k + 3] = 0.0;
                        S.QH[QHS * k + 5] = 0.0;
                        *reinterpret_cast<double2*>(S.gh + 2 * (k - 1)) =
                            make_double2(g0 - fma(R0, pu0, R0 * ub0), g1 - fma(R1, pu1, R1 * ub1));
                    }
                    wave_sync();
                    // the crossover (phase 0) solves in K-row form wherever the two-phase launch exists
                    // (G >= 2): the MODE_XO launch has no AC rows (lite LDS layout), and MODE_FULL must give
                    // bit-identical results.  GL = 64 (G = 1) is never split and keeps the AC rows (the
                    // K-row crossover cost C5 4%).
                    if (ACL && (phase == 1 || GL == 64)) riccati_solve<NTR, ACL>(S, N, dt, gl);
                    else riccati_solve<NTR, false>(S, N, dt, gl);
                    {
                        double dx4[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) dx4[a] = live ? S.dX[5 * k + st4(a)] : 0.0;
#pragma unroll
                        for (int j = 0; j < NR; ++j)
                            if (cls[j] == 1) tl[j] += (r2[j] - rdot(rid<OBS>(j), cf[j], dx4)) * (1.0 / POLISH_DELTA);
                        const double dd0 = live ? S.dud[2 * (k - 1)] : 0.0, dd1 = live ? S.dud[2 * (k - 1) + 1] : 0.0;
#pragma unroll
                        for (int j = 0; j < NBOX; ++j)
                            if (clb[j] == 1) tlb[j] += (r2b[j] - bsign(j) * (j < 2 ? dd0 : dd1)) * (1.0 / POLISH_DELTA);
#pragma unroll
                        for (int a = 0; a < 4; ++a) xp[a] += dx4[a];
                        pu0 += dd0;
                        pu1 += dd1;
                    }
                    wave_sync();
                }
                // acceptance: KKT consistency; otherwise flip every offending row and retry
                double lmax = 1.0;
#pragma unroll
                for (int j = 0; j < NR; ++j)
                    if (cls[j] == 1) lmax = vmaxabs(lmax, tl[j]);
#pragma unroll
                for (int j = 0; j < NBOX; ++j)
                    if (clb[j] == 1) lmax = vmaxabs(lmax, tlb[j]);
                lmax = Q.max(lmax);
                // a row is offending when its KKT condition fails (oracle polish_from: bad > 0); only the
                // flags matter, so no division by the scales (each IEEE division is ~10 instructions)
                double worst = 0.0, nviol = 0.0, finite = 1.0;
                bool flip[NR], flipb[NBOX];
                if (live && (!(pu0 == pu0) || !(pu1 == pu1))) finite = 0.0;
#pragma unroll
                for (int j = 0; j < NR; ++j) {
                    flip[j] = false;
                    if (!ron[j]) continue;
                    const double bsc = 1.0 + fabs(bkp[j]);
                    const double r = rdot(rid<OBS>(j), cf[j], xp) - bkp[j];
                    bool badv;
                    if (cls[j] == 1) {
                        badv = tl[j] < -1e-9 * lmax || tl[j] > rho * (1.0 + 1e-9) || fabs(r) > 1e-7 * bsc;
                    } else if (cls[j] == 2) {
                        badv = r > 1e-9 * bsc;
                        if (r < -1e-6 * bsc) nviol += 1.0;
                    } else {
                        badv = r < -1e-9 * bsc;
                    }
                    if (badv) worst = 1.0;
                    flip[j] = badv;
                }
#pragma unroll
                for (int j = 0; j < NBOX; ++j) {
                    flipb[j] = false;
                    if (!live) continue;
                    const double bsc = 1.0 + fabs(bbp[j]);
                    const double r = bsign(j) * (j < 2 ? pu0 : pu1) - bbp[j];
                    const bool badv = clb[j] == 1 ? (tlb[j] < -1e-9 * lmax || fabs(r) > 1e-7 * bsc) : r < -1e-9 * bsc;
                    if (badv) worst = 1.0;
                    flipb[j] = badv;
                }
                worst = Q.max(worst);
                nviol = Q.sum(nviol);
                finite = Q.min(finite);
                if (finite == 0.0) break;
                if (worst == 0.0) {
                    accepted = true;
                    nviol_acc = nviol;
                    break;
                }
#pragma unroll
                for (int j = 0; j < NR; ++j)
                    if (flip[j]) cls[j] = (cls[j] == 1) ? (tl[j] > rho ? 2 : 0) : 1;
#pragma unroll
                for (int j = 0; j < NBOX; ++j)
                    if (flipb[j]) clb[j] = 1 - clb[j];
                wave_sync();
            }
            if (MODE == MODE_FULL && nsqp > 1) {
                wcls = 0;
#pragma unroll
                for (int j = 0; j < NR; ++j) wcls |= cls[j] << (2 * j);
#pragma unroll
                for (int j = 0; j < NBOX; ++j) wcls |= clb[j] << (2 * NR + j);
            }
            if (accepted) {
                du0 = pu0;
                du1 = pu1;
                st_here = nviol_acc > 0.0 ? MPC_INFEASIBLE : MPC_OK;
            }
            wave_sync();
        }
        if (chk) {
            if (!accepted) {          // not certified: the interior point continues from the unchanged iterate
                chk = false;
                checked = true;
                continue;
            }
            total_it += it;
        }
        break;
        }   // segments
        if (phase == 0) xo_ok = accepted;
        if (accepted || phase == 1) break;
        }   // phases
        status = st_here;
        double ua0 = 0.0, ua1 = 0.0;       // this QP's linearisation point: U one QP back
        if (live) {
            ua0 = S.ub[2 * (k - 1)];
            ua1 = S.ub[2 * (k - 1) + 1];
            S.ub[2 * (k - 1)] = ua0 + du0;
            S.ub[2 * (k - 1) + 1] = ua1 + du1;
        }
        wave_sync();
        // SQP: stop once the re-linearised QP no longer moves U, on a 2-cycle, or after SQP_INF_STREAK elastic
        // QPs in a row (oracle orc_solve; all group-uniform)
        if (nsqp > 1) {
            const double stp = Q.max(live ? vmaxabs(fabs(du0), du1) : 0.0);
            const double b2 = Q.max(live ? vmaxabs(fabs((ua0 + du0) - pb0), (ua1 + du1) - pb1) : 0.0);
            pb0 = ua0;
            pb1 = ua1;
            ninf = status == MPC_INFEASIBLE ? ninf + 1 : 0;
            if (stp <= Pr.sqp_tol) { sqp_conv = true; break; }
            if (Pr.sqp_tol > 0.0 && ((sqp >= 2 && b2 <= SQP_CYCLE_REL * stp) || ninf >= SQP_INF_STREAK)) break;
        }
    }

    if (MODE == MODE_FULL && nsqp > 1 && Pr.sqp_tol > 0.0 && !sqp_conv) status |= MPC_SQP_UNCONVERGED;

    // ---- K5: outputs: U*, u0, predict(x0, U*) ----------------------------------------------
    PROF(9)
    // The instance index and x0 are recomputed / re-read here (from the lane id, the work list and an
    // opaque index that defeats CSE with the first load) rather than held in registers across the
    // interior point, where they would be spilled to scratch.
    int ln2 = __lane_id();
    asm volatile("" : "+v"(ln2));
    const int grp2 = ln2 / GL;
    {
        if (MODE == MODE_IPM) {
            const int cnt = *wcount;
            const int slot = blockIdx.x * G + grp2;
            bvalid = slot < cnt;
            b = wlist[bvalid ? slot : cnt - 1];
        } else {
            b = blockIdx.x * G + grp2;
            bvalid = b < B;
            if (!bvalid) b = B - 1;
        }
#pragma unroll
        for (int j = 0; j < 5; ++j) x0[j] = x0g[5 * (size_t)b + j];
    }
    predict_grp(tab, N, dt, x0, S.ub, S.Xr, S.kap, gl);
    if (MODE == MODE_XO && !xo_ok) {
        // not certified: defer to the MODE_IPM launch (group-uniform); S.ub is still the warm start and
        // S.Xr its rollout (a failed crossover leaves no state behind), which the stage cache keeps
        int slot = 0;
        if (bvalid && gl == 0) {
            if (Pr.dbg & 1) {
                slot = b;
            } else {
                slot = atomicAdd(wcount, 1);
                wlist[slot] = b;
            }
        }
        slot = __shfl(slot, grp2 * GL, WAVE);
        if (bvalid && stc) {
            double* o = stc + (size_t)slot * stage_cache_doubles(N);
            if (gl < N) {
                o[2 * gl] = S.ub[2 * gl];
                o[2 * gl + 1] = S.ub[2 * gl + 1];
            }
            for (int i = gl; i < 5 * NP; i += GL) o[2 * N + i] = S.Xr[i];
            if (LKC && gl <= N) {
                double2* lk = reinterpret_cast<double2*>(o + stage_cache_lk(N) + 8 * gl);
                lk[0] = make_double2(refk[1], refk[2]);
                lk[1] = make_double2(refk[3], refk[4]);
                lk[2] = make_double2(slk[0], slk[1]);
                lk[3] = make_double2(slk[2], slk[3]);
            }
            // the crossover's solve (the interior point's start): still in dud / dX (the epilogue's rollout
            // writes Xr and kap only)
            if (gl < N) {
                double* xo = o + stage_cache_xo(N) + 6 * gl;
                xo[0] = S.dud[2 * gl];
                xo[1] = S.dud[2 * gl + 1];
#pragma unroll
                for (int a = 0; a < 4; ++a) xo[2 + a] = S.dX[5 * (gl + 1) + st4(a)];
            }
        }
    } else if (bvalid) {
        // one 16-B store per lane (full cache lines, not two half-filled strided stores) when the caller's
        // buffers allow it; 8-B aligned views (e.g. a tensor slice at an odd offset) take two 8-B stores
        const bool a16 = ((((uintptr_t)Ug) | ((uintptr_t)u0g)) & 15) == 0;
        if (gl < N && Ug) {
            double* o = Ug + (size_t)b * 2 * N + 2 * gl;
            if (a16) {
                *reinterpret_cast<double2*>(o) = make_double2(S.ub[2 * gl], S.ub[2 * gl + 1]);
            } else {
                o[0] = S.ub[2 * gl];
                o[1] = S.ub[2 * gl + 1];
            }
        }
        if (Xg)
            for (int i = gl; i < 5 * NP; i += GL) Xg[(size_t)b * 5 * NP + i] = S.Xr[i];
        if (gl == 0) {
            if (u0g) {
                double* o = u0g + 2 * (size_t)b;
                if (a16) {
                    *reinterpret_cast<double2*>(o) = make_double2(S.ub[0], S.ub[1]);
                } else {
                    o[0] = S.ub[0];
                    o[1] = S.ub[1];
                }
            }
            if (statusg) statusg[b] = status;
            if (itersg) itersg[b] = total_it;
        }
    }
    PROF(10)
    PROF_END
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
// batched closed loop: run_simulation, trajectory_tracking.py:377-443, per ego,
// with the ObstaclesFSM of :266-374.  One thread per ego for the FSM and the plant; the solve in
// between is the batched solver kernel.  Same arithmetic order as the reference (numpy), so a
// closed loop on the device reproduces the host loop bit for bit.
// ------------------------------------------------------------------------------------------
struct ClState {
    double* x;          // [B][5]    current state
    double* obs;        // [B][2][2] obstacle slab of this step (car first, then the light: :341-358)
    int* nobs;          // [B]
    int* active;        // [B]       still inside the loop condition s <= s_stop (:395)
    double* obs_s;      // [B]       dynamic obstacle position
    double* tl_timer;   // [B]
    int* fsm_flags;     // [B][4]    obs_active, obs_has_triggered, tl_green, tl_waiting
    int* n_active;      // [1]
    // the solver runs on the egos still in the loop only: alist [B] holds their ids (increasing, rebuilt by
    // cl_compact_kernel whenever egos have left), and the solve reads / writes the packed slabs below
    int* alist;         // [B]
    int* n_list;        // [1]
    double* xa;         // [B][5]
    double* obsa;       // [B][2][2]
    int* nobsa;         // [B]
    double* u0a;        // [B][2]
    int* sta;           // [B]
};

// ids of the egos still in the loop, in increasing order (deterministic): one workgroup of 1024 lanes,
// wave ballots and a scan of the 16 wave counts per chunk
__global__ void __launch_bounds__(1024) cl_compact_kernel(int B, ClState C) {
    __shared__ int wsum[16];
    __shared__ int base;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c0 = 0; c0 < B; c0 += 1024) {
        const int e = c0 + threadIdx.x;
        const bool f = e < B && C.active[e];
        const unsigned long long m = __ballot(f);
        const int pre = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int i = 0; i < w; ++i) off += wsum[i];
        if (f) C.alist[off + pre] = e;
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int i = 0; i < 16; ++i) t += wsum[i];
            base += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *C.n_list = base;
}

// packs the listed egos' state and obstacle slab for the solve (slot i <- ego alist[i])
__global__ void cl_gather_kernel(int nl, ClState C) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const int e = C.alist[i];
    for (int j = 0; j < 5; ++j) C.xa[5 * (size_t)i + j] = C.x[5 * (size_t)e + j];
    for (int j = 0; j < 4; ++j) C.obsa[4 * (size_t)i + j] = C.obs[4 * (size_t)e + j];
    C.nobsa[i] = C.nobs[e];
}

// ObstaclesFSM.update(dt, s, v) (trajectory_tracking.py:330-374) for every active ego
__global__ void cl_fsm_kernel(int B, mpc_fsm F, double dt, ClState C, double* hist_obs_s, int* hist_tl, int step,
                              int max_steps) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    if (!C.active[b]) { C.nobs[b] = 0; return; }
    const double s = C.x[5 * (size_t)b], v = C.x[5 * (size_t)b + 4];
    int* fl = C.fsm_flags + 4 * (size_t)b;
    double* o = C.obs + 4 * (size_t)b;
    int n = 0;
    double car_s = NAN;
    if (F.dynamic_obstacle) {
        if (!fl[1] && s >= F.obs_trigger_s) { fl[1] = 1; fl[0] = 1; }
        if (fl[0]) {
            const double os = C.obs_s[b] + F.obs_v * dt;
            C.obs_s[b] = os;
            if (os > F.obs_end_s) {
                fl[0] = 0;
            } else {
                o[0] = os;
                o[1] = F.obs_v;
                n = 1;
                car_s = os;
            }
        }
    }
    if (F.traffic_light && !fl[2]) {
        const double dist = F.tl_pos - s;
        if (0.0 < dist && dist < F.tl_trigger_s) {
            o[2 * n] = F.tl_pos;
            o[2 * n + 1] = 0.0;
            ++n;
            if (v < 0.1 && dist < 10.0) fl[3] = 1;
        }
        if (fl[3]) {
            C.tl_timer[b] += dt;
            if (C.tl_timer[b] >= F.tl_stop_duration) { fl[2] = 1; fl[3] = 0; }
        }
    }
    C.nobs[b] = n;
    if (hist_obs_s) hist_obs_s[(size_t)b * max_steps + step] = car_s;
    if (hist_tl) hist_tl[(size_t)b * max_steps + step] = fl[2];
}

// plant step x <- x + dt * dynamics(x, u0, k_ref(x_s)) (:403-406) and the histories (:412-421), for the
// listed egos (slot i: ego alist[i], its control at u0a[i])
__global__ void cl_plant_kernel(DevTable tab, int nl, double dt, ClState C, double s_stop, double* hist_x,
                                double* hist_u, int* hist_status, int* n_steps, int step, int max_steps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const int b = C.alist[i];
    if (!C.active[b]) return;
    double x[5], st[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) x[j] = C.x[5 * (size_t)b + j];
    const double u1 = C.u0a[2 * (size_t)i], u2 = C.u0a[2 * (size_t)i + 1];
    get_state(tab, x[0], st, nullptr);
    const double xd[5] = {x[4], x[4] * x[2], x[4] * (x[3] - st[3]), u1, u2};
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        x[j] = x[j] + dt * xd[j];
        C.x[5 * (size_t)b + j] = x[j];
        if (hist_x) hist_x[((size_t)b * (max_steps + 1) + step + 1) * 5 + j] = x[j];
    }
    if (hist_u) {
        hist_u[((size_t)b * max_steps + step) * 2] = u1;
        hist_u[((size_t)b * max_steps + step) * 2 + 1] = u2;
    }
    if (hist_status) hist_status[(size_t)b * max_steps + step] = C.sta[i];
    n_steps[b] = step + 1;
    if (!(x[0] <= s_stop)) C.active[b] = 0;
    else atomicAdd(C.n_active, 1);
}

__global__ void cl_init_kernel(int B, mpc_fsm F, ClState C, const double* x_init, double s_stop, double* hist_x,
                               int* n_steps, int max_steps) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    for (int j = 0; j < 5; ++j) {
        C.x[5 * (size_t)b + j] = x_init[5 * (size_t)b + j];
        if (hist_x) hist_x[(size_t)b * (max_steps + 1) * 5 + j] = x_init[5 * (size_t)b + j];
    }
    C.active[b] = x_init[5 * (size_t)b] <= s_stop ? 1 : 0;
    C.obs_s[b] = F.obs_start_s;
    C.tl_timer[b] = 0.0;
    for (int j = 0; j < 4; ++j) C.fsm_flags[4 * (size_t)b + j] = 0;
    for (int j = 0; j < 4; ++j) C.obs[4 * (size_t)b + j] = 0.0;
    C.nobs[b] = 0;
    n_steps[b] = 0;
}

// TrajectoryLoader.get_global_pose(s, d) (trajectory_loader.py:104-116), batched
__global__ void mpc_pose_kernel(DevTable tab, int n, const double* __restrict__ s, const double* __restrict__ d,
                                double* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double si = s[i];
    if (si > tab.smax) si = tab.smax;
    const int j = seg_t(tab, tab.T, si);
    const double xr = lin(tab.s, tab.gx, j, si), yr = lin(tab.s, tab.gy, j, si), psi = lin(tab.s, tab.gpsi, j, si);
    out[3 * (size_t)i] = xr - d[i] * sin(psi);
    out[3 * (size_t)i + 1] = yr + d[i] * cos(psi);
    out[3 * (size_t)i + 2] = psi;
}

// ------------------------------------------------------------------------------------------
// host side: C ABI
// ------------------------------------------------------------------------------------------
static thread_local std::string g_err = "";

static int fail(int code, const std::string& msg);

// a host-backend call behind an extern "C" entry: no C++ exception crosses the ABI (worker threads that
// cannot start, or allocations that fail, become MPC_E_ALLOC)
template <typename F>
static int host_call(F&& f) {
    try {
        f();
        return MPC_SUCCESS;
    } catch (const std::bad_alloc&) {
        return fail(MPC_E_ALLOC, "host backend: out of memory");
    } catch (const std::exception& e) {
        return fail(MPC_E_ALLOC, std::string("host backend: ") + e.what());
    } catch (...) {
        return fail(MPC_E_ALLOC, "host backend: unexpected exception");
    }
}

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
    mpcqp_cpu::Backend* cpu;    // device = -1: the host backend (cpu_backend.h); no HIP state is created
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
    // work list of the two-phase launch: wl[0], wl[1] = counts of the eager calls (alternating), wl[2] = count
    // of a call captured into a graph, wl[3..cap_wl + 2] = deferred instance ids
#define MPC_WORKLIST_CAP (1 << 20)
#define MPC_WL_HEAD 3
    int* wl;
    int wl_epoch;       // counter wl[wl_epoch] serves the next eager call; wl[wl_epoch ^ 1] is zeroed by it
    bool wl_memset;     // MPC_WL_MEMSET=1: reset the count by a memset launch before every call (A/B switch)
    size_t cap_wl;
    bool two_phase;     // MPC_TWO_PHASE=0 in the environment selects the single MODE_FULL launch
    // the work list is reused by every call: a call on a different stream than the previous one
    // first waits for the previous call's last kernel (wl_done, recorded after each split launch)
    hipEvent_t wl_done;
    hipStream_t wl_stream;
    bool wl_pending;
    // stage cache of the split launch (same ordering as the work list): per deferred instance, the
    // linearisation point and nominal rollout that MODE_XO computed, read back by MODE_IPM.  Off by
    // default (MPC_STAGE_CACHE=1 enables it): the repeated setup is ~1% of the slowest instance, and the
    // A/B is within noise (C2 0.4288 vs 0.4288 ms, C3 0.4977 vs 0.5004, C4 0.6078 vs 0.6107, two runs
    // each) while the cache moves 2.9 MB more per C2 step.  Grown on demand by eager calls; a captured
    // call that finds it too small runs without it (same results)
    double* stc;
    size_t cap_stc;     // doubles
    bool use_stc;
    // MPC_IPM_GL64=1: the N = 20 interior-point launch of the split path with one deferred instance per
    // wavefront (GL = 64) instead of two (A/B switch)
    bool ipm_gl64;
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
    p->polish = 2;
    p->sqp_tol = 1e-10;
}

extern "C" const char* mpc_last_error(void) { return g_err.c_str(); }

#ifdef MPC_PROF
// diagnostic build only: accumulated shader cycles per kernel phase (lane 0 of every instance)
extern "C" int mpc_debug_prof(unsigned long long* out, int reset) {
    if (out) HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 16), MPC_E_DEVICE);
    if (reset) {
        unsigned long long z[16] = {0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)), MPC_E_DEVICE);
    }
    return MPC_SUCCESS;
}
#endif
extern "C" int mpc_version(void) { return MPCQP_VERSION; }

static int check_params(const mpc_params* p) {
    if (!p) return fail(MPC_E_ARG, "params is NULL");
    if (p->N < 1 || p->N > MPC_MAX_N) return fail(MPC_E_ARG, "N out of range [1, 63]");
    if (p->max_obs < 0 || p->max_obs > MPC_MAX_OBS) return fail(MPC_E_ARG, "max_obs out of range [0, 64]");
    if (!(p->dt > 0)) return fail(MPC_E_ARG, "dt must be > 0");
    if (p->max_iter < 1) return fail(MPC_E_ARG, "max_iter must be >= 1");
    if (p->sqp_iters < 0 || p->sqp_iters > 100) return fail(MPC_E_ARG, "sqp_iters out of range [0, 100]");
    if (!(p->elastic_rho > 1.0)) return fail(MPC_E_ARG, "elastic_rho must be > 1");
    if (!(p->sqp_tol >= 0.0)) return fail(MPC_E_ARG, "sqp_tol must be >= 0");
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
    k.sqp_tol = p->sqp_tol;
    const char* dbg = std::getenv("MPC_DBG");
    k.dbg = dbg ? std::atoi(dbg) : 0;
    k.mu_check = mpcqp_cpu::checkpoint_on() ? MU_CHECK : -1.0;
    return k;
}

extern "C" int mpc_create(const double* X, int T, const double* U, int Tu, const mpc_params* p, int device,
                          mpc_ctx** out) {
    if (!out) return fail(MPC_E_ARG, "out is NULL");
    *out = nullptr;
    if (!X || !U || T < 2 || Tu < 2) return fail(MPC_E_ARG, "trajectory table needs T >= 2, Tu >= 2");
    int rc = check_params(p);
    if (rc) return rc;
    if (device < -1) return fail(MPC_E_DEVICE, "device index out of range (-1 = CPU backend)");
    if (device == -1) {
        // host backend: the same table build, the solver on host threads (cpu_backend.h)
        mpcqp_host::HostTable ht;
        if (!mpcqp_host::build_host_table(X, T, U, Tu, ht)) return fail(MPC_E_ARG, "bad trajectory table");
        mpc_ctx* c = (mpc_ctx*)std::calloc(1, sizeof(mpc_ctx));
        if (!c) return fail(MPC_E_ALLOC, "calloc");
        c->device = -1;
        c->p = *p;
        c->cpu = new (std::nothrow) mpcqp_cpu::Backend(std::move(ht));
        if (!c->cpu) {
            std::free(c);
            return fail(MPC_E_ALLOC, "host backend");
        }
        *out = c;
        return MPC_SUCCESS;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(MPC_E_DEVICE, "no HIP device available (device = -1 selects the CPU backend)");
    if (device < 0 || device >= ndev) return fail(MPC_E_DEVICE, "device index out of range (-1 = CPU backend)");
    HIPCHK(hipSetDevice(device), MPC_E_DEVICE);
    mpcqp_host::HostTable ht;      // monotone s fix, interp columns, global line, bucket index (host_table.h)
    if (!mpcqp_host::build_host_table(X, T, U, Tu, ht)) return fail(MPC_E_ARG, "bad trajectory table");
    const std::vector<double>& h = ht.buf;
    const int tu = ht.tu;
    mpc_ctx* c = (mpc_ctx*)std::calloc(1, sizeof(mpc_ctx));
    if (!c) return fail(MPC_E_ALLOC, "calloc");
    c->device = device;
    c->p = *p;
    {
        const char* e = std::getenv("MPC_TWO_PHASE");
        c->two_phase = !(e && e[0] == '0');
        const char* e2 = std::getenv("MPC_STAGE_CACHE");
        c->use_stc = !(e2 && e2[0] == '0');     // on by default since round 6 (it carries the interior point's start)
        const char* e3 = std::getenv("MPC_WL_MEMSET");
        c->wl_memset = e3 && e3[0] == '1';
        const char* e4 = std::getenv("MPC_IPM_GL64");
        c->ipm_gl64 = e4 && e4[0] == '1';
    }
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
    c->tab.gx = c->table_buf + 5 * T + 2 * tu;
    c->tab.gy = c->tab.gx + T;
    c->tab.gpsi = c->tab.gy + T;
    c->tab.T = T;
    c->tab.Tu = tu;
    c->tab.smax = ht.smax;
    c->tab.bidx = reinterpret_cast<const int*>(c->table_buf + ht.off_bidx);
    c->tab.nb = ht.nb;
    c->tab.s0 = ht.s0;
    c->tab.ibh = ht.ibh;
    for (int j = 0; j < 5; ++j) c->tab.last[j] = ht.last[j];
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        hipFree(c->table_buf);
        std::free(c);
        return fail(MPC_E_DEVICE, "hipStreamCreate");
    }
    // work list of the two-phase launch (count + ids), allocated here once so that no solve call
    // allocates; without it every batch runs the single-kernel path
    if (hipMalloc(&c->wl, sizeof(int) * ((size_t)MPC_WORKLIST_CAP + MPC_WL_HEAD)) == hipSuccess &&
        hipMemset(c->wl, 0, sizeof(int) * MPC_WL_HEAD) == hipSuccess &&
        hipEventCreateWithFlags(&c->wl_done, hipEventDisableTiming) == hipSuccess) {
        c->cap_wl = MPC_WORKLIST_CAP;
    } else {
        hipFree(c->wl);
        c->wl = nullptr;
        c->cap_wl = 0;
        (void)hipGetLastError();
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
    if (c->cpu) {
        delete c->cpu;
        std::free(c);
        return;
    }
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    free_staging(c);
    hipFree(c->ls); hipFree(c->lst); hipFree(c->lct);
    if (c->wl) hipEventDestroy(c->wl_done);
    hipFree(c->wl);
    hipFree(c->stc);
    hipFree(c->table_buf);
    hipStreamDestroy(c->stream);
    std::free(c);
}

// launch of the solver kernel for an already validated parameter set
#define MPC_STAGE_CACHE_CAP ((size_t)1 << 27)
static int launch_solve(mpc_ctx* c, const KParams& kp, int B, const double* x0, const double* obs, const int* n_obs,
                        const double* ubar, double* u0, double* U, double* Xpred, int* status, int* iters,
                        hipStream_t st) {
    // G = 64 / GL instances per wavefront: the smallest lane group holding the N + 1 stages
    const int* nob = obs ? n_obs : nullptr;
    const int GL = kp.N + 1 <= 16 ? 16 : (kp.N + 1 <= 32 ? 32 : 64);
    const int G = WAVE / GL;
    const bool nt20 = kp.N == 20 && !MPC_NO_NT20;
    const bool nt40 = kp.N == 40 && !MPC_NO_NT20;
    const bool nt30 = kp.N == 30 && !MPC_NO_NT20;
    const int ntv = nt20 ? 20 : (nt40 ? 40 : (nt30 ? 30 : 0));
    const size_t lds_wave = sizeof(double) * (size_t)lds_doubles(kp.N, acl_on(GL, ntv)) * G;
    if (lds_wave > 160 * 1024) return fail(MPC_E_ARG, "horizon too long for LDS");
    const size_t lds_lite = sizeof(double) * (size_t)lds_doubles(kp.N, false, true) * G;   // MODE_XO
    const dim3 grid((B + G - 1) / G);
    // Two-phase launch (MODE_XO then MODE_IPM) for single-QP solves with the crossover on; the work
    // list lives in the context (one list per context: a context is not re-entrant, include/mpcqp.h).
    // With one instance per wavefront (G = 1, N > 31) nothing is stranded behind a slower partner, and
    // the crossover rarely certifies at those horizons (C5: 9%), so the split only repeats the setup.
    // The list is allocated once by mpc_create (MPC_WORKLIST_CAP ids), so this path allocates nothing
    // and stays graph-capturable; a larger batch runs the single-kernel path (same results).
    const bool split = kp.polish >= 2 && kp.sqp_iters == 1 && c->two_phase && G >= 2 && (size_t)B <= c->cap_wl;
    int* wl = split ? c->wl + MPC_WL_HEAD : nullptr;
    int* wcnt = nullptr;
    int* wnext = nullptr;
    // Under stream capture (a HIP graph being recorded) the cross-call ordering below is left out: waiting
    // on wl_done, recorded outside the capture, would be a cross-capture dependency that invalidates the
    // capture, and an event recorded inside it belongs to the graph.  Replays of a captured graph are
    // therefore ordered against eager calls on the same context only by the caller (include/mpcqp.h).
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (split) HIPCHK(hipStreamIsCapturing(st, &cap), MPC_E_DEVICE);
    const bool capturing = cap != hipStreamCaptureStatusNone;
    double* stc = nullptr;
    if (split) {
        // the previous split launch may still be reading the list on another stream: order after it
        if (!capturing && c->wl_pending && c->wl_stream != st)
            HIPCHK(hipStreamWaitEvent(st, c->wl_done, 0), MPC_E_DEVICE);
        const size_t need = (size_t)B * stage_cache_doubles(kp.N);
        // the cache is sized for B records (only the deferred instances write one); above MPC_STAGE_CACHE_CAP
        // doubles (1 GiB) the call runs without it (the same results: the start is recomputed bit for bit)
        if (c->use_stc && need > c->cap_stc && need <= MPC_STAGE_CACHE_CAP && !capturing) {
            // hipFree waits for the device, so no launch still reads the old buffer
            hipFree(c->stc);
            c->stc = nullptr;
            c->cap_stc = 0;
            if (hipMalloc(&c->stc, need * sizeof(double)) == hipSuccess) c->cap_stc = need;
            else { c->stc = nullptr; (void)hipGetLastError(); }
        }
        // a captured call runs without the stage cache: a later eager call may grow (free and reallocate) it,
        // and a graph holding the old pointer would then replay into freed memory
        if (c->use_stc && need <= c->cap_stc && !capturing) stc = c->stc;
        if (capturing || c->wl_memset) {
            // a captured call resets its own count by a memset inside the graph, so every replay starts
            // from zero (an eager call's reset would not be replayed)
            wcnt = capturing ? c->wl + 2 : c->wl + c->wl_epoch;
            HIPCHK(hipMemsetAsync(wcnt, 0, sizeof(int), st), MPC_E_DEVICE);
        } else {
            // eager calls alternate between two counts: this call's MODE_XO zeroes the other one, which the
            // next call (same stream, or ordered after this one by wl_done) uses; no memset launch
            wcnt = c->wl + c->wl_epoch;
            wnext = c->wl + (c->wl_epoch ^ 1);
        }
    }
    // obstacle rows exist only when obstacles are passed
#define MPC_LAUNCH(GLV, OBSV, MODEV, NTV)                                                                   \
    hipLaunchKernelGGL((mpc_solve_kernel<GLV, OBSV, MODEV, NTV>), grid, dim3(WAVE),                    \
                       MODEV == MODE_XO ? lds_lite : lds_wave, st, c->tab, kp, B,                           \
                       x0, obs, nob, ubar, u0, U, Xpred, status, iters, wl, wcnt, stc,                 \
                       MODEV == MODE_XO ? wnext : nullptr)
    // horizon-specialised kernels for the BASELINE horizons (N = 20: C2, C3; N = 30: C4; N = 40: C5), whose
    // unrolled recursions pay for their code size (C4 0.89 -> 0.66 ms, C5 5.67 -> 4.16 ms)
#ifdef MPC_AB_NT20ONLY
    // experiment builds only (tools/build_variant.sh): the N = 20 kernels alone, which compile ~4x faster
#define MPC_LAUNCH_GL(MODEV)                                                                   \
    do {                                                                                       \
        if (!nt20) return fail(MPC_E_ARG, "MPC_AB_NT20ONLY build: N = 20 only");             \
        if (with_obs) MPC_LAUNCH(32, true, MODEV, 20); else MPC_LAUNCH(32, false, MODEV, 20);  \
    } while (0)
#else
#define MPC_LAUNCH_GL(MODEV)                                                                   \
    do {                                                                                       \
        if (nt20) { if (with_obs) MPC_LAUNCH(32, true, MODEV, 20); else MPC_LAUNCH(32, false, MODEV, 20); } \
        else if (nt30) { if (with_obs) MPC_LAUNCH(32, true, MODEV, 30); else MPC_LAUNCH(32, false, MODEV, 30); } \
        else if (nt40) { if (with_obs) MPC_LAUNCH(64, true, MODEV, 40); else MPC_LAUNCH(64, false, MODEV, 40); } \
        else if (GL == 16) { if (with_obs) MPC_LAUNCH(16, true, MODEV, 0); else MPC_LAUNCH(16, false, MODEV, 0); } \
        else if (GL == 32) { if (with_obs) MPC_LAUNCH(32, true, MODEV, 0); else MPC_LAUNCH(32, false, MODEV, 0); } \
        else { if (with_obs) MPC_LAUNCH(64, true, MODEV, 0); else MPC_LAUNCH(64, false, MODEV, 0); } \
    } while (0)
#endif
    const bool with_obs = obs != nullptr && kp.max_obs > 0;
    if (split) {
        MPC_LAUNCH_GL(MODE_XO);
        HIPCHK(hipGetLastError(), MPC_E_LAUNCH);
        // the launched MODE_XO zeroed wl[epoch ^ 1] and uses wl[epoch]: the next eager call takes the other
        if (wnext) c->wl_epoch ^= 1;
#ifndef MPC_AB_NT20ONLY
        if (nt20 && c->ipm_gl64) {
            // one deferred instance per wavefront: B waves at most, the wave's LDS for one group
            const size_t lds_one = sizeof(double) * (size_t)lds_doubles(kp.N, true);
            if (with_obs)
                hipLaunchKernelGGL((mpc_solve_kernel<64, true, MODE_IPM, 20>), dim3(B), dim3(WAVE), lds_one, st,
                                   c->tab, kp, B, x0, obs, nob, ubar, u0, U, Xpred, status, iters, wl, wcnt, stc,
                                   nullptr);
            else
                hipLaunchKernelGGL((mpc_solve_kernel<64, false, MODE_IPM, 20>), dim3(B), dim3(WAVE), lds_one, st,
                                   c->tab, kp, B, x0, obs, nob, ubar, u0, U, Xpred, status, iters, wl, wcnt, stc,
                                   nullptr);
        } else
#endif
        {
            MPC_LAUNCH_GL(MODE_IPM);
        }
        HIPCHK(hipGetLastError(), MPC_E_LAUNCH);
        if (!capturing) {
            HIPCHK(hipEventRecord(c->wl_done, st), MPC_E_DEVICE);
            c->wl_stream = st;
            c->wl_pending = true;
        }
    } else if (kp.sqp_iters == 1) {
        MPC_LAUNCH_GL(MODE_ONE);
    } else {
        MPC_LAUNCH_GL(MODE_FULL);
    }
#undef MPC_LAUNCH_GL
#undef MPC_LAUNCH
    HIPCHK(hipGetLastError(), MPC_E_LAUNCH);
    return MPC_SUCCESS;
}

extern "C" int mpc_solve_batch_device(mpc_ctx* c, int B, const double* x0, const double* obs, const int* n_obs,
                                      const double* ubar, double* u0, double* U, double* Xpred, int* status,
                                      int* iters, void* stream) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    if (B < 0) return fail(MPC_E_ARG, "B < 0");
    if (B == 0) return MPC_SUCCESS;
    if (!x0) return fail(MPC_E_ARG, "x0 is NULL");
    if (c->p.max_obs > 0 && n_obs && !obs) return fail(MPC_E_ARG, "n_obs given but obs is NULL");
    if (obs && c->p.max_obs == 0)
        return fail(MPC_E_ARG, "obs given but params.max_obs == 0 (the obstacles would be ignored)");
    int rc = check_params(&c->p);
    if (rc) return rc;
    if (((uintptr_t)u0 | (uintptr_t)U | (uintptr_t)x0 | (uintptr_t)Xpred | (uintptr_t)obs | (uintptr_t)ubar) & 7)
        return fail(MPC_E_ARG, "double arrays must be 8-byte aligned");
    if (c->cpu) {
        // host context: the pointers are host memory and the call is synchronous (stream ignored)
        return host_call([&] { c->cpu->solve_batch(c->p, B, x0, obs, n_obs, ubar, u0, U, Xpred, status, iters); });
    }
    KParams kp = kparams(&c->p);
    if (!obs) kp.max_obs = 0;
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    return launch_solve(c, kp, B, x0, obs, n_obs, ubar, u0, U, Xpred, status, iters, (hipStream_t)stream);
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
    const int N = c->p.N, mo = c->p.max_obs;
    if (obs && mo == 0) return fail(MPC_E_ARG, "obs given but params.max_obs == 0 (the obstacles would be ignored)");
    if (c->cpu)
        return host_call([&] {
            c->cpu->solve_batch(c->p, B, x0, mo > 0 ? obs : nullptr, n_obs, ubar, u0, U, Xpred, status, iters);
        });
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
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
        if (n_obs) HIPCHK(hipMemcpyAsync(c->nobs, n_obs, sizeof(int) * B, hipMemcpyHostToDevice, s), MPC_E_DEVICE);
    }
    if (ubar) HIPCHK(hipMemcpyAsync(c->ub, ubar, sizeof(double) * 2 * N * B, hipMemcpyHostToDevice, s), MPC_E_DEVICE);
    rc = mpc_solve_batch_device(c, B, c->x0, use_obs ? c->obs : nullptr, use_obs && n_obs ? c->nobs : nullptr,
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

extern "C" void mpc_default_fsm(mpc_fsm* f) {
    std::memset(f, 0, sizeof(*f));
    // the trajectory2.json preset, active in the reference (trajectory_tracking.py:292-308)
    f->obs_trigger_s = 710.0;
    f->obs_start_s = 780.0;
    f->obs_v = 4.0;
    f->obs_end_s = 1050.0;
    f->tl_pos = 550.0;
    f->tl_trigger_s = 100.0;
    f->tl_stop_duration = 20.0;
}

extern "C" int mpc_closed_loop(mpc_ctx* c, int B, const double* x_init, const mpc_fsm* fsm, int max_steps,
                               double s_stop, double* hist_x, double* hist_u, double* hist_obs_s, int* hist_tl,
                               int* hist_status, int* n_steps, double* step_ms) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    if (B < 0 || max_steps < 1) return fail(MPC_E_ARG, "B < 0 or max_steps < 1");
    if (B == 0) return MPC_SUCCESS;
    if (!x_init || !n_steps) return fail(MPC_E_ARG, "x_init and n_steps are required");
    int rc = check_params(&c->p);
    if (rc) return rc;
    mpc_fsm F;
    if (fsm) F = *fsm; else mpc_default_fsm(&F);     // NULL: both scenarios off
    const bool with_fsm = fsm && (F.dynamic_obstacle || F.traffic_light);
    if (c->cpu) {
        int hrc = MPC_SUCCESS;
        const int erc = host_call([&] {
            hrc = c->cpu->closed_loop(c->p, B, x_init, F, with_fsm, max_steps, s_stop, hist_x, hist_u, hist_obs_s,
                                      hist_tl, hist_status, n_steps, step_ms);
        });
        return erc != MPC_SUCCESS ? erc : hrc;
    }
    KParams kp = kparams(&c->p);
    kp.max_obs = with_fsm ? 2 : 0;          // the FSM yields at most the car and the light
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    const size_t nb = (size_t)B, ns = (size_t)max_steps;
    std::vector<void*> bufs;
    auto dalloc = [&](size_t bytes) -> void* {
        void* ptr = nullptr;
        if (hipMalloc(&ptr, bytes) != hipSuccess) return nullptr;
        bufs.push_back(ptr);
        return ptr;
    };
    auto release = [&]() { for (void* q : bufs) hipFree(q); };
    ClState C;
    C.x = (double*)dalloc(nb * 5 * 8);
    C.obs = (double*)dalloc(nb * 4 * 8);
    C.nobs = (int*)dalloc(nb * 4);
    C.active = (int*)dalloc(nb * 4);
    C.obs_s = (double*)dalloc(nb * 8);
    C.tl_timer = (double*)dalloc(nb * 8);
    C.fsm_flags = (int*)dalloc(nb * 4 * 4);
    C.n_active = (int*)dalloc(4);
    C.alist = (int*)dalloc(nb * 4);
    C.n_list = (int*)dalloc(4);
    C.xa = (double*)dalloc(nb * 5 * 8);
    C.obsa = (double*)dalloc(nb * 4 * 8);
    C.nobsa = (int*)dalloc(nb * 4);
    C.u0a = (double*)dalloc(nb * 2 * 8);
    C.sta = (int*)dalloc(nb * 4);
    double* d_xinit = (double*)dalloc(nb * 5 * 8);
    double* d_hx = hist_x ? (double*)dalloc(nb * (ns + 1) * 5 * 8) : nullptr;
    double* d_hu = hist_u ? (double*)dalloc(nb * ns * 2 * 8) : nullptr;
    double* d_ho = hist_obs_s ? (double*)dalloc(nb * ns * 8) : nullptr;
    int* d_ht = hist_tl ? (int*)dalloc(nb * ns * 4) : nullptr;
    int* d_hs = hist_status ? (int*)dalloc(nb * ns * 4) : nullptr;
    int* d_ns = (int*)dalloc(nb * 4);
    for (void* q : bufs)
        if (!q) { release(); return fail(MPC_E_ALLOC, "hipMalloc closed-loop buffers"); }
    if ((hist_x && !d_hx) || (hist_u && !d_hu) || (hist_obs_s && !d_ho) || (hist_tl && !d_ht) || (hist_status && !d_hs)) {
        release();
        return fail(MPC_E_ALLOC, "hipMalloc closed-loop histories");
    }
    hipStream_t st = c->stream;
    std::vector<hipEvent_t> ev;
    auto cleanup = [&]() {
        hipStreamSynchronize(st);
        for (auto& e : ev)
            if (e) hipEventDestroy(e);
        release();
    };
    // steps that never run stay NaN / -1 (all-ones bytes)
    bool ok0 = true;
    if (d_hx) ok0 = ok0 && hipMemsetAsync(d_hx, 0xff, nb * (ns + 1) * 5 * 8, st) == hipSuccess;
    if (d_hu) ok0 = ok0 && hipMemsetAsync(d_hu, 0xff, nb * ns * 2 * 8, st) == hipSuccess;
    if (d_ho) ok0 = ok0 && hipMemsetAsync(d_ho, 0xff, nb * ns * 8, st) == hipSuccess;
    if (d_ht) ok0 = ok0 && hipMemsetAsync(d_ht, 0xff, nb * ns * 4, st) == hipSuccess;
    if (d_hs) ok0 = ok0 && hipMemsetAsync(d_hs, 0xff, nb * ns * 4, st) == hipSuccess;
    ok0 = ok0 && hipMemcpyAsync(d_xinit, x_init, nb * 5 * 8, hipMemcpyHostToDevice, st) == hipSuccess;
    if (!ok0) {
        cleanup();
        return fail(MPC_E_DEVICE, "closed-loop buffer initialisation");
    }
    const dim3 tb(256), tg((B + 255) / 256);
    hipLaunchKernelGGL(cl_init_kernel, tg, tb, 0, st, B, F, C, d_xinit, s_stop, d_hx, d_ns, max_steps);
    if (step_ms) {
        ev.assign(ns + 1, nullptr);
        for (auto& e : ev)
            if (hipEventCreate(&e) != hipSuccess) {
                e = nullptr;
                cleanup();
                return fail(MPC_E_DEVICE, "hipEventCreate (step timing)");
            }
        if (hipEventRecord(ev[0], st) != hipSuccess) {
            cleanup();
            return fail(MPC_E_DEVICE, "hipEventRecord (step timing)");
        }
    }
    int steps_run = 0;
    rc = MPC_SUCCESS;
    // the solve runs on the egos still in the loop: the list is rebuilt at the host syncs below whenever
    // egos have left, so retired egos stop costing solver work (results are per ego, unchanged)
    hipLaunchKernelGGL(cl_compact_kernel, dim3(1), dim3(1024), 0, st, B, C);
    int nl = 0;
    if (hipMemcpyAsync(&nl, C.n_list, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        cleanup();
        return fail(MPC_E_DEVICE, "closed-loop initial ego list");
    }
    for (int step = 0; step < max_steps && nl > 0; ++step) {
        // runs without scenarios too: records the RED light / no-car histories like the reference
        hipLaunchKernelGGL(cl_fsm_kernel, tg, tb, 0, st, B, F, kp.dt, C, d_ho, d_ht, step, max_steps);
        const dim3 lg((nl + 255) / 256);
        hipLaunchKernelGGL(cl_gather_kernel, lg, tb, 0, st, nl, C);
        rc = launch_solve(c, kp, nl, C.xa, with_fsm ? C.obsa : nullptr, with_fsm ? C.nobsa : nullptr, nullptr, C.u0a,
                          nullptr, nullptr, C.sta, nullptr, st);
        if (rc) break;
        if (hipMemsetAsync(C.n_active, 0, 4, st) != hipSuccess) {
            rc = fail(MPC_E_DEVICE, "closed-loop active-count reset");
            break;
        }
        hipLaunchKernelGGL(cl_plant_kernel, lg, tb, 0, st, c->tab, nl, kp.dt, C, s_stop, d_hx, d_hu, d_hs, d_ns, step,
                           max_steps);
        if (step_ms && hipEventRecord(ev[step + 1], st) != hipSuccess) {
            rc = fail(MPC_E_DEVICE, "hipEventRecord (step timing)");
            break;
        }
        steps_run = step + 1;
        if ((step & 7) == 7 || step == max_steps - 1) {     // every 8 steps: has every ego left the loop?
            int na = 0;
            if (hipMemcpyAsync(&na, C.n_active, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                rc = fail(MPC_E_DEVICE, "closed-loop step sync");
                break;
            }
            if (na == 0) break;
            if (na < nl) {                                  // egos left: shrink the solver's list
                hipLaunchKernelGGL(cl_compact_kernel, dim3(1), dim3(1024), 0, st, B, C);
                if (hipMemcpyAsync(&nl, C.n_list, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess) {
                    rc = fail(MPC_E_DEVICE, "closed-loop ego list");
                    break;
                }
            }
        }
    }
    if (rc == MPC_SUCCESS && hipGetLastError() != hipSuccess) rc = fail(MPC_E_LAUNCH, "closed-loop kernel launch");
    if (rc == MPC_SUCCESS) {
        bool ok = hipMemcpyAsync(n_steps, d_ns, nb * 4, hipMemcpyDeviceToHost, st) == hipSuccess;
        if (hist_x) ok = ok && hipMemcpyAsync(hist_x, d_hx, nb * (ns + 1) * 5 * 8, hipMemcpyDeviceToHost, st) == hipSuccess;
        if (hist_u) ok = ok && hipMemcpyAsync(hist_u, d_hu, nb * ns * 2 * 8, hipMemcpyDeviceToHost, st) == hipSuccess;
        if (hist_obs_s) ok = ok && hipMemcpyAsync(hist_obs_s, d_ho, nb * ns * 8, hipMemcpyDeviceToHost, st) == hipSuccess;
        if (hist_tl) ok = ok && hipMemcpyAsync(hist_tl, d_ht, nb * ns * 4, hipMemcpyDeviceToHost, st) == hipSuccess;
        if (hist_status) ok = ok && hipMemcpyAsync(hist_status, d_hs, nb * ns * 4, hipMemcpyDeviceToHost, st) == hipSuccess;
        ok = ok && hipStreamSynchronize(st) == hipSuccess;
        if (!ok) rc = fail(MPC_E_DEVICE, "closed-loop copy-back");
    }
    if (step_ms) {
        for (size_t i = 0; i < ns; ++i) {
            float ms = NAN;
            if ((int)i < steps_run && hipEventElapsedTime(&ms, ev[i], ev[i + 1]) != hipSuccess) ms = NAN;
            step_ms[i] = ms;
        }
    }
    cleanup();
    return rc;
}

extern "C" int mpc_global_pose(mpc_ctx* c, int n, const double* s, const double* d, double* out) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    if (n < 0 || (n > 0 && (!s || !d || !out))) return fail(MPC_E_ARG, "bad global-pose arguments");
    if (n == 0) return MPC_SUCCESS;
    if (c->cpu) {
        c->cpu->pose(n, s, d, out);
        return MPC_SUCCESS;
    }
    HIPCHK(hipSetDevice(c->device), MPC_E_DEVICE);
    double* buf = nullptr;
    HIPCHK(hipMalloc(&buf, sizeof(double) * 5 * (size_t)n), MPC_E_ALLOC);
    hipStream_t st = c->stream;
    int rc = MPC_SUCCESS;
    if (hipMemcpyAsync(buf, s, sizeof(double) * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(buf + n, d, sizeof(double) * n, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = fail(MPC_E_DEVICE, "hipMemcpy global pose inputs");
    } else {
        hipLaunchKernelGGL(mpc_pose_kernel, dim3((n + 255) / 256), dim3(256), 0, st, c->tab, n, buf, buf + n, buf + 2 * n);
        if (hipGetLastError() != hipSuccess) rc = fail(MPC_E_LAUNCH, "global pose kernel");
        else if (hipMemcpyAsync(out, buf + 2 * n, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                 hipStreamSynchronize(st) != hipSuccess)
            rc = fail(MPC_E_DEVICE, "hipMemcpy global pose");
    }
    hipStreamSynchronize(st);
    hipFree(buf);
    return rc;
}

extern "C" int mpc_read_trajectory_json(const char* path, double* X, int maxT, double* U, int maxTu, int* T,
                                        int* Tu) {
    if (!path || !T || !Tu) return fail(MPC_E_ARG, "path, T and Tu are required");
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(MPC_E_ARG, std::string("File not found : ") + path + ".");   // trajectory_loader.py:18
    std::string text;
    char chunk[65536];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof(chunk), f)) > 0) text.append(chunk, got);
    std::fclose(f);
    // host_table.h: json.load semantics (last duplicate key wins, bounded nesting, no trailing data)
    std::vector<double> xs, us;
    int tx = 0, tu = 0;
    std::string err;
    if (!mpcqp_host::read_trajectory_json_text(text, xs, tx, us, tu, err)) return fail(MPC_E_ARG, err);
    *T = tx;
    *Tu = tu;
    if (X) {
        if (maxT < tx) return fail(MPC_E_ARG, "X buffer too small");
        std::memcpy(X, xs.data(), sizeof(double) * 5 * (size_t)tx);
    }
    if (U) {
        if (maxTu < tu) return fail(MPC_E_ARG, "U buffer too small");
        std::memcpy(U, us.data(), sizeof(double) * 2 * (size_t)tu);
    }
    return MPC_SUCCESS;
}

extern "C" int mpc_create_from_json(const char* path, const mpc_params* p, int device, mpc_ctx** out) {
    int T = 0, Tu = 0;
    int rc = mpc_read_trajectory_json(path, nullptr, 0, nullptr, 0, &T, &Tu);
    if (rc) return rc;
    std::vector<double> X((size_t)5 * T), U((size_t)2 * Tu);
    rc = mpc_read_trajectory_json(path, X.data(), T, U.data(), Tu, &T, &Tu);
    if (rc) return rc;
    return mpc_create(X.data(), T, U.data(), Tu, p, device, out);
}

extern "C" int mpc_lookup(mpc_ctx* c, int n, const double* s, double* out_state, double* out_control) {
    if (!c) return fail(MPC_E_ARG, "ctx is NULL");
    if (n < 0 || (n > 0 && !s)) return fail(MPC_E_ARG, "bad lookup arguments");
    if (n == 0) return MPC_SUCCESS;
    if (c->cpu) {
        c->cpu->lookup(n, s, out_state, out_control);
        return MPC_SUCCESS;
    }
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

// multi-GPU: the ego-shard communicator (RCCL gather behind the C ABI)
#include "comm.h"

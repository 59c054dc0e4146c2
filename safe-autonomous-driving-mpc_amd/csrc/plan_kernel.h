// plan_kernel.h — the planner's device code (one wavefront per chunk, LDS working set); included by plan.hip
// and, with tools/plan_emu.cpp's definitions of the HIP built-ins, by the host emulation used to debug it
// under AddressSanitizer.  See plan.hip for the design.
#pragma once
#include <cmath>
#include "../../include/mpcplan.h"

#ifndef PLAN_LDS_DECL
#define PLAN_LDS_DECL extern __shared__ double lds[]
#endif
#ifndef PLAN_LDS_AS
#define PLAN_LDS_AS __attribute__((address_space(3)))
#endif
typedef PLAN_LDS_AS double ldsd;

#ifdef PLAN_PROF
__device__ unsigned long long g_plan_prof[16];
#endif

namespace {

constexpr int WAVE = 64;
constexpr int NZ = 8;             // stage variables: x (s, d, o, k, v), w (u1, u2, S)
constexpr int NR = 11;            // rows per stage at most
constexpr int RS = 11;            // row slots per stage in LDS: one per row kind (kind_slot), so every row visit
                                  // has a compile-time slot; a stage's missing kinds leave their slots unused
constexpr int NH = 36;            // packed symmetric 8x8
// LDS strides of the per-stage 8-vectors and stage Hessians: one double of padding each, so the lanes of a
// stage-parallel loop (lane k on stage k) spread over the LDS banks (a stride of 8 doubles = 16 dwords put
// every fourth lane on the same bank group: SQ_LDS_BANK_CONFLICT was 39% of the LDS-active cycles)
constexpr int ZS = NZ + 1;
constexpr int HSTR = NH + 9;     // a stage's H block: packed H (36), the factorisation's 8 slots (hs_slot), 1 / HT(7, 7)
constexpr double RHO = 1e8;       // penalty of the active rows in the equality-constrained solve
constexpr int AL_STEPS = 4;
constexpr double AL_TOL = 1e-13;   // refinements stop once the multiplier update is at rounding level
constexpr int POLISH_ROUNDS = 6;
constexpr int WARM_ROUNDS = 5;      // active-set rounds from the previous QP's classification (oracle qp_solve)
constexpr double MU_CHECK = 1e-4;   // interior-point checkpoint: a polish is tried once mu and phi are below this ...
constexpr double CHECK_SEP = 100.0; // ... and every row's s and lambda differ by this factor (no near-tie)
constexpr int CHECK_ROUNDS = 2;     // polish rounds at the checkpoint (the interior point resumes if they fail)
constexpr double SHIFT0 = 1.0;
constexpr double TAU = 0.995;
constexpr double CYCLE_REL = 1e-6;
constexpr double DELTA0 = 1e-6;
constexpr double DELTA_MAX = 1e4;
constexpr double EXACT_STEP = 0.1;
constexpr int EXACT_AFTER = 20;      // exact Hessian from this SQP iteration on as well (oracle EXACT_AFTER)
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
    // uniform grid over [s[0], s[M-1]]: grid[j] = first i with s[i] >= s[0] + j / ginv (route_grid), so a
    // search starts at most a cell's worth of way-points before its answer (one load instead of a binary
    // search's ~log2 M dependent loads from HBM)
    const int* grid;
    int T;
    double ginv;
};

// the grid of DevRoute (host side; T cells of equal length)
inline void route_grid(const double* s, int M, int T, int* grid, double* ginv) {
    const double h = (s[M - 1] - s[0]) / T;
    *ginv = 1.0 / h;
    int i = 0;
    for (int j = 0; j < T; ++j) {
        const double c = s[0] + j * h;
        while (i < M && s[i] < c) ++i;
        grid[j] = i;
    }
}

// LDS layout of one chunk (doubles; per-stage counts times NP = Nmax + 1).  Arrays used only by the interior
// point alias the polish's: DSA = Y, DLA = TLAM, DS = TZ (the polish runs after the interior point is done).
struct Layout {
    int NP;
    int oAB, oH, oGQ, oG, oK, oL, oEZ, oZ, oS, oLAM, oGL, oDZ, oDSA, oDLA, oDS, oDL, oMY, oMLAT, oZB,
        oZ2, oDZV, oPI, oVLIM, oVL, oACT, oTACT, oSC;
    int oY, oTLAM, oTZ;
    int total;
};

__host__ __device__ Layout make_layout(int Nmax) {
    Layout y;
    y.NP = Nmax + 1;
    int o = 0;
    const int np = y.NP;
    y.oAB = o; o += 40 * np;         // the dynamics [A B c] by rows (ab_at): A(l, j) at 8 l + j, B(l, r) (u1, u2;
                                     // the slack's column is zero) at 8 l + 5 + r, c(l) at 8 l + 7
    y.oH = o; o += HSTR * np;        // packed H, then at NH + slot the factorisation's stage Hessian H + delta I +
                                     // row weights at the 8 entries rows touch (hs_slot; elsewhere it is H + delta I), then
                                     // 1 / HT(7, 7)
    y.oGQ = o; o += ZS * np;
    y.oG = o; o += RS * np;
    y.oK = o; o += 15 * np;
    y.oL = o; o += 6 * np;
    y.oEZ = o; o += 2 * ZS * np;
    y.oZ = o; o += ZS * np;
    y.oS = o; o += RS * np;
    y.oLAM = o; o += RS * np;
    y.oGL = o; o += ZS * np;
    y.oDZ = o; o += ZS * np;
    y.oDSA = o; o += RS * np;
    y.oDLA = o; o += RS * np;
    y.oDS = o; o += RS * np;
    y.oDL = o; o += RS * np;
    y.oMY = o; o += 5 * np;
    y.oMLAT = o; o += 2 * np;
    y.oZB = o; o += ZS * np;
    y.oZ2 = o; o += ZS * np;
    y.oDZV = o; o += ZS * np;
    y.oVLIM = o; o += np;
    y.oVL = o; o += np;
    y.oACT = o; o += np;             // active-row bit masks (bit = slot, kind_slot), stored as doubles
    y.oTACT = o; o += np;
    y.oSC = o; o += 16;              // scalars shared by the wave
#ifdef PLAN_PROF
    o += 16;                         // phase counters of the diagnostic build
#endif
    y.oY = y.oDSA;
    y.oTLAM = y.oDLA;
    y.oTZ = y.oDS;
    y.oPI = y.oDZ;                   // co-states of the multiplier recovery (after the QP's last solve)
    y.total = o;
    return y;
}

// UNI(i): a wave-uniform int (an LDS offset of the context) in a scalar register.  The hot loops take their
// offsets and scalars into locals first: the context lives in private memory and is reached through a
// generic pointer in the non-inlined phases, which an LDS store may alias as far as the compiler knows, so
// a field read inside a loop is a flat load (and a wait on it) per trip.
#ifndef PLAN_HOST_EMU
#define UNI(i) __builtin_amdgcn_readfirstlane(i)
#else
#define UNI(i) (i)
#endif
// the layout's offsets in scalar registers (a hot function's copy of X.Y): recomputed from the uniform Nmax
// (make_layout is integer arithmetic), one private-memory read instead of one per field
__device__ inline Layout uni_layout(const Layout& y) { return make_layout(UNI(y.NP) - 1); }

// phases of the diagnostic build
enum { PH_OTHER, PH_BUILD, PH_HESS, PH_FACTOR, PH_SOLVE, PH_IPM, PH_EQP, PH_MULT, PH_LSEARCH, PH_ROLLOUT, PH_COUNT };
// call counters of the diagnostic build (slots after the phases)
enum { PH_NFACTOR = PH_COUNT, PH_NSOLVE, PH_IGRAD, PH_IDIR, PH_IRED, PH_NSLOTS };   // slot 15: chunks
// (PH_IGRAD / PH_IDIR / PH_IRED: the interior point's gradient rows, direction rows, and its reductions, ratio
// tests and updates)

// scalar slots (oSC + ...)
enum { SC_DELTA, SC_NU0, SC_NU1, SC_EM0, SC_EM1, SC_EM2, SC_EM3, SC_FLAG };

// ------------------------------------------------------------------------------------------------------
// wave reductions
// ------------------------------------------------------------------------------------------------------
__device__ inline double wmax(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
    return v;
}
__device__ inline double wmin(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
    return v;
}
__device__ inline double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ inline int wsumi(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}

// ------------------------------------------------------------------------------------------------------
// route: k_ref_fun (:445-459) and v_max_fun (:470-473)
// ------------------------------------------------------------------------------------------------------
__device__ inline int imin(int a, int b) { return a < b ? a : b; }

// first i with x[i] >= v (std::lower_bound over R.s; NaN -> 0), from the grid cell of v
__device__ int lower_bound_g(const DevRoute& R, double v) {
    const double* x = R.s;
    int j;
    if (!(v > x[0])) return 0;
    if (!(v < x[R.M - 1])) j = R.T - 1;
    else j = imin(R.T - 1, (int)((v - x[0]) * R.ginv));
    int i = R.grid[j];
    while (i > 0 && x[i - 1] >= v) --i;      // the cell index may round up past v
    while (i < R.M && x[i] < v) ++i;
    return i;
}

// first i with x[i] > v (std::upper_bound over R.s; NaN -> 0), from the grid cell of v
__device__ int upper_bound_g(const DevRoute& R, double v) {
    const double* x = R.s;
    int j;
    if (!(v >= x[0])) return 0;
    if (!(v < x[R.M - 1])) j = R.T - 1;
    else j = imin(R.T - 1, (int)((v - x[0]) * R.ginv));
    int i = R.grid[j];
    while (i > 0 && x[i - 1] > v) --i;
    while (i < R.M && x[i] <= v) ++i;
    return i;
}

// kappa(s) with d/ds and d2/ds2 (k2 may be null): s_to_t linear (searchsorted left, clipped to [1, M-1]),
// spline piece floor(t) clipped to [0, M-2]
__device__ double route_kappa(const DevRoute& R, double s, double* k1, double* k2) {
    const int M = R.M;
    int i = lower_bound_g(R, s);
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
    const int i = upper_bound_g(R, s);
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

// the rows of stage k, in order: [v_min, v_max, (k > 0) lateral +, lateral -] unless the final chunk's last
// stage; (k > 0) curvature min, max; (k < N) u1 min, max, u2 min, max, slack; the intermediate chunk's
// terminal row at k = N.  Counted and indexed arithmetically (no per-lane array, which would live in
// scratch memory).
__host__ __device__ constexpr int stage_nrows(int k, int N, int fin) {
    return ((fin && k == N) ? 0 : (k > 0 ? 4 : 2)) + (k > 0 ? 2 : 0) + (k < N ? 5 : 0) + ((k == N && !fin) ? 1 : 0);
}
__host__ __device__ constexpr int row_kind(int k, int N, int fin, int j) {
    const int n0 = (fin && k == N) ? 0 : (k > 0 ? 4 : 2);
    if (j < n0) return j;                                   // ROW_VMIN, ROW_VMAX, ROW_LATP, ROW_LATM
    j -= n0;
    const int n1 = k > 0 ? 2 : 0;
    if (j < n1) return ROW_KMIN + j;
    j -= n1;
    if (k < N) return ROW_U1MIN + j;                        // ROW_U1MIN .. ROW_S
    return ROW_STERM;
}

// Row coefficients over (x_k, w_k) at the SQP iterate's (k, v) of stage k, sparse: every row touches one or
// two of the 8 stage variables, so instead of a dense 8-vector the loops visit the 12 row kinds in a fully
// unrolled loop
// (for_rows), where each kind, and with it the indices of its nonzero coefficients, is a compile-time
// constant.  Adding only the nonzero terms, in the same order, gives the dense loops' values (a skipped
// term is an exact zero).
// the LDS slot of a row kind: its own, except the intermediate chunk's terminal row (k = N only), which takes
// the u1-min slot (no stage has both), so a stage's rows fit in NR slots in row order
__host__ __device__ constexpr int kind_slot(int kind) { return kind == ROW_STERM ? ROW_U1MIN : kind; }
__host__ __device__ constexpr bool row_on(int kind, int k, int N, int fin) {
    switch (kind) {
        case ROW_VMIN: case ROW_VMAX: return !(fin && k == N);
        case ROW_LATP: case ROW_LATM: return !(fin && k == N) && k > 0;
        case ROW_KMIN: case ROW_KMAX: return k > 0;
        case ROW_STERM: return k == N && !fin;
        default: return k < N;
    }
}
struct RowSp {
    int i0, i1;          // indices of the coefficients (i0 < i1)
    double c0, c1;
    bool two;            // c1 present
};
__device__ __forceinline__ RowSp row_sp(int kind, bool has_w, double kb, double vb) {
    switch (kind) {
        case ROW_VMIN: return {4, 7, 1.0, 1.0, has_w};
        case ROW_VMAX: return {4, 7, -1.0, -1.0, has_w};
        case ROW_LATP: return {3, 4, -vb * vb, -2.0 * kb * vb, true};
        case ROW_LATM: return {3, 4, vb * vb, 2.0 * kb * vb, true};
        case ROW_KMIN: return {3, 3, 1.0, 0.0, false};
        case ROW_KMAX: return {3, 3, -1.0, 0.0, false};
        case ROW_U1MIN: return {5, 5, 1.0, 0.0, false};
        case ROW_U1MAX: return {5, 5, -1.0, 0.0, false};
        case ROW_U2MIN: return {6, 6, 1.0, 0.0, false};
        case ROW_U2MAX: return {6, 6, -1.0, 0.0, false};
        case ROW_S: return {7, 7, 1.0, 0.0, false};
        default: return {0, 0, 1.0, 0.0, false};        // ROW_STERM
    }
}
// f(kind, j, on) for every row kind of stage k, in storage order: j = the row's slot (kind_slot, a compile-time
// constant), on = the stage has the row (else the slot's values are not the body's to use).  The body runs
// unconditionally -- loads, divisions and all -- and applies its results under `on` (selects, masked stores):
// no branch per kind, so the scheduler overlaps the rows' independent chains (one lane serves a stage, so
// the rows are its serial work); every on-row value is computed by the same operations as before.
// (a compile-time recursion over the kinds: a loop the unroller gives up on in a large function would index
// the callers' per-lane arrays at run time, which puts them in scratch memory)
template <int KIND, class F>
__device__ __forceinline__ void for_rows_from(int k, int N, int fin, int j, F& f) {
    if constexpr (KIND <= ROW_STERM) {
        f(KIND, kind_slot(KIND), row_on(KIND, k, N, fin));
        for_rows_from<KIND + 1>(k, N, fin, j, f);
    }
}
template <class F>
__device__ __forceinline__ void for_rows(int k, int N, int fin, F&& f) {
    for_rows_from<0>(k, N, fin, 0, f);
}
// g + a . z
__device__ __forceinline__ double sp_dot(const RowSp& r, double g, const double z[NZ]) {
    double v = g + r.c0 * z[r.i0];
    if (r.two) v += r.c1 * z[r.i1];
    return v;
}

// Row-parallel visits: slot q = RS k + j of the row arrays (S, LAM, G, DS, ...), lane q, q + 64, ...: the
// interior point's per-row divisions and ratio tests run on (N + 1) RS / 64 slots per lane instead of a
// stage's rows on each of N + 1 lanes.  The row's stage, kind and coefficients come arithmetically from
// q (no branch per kind): the same values row_sp gives (c0 = -vb vb for ROW_LATP is (-vb) vb exactly,
// c1 = (-2 kb) vb likewise), so every row value is formed by the same operations as in for_rows.
struct RowAt {
    int k, i0, i1;
    bool on, two;
    double c0, c1;
};
// the slots a stage's rows occupy, one bit per slot, for the four stage shapes: first stage (k = 0 < N),
// interior, last stage of the final chunk, last stage of an intermediate chunk (row_on tabulated)
__host__ __device__ constexpr unsigned on_tab(int k, int N, int fin) {
    unsigned m = 0;
    for (int kind = 0; kind <= ROW_STERM; ++kind) m |= row_on(kind, k, N, fin) ? 1u << kind_slot(kind) : 0u;
    return m;
}
// the kind in slot j of stage k (the slot it shares decides: the terminal row at k = N)
__host__ __device__ constexpr int slot_kind(int j, int k, int N) { return (k == N && j == ROW_U1MIN) ? ROW_STERM : j; }
constexpr unsigned ON_FIRST = on_tab(0, 2, 0), ON_MID = on_tab(1, 2, 0), ON_LASTF = on_tab(2, 2, 1), ON_LASTI = on_tab(2, 2, 0);
__device__ inline unsigned stage_on(int k, int N, int fin) {
    return k == N ? (fin ? ON_LASTF : ON_LASTI) : (k == 0 ? ON_FIRST : ON_MID);
}
__device__ inline RowAt row_at(const ldsd* L, int oZB, int q, int N, int fin) {
    RowAt r;
    const int k = q / RS, j = q - RS * k, kind = slot_kind(j, k, N);
    r.k = k;
    r.on = (stage_on(k, N, fin) >> j) & 1u;
    // nibble tables over the kinds (ROW_VMIN .. ROW_STERM): first and second coefficient's variable
    constexpr unsigned long long I0TAB = 0x076655333344ull;   // kind 0..11: 4 4 3 3 3 3 5 5 6 6 7 0
    constexpr unsigned long long I1TAB = 0x076655334477ull;   // kind 0..11: 7 7 4 4 3 3 5 5 6 6 7 0
    r.i0 = (int)((I0TAB >> (4 * kind)) & 15ull);
    r.i1 = (int)((I1TAB >> (4 * kind)) & 15ull);
    const bool neg = (0x2A6u >> kind) & 1u;                            // VMAX, LATP, KMAX, U1MAX, U2MAX
    const bool lat = kind == ROW_LATP || kind == ROW_LATM;
    r.two = lat || (kind <= ROW_VMAX && k < N);
    const double kb = L[oZB + ZS * k + 3], vb = L[oZB + ZS * k + 4];
    const double vv = neg ? -vb * vb : vb * vb;
    r.c0 = lat ? vv : (neg ? -1.0 : 1.0);
    const double kk2 = neg ? -2.0 * kb : 2.0 * kb;
    r.c1 = lat ? kk2 * vb : (neg ? -1.0 : 1.0);
    return r;
}

// Gaussian elimination with partial pivoting on a 5x5 system with NC right-hand sides, in registers: the pivot
// row is found and swapped by selects (every candidate row compared, the one chosen exchanged), so no array is
// indexed at run time (a run-time row index would put M and R in scratch memory); columns left of the pivot
// column are never read again and are not exchanged.  The first largest |M(i, c)| wins, as in the oracle.
template <int NC>
__device__ bool solve5(double M[25], double R[5 * NC]) {
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        int pr = c;
        double best = fabs(M[5 * c + c]);
#pragma unroll
        for (int i = c + 1; i < 5; ++i) {
            const double a = fabs(M[5 * i + c]);
            pr = a > best ? i : pr;
            best = a > best ? a : best;
        }
#pragma unroll
        for (int i = c + 1; i < 5; ++i) {
            const bool sw = pr == i;
#pragma unroll
            for (int j = c; j < 5; ++j) {
                const double t = M[5 * c + j];
                M[5 * c + j] = sw ? M[5 * i + j] : t;
                M[5 * i + j] = sw ? t : M[5 * i + j];
            }
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const double t = R[NC * c + j];
                R[NC * c + j] = sw ? R[NC * i + j] : t;
                R[NC * i + j] = sw ? t : R[NC * i + j];
            }
        }
        if (M[5 * c + c] == 0.0) return false;
#pragma unroll
        for (int i = c + 1; i < 5; ++i) {
            const double f = M[5 * i + c] / M[5 * c + c];
#pragma unroll
            for (int j = c; j < 5; ++j) M[5 * i + j] -= f * M[5 * c + j];
#pragma unroll
            for (int j = 0; j < NC; ++j) R[NC * i + j] -= f * R[NC * c + j];
        }
    }
#pragma unroll
    for (int c = 4; c >= 0; --c)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            double v = R[NC * c + j];
#pragma unroll
            for (int k = c + 1; k < 5; ++k) v -= M[5 * c + k] * R[NC * k + j];
            R[NC * c + j] = v / M[5 * c + c];
        }
    return true;
}

// H (3 x 3, symmetric positive definite) = L D L' with L unit lower triangular, stored as {1/d0, l10, 1/d1,
// l20, l21, 1/d2}: no square roots, three divisions per factorisation and none in the solves, which sit on
// the solves' dependent chains (oracle/plan_oracle.c uses the same form and rounding).  Fails (false) when a
// pivot is not positive, the Cholesky condition.
__device__ bool chol3(const double H[3][3], double L[6]) {
    const double d0 = H[0][0];
    if (!(d0 > 0.0)) return false;
    L[0] = 1.0 / d0;
    L[1] = H[1][0] * L[0];
    const double d1 = H[1][1] - L[1] * H[1][0];
    if (!(d1 > 0.0)) return false;
    L[2] = 1.0 / d1;
    L[3] = H[2][0] * L[0];
    const double e21 = H[2][1] - L[3] * H[1][0];
    L[4] = e21 * L[2];
    const double d2 = H[2][2] - L[3] * H[2][0] - L[4] * e21;
    if (!(d2 > 0.0)) return false;
    L[5] = 1.0 / d2;
    return true;
}

// b <- (L D L')^-1 b
__device__ inline void chol3_solve(const double L[6], double b[3]) {
    const double y0 = b[0];
    const double y1 = b[1] - L[1] * y0;
    const double y2 = b[2] - L[3] * y0 - L[4] * y1;
    b[2] = y2 * L[5];
    b[1] = y1 * L[2] - L[4] * b[2];
    b[0] = y0 * L[0] - L[1] * b[1] - L[3] * b[2];
}

__host__ __device__ constexpr int hx(int i, int j) {   // packed index of the symmetric 8x8 (i <= j)
    return i * NZ - (i * (i - 1)) / 2 + (j - i);
}
__device__ inline int hidx(int i, int j) { return i <= j ? hx(i, j) : hx(j, i); }
// [A B c] of stage k, row l, column c (0..4 A, 5..6 B, 7 c): one stride per stage and per row, so a lane that
// reads a column (or a row) adds one offset per stage and takes the rest as immediate offsets
__host__ __device__ constexpr int ab_at(int k, int l, int c) { return 40 * k + 8 * l + c; }

// the 8 entries of a stage Hessian the rows touch, slots 0..7: (0,0) terminal row; (3,3), (3,4), (4,4) curvature
// and lateral rows; (4,7) and (7,7) speed and slack rows (with (4,4)); (5,5), (6,6) control boxes
__device__ inline int hs_slot(int u, int w) {
    const int a = u < w ? u : w, b = u < w ? w : u;
    if (a == b) return a == 0 ? 0 : a == 3 ? 1 : a == 4 ? 3 : a == 5 ? 5 : a == 6 ? 6 : a == 7 ? 7 : -1;
    return (a == 3 && b == 4) ? 2 : (a == 4 && b == 7) ? 4 : -1;
}

// ------------------------------------------------------------------------------------------------------
// the chunk: LDS working set, per-lane view
// ------------------------------------------------------------------------------------------------------
struct Ctx {
    DevRoute R;
    plan_params P;
    Layout Y;
    ldsd* L;            // the chunk's LDS block (explicit address space: ds_read / ds_write, never flat)
    int ln;             // lane
    int N, fin;
    int dbg;            // A/B timing switches (PLAN_DBG, plan.hip): repeat a phase, results unchanged
    double x0[5], st, den;
    double delta;       // uniform
    double xi0[5], e[2], nu[2];
};

// phase-time instrumentation of the diagnostic build (-DPLAN_PROF, libmpcplan_prof.so, tools/plan_phase.py):
// each scope adds its own elapsed s_memtime ticks (inclusive of the phases nested in it) to an LDS counter
// (lane 0), summed into g_plan_prof at the end of the chunk
#ifdef PLAN_PROF
struct PhScope {
    ldsd* L;
    int off, ln;
    unsigned long long t0;
    __device__ PhScope(const Ctx& X, int p) : L(X.L), off(X.Y.oSC + 16 + p), ln(X.ln), t0(__builtin_amdgcn_s_memtime()) {}
    __device__ ~PhScope() {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (ln == 0) {
            PLAN_LDS_AS unsigned long long* q = (PLAN_LDS_AS unsigned long long*)(L + off);
#ifdef PLAN_PROF_COUNT
            *q += 1;                  // host emulation: entries per phase
#else
            *q += t - t0;
#endif
        }
    }
};
#define PHASE(p) PhScope ph_scope_(X, p)
// an explicitly closed span (phases that are not a scope of their own)
#define PhOpen(v, X, p) const unsigned long long v##_t0 = __builtin_amdgcn_s_memtime(); const int v##_p = (p)
#define PhClose(v)                                                                                              \
    do {                                                                                                        \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                             \
        if (X.ln == 0) *(PLAN_LDS_AS unsigned long long*)(X.L + X.Y.oSC + 16 + v##_p) += t_ - v##_t0;          \
    } while (0)
// calls of a phase (factorisations, solves), so that tools/plan_phase.py can report cycles per call and stage
#define PROF_COUNT(p)                                                                        \
    do {                                                                                     \
        if (X.ln == 0) *(PLAN_LDS_AS unsigned long long*)(X.L + X.Y.oSC + 16 + (p)) += 1ull; \
    } while (0)
#else
#define PHASE(p)
#define PROF_COUNT(p)
#define PhOpen(v, X, p)
#define PhClose(v)
#endif

__device__ inline bool act_bit(const Ctx& X, int o, int k, int j) {
    return (((unsigned)X.L[o + k]) >> j) & 1u;
}

__device__ inline void sync() { __syncthreads(); }

// interval Jacobians at the iterate: D1 = d def / d x_{k+1}, and (when R given) the rhs [-D0 | sg h e3, e4 | -def]
__device__ void interval_jac(const Ctx& X, const double xa[5], const double xb[5], double u1, double u2, double D1[25],
                             double* R) {
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
    dyn_jac(xa, ka, dka, Fa);
    dyn_jac(xb, kb, dkb, Fb);
    dyn_jac(xm, km, dkm, Fm);
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
            if (R) R[8 * i + j] = -((i == j ? -1.0 : 0.0) - sg * (h / 6.0) * (Fa[5 * i + j] + 4.0 * m0));
            D1[5 * i + j] = (i == j ? 1.0 : 0.0) - sg * (h / 6.0) * (4.0 * m1 + Fb[5 * i + j]);
        }
    if (R) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const double def = xb[i] - (xa[i] + sg * (h / 6.0) * (fa[i] + 4.0 * fm[i] + fb[i]));
            R[8 * i + 5] = i == 3 ? sg * h : 0.0;
            R[8 * i + 6] = i == 4 ? sg * h : 0.0;
            R[8 * i + 7] = -def;
        }
    }
}

// interval k's share of the Lagrangian Hessian (-y . def_k over (x_a, x_b)) folded into stage k's Hessian
// and gradient along x_{k+1} = A x_k + B w_k + c (A, B, c of this stage already in LDS)
__device__ void interval_hess_fold(Ctx& X, int k, const double xa[5], const double xb[5], double u1, double u2,
                                   const double y[5]) {
    ldsd* L = X.L;
    const Layout& Y = X.Y;
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
    double T[5][NZ], c[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
#pragma unroll
        for (int j = 0; j < 7; ++j) T[i][j] = L[Y.oAB + ab_at(k, i, j)];
        T[i][7] = 0.0;
        c[i] = L[Y.oAB + ab_at(k, i, 7)];
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
        for (int j = i; j < NZ; ++j) {
            double v = 0.0;
#pragma unroll
            for (int l = 0; l < 5; ++l) v += T[l][i] * HbT[l][j];
            if (i < 5) v += HabT[i][j];
            if (j < 5) v += HabT[j][i];
            if (i < 5 && j < 5) v += Haa[5 * i + j];
            L[Y.oH + HSTR * k + hx(i, j)] += v;
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
        L[Y.oGQ + ZS * k + i] += v;
    }
}

// the QP at the SQP iterate in ZB (stage-parallel); returns false (uniform) when a defect Jacobian is singular
__device__ bool build_qp(Ctx& X, bool frozen, bool exact) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    PHASE(PH_BUILD);
    const int N = UNI(X.N);
    const int fin_u = UNI(X.fin);
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    const plan_params& P = X.P;
    const double den = X.den;
    bool ok = true;
    for (int k = ln; k <= N; k += WAVE) {
        double x[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = L[Y.oZB + ZS * k + i];
#pragma unroll
        for (int i = 0; i < NH; ++i) L[Y.oH + HSTR * k + i] = 0.0;
#pragma unroll
        for (int i = 0; i < NZ; ++i) L[Y.oGQ + ZS * k + i] = 0.0;
        const double u1 = k < N ? L[Y.oZB + ZS * k + 5] : 0.0, u2 = k < N ? L[Y.oZB + ZS * k + 6] : 0.0;
        const double sl = k < N ? L[Y.oZB + ZS * k + 7] : 0.0;
        if (k < N) {
            L[Y.oH + HSTR * k + hx(0, 0)] = 2.0 * P.w_s / (den * den);
            L[Y.oH + HSTR * k + hx(1, 1)] = 2.0 * P.w_y;
            L[Y.oH + HSTR * k + hx(2, 2)] = 2.0 * P.w_y;
            L[Y.oH + HSTR * k + hx(5, 5)] = 2.0 * P.w_u;
            L[Y.oH + HSTR * k + hx(6, 6)] = 2.0 * P.w_u;
            L[Y.oH + HSTR * k + hx(7, 7)] = 2.0 * P.w_slack;
            L[Y.oGQ + ZS * k + 0] = -2.0 * P.w_s * (X.R.s_total - x[0]) / (den * den);
            L[Y.oGQ + ZS * k + 1] = 2.0 * P.w_y * x[1];
            L[Y.oGQ + ZS * k + 2] = 2.0 * P.w_y * x[2];
            L[Y.oGQ + ZS * k + 5] = 2.0 * P.w_u * u1;
            L[Y.oGQ + ZS * k + 6] = 2.0 * P.w_u * u2;
            L[Y.oGQ + ZS * k + 7] = 2.0 * P.w_slack * sl;
            double xb[5], D1[25], R[5 * 8];
#pragma unroll
            for (int i = 0; i < 5; ++i) xb[i] = L[Y.oZB + ZS * (k + 1) + i];
            interval_jac(X, x, xb, u1, u2, D1, R);
            if (!solve5<8>(D1, R)) {
                ok = false;
            } else {
#pragma unroll
                for (int i = 0; i < 5; ++i)
#pragma unroll
                    for (int j = 0; j < 8; ++j) L[Y.oAB + ab_at(k, i, j)] = R[8 * i + j];   // R's rows are [A B c]
                if (exact) {
                    double y[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) y[i] = L[Y.oMY + 5 * k + i];
                    interval_hess_fold(X, k, x, xb, u1, u2, y);
                }
            }
        }
        const double kk = x[3], v = x[4];
        const unsigned son = stage_on(k, N, fin_u);
        for (int j = 0; j < RS; ++j) {             // slot j (kind_slot); a slot without a row gets 0
            double gv = 0.0;
            switch ((son >> j) & 1u ? slot_kind(j, k, N) : -1) {
                case ROW_VMIN: gv = v + sl - P.v_min; break;
                case ROW_VMAX: gv = (frozen ? L[Y.oVLIM + k] : route_vmax(X.R, x[0])) - (v + sl); break;
                case ROW_LATP: gv = P.a_max - kk * v * v; break;
                case ROW_LATM: gv = P.a_max + kk * v * v; break;
                case ROW_KMIN: gv = kk - P.k_min; break;
                case ROW_KMAX: gv = P.k_max - kk; break;
                case ROW_U1MIN: gv = u1 - P.u_min[0]; break;
                case ROW_U1MAX: gv = P.u_max[0] - u1; break;
                case ROW_U2MIN: gv = u2 - P.u_min[1]; break;
                case ROW_U2MAX: gv = P.u_max[1] - u2; break;
                case ROW_S: gv = sl; break;
                case ROW_STERM: gv = x[0] - X.st / 2.0; break;
                default: gv = 0.0; break;
            }
            L[Y.oG + RS * k + j] = gv;
        }
        if (exact && k > 0 && !(fin_u && k == N)) {
            const double lp = L[Y.oMLAT + 2 * k], lm = L[Y.oMLAT + 2 * k + 1];
            L[Y.oH + HSTR * k + hx(3, 4)] += 2.0 * v * (lp - lm);
            L[Y.oH + HSTR * k + hx(4, 4)] += 2.0 * kk * (lp - lm);
        }
    }
    ok = wmin(ok ? 1.0 : 0.0) > 0.0;
    sync();
#pragma unroll
    for (int i = 0; i < 5; ++i) X.xi0[i] = X.x0[i] - L[Y.oZB + i];
    X.e[0] = X.st - L[Y.oZB + ZS * N + 0];
    X.e[1] = -L[Y.oZB + ZS * N + 4];
    X.delta = 0.0;
    return ok;
}

// the factorisation's stage Hessians HT = H + delta I + sum w a a' (stage-parallel); mode 0: w = lam / s
// (interior point), 1: RHO on the TACT rows (polish)
__device__ void stage_hess_par(Ctx& X, int mode) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    PHASE(PH_HESS);
    const int N = UNI(X.N);
    const int fin_u = UNI(X.fin);
    ldsd* L = X.L;
    const Layout Y = uni_layout(X.Y);
    if (mode == 0) {
        // the barrier weights w = lam / s, row-parallel, into DS (free at the top of an interior-point
        // iteration: the previous step has been taken)
        for (int q = ln; q < (N + 1) * RS; q += WAVE) {
            const RowAt r = row_at(L, Y.oZB, q, N, fin_u);
            const double w = L[Y.oLAM + q] / L[Y.oS + q];
            if (r.on) L[Y.oDS + q] = w;
        }
        sync();
    }
    for (int k = ln; k <= N; k += WAVE) {
        // only the 8 entries rows touch are stored (hs_slot); the rest of the factorisation Hessian is
        // H + delta I, formed where it is read (ht_at)
        double H[NH];
#pragma unroll
        for (int i = 0; i < NH; ++i) H[i] = 0.0;
        H[hx(0, 0)] = L[Y.oH + HSTR * k + hx(0, 0)];
        H[hx(3, 3)] = L[Y.oH + HSTR * k + hx(3, 3)];
        H[hx(3, 4)] = L[Y.oH + HSTR * k + hx(3, 4)];
        H[hx(4, 4)] = L[Y.oH + HSTR * k + hx(4, 4)];
        H[hx(4, 7)] = L[Y.oH + HSTR * k + hx(4, 7)];
        H[hx(5, 5)] = L[Y.oH + HSTR * k + hx(5, 5)];
        H[hx(6, 6)] = L[Y.oH + HSTR * k + hx(6, 6)];
        H[hx(7, 7)] = L[Y.oH + HSTR * k + hx(7, 7)];
        const int nv = k < N ? NZ : 5;
#pragma unroll
        for (int i = 0; i < NZ; ++i)
            if (i < nv) H[hx(i, i)] += X.delta;
        const double kb = L[Y.oZB + ZS * k + 3], vb = L[Y.oZB + ZS * k + 4];
        const unsigned act = mode == 0 ? 0u : (unsigned)L[Y.oTACT + k];
        for_rows(k, N, fin_u, [&](int kind, int j, bool on) {
            const double w = mode == 0 ? L[Y.oDS + RS * k + j] : (((act >> j) & 1u) ? RHO : 0.0);
            const bool use = on && w != 0.0;
            const RowSp r = row_sp(kind, k < N, kb, vb);
            const int a = hx(r.i0, r.i0), b = hx(r.i0, r.i1), c = hx(r.i1, r.i1);
            const double ha = H[a] + w * r.c0 * r.c0;
            H[a] = use ? ha : H[a];
            if (r.two) {
                const double hb = H[b] + w * r.c0 * r.c1;
                H[b] = use ? hb : H[b];
                const double hc = H[c] + w * r.c1 * r.c1;
                H[c] = use ? hc : H[c];
            }
        });
        ldsd* hs = L + Y.oH + HSTR * k + NH;
        hs[0] = H[hx(0, 0)];
        hs[1] = H[hx(3, 3)];
        hs[2] = H[hx(3, 4)];
        hs[3] = H[hx(4, 4)];
        hs[4] = H[hx(4, 7)];
        hs[5] = H[hx(5, 5)];
        hs[6] = H[hx(6, 6)];
        hs[7] = H[hx(7, 7)];
        hs[8] = 1.0 / H[hx(7, 7)];          // the third pivot's reciprocal, formed here stage-parallel (factor_par)
    }
}

// ------------------------------------------------------------------------------------------------------
// Riccati recursions on lanes 0..7 with DPP broadcasts (round 5; round 4 read P and [A B] element by element
// from LDS in every lane of an entry-parallel factorisation and broadcast the solves' vectors by readlane).
// Lane j holds column j of the stage matrices: of P (j < 5; P is symmetric, so its columns are its rows), of
// P [A B] and of M = HT + [A B]' P [A B] (j < 7: the five state columns, then u1, u2); in the solves and
// rollouts, component i of the co-state / state.  Every cross-lane term is one v_fmac_f64_dpp with
// row_newbcast:l -- lane l's register broadcast within the 16-lane row, fused into the FMA, one issue slot --
// so nothing of a recursion goes through LDS but the stage data it consumes.  Each sum accumulates its terms
// in the order oracle/plan_oracle.c uses (factor(), solve_core(), rollout(), multipliers()), one rounding per
// term, so the two agree bit for bit.  The symmetrisation P <- (Pn + Pn') / 2 pairs lane j's column with the
// row lane j needs from the other lanes by a per-lane selector (0.5 on the lane's own index, 0 elsewhere):
// fma(0.5, Pn(j, i), 0.5 Pn(i, j)) = 0.5 (Pn(i, j) + Pn(j, i)) exactly (scaling by 2 commutes with rounding).
// The recursions run on the whole wave (REC_LANES): the four 16-lane rows compute the same values (each
// broadcast stays within its row; lanes 7..15 of a row carry a zero column) and only row 0 stores.  Narrowing
// exec to lanes 0..7 made every FP64 instruction slower (tools/micro/dpp_lat.hip on the MI355X: v_fmac_f64
// 5.4 -> 7.2 cycles, its DPP form 7.3 -> 9.5, a division 77 -> 100), so the replicas cost nothing and save
// a quarter.  The host emulation (tools/plan_emu.cpp) runs every lane the same way.
// ------------------------------------------------------------------------------------------------------

#define REC_LANES(ln) true
#ifndef PLAN_HOST_EMU
// d += s@L * c: s broadcast from lane L of the 16-lane row (DPP row_newbcast), fused into the FMA.  Every asm
// block starts with s_nop 1, the two wait states a DPP read needs after a VALU write of its source.
#define PF(d, s, c, L) "v_fmac_f64_dpp " d ", " s ", " c " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#endif

// acc += sum_l src@l * c[l] (l = 0..4, in that order): one lane's dot product with a vector held one
// component per lane (the solves' A' p, A x, K x rows)
__device__ inline void dot5_lanes(double& acc, double src, const double c[5]) {
#ifndef PLAN_HOST_EMU
    asm("s_nop 1\n\t" PF("%0", "%1", "%2", 0) PF("%0", "%1", "%3", 1) PF("%0", "%1", "%4", 2) PF("%0", "%1", "%5", 3)
        PF("%0", "%1", "%6", 4)
        : "+&v"(acc) : "v"(src), "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]));
#else
    for (int l = 0; l < 5; ++l) acc = fma(dpp_row_bcast(src, l), c[l], acc);
#endif
}

// column j of P [A B]: q[i] = sum_l P(i, l) AB(l, j), P(i, l) = register i of lane l (oracle factor(): PA, PB)
__device__ inline void fac_pab(double q[5], const double Pc[5], const double abc[5]) {
#ifndef PLAN_HOST_EMU
#define PAB_L(L, A) PF("%0", "%5", A, L) PF("%1", "%6", A, L) PF("%2", "%7", A, L) PF("%3", "%8", A, L) PF("%4", "%9", A, L)
    asm("s_nop 1\n\t" PAB_L(0, "%10") PAB_L(1, "%11") PAB_L(2, "%12") PAB_L(3, "%13") PAB_L(4, "%14")
        : "+&v"(q[0]), "+&v"(q[1]), "+&v"(q[2]), "+&v"(q[3]), "+&v"(q[4])
        : "v"(Pc[0]), "v"(Pc[1]), "v"(Pc[2]), "v"(Pc[3]), "v"(Pc[4]), "v"(abc[0]), "v"(abc[1]), "v"(abc[2]), "v"(abc[3]),
          "v"(abc[4]));
#undef PAB_L
#else
    for (int l = 0; l < 5; ++l)
        for (int i = 0; i < 5; ++i) q[i] = fma(dpp_row_bcast(Pc[i], l), abc[l], q[i]);
#endif
}

// column j of M: m[u] += sum_l AB(l, u) (P [A B])(l, j), AB(l, u) = register l of lane u (oracle factor():
// the A'PA part of Pn, Hwx, Hww)
__device__ inline void fac_m(double m[8], const double abc[5], const double q[5]) {
#ifndef PLAN_HOST_EMU
#define M_L(S, C) PF("%0", S, C, 0) PF("%1", S, C, 1) PF("%2", S, C, 2) PF("%3", S, C, 3) PF("%4", S, C, 4) \
    PF("%5", S, C, 5) PF("%6", S, C, 6)
    asm("s_nop 1\n\t" M_L("%7", "%12") M_L("%8", "%13") M_L("%9", "%14") M_L("%10", "%15") M_L("%11", "%16")
        : "+&v"(m[0]), "+&v"(m[1]), "+&v"(m[2]), "+&v"(m[3]), "+&v"(m[4]), "+&v"(m[5]), "+&v"(m[6])
        : "v"(abc[0]), "v"(abc[1]), "v"(abc[2]), "v"(abc[3]), "v"(abc[4]), "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[3]),
          "v"(q[4]));
#undef M_L
#else
    for (int l = 0; l < 5; ++l)
        for (int u = 0; u < 7; ++u) m[u] = fma(dpp_row_bcast(abc[l], u), q[l], m[u]);
#endif
}

// the control block of M in every lane: (M55, M65, M66) = lane 5's m5, m6 and lane 6's m6
__device__ inline void fac_mww(double t[3], double m5, double m6) {
    t[0] = t[1] = t[2] = 0.0;
#ifndef PLAN_HOST_EMU
    const double one = 1.0;
    asm("s_nop 1\n\t" PF("%0", "%3", "%5", 5) PF("%1", "%4", "%5", 5) PF("%2", "%4", "%5", 6)
        : "+&v"(t[0]), "+&v"(t[1]), "+&v"(t[2]) : "v"(m5), "v"(m6), "v"(one));
#else
    t[0] = fma(dpp_row_bcast(m5, 5), 1.0, t[0]);
    t[1] = fma(dpp_row_bcast(m6, 5), 1.0, t[1]);
    t[2] = fma(dpp_row_bcast(m6, 6), 1.0, t[2]);
#endif
}

// column j of Pn = M_xx + Hwx' K: pn[i] += sum_r Hwx(r, i) K(r, j), Hwx(r, i) = m[5 + r] of lane i
__device__ inline void fac_pn(double pn[5], double m5, double m6, double m7, const double kc[3]) {
#ifndef PLAN_HOST_EMU
#define PN_I(D, L) PF(D, "%5", "%8", L) PF(D, "%6", "%9", L) PF(D, "%7", "%10", L)
    asm("s_nop 1\n\t" PN_I("%0", 0) PN_I("%1", 1) PN_I("%2", 2) PN_I("%3", 3) PN_I("%4", 4)
        : "+&v"(pn[0]), "+&v"(pn[1]), "+&v"(pn[2]), "+&v"(pn[3]), "+&v"(pn[4])
        : "v"(m5), "v"(m6), "v"(m7), "v"(kc[0]), "v"(kc[1]), "v"(kc[2]));
#undef PN_I
#else
    for (int i = 0; i < 5; ++i) {
        pn[i] = fma(dpp_row_bcast(m5, i), kc[0], pn[i]);
        pn[i] = fma(dpp_row_bcast(m6, i), kc[1], pn[i]);
        pn[i] = fma(dpp_row_bcast(m7, i), kc[2], pn[i]);
    }
#endif
}

// P column j = (Pn + Pn')(:, j) / 2: s[i] = 0.5 Pn(i, j) + sum_r Pn(r, i) sel[r] with sel[r] = 0.5 on lane r
__device__ inline void fac_sym(double s[5], const double pn[5], const double sel[5]) {
#pragma unroll
    for (int i = 0; i < 5; ++i) s[i] = 0.5 * pn[i];
#ifndef PLAN_HOST_EMU
#define SY_I(D, L) PF(D, "%5", "%10", L) PF(D, "%6", "%11", L) PF(D, "%7", "%12", L) PF(D, "%8", "%13", L) \
    PF(D, "%9", "%14", L)
    asm("s_nop 1\n\t" SY_I("%0", 0) SY_I("%1", 1) SY_I("%2", 2) SY_I("%3", 3) SY_I("%4", 4)
        : "+&v"(s[0]), "+&v"(s[1]), "+&v"(s[2]), "+&v"(s[3]), "+&v"(s[4])
        : "v"(pn[0]), "v"(pn[1]), "v"(pn[2]), "v"(pn[3]), "v"(pn[4]), "v"(sel[0]), "v"(sel[1]), "v"(sel[2]),
          "v"(sel[3]), "v"(sel[4]));
#undef SY_I
#else
    for (int i = 0; i < 5; ++i)
        for (int r = 0; r < 5; ++r) s[i] = fma(dpp_row_bcast(pn[r], i), sel[r], s[i]);
#endif
}

// acc += src@0 * c0 + src@1 * c1 (in that order): the lanes 0 and 1 components of a vector held one component
// per lane, into every lane's sum (the solves' B w and K' h terms)
__device__ inline void dot2_lanes(double& acc, double src, double c0, double c1) {
#ifndef PLAN_HOST_EMU
    asm("s_nop 1\n\t" PF("%0", "%1", "%2", 0) PF("%0", "%1", "%3", 1) : "+&v"(acc) : "v"(src), "v"(c0), "v"(c1));
#else
    acc = fma(dpp_row_bcast(src, 0), c0, acc);
    acc = fma(dpp_row_bcast(src, 1), c1, acc);
#endif
}

// LQ solve over the wave with zero initial state and homogeneous dynamics: stage linear terms at ogl -> odz
// (the caller syncs before reading odz).  Backward: p_{k} = gx_k + A_k' p_{k+1} + K_k' h_k with h = gw + B' p;
// lane i holds p_i and, for i < 2, h_i (its own dot product with B's column i), which the co-state update
// takes by broadcast; the control right-hand sides h_k go to odz's w slots, and after the recursion every
// stage forms its feed-forward kk_k = -(L D L')^-1 h_k at once (lane k).  Forward: x <- A x + B w with
// w = kk + K x; lane i holds x_i and, for i < 3, w_i (K's row i against x).  Each recursion loads stage k - 1's
// (k + 1's) data while it works on stage k.  Every sum keeps oracle solve_core()'s terms and order.
struct SolBk { double Br[5], Ac[5], Kc[3], h, h2, gx; };
struct SolFw { double Kr[5], Ar[5], b0, b1, t; };
__device__ inline void sol_load_bk(const ldsd* L, const Layout& Y, int ogl, int k, int me, int rh, SolBk& R) {
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        R.Br[l] = L[Y.oAB + ab_at(k, l, 5 + rh)];
        R.Ac[l] = L[Y.oAB + ab_at(k, l, me)];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) R.Kc[r] = L[Y.oK + 15 * k + 5 * r + me];
    R.h = L[ogl + ZS * k + 5 + rh];
    R.h2 = L[ogl + ZS * k + 7];
    R.gx = L[ogl + ZS * k + me];
}
__device__ inline void sol_load_fw(const ldsd* L, const Layout& Y, int odz, int k, int me, int rw, SolFw& R) {
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        R.Kr[l] = L[Y.oK + 15 * k + 5 * rw + l];
        R.Ar[l] = L[Y.oAB + ab_at(k, me, l)];
    }
    R.b0 = L[Y.oAB + ab_at(k, me, 5)];
    R.b1 = L[Y.oAB + ab_at(k, me, 6)];
    R.t = L[odz + ZS * k + 5 + rw];
}
__device__ void solve_core(const Ctx& X, int ogl, int odz) {
    const int N = UNI(X.N), ln = X.ln;
    ldsd* L = X.L;
    const Layout Y = uni_layout(X.Y);
    if (REC_LANES(ln)) {
        const int me = (ln & 15) < 5 ? (ln & 15) : 4, rh = (ln & 15) < 2 ? (ln & 15) : 1;
        double p = (ln & 15) < 5 ? L[ogl + ZS * N + me] : 0.0;
        auto step = [&](const SolBk& c, int k) {
            double h = c.h;                       // h_rh = gw_rh + sum_l B(l, rh) p_l
            dot5_lanes(h, p, c.Br);
            if (ln < 3) L[odz + ZS * k + 5 + ln] = ln < 2 ? h : c.h2;    // the w slots: h_0, h_1, h2 (one store)
            double v = c.gx;
            dot5_lanes(v, p, c.Ac);
            dot2_lanes(v, h, c.Kc[0], c.Kc[1]);   // + K(0, me) h_0 + K(1, me) h_1
            v = fma(c.Kc[2], c.h2, v);
            p = v;
        };
        // two stages per trip, alternating buffers: each stage's loads are in flight during the other's work
        SolBk ra, rb;
        sol_load_bk(L, Y, ogl, N - 1, me, rh, ra);
        int k = N - 1;
        for (; k >= 1; k -= 2) {
            sol_load_bk(L, Y, ogl, k - 1, me, rh, rb);
            step(ra, k);
            sol_load_bk(L, Y, ogl, k >= 2 ? k - 2 : 0, me, rh, ra);
            step(rb, k - 1);
        }
        if (k == 0) step(ra, 0);
    }
    sync();
    // feed-forward terms, stage-parallel: kk_k = -(L D L')^-1 h_k (oracle: the same chol3_solve per stage)
    for (int k = ln; k < N; k += WAVE) {
        double Lc[6], t[3];
#pragma unroll
        for (int i = 0; i < 6; ++i) Lc[i] = L[Y.oL + 6 * k + i];
#pragma unroll
        for (int r = 0; r < 3; ++r) t[r] = -L[odz + ZS * k + 5 + r];
        chol3_solve(Lc, t);
#pragma unroll
        for (int r = 0; r < 3; ++r) L[odz + ZS * k + 5 + r] = t[r];
    }
    sync();
    if (REC_LANES(ln)) {
        const int me = (ln & 15) < 5 ? (ln & 15) : 4, rw = (ln & 15) < 3 ? (ln & 15) : 2;
        double x = 0.0;
        auto step = [&](const SolFw& c, int k) {
            double w = c.t;                       // w_rw = kk_rw + sum_l K(rw, l) x_l
            dot5_lanes(w, x, c.Kr);
            double xn = 0.0;
            dot5_lanes(xn, x, c.Ar);
            dot2_lanes(xn, w, c.b0, c.b1);        // + B(me, 0) w_0 + B(me, 1) w_1
            // stage k overwritten after every lane has read its feed-forward term (program order within the
            // wave; the emulation's broadcasts above are barriers)
            // x_0..4 from lanes 0..4, w_0..2 from lanes 16..18 (row 1's copies of lanes 0..2): one store
            if (ln < 5 || (ln >= 16 && ln < 19)) L[odz + ZS * k + (ln < 16 ? ln : ln - 11)] = ln < 16 ? x : w;
            x = xn;
        };
        // two stages per trip, alternating buffers; a stage's feed-forward slots are read before the stage
        // before it is overwritten (the loads are issued first)
        SolFw fa, fb;
        sol_load_fw(L, Y, odz, 0, me, rw, fa);
        int k = 0;
        for (; k + 1 < N; k += 2) {
            sol_load_fw(L, Y, odz, k + 1, me, rw, fb);
            step(fa, k);
            sol_load_fw(L, Y, odz, k + 2 < N ? k + 2 : k + 1, me, rw, fa);
            step(fb, k + 1);
        }
        if (k < N) step(fa, k);
        if (ln < 5) L[odz + ZS * N + ln] = x;
        if (ln == 0)
#pragma unroll
            for (int i = 5; i < NZ; ++i) L[odz + ZS * N + i] = 0.0;
    }
}

// Riccati factorisation of the HT stage Hessians (uniform result: false when a control pivot is not positive,
// or the final chunk's terminal system is singular).  Per stage, backwards, lane j (oracle factor()):
//   q = P [A B](:, j)                        25 broadcast FMAs (P(i, l) from lane l)
//   m = HT(:, j) + [A B]' q                  35 broadcast FMAs ([A B](l, u) from lane u)
//   Mww = L D L' (every lane, from lanes 5 and 6), K(:, j) = -Mww^-1 Mwx(:, j), lanes 0..4 store it
//   P(:, j) <- sym(Mxx + Mwx' K)(:, j)       15 + 25 broadcast FMAs
// The slack has no dynamics (B's third column is zero), so its rows of Mww and Mwx are HT's: the third pivot
// is HT(7, 7) and the factor's (2, 0), (2, 1) entries are exact zeros, as in the oracle's chol3 of the same
// matrix.  Column j of HT comes from the packed H (+ delta on the diagonal) except at the 8 entries rows
// touch, which stage_hess_par stored in HS (ht_at).
__device__ bool factor_par(const Ctx& X) {
    const int N = UNI(X.N), ln = X.ln;
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    const int oAB = UNI(Y.oAB), oH = UNI(Y.oH), oK = UNI(Y.oK), oL = UNI(Y.oL);
    const double delta = X.delta;
    int okw = 1;
    if (REC_LANES(ln)) {
        const int j = (ln & 15) < 7 ? (ln & 15) : 7;
        // HT(u, j) of stage k: the slot or the packed H entry, at a per-lane offset in the stage's H block (no
        // select per stage); the non-slot diagonal entries (1, 1), (2, 2) add delta (ht_at: h + delta there):
        // v + dg1 with dg1 = delta on lane 1 and +0 elsewhere is fma(j == 1, delta, v) bit for bit
        int hoff[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int sl = hs_slot(u, j);
            hoff[u] = sl >= 0 ? NH + sl : hidx(u, j);
        }
        const double dg1 = j == 1 ? delta : 0.0, dg2 = j == 2 ? delta : 0.0;
        auto ht = [&](int k, int u) {
            const double v = L[oH + HSTR * k + hoff[u]];
            return u == 1 ? v + dg1 : (u == 2 ? v + dg2 : v);
        };
        double Pc[5], sel[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            Pc[i] = ht(N, i);
            sel[i] = (j == i) ? 0.5 : 0.0;
        }
        // column j of [A B c] (lanes 7..15: the c column, whose values no other lane reads), one stage offset
        const int abase = oAB + j;
        // one stage's inputs: column j of [A B], of HT (with delta) and HT(7, 7)
        struct FacIn { double abc[5], m[8], h77, r77; };
        auto load = [&](int k, FacIn& R) {
#pragma unroll
            for (int l = 0; l < 5; ++l) R.abc[l] = L[abase + ab_at(k, l, 0)];
#pragma unroll
            for (int u = 0; u < 8; ++u) R.m[u] = ht(k, u);
            R.h77 = L[oH + HSTR * k + NH + 7];
            R.r77 = L[oH + HSTR * k + NH + 8];
        };
        // one stage; false (uniform: every operand of a pivot is a broadcast or a uniform load) when a pivot is not
        // positive, after which the stage's stores are garbage the caller never reads
        auto step = [&](FacIn& c, int k) -> int {
            double* m = c.m;                  // M's column, formed in place over HT's (no register copies)
            double q[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
            fac_pab(q, Pc, c.abc);
            fac_m(m, c.abc, q);
            double t[3], Lc[6];
            fac_mww(t, m[5], m[6]);
            // chol3 of [[M55, ., .], [M65, M66, .], [0, 0, HT77]] (oracle chol3, same operations)
            const double d0 = t[0];
            Lc[0] = 1.0 / d0;
            Lc[1] = t[1] * Lc[0];
            const double d1 = t[2] - Lc[1] * t[1];
            Lc[2] = 1.0 / d1;
            Lc[3] = 0.0;
            Lc[4] = 0.0;
            Lc[5] = c.r77;                    // 1.0 / HT(7, 7), from stage_hess_par
            const int ok = d0 > 0.0 && d1 > 0.0 && c.h77 > 0.0;
            double kc[3] = {-m[5], -m[6], -m[7]};
            chol3_solve(Lc, kc);
            if (ln < 5)
#pragma unroll
                for (int r = 0; r < 3; ++r) L[oK + 15 * k + 5 * r + ln] = kc[r];
            if (ln == 0)
#pragma unroll
                for (int i = 0; i < 6; ++i) L[oL + 6 * k + i] = Lc[i];
            if (k > 0) {
                fac_pn(m, m[5], m[6], m[7], kc);    // Pn's column over M_xx's, in place
                fac_sym(Pc, m, sel);
            }
            return ok;
        };
        // two stages per trip, alternating buffers: a stage's inputs are in flight during the other's work; the
        // pivot test is a scalar branch
        FacIn fa, fb;
        load(N - 1, fa);
        int k = N - 1;
        for (; k >= 1; k -= 2) {
            load(k - 1, fb);
            okw = UNI(step(fa, k));
            if (!okw) break;
            load(k >= 2 ? k - 2 : 0, fa);
            okw = UNI(step(fb, k - 1));
            if (!okw) break;
        }
        if (okw && k == 0) okw = UNI(step(fa, 0));
    }
    if (!okw) return false;
    sync();
    if (X.fin) {
        for (int c = 0; c < 2; ++c) {
            for (int k = ln; k <= N; k += WAVE)
#pragma unroll
                for (int i = 0; i < NZ; ++i) L[Y.oGL + ZS * k + i] = (k == N && i == (c == 0 ? 0 : 4)) ? 1.0 : 0.0;
            sync();
            solve_core(X, Y.oGL, Y.oDZ);
            sync();
            for (int k = ln; k <= N; k += WAVE)
#pragma unroll
                for (int i = 0; i < NZ; ++i) L[Y.oEZ + 2 * ZS * k + ZS * c + i] = L[Y.oDZ + ZS * k + i];
            sync();
        }
        const double e0 = L[Y.oEZ + 2 * ZS * N + 0], e1 = L[Y.oEZ + 2 * ZS * N + ZS + 0];
        const double e2 = L[Y.oEZ + 2 * ZS * N + 4], e3 = L[Y.oEZ + 2 * ZS * N + ZS + 4];
        if (ln == 0) {
            L[Y.oSC + SC_EM0] = e0;
            L[Y.oSC + SC_EM1] = e1;
            L[Y.oSC + SC_EM2] = e2;
            L[Y.oSC + SC_EM3] = e3;
        }
        const double det = e0 * e3 - e1 * e2;
        if (!(fabs(det) > 0.0) || !isfinite(det)) return false;
    }
    return true;
}

// factorisation with the regularisation raised until the pivots are positive (uniform result)
__device__ bool factor_reg(Ctx& X, int mode) {
    for (;;) {
        stage_hess_par(X, mode);
        sync();
        bool ok;
        {
            PHASE(PH_FACTOR);
            ok = factor_par(X);
            sync();
        }
        PROF_COUNT(PH_NFACTOR);
        if (ok) return true;
        if (X.delta >= DELTA_MAX) return false;
        X.delta = X.delta > 0.0 ? 10.0 * X.delta : DELTA0;
    }
}

// full solve (GL filled and synced): DZ; meets E dz_N = rE exactly (final chunk); X.nu = terminal forces
__device__ void solve(Ctx& X, const double rE[2]) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    PHASE(PH_SOLVE);
    PROF_COUNT(PH_NSOLVE);
    ldsd* L = X.L;
    const Layout Y = uni_layout(X.Y);
    const int N = UNI(X.N);
    solve_core(X, Y.oGL, Y.oDZ);
    sync();
    double n0 = 0.0, n1 = 0.0;
    const int fin = UNI(X.fin);
    if (fin) {
        const double b0 = rE[0] - L[Y.oDZ + ZS * N + 0], b1 = rE[1] - L[Y.oDZ + ZS * N + 4];
        const double e0 = L[Y.oSC + SC_EM0], e1 = L[Y.oSC + SC_EM1], e2 = L[Y.oSC + SC_EM2], e3 = L[Y.oSC + SC_EM3];
        const double det = e0 * e3 - e1 * e2;
        n0 = (b0 * e3 - e1 * b1) / det;
        n1 = (e0 * b1 - e2 * b0) / det;
    }
    X.nu[0] = n0;
    X.nu[1] = n1;
    sync();
    if (fin)
        for (int k = ln; k <= N; k += WAVE)
#pragma unroll
            for (int i = 0; i < NZ; ++i)
                L[Y.oDZ + ZS * k + i] += n0 * L[Y.oEZ + 2 * ZS * k + i] + n1 * L[Y.oEZ + 2 * ZS * k + ZS + i];
    sync();
}

// dynamics-feasible start at oz: dx_0 = xi0, dw = 0 (lane i: x_i, the A x products broadcast by DPP; oracle
// rollout())
__device__ void rollout(const Ctx& X, int oz) {
    PHASE(PH_ROLLOUT);
    const int N = UNI(X.N), ln = X.ln;
    ldsd* L = X.L;
    const Layout Y = uni_layout(X.Y);
    if (REC_LANES(ln)) {
        const int me = (ln & 15) < 5 ? (ln & 15) : 4;
        double x = X.xi0[me];
        for (int k = 0; k <= N; ++k) {
            if (ln < 5) L[oz + ZS * k + ln] = x;
            if (ln == 0)
#pragma unroll
                for (int i = 5; i < NZ; ++i) L[oz + ZS * k + i] = 0.0;
            if (k == N) break;
            double Ar[5];
#pragma unroll
            for (int l = 0; l < 5; ++l) Ar[l] = L[Y.oAB + ab_at(k, me, l)];
            double v = L[Y.oAB + ab_at(k, me, 7)];
            dot5_lanes(v, x, Ar);
            x = v;
        }
    }
    sync();
}

// gradient of the QP objective 1/2 z'(H + delta I)z + gq'z at stage k
__device__ __forceinline__ void grad_f(const ldsd* L, const Layout& Y, int N, double delta, int k, int oz, double g[NZ]) {
    const int nv = k < N ? NZ : 5;
    double z[NZ], H[NH];
#pragma unroll
    for (int i = 0; i < NZ; ++i) z[i] = L[oz + ZS * k + i];
#pragma unroll
    for (int i = 0; i < NH; ++i) H[i] = L[Y.oH + HSTR * k + i];
#pragma unroll
    for (int i = 0; i < NZ; ++i) {
        double v = L[Y.oGQ + ZS * k + i] + (i < nv ? delta * z[i] : 0.0);
#pragma unroll
        for (int j = 0; j < NZ; ++j) v += H[hidx(i, j)] * z[j];
        g[i] = i < nv ? v : 0.0;
    }
}

// equality-constrained QP on the TACT rows (estimates TLAM), solution into TZ / TLAM; 0 = KKT-consistent,
// > 0 = offending rows (flipped in TACT), -1 = breakdown (uniform)
__device__ int eqp(Ctx& X, double scale) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    PHASE(PH_EQP);
    const int N = UNI(X.N);
    ldsd* L = X.L;
    const Layout Y = uni_layout(X.Y);
    const int fin_c = UNI(X.fin);
    const double e0 = X.e[0], e1 = X.e[1];
    for (int k = ln; k <= N; k += WAVE)
#pragma unroll
        for (int j = 0; j < RS; ++j) L[Y.oY + RS * k + j] = act_bit(X, Y.oTACT, k, j) ? L[Y.oTLAM + RS * k + j] : 0.0;
    sync();
    if (!factor_reg(X, 1)) return -1;
    const double delta = X.delta;
    rollout(X, Y.oTZ);
    for (int it = 0; it < AL_STEPS; ++it) {
        for (int k = ln; k <= N; k += WAVE) {
            double g[NZ], z[NZ];
            grad_f(L, Y, N, delta, k, Y.oTZ, g);
#pragma unroll
            for (int u = 0; u < NZ; ++u) z[u] = L[Y.oTZ + ZS * k + u];
            const double kb = L[Y.oZB + ZS * k + 3], vb = L[Y.oZB + ZS * k + 4];
            const unsigned act = (unsigned)L[Y.oTACT + k];
            for_rows(k, N, fin_c, [&](int kind, int j, bool on) {
                const bool use = on && ((act >> j) & 1u);
                const RowSp r = row_sp(kind, k < N, kb, vb);
                const double f = RHO * sp_dot(r, L[Y.oG + RS * k + j], z) - L[Y.oY + RS * k + j];
                const double g0 = g[r.i0] + f * r.c0;
                g[r.i0] = use ? g0 : g[r.i0];
                if (r.two) {
                    const double g1 = g[r.i1] + f * r.c1;
                    g[r.i1] = use ? g1 : g[r.i1];
                }
            });
#pragma unroll
            for (int u = 0; u < NZ; ++u) L[Y.oGL + ZS * k + u] = g[u];
        }
        sync();
        const double rE[2] = {e0 - L[Y.oTZ + ZS * N + 0], e1 - L[Y.oTZ + ZS * N + 4]};
        solve(X, rE);
        double upd = 0.0, ym = 0.0;
        for (int k = ln; k <= N; k += WAVE) {
#pragma unroll
            for (int u = 0; u < NZ; ++u) L[Y.oTZ + ZS * k + u] += L[Y.oDZ + ZS * k + u];
            double z[NZ];
#pragma unroll
            for (int u = 0; u < NZ; ++u) z[u] = L[Y.oTZ + ZS * k + u];
            const double kb = L[Y.oZB + ZS * k + 3], vb = L[Y.oZB + ZS * k + 4];
            const unsigned act = (unsigned)L[Y.oTACT + k];
            for_rows(k, N, fin_c, [&](int kind, int j, bool on) {
                const bool use = on && ((act >> j) & 1u);
                const double d = RHO * sp_dot(row_sp(kind, k < N, kb, vb), L[Y.oG + RS * k + j], z);
                const double y0 = L[Y.oY + RS * k + j], y = y0 - d;
                L[Y.oY + RS * k + j] = use ? y : y0;             // unpredicated store (no exec mask per row)
                upd = use ? fmax(upd, fabs(d)) : upd;
                ym = use ? fmax(ym, fabs(y)) : ym;
            });
        }
        upd = wmax(upd);
        ym = wmax(ym);
        sync();
        // the multiplier update has reached rounding level: further refinements change nothing
        if (upd <= AL_TOL * (1.0 + ym)) break;
    }
    double fin = 1.0;
    int bad = 0;
    const double tr = 1e-9 * scale, tl = 1e-9 * scale;
    for (int k = ln; k <= N; k += WAVE) {
#pragma unroll
        for (int u = 0; u < NZ; ++u) fin = isfinite(L[Y.oTZ + ZS * k + u]) ? fin : 0.0;
        unsigned mask = (unsigned)L[Y.oTACT + k];
        double z[NZ];
#pragma unroll
        for (int u = 0; u < NZ; ++u) z[u] = L[Y.oTZ + ZS * k + u];
        const double kb = L[Y.oZB + ZS * k + 3], vb = L[Y.oZB + ZS * k + 4];
        for_rows(k, N, fin_c, [&](int kind, int j, bool on) {
            const double rv = sp_dot(row_sp(kind, k < N, kb, vb), L[Y.oG + RS * k + j], z);
            const double y = L[Y.oY + RS * k + j];
            const bool in = (mask >> j) & 1u;
            if (on) L[Y.oTLAM + RS * k + j] = in ? y : 0.0;   // predicated: the terminal row shares a slot
            // bitwise, not short-circuit: no branch per row
            const bool flip = on & (in ? ((y < -tl) | (fabs(rv) > tr)) : (rv < -tr));
            mask = flip ? (mask ^ (1u << j)) : mask;
            bad += flip ? 1 : 0;
        });
        L[Y.oTACT + k] = (double)mask;
    }
    fin = wmin(fin);
    bad = wsumi(bad);
    sync();
    if (fin == 0.0) return -1;
    return bad;
}

// Mehrotra predictor-corrector interior point; solution in Z, S, LAM; 0 converged, 1 cap, -1 breakdown, 2
// checkpoint (first call only: mu and phi below MU_CHECK, every row's s and lambda CHECK_SEP apart); resume
// continues from Z, S, LAM, *iters, *phi_io (oracle ipm)
__device__ int ipm(Ctx& X, int* iters, bool resume, double* phi_io) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    PHASE(PH_IPM);
    const int N = UNI(X.N);
    ldsd* L = X.L;
    const Layout Y = uni_layout(X.Y);
    const int nq = (N + 1) * RS, nzq = (N + 1) * ZS;      // row slots, stage-variable slots
    // the context's scalars the iterations read, taken once (the context lives in private memory)
    const int dbg = UNI(X.dbg), fin_c = UNI(X.fin), max_iter = UNI(X.P.max_iter);
    const double tol = X.P.tol, e0 = X.e[0], e1 = X.e[1];
    if (!resume) rollout(X, Y.oZ);
    int m = 0;
    for (int k = ln; k <= N; k += WAVE) {
        double z[NZ];
#pragma unroll
        for (int u = 0; u < NZ; ++u) z[u] = L[Y.oZ + ZS * k + u];
        const double kb = L[Y.oZB + ZS * k + 3], vb = L[Y.oZB + ZS * k + 4];
        for_rows(k, N, fin_c, [&](int kind, int j, bool on) {
            if (!resume) {
                const double rv = sp_dot(row_sp(kind, k < N, kb, vb), L[Y.oG + RS * k + j], z);
                if (on) {
                    L[Y.oS + RS * k + j] = (rv > 0.0 ? rv : 0.0) + SHIFT0;
                    L[Y.oLAM + RS * k + j] = 1.0;
                }
            }
            m += on ? 1 : 0;
        });
    }
    m = wsumi(m);
    sync();
    double phi = resume ? *phi_io : 1.0;
    int it = resume ? *iters : 0, rc = 1;
    for (; it < max_iter; ++it) {
        double mu = 0.0;
        PhOpen(ph_red, X, PH_IRED);
        for (int k = ln; k <= N; k += WAVE) {
            const unsigned son = stage_on(k, N, fin_c);
#pragma unroll
            for (int j = 0; j < RS; ++j) {      // every slot, the stage's rows applied (see for_rows)
                const double t = mu + L[Y.oS + RS * k + j] * L[Y.oLAM + RS * k + j];
                mu = (son >> j) & 1u ? t : mu;
            }
        }
        mu = wsum(mu) / m;
        PhClose(ph_red);
        if (!isfinite(mu)) { rc = -1; break; }
        if (mu <= tol && phi <= 1e-12) { rc = 0; break; }
        if (!resume && mu <= MU_CHECK && phi <= MU_CHECK) {
            double tie = 0.0;
            for (int q = ln; q < nq; q += WAVE) {
                const RowAt r = row_at(L, Y.oZB, q, N, fin_c);
                const double sv = L[Y.oS + q], lv = L[Y.oLAM + q];
                if (r.on && !(sv > CHECK_SEP * lv || lv > CHECK_SEP * sv)) tie = 1.0;
            }
            if (wmax(tie) == 0.0) { rc = 2; break; }
        }
        if (dbg & 1) (void)factor_reg(X, 0);
        if (!factor_reg(X, 0)) { rc = -1; break; }
        const double delta = X.delta;
        const double rE[2] = {e0 - L[Y.oZ + ZS * N + 0], e1 - L[Y.oZ + ZS * N + 4]};
        for (int pass = 0; pass < 2; ++pass) {
            double sigma_mu = 0.0;
            if (pass == 1) {
                PhOpen(ph_r1, X, PH_IRED);
                double am = 1.0;
                for (int q = ln; q < nq; q += WAVE) {
                    const RowAt r = row_at(L, Y.oZB, q, N, fin_c);
                    const double dsa = L[Y.oDSA + q], dla = L[Y.oDLA + q];
                    const double rs = -L[Y.oS + q] / dsa, rl = -L[Y.oLAM + q] / dla;
                    am = (r.on && dsa < 0.0) ? fmin(am, rs) : am;
                    am = (r.on && dla < 0.0) ? fmin(am, rl) : am;
                }
                am = wmin(am);
                double mua = 0.0;
                for (int k = ln; k <= N; k += WAVE) {
                    const unsigned son = stage_on(k, N, fin_c);
#pragma unroll
                    for (int j = 0; j < RS; ++j) {
                        const double t = mua + (L[Y.oS + RS * k + j] + am * L[Y.oDSA + RS * k + j]) *
                                                   (L[Y.oLAM + RS * k + j] + am * L[Y.oDLA + RS * k + j]);
                        mua = (son >> j) & 1u ? t : mua;
                    }
                }
                mua = wsum(mua) / m;
                const double ratio = mua / mu;
                sigma_mu = ratio * ratio * ratio * mu;
                PhClose(ph_r1);
            }
            PhOpen(ph_g, X, PH_IGRAD);
            for (int rp_ = 0; rp_ < 1 + ((dbg >> 2) & 1); ++rp_) {
                // each row's f = l + (rs - l rp) / s, row-parallel, into DS (free until this pass's
                // direction rows write it); then each stage folds its rows into the gradient in row order
                for (int q = ln; q < nq; q += WAVE) {
                    const RowAt r = row_at(L, Y.oZB, q, N, fin_c);
                    const double s = L[Y.oS + q], l = L[Y.oLAM + q];
                    double rs = -s * l;
                    if (pass == 1) rs += sigma_mu - L[Y.oDSA + q] * L[Y.oDLA + q];
                    double sp = L[Y.oG + q] + r.c0 * L[Y.oZ + ZS * r.k + r.i0];
                    const double sp2 = sp + r.c1 * L[Y.oZ + ZS * r.k + r.i1];
                    sp = r.two ? sp2 : sp;
                    const double rp = sp - s;
                    const double f = l + (rs - l * rp) / s;
                    if (r.on) L[Y.oDS + q] = f;
                }
                sync();
                for (int k = ln; k <= N; k += WAVE) {
                    double g[NZ];
                    grad_f(L, Y, N, delta, k, Y.oZ, g);
                    const double kb = L[Y.oZB + ZS * k + 3], vb = L[Y.oZB + ZS * k + 4];
                    for_rows(k, N, fin_c, [&](int kind, int j, bool on) {
                        const RowSp r = row_sp(kind, k < N, kb, vb);
                        const double f = L[Y.oDS + RS * k + j];
                        const double g0 = g[r.i0] - f * r.c0;
                        g[r.i0] = on ? g0 : g[r.i0];
                        if (r.two) {
                            const double g1 = g[r.i1] - f * r.c1;
                            g[r.i1] = on ? g1 : g[r.i1];
                        }
                    });
#pragma unroll
                    for (int u = 0; u < NZ; ++u) L[Y.oGL + ZS * k + u] = g[u];
                }
                sync();
            }
            PhClose(ph_g);
            if (dbg & 2) solve(X, rE);
            solve(X, rE);
            const int ods = pass == 0 ? Y.oDSA : Y.oDS, odl = pass == 0 ? Y.oDLA : Y.oDL;
            PhOpen(ph_d, X, PH_IDIR);
            for (int rp_ = 0; rp_ < 1 + ((dbg >> 3) & 1); ++rp_)
            for (int q = ln; q < nq; q += WAVE) {
                const RowAt r = row_at(L, Y.oZB, q, N, fin_c);
                const double s = L[Y.oS + q], l = L[Y.oLAM + q];
                double rs = -s * l;
                if (pass == 1) rs += sigma_mu - L[Y.oDSA + q] * L[Y.oDLA + q];
                const int zk = ZS * r.k;
                double v = L[Y.oG + q] + r.c0 * L[Y.oZ + zk + r.i0];
                const double v2 = v + r.c1 * L[Y.oZ + zk + r.i1];
                v = r.two ? v2 : v;
                v -= s;
                v += r.c0 * L[Y.oDZ + zk + r.i0];
                const double v3 = v + r.c1 * L[Y.oDZ + zk + r.i1];
                v = r.two ? v3 : v;
                const double dl = (rs - l * v) / s;
                if (r.on) {
                    L[ods + q] = v;
                    L[odl + q] = dl;
                }
            }
            sync();
            PhClose(ph_d);
        }
        PhOpen(ph_r2, X, PH_IRED);
        double amax = 1.0 / TAU, fin = 1.0;
        for (int q = ln; q < nq; q += WAVE) {
            const RowAt r = row_at(L, Y.oZB, q, N, fin_c);
            const double ds = L[Y.oDS + q], dl = L[Y.oDL + q];
            const double rs = -L[Y.oS + q] / ds, rl = -L[Y.oLAM + q] / dl;
            amax = (r.on && ds < 0.0) ? fmin(amax, rs) : amax;
            amax = (r.on && dl < 0.0) ? fmin(amax, rl) : amax;
        }
        for (int q = ln; q < nzq; q += WAVE)
            if (q % ZS < NZ) fin = isfinite(L[Y.oDZ + q]) ? fin : 0.0;
        amax = wmin(amax);
        fin = wmin(fin);
        const double alpha = fmin(1.0, TAU * amax);
        if (!isfinite(alpha) || fin == 0.0) { rc = -1; break; }
        for (int q = ln; q < nzq; q += WAVE)
            if (q % ZS < NZ) L[Y.oZ + q] += alpha * L[Y.oDZ + q];
        for (int q = ln; q < nq; q += WAVE) {
            const RowAt r = row_at(L, Y.oZB, q, N, fin_c);
            const double sn = L[Y.oS + q] + alpha * L[Y.oDS + q];
            const double ln_ = L[Y.oLAM + q] + alpha * L[Y.oDL + q];
            if (r.on) {
                L[Y.oS + q] = sn;
                L[Y.oLAM + q] = ln_;
            }
        }
        sync();
        PhClose(ph_r2);
        phi *= 1.0 - alpha;
    }
    sync();
    *iters = it;
    *phi_io = phi;
    return rc;
}

// copy the polish result (TZ, TLAM, TACT) to the solution (Z, LAM, ACT)
__device__ void accept_polish(const Ctx& X, bool with_act) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    for (int k = ln; k <= X.N; k += WAVE) {
#pragma unroll
        for (int u = 0; u < NZ; ++u) L[Y.oZ + ZS * k + u] = L[Y.oTZ + ZS * k + u];
#pragma unroll
        for (int j = 0; j < RS; ++j) L[Y.oLAM + RS * k + j] = L[Y.oTLAM + RS * k + j];
        if (with_act) L[Y.oACT + k] = L[Y.oTACT + k];
    }
    sync();
}

// interior-point classification (s < lam) of stage k as a bit mask
__device__ double ipm_mask(const Ctx& X, int k) {
    const unsigned son = stage_on(k, X.N, X.fin);
    unsigned m = 0;
#pragma unroll
    for (int j = 0; j < RS; ++j)
        if (((son >> j) & 1u) && X.L[X.Y.oS + RS * k + j] < X.L[X.Y.oLAM + RS * k + j]) m |= 1u << j;
    return (double)m;
}

// one QP: 0 solved (KKT point), 1 interior-point answer without a certified polish, -1 failure (uniform)
__device__ int qp_solve(Ctx& X, bool have_cls, int* iters) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    const int N = UNI(X.N);
    const int fin_u = UNI(X.fin);
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    double scale = 1.0;
    for (int k = ln; k <= N; k += WAVE) {
        const unsigned son = stage_on(k, N, fin_u);
#pragma unroll
        for (int j = 0; j < RS; ++j) scale = (son >> j) & 1u ? fmax(scale, fabs(L[Y.oG + RS * k + j])) : scale;
    }
    scale = wmax(scale);
    *iters = 0;
    if (have_cls) {
        for (int k = ln; k <= N; k += WAVE) {
            L[Y.oTACT + k] = L[Y.oACT + k];
#pragma unroll
            for (int j = 0; j < RS; ++j) L[Y.oTLAM + RS * k + j] = L[Y.oLAM + RS * k + j];
        }
        sync();
        for (int round = 0; round < WARM_ROUNDS; ++round) {
            const int bad = eqp(X, scale);
            if (bad < 0) break;
            if (bad == 0) {
                accept_polish(X, true);
                return 0;
            }
        }
    }
    double phi = 1.0;
    int rc = ipm(X, iters, false, &phi);
    if (rc == 2) {
        // checkpoint (oracle qp_solve): polish from the loose interior point's classification; the interior
        // point resumes where it stopped if that does not certify
        for (int k = ln; k <= N; k += WAVE) {
            L[Y.oTACT + k] = ipm_mask(X, k);
#pragma unroll
            for (int j = 0; j < RS; ++j) L[Y.oTLAM + RS * k + j] = L[Y.oLAM + RS * k + j];
        }
        sync();
        for (int round = 0; round < CHECK_ROUNDS; ++round) {
            const int bad = eqp(X, scale);
            if (bad < 0) break;
            if (bad == 0) {
                accept_polish(X, true);
                return 0;
            }
        }
        rc = ipm(X, iters, true, &phi);
    }
    if (rc < 0) return -1;
    const double nu_ipm[2] = {X.nu[0], X.nu[1]};
    for (int k = ln; k <= N; k += WAVE) {
        L[Y.oTACT + k] = ipm_mask(X, k);
#pragma unroll
        for (int j = 0; j < RS; ++j) L[Y.oTLAM + RS * k + j] = L[Y.oLAM + RS * k + j];
    }
    sync();
    for (int round = 0; round < POLISH_ROUNDS; ++round) {
        const int bad = eqp(X, scale);
        if (bad < 0) break;
        if (bad == 0) {
            accept_polish(X, true);
            return 0;
        }
    }
    for (int k = ln; k <= N; k += WAVE) L[Y.oACT + k] = ipm_mask(X, k);
    sync();
    X.nu[0] = nu_ipm[0];
    X.nu[1] = nu_ipm[1];
    return rc == 0 ? 1 : -1;
}

// NLP multipliers from the QP solution (oracle multipliers()): MY, MLAT
__device__ void multipliers(Ctx& X) {
    PHASE(PH_MULT);
    const int N = UNI(X.N);
    const int fin_u = UNI(X.fin);
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    // stage gradients of the Lagrangian minus the rows (x part) into GL; lateral multipliers
    for (int k = X.ln; k <= N; k += WAVE) {
        double g[NZ];
        grad_f(L, Y, N, X.delta, k, Y.oZ, g);
        L[Y.oMLAT + 2 * k] = 0.0;
        L[Y.oMLAT + 2 * k + 1] = 0.0;
        const double kb = L[Y.oZB + ZS * k + 3], vb = L[Y.oZB + ZS * k + 4];
        for_rows(k, N, fin_u, [&](int kind, int j, bool on) {
            const RowSp r = row_sp(kind, k < N, kb, vb);
            const double l = L[Y.oLAM + RS * k + j];
            const double g0 = g[r.i0] - l * r.c0;
            g[r.i0] = on ? g0 : g[r.i0];
            if (r.two) {
                const double g1 = g[r.i1] - l * r.c1;
                g[r.i1] = on ? g1 : g[r.i1];
            }
            if (on && kind == ROW_LATP) L[Y.oMLAT + 2 * k] = l;
            if (on && kind == ROW_LATM) L[Y.oMLAT + 2 * k + 1] = l;
        });
#pragma unroll
        for (int u = 0; u < 5; ++u) L[Y.oGL + ZS * k + u] = g[u];
    }
    sync();
    // co-states: PI[k] = pi_{k+1} (lane i: pi_i, the A' pi products broadcast by DPP)
    if (REC_LANES(X.ln)) {
        const int ln = X.ln, me = (ln & 15) < 5 ? (ln & 15) : 4;
        double pi = L[Y.oGL + ZS * N + me];
        if (fin_u) pi += me == 0 ? X.nu[0] : (me == 4 ? X.nu[1] : 0.0);
        for (int k = N - 1; k >= 0; --k) {
            if (ln < 5) L[Y.oPI + 5 * k + ln] = pi;
            if (k > 0) {
                double Ac[5];
#pragma unroll
                for (int l = 0; l < 5; ++l) Ac[l] = L[Y.oAB + ab_at(k, l, me)];
                double v = L[Y.oGL + ZS * k + me];
                dot5_lanes(v, pi, Ac);
                pi = v;
            }
        }
    }
    // y_k = D1_k^-T pi_{k+1} (stage-parallel; D1 at the iterate ZB)
    for (int k = X.ln; k < N; k += WAVE) {
        double xa[5], xb[5], D1[25], D1t[25], y[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            xa[i] = L[Y.oZB + ZS * k + i];
            xb[i] = L[Y.oZB + ZS * (k + 1) + i];
        }
        interval_jac(X, xa, xb, L[Y.oZB + ZS * k + 5], L[Y.oZB + ZS * k + 6], D1, nullptr);
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) D1t[5 * i + j] = D1[5 * j + i];
#pragma unroll
        for (int i = 0; i < 5; ++i) y[i] = L[Y.oPI + 5 * k + i];
        const bool ok = solve5<1>(D1t, y);
#pragma unroll
        for (int i = 0; i < 5; ++i) L[Y.oMY + 5 * k + i] = ok ? y[i] : 0.0;
    }
    sync();
}

// the NLP's cost (:128-170) and L1 violation at ZB + alpha * DZV (stage-parallel, reduced)
// cost and violation at ZB + alpha DZV.  GS < WAVE: each group of GS lanes (GS >= N + 1) evaluates its own
// alpha, the sums reduced within the group -- the same butterfly as wsum's last log2(GS) levels, whose first
// levels only add the idle lanes' exact zeros, so every group's sums are wsum's for its alpha bit for bit
__device__ void cost_viol(const Ctx& X, double alpha, double* f, double* viol, int GS = WAVE) {
    const int ln = X.ln & (GS - 1);      // the lane within its group
    PHASE(PH_LSEARCH);
    const int N = UNI(X.N);
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    const plan_params& P = X.P;
    auto zv = [&](int k, int i) { return L[Y.oZB + ZS * k + i] + (alpha != 0.0 ? alpha * L[Y.oDZV + ZS * k + i] : 0.0); };
    double c = 0.0, v = 0.0;
    if (ln == 0)
        for (int i = 0; i < 5; ++i) v += fabs(zv(0, i) - X.x0[i]);
    for (int k = ln; k <= N; k += GS) {
        double x[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = zv(k, i);
        const double u1 = k < N ? zv(k, 5) : 0.0, u2 = k < N ? zv(k, 6) : 0.0, sl = k < N ? zv(k, 7) : 0.0;
        if (k < N) {
            const double e = (X.R.s_total - x[0]) / X.den;
            c += P.w_y * (x[1] * x[1] + x[2] * x[2]) + P.w_s * e * e + P.w_u * (u1 * u1 + u2 * u2) + P.w_slack * (sl * sl);
            double xb[5], def[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) xb[i] = zv(k + 1, i);
            defect(X.R, P, x, xb, u1, u2, def);
#pragma unroll
            for (int i = 0; i < 5; ++i) v += fabs(def[i]);
        }
        const double kk = x[3], vv = x[4];
        // the rows' violations in storage order (a per-lane array indexed at run time would live in scratch)
        auto add = [&](bool on, double g) { v = on ? v + (g < 0.0 ? -g : 0.0) : v; };
        const bool sp = !(X.fin && k == N);
        add(sp, vv + sl - P.v_min);
        add(sp, L[Y.oVL + k] - (vv + sl));
        add(sp && k > 0, P.a_max - kk * vv * vv);
        add(sp && k > 0, P.a_max + kk * vv * vv);
        add(k > 0, kk - P.k_min);
        add(k > 0, P.k_max - kk);
        add(k < N, u1 - P.u_min[0]);
        add(k < N, P.u_max[0] - u1);
        add(k < N, u2 - P.u_min[1]);
        add(k < N, P.u_max[1] - u2);
        add(k < N, sl);
        add(k == N && !X.fin, x[0] - X.st / 2.0);
        if (k == N && X.fin) v += fabs(x[0] - X.st) + fabs(x[4]);
    }
    for (int o = GS >> 1; o > 0; o >>= 1) {
        c += __shfl_xor(c, o, WAVE);
        v += __shfl_xor(v, o, WAVE);
    }
    *f = c;
    *viol = v;
}

__device__ double cost_dir(const Ctx& X) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    PHASE(PH_LSEARCH);
    const int N = UNI(X.N);
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    const plan_params& P = X.P;
    double v = 0.0;
    for (int k = ln; k < N; k += WAVE) {
        v += 2.0 * P.w_y * (L[Y.oZB + ZS * k + 1] * L[Y.oDZV + ZS * k + 1] + L[Y.oZB + ZS * k + 2] * L[Y.oDZV + ZS * k + 2]);
        v += -2.0 * P.w_s * (X.R.s_total - L[Y.oZB + ZS * k]) / (X.den * X.den) * L[Y.oDZV + ZS * k];
        v += 2.0 * P.w_u * (L[Y.oZB + ZS * k + 5] * L[Y.oDZV + ZS * k + 5] + L[Y.oZB + ZS * k + 6] * L[Y.oDZV + ZS * k + 6]);
        v += 2.0 * P.w_slack * L[Y.oZB + ZS * k + 7] * L[Y.oDZV + ZS * k + 7];
    }
    return wsum(v);
}

__device__ inline ldsd* lds_p(const Ctx& X) { return X.L; }

// one chunk NLP (trajectory_planning.py:351-390) at X.x0, X.st, X.fin, X.N, set by the caller: the plan is
// left in the LDS block (ZB); returns the status, the interior-point iterations and QPs in *total_out, *nq_out
__device__ __forceinline__ int solve_chunk(Ctx& X, int* total_out, int* nq_out) {
    const int ln = X.ln;            // the lane, once (the context lives in private memory)
    const int N = UNI(X.N);
    X.den = fmax(1.0, X.R.s_total - X.x0[0]);
    X.nu[0] = X.nu[1] = 0.0;
    X.delta = 0.0;
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    // initial guess (:357-376)
    const double dss = (X.st - X.x0[0]) / N;
    for (int k = ln; k <= N; k += WAVE) {
#pragma unroll
        for (int i = 0; i < NZ; ++i) L[Y.oZB + ZS * k + i] = 0.0;
        L[Y.oZB + ZS * k + 0] = k == N ? X.st : X.x0[0] + k * dss;
        L[Y.oZB + ZS * k + 4] = X.fin ? (k == N ? 0.0 : X.x0[4] + k * ((0.0 - X.x0[4]) / N)) : X.x0[4];
#pragma unroll
        for (int i = 0; i < NZ; ++i) L[Y.oZ2 + ZS * k + i] = L[Y.oZB + ZS * k + i];
    }
    sync();
    int status = PLAN_NOT_CONVERGED, total = 0, nq = 0, since = 0;
    bool have_cls = false, frozen = false;
    double last = INFINITY, mu_m = 0.0, hf[LS_MEMORY], hv[LS_MEMORY];
    int nh = 0;
    for (int it = 0; it < X.P.sqp_iters; ++it, ++since) {
        bool exact = last <= EXACT_STEP || it >= EXACT_AFTER;
        int rc = -1;
        for (;;) {
            if (X.dbg & 16) (void)build_qp(X, frozen, exact);
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
        if (X.dbg & 32) multipliers(X);
        multipliers(X);
        double full = 0.0, mu_l = 0.0;
        for (int k = ln; k <= N; k += WAVE) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                const double d = (k < N || i < 5) ? L[Y.oZ + ZS * k + i] : 0.0;
                L[Y.oDZV + ZS * k + i] = d;
                full = fmax(full, fabs(d));
            }
            if (k < N)
#pragma unroll
                for (int i = 0; i < 5; ++i) mu_l = fmax(mu_l, 2.0 * fabs(L[Y.oMY + 5 * k + i]));
            const unsigned son = stage_on(k, N, X.fin);
#pragma unroll
            for (int j = 0; j < RS; ++j) mu_l = (son >> j) & 1u ? fmax(mu_l, 2.0 * fabs(L[Y.oLAM + RS * k + j])) : mu_l;
        }
        full = wmax(full);
        mu_m = fmax(mu_m, wmax(mu_l));
        if (X.fin) mu_m = fmax(mu_m, 2.0 * fmax(fabs(X.nu[0]), fabs(X.nu[1])));
        sync();
        double alpha = 1.0;
        if (full > LS_FULL) {
            for (int k = ln; k <= N; k += WAVE) L[Y.oVL + k] = frozen ? L[Y.oVLIM + k] : route_vmax(X.R, L[Y.oZB + ZS * k]);
            sync();
            double f0, v0;
            cost_viol(X, 0.0, &f0, &v0);
            const double dd = cost_dir(X) - mu_m * v0;
            hf[nh % LS_MEMORY] = f0;
            hv[nh % LS_MEMORY] = v0;
            ++nh;
            double m0 = -INFINITY;
            for (int i = 0; i < (nh < LS_MEMORY ? nh : LS_MEMORY); ++i) m0 = fmax(m0, hf[i] + mu_m * hv[i]);
            // backtracking alpha = 1, 1/2, ...: G = WAVE / GS trials at once, trial ls + g on lane group g (the
            // halvings are exact, so group g's alpha * 2^-g is the serial loop's alpha); the first accepted trial
            // in order wins, the last one (LS_STEPS - 1) unconditionally, as in the serial loop
            const int GS = N + 1 <= 16 ? 16 : (N + 1 <= 32 ? 32 : WAVE), G = WAVE / GS, g = ln / GS;
            const double gsc = g == 0 ? 1.0 : (g == 1 ? 0.5 : (g == 2 ? 0.25 : 0.125)), gstep = G == 4 ? 0.0625 : (G == 2 ? 0.25 : 0.5);
            for (int ls = 0;; ls += G) {
                const double ag = alpha * gsc;
                double f1, v1;
                if (X.dbg & 64) cost_viol(X, ag, &f1, &v1, GS);
                cost_viol(X, ag, &f1, &v1, GS);
                const bool acc = ls + g < LS_STEPS && (f1 + mu_m * v1 <= m0 + LS_ARMIJO * ag * dd || ls + g == LS_STEPS - 1);
                const double first = wmin(acc ? (double)g : (double)G);
                if (first < (double)G) {
                    alpha *= first == 0.0 ? 1.0 : (first == 1.0 ? 0.5 : (first == 2.0 ? 0.25 : 0.125));
                    break;
                }
                alpha *= gstep;
            }
        }
        double step = 0.0, back2 = 0.0, fin = 1.0;
        for (int k = ln; k <= N; k += WAVE)
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                if (k == N && i >= 5) continue;
                const double zo = L[Y.oZB + ZS * k + i];
                const double zn = zo + alpha * L[Y.oDZV + ZS * k + i];
                step = fmax(step, fabs(zn - zo));
                back2 = fmax(back2, fabs(zn - L[Y.oZ2 + ZS * k + i]));
                fin = isfinite(zn) ? fin : 0.0;
            }
        step = wmax(step);
        back2 = wmax(back2);
        fin = wmin(fin);
        if (fin == 0.0) { status = PLAN_NUMERICAL; break; }
        for (int k = ln; k <= N; k += WAVE)
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                if (k == N && i >= 5) continue;
                const double zo = L[Y.oZB + ZS * k + i];
                L[Y.oZ2 + ZS * k + i] = zo;
                L[Y.oZB + ZS * k + i] = zo + alpha * L[Y.oDZV + ZS * k + i];
            }
        sync();
        last = step;
        if (step <= X.P.sqp_tol) { status = frozen ? PLAN_FROZEN_LIMITS : PLAN_OK; break; }
        if (since >= 2 && back2 <= CYCLE_REL * step) {
            if (frozen) break;
            for (int k = ln; k <= N; k += WAVE)
                L[Y.oVLIM + k] = fmin(route_vmax(X.R, L[Y.oZB + ZS * k]), route_vmax(X.R, L[Y.oZ2 + ZS * k]));
            frozen = true;
            since = -1;
            for (int k = ln; k <= N; k += WAVE)
#pragma unroll
                for (int i = 0; i < NZ; ++i) L[Y.oZ2 + ZS * k + i] = L[Y.oZB + ZS * k + i];
            sync();
        }
    }
    if (status == PLAN_FROZEN_LIMITS) {
        double bad = 0.0;
        for (int k = ln; k <= N; k += WAVE)
            if (L[Y.oZB + ZS * k + 4] + (k < N ? L[Y.oZB + ZS * k + 7] : 0.0) > route_vmax(X.R, L[Y.oZB + ZS * k]) + 1e-9)
                bad = 1.0;
        if (wmax(bad) > 0.0) status = PLAN_NOT_CONVERGED;
    }
    *total_out = total;
    *nq_out = nq;
    return status;
}

struct KArgs {
    DevRoute R;
    plan_params P;
    int B, Nmax, Nfixed, dbg;
    const int* order;          // dispatch order (plan_order_kernels): workgroup w solves chunk order[w]; NULL = w
    const int* N;
    const double *x0, *st;
    const int* fin;
    double *X, *U, *S;
    int *status, *iters, *sqp;
};

__global__ void __launch_bounds__(WAVE) plan_chunk_kernel(KArgs a) {
    PLAN_LDS_DECL;
    const int b = a.order ? a.order[blockIdx.x] : (int)blockIdx.x;
    Ctx X;
    X.R = a.R;
    X.P = a.P;
    X.Y = make_layout(a.Nmax);
    X.L = (ldsd*)lds;
    X.ln = threadIdx.x;
    X.dbg = a.dbg;
    X.N = a.N ? a.N[b] : a.Nfixed;
    if (X.N < 1 || X.N > a.Nmax) {
        // a per-chunk horizon outside [1, Nmax] (device arrays are not validated on the host): no solve, zero
        // plan, status PLAN_NUMERICAL (the chunk's LDS block is sized for Nmax)
        for (int k = threadIdx.x; k <= a.Nmax; k += WAVE) {
            if (a.X)
                for (int i = 0; i < 5; ++i) a.X[((size_t)b * (a.Nmax + 1) + k) * 5 + i] = 0.0;
            if (k < a.Nmax) {
                if (a.U) a.U[((size_t)b * a.Nmax + k) * 2] = a.U[((size_t)b * a.Nmax + k) * 2 + 1] = 0.0;
                if (a.S) a.S[(size_t)b * a.Nmax + k] = 0.0;
            }
        }
        if (threadIdx.x == 0) {
            if (a.status) a.status[b] = PLAN_NUMERICAL;
            if (a.iters) a.iters[b] = 0;
            if (a.sqp) a.sqp[b] = 0;
        }
        return;
    }
    const int N = UNI(X.N);
    X.fin = a.fin ? (a.fin[b] != 0) : 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) X.x0[i] = a.x0[5 * (size_t)b + i];
    X.st = a.st[b];
#ifdef PLAN_PROF
    if (X.ln == 0)
        for (int i = 0; i < 16; ++i) *(PLAN_LDS_AS unsigned long long*)(lds_p(X) + X.Y.oSC + 16 + i) = 0ull;
    sync();
    const unsigned long long t_total0 = __builtin_amdgcn_s_memtime();
#endif
    int total = 0, nq = 0;
    const int status = solve_chunk(X, &total, &nq);
    ldsd* L = X.L;
    const Layout& Y = X.Y;
    // outputs: rows past this chunk's N are zero
    const int Nm = a.Nmax;
    for (int k = X.ln; k <= Nm; k += WAVE) {
        if (a.X)
#pragma unroll
            for (int i = 0; i < 5; ++i) a.X[((size_t)b * (Nm + 1) + k) * 5 + i] = k <= N ? L[Y.oZB + ZS * k + i] : 0.0;
        if (k < Nm) {
            if (a.U) {
                a.U[((size_t)b * Nm + k) * 2 + 0] = k < N ? L[Y.oZB + ZS * k + 5] : 0.0;
                a.U[((size_t)b * Nm + k) * 2 + 1] = k < N ? L[Y.oZB + ZS * k + 6] : 0.0;
            }
            if (a.S) a.S[(size_t)b * Nm + k] = k < N ? L[Y.oZB + ZS * k + 7] : 0.0;
        }
    }
    if (X.ln == 0) {
        if (a.status) a.status[b] = status;
        if (a.iters) a.iters[b] = total;
        if (a.sqp) a.sqp[b] = nq;
    }
#ifdef PLAN_PROF
    if (X.ln == 0) {
        *(PLAN_LDS_AS unsigned long long*)(lds_p(X) + X.Y.oSC + 16 + PH_OTHER) = __builtin_amdgcn_s_memtime() - t_total0;
        for (int i = 0; i < PH_NSLOTS; ++i)
            atomicAdd(&g_plan_prof[i], *(PLAN_LDS_AS unsigned long long*)(lds_p(X) + X.Y.oSC + 16 + i));
        atomicAdd(&g_plan_prof[15], 1ull);
    }
#endif
}

// The receding-horizon loop of optimize_full_trajectory (trajectory_planning.py:491-548) on the device: wave
// b runs plan b's chunks one after another from starts[b], with no barrier across plans (a launch over B plans
// lasts as long as the slowest plan's chain of chunks, not the sum over rounds of each round's slowest chunk).
// Chunk n of plan b: remaining = s_total - s; final when remaining < 2 max_chunk_size (size = remaining, else
// max_chunk_size); N = ceil(size / avg[int(s / 5)] * 2 / 0.3) with avg[i] = mean(vmax[i:]) (the reference's
// np.mean over the speed-limit array, :507, computed by the caller); the chunk's plan, horizon, final flag and
// status go to slot (b, n); the next start is X[N/2] (the reference's commit of the first int(N/2)
// intervals, :523-541) or X[N] after a final chunk.  The loop ends when remaining <= 0.1 or after
// max_chunks chunks; nchunks[b] = chunks run, or -(n + 1) when chunk n's horizon is outside [1, Nmax] (or
// int(s / 5) past the end of avg), the reference's ValueError.
struct LArgs {
    DevRoute R;
    plan_params P;
    int B, Nmax, max_chunks, nav;
    double max_chunk_size;
    const double* avg;
    const double* starts;
    double *X, *U, *S;
    int *N, *fin, *status, *iters, *sqp, *nchunks;
};

__global__ void __launch_bounds__(WAVE) plan_loop_kernel(LArgs a) {
    PLAN_LDS_DECL;
    const int b = blockIdx.x;
    Ctx X;
    X.R = a.R;
    X.P = a.P;
    X.Y = make_layout(a.Nmax);
    X.L = (ldsd*)lds;
    X.ln = threadIdx.x;
    X.dbg = 0;
    const Layout& Y = X.Y;
    const int Nm = a.Nmax;
    double x0[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) x0[i] = a.starts[5 * (size_t)b + i];
    int n = 0;
    bool err = false;
    for (; n < a.max_chunks; ++n) {
        const double rem = a.R.s_total - x0[0];
        if (!(rem > 0.1)) break;
        const int fin = rem < a.max_chunk_size * 2.0 ? 1 : 0;
        const double size = fin ? rem : a.max_chunk_size;
        // vmax[int(s / 5):] with Python's slice rules: truncation toward zero, a negative index counts from the
        // end (clamped at the start), an index past the end leaves an empty slice (nan: the reference raises)
        const double si = x0[0] / 5.0;
        if (!(si < (double)a.nav)) { err = true; break; }
        int idx = si <= -(double)a.nav ? 0 : (int)si;
        if (idx < 0) idx += a.nav;
        const double hz = ceil(size / a.avg[idx] * 2.0 / 0.3);
        if (!(hz >= 1.0 && hz <= (double)Nm)) { err = true; break; }
        X.N = (int)hz;
        X.fin = fin;
#pragma unroll
        for (int i = 0; i < 5; ++i) X.x0[i] = x0[i];
        X.st = x0[0] + size;
        int total = 0, nq = 0;
        const int status = solve_chunk(X, &total, &nq);
        const int N = UNI(X.N);
        const size_t slot = (size_t)b * a.max_chunks + n;
        ldsd* L = X.L;
        for (int k = X.ln; k <= Nm; k += WAVE) {
#pragma unroll
            for (int i = 0; i < 5; ++i) a.X[(slot * (Nm + 1) + k) * 5 + i] = k <= N ? L[Y.oZB + ZS * k + i] : 0.0;
            if (k < Nm) {
                a.U[(slot * Nm + k) * 2 + 0] = k < N ? L[Y.oZB + ZS * k + 5] : 0.0;
                a.U[(slot * Nm + k) * 2 + 1] = k < N ? L[Y.oZB + ZS * k + 6] : 0.0;
                a.S[slot * Nm + k] = k < N ? L[Y.oZB + ZS * k + 7] : 0.0;
            }
        }
        if (X.ln == 0) {
            a.N[slot] = N;
            a.fin[slot] = fin;
            a.status[slot] = status;
            a.iters[slot] = total;
            a.sqp[slot] = nq;
        }
        const int c = fin ? N : N / 2;
#pragma unroll
        for (int i = 0; i < 5; ++i) x0[i] = L[Y.oZB + ZS * c + i];
        sync();          // every lane has its next start before the next chunk rewrites the block
    }
    if (X.ln == 0) a.nchunks[b] = err ? -(n + 1) : n;
}

// Longest-first dispatch (a scheduling hint; every chunk's result is independent of the order).  A launch
// lasts as long as its slowest chunk, and the slow chunks are the ones whose path the vehicle cannot follow
// at the speed limit: a route curvature beyond the curvature bound, or one whose lateral acceleration at
// the limit exceeds a_max (on traj3 a spike of |kappa| = 1 at s = 720 m makes chunks nearby need 50-100 SQP
// iterations and up to 2000 interior-point iterations).  Score of chunk b: the largest of |kappa| / k_max and
// |kappa| vmax^2 / a_max over ORDER_SAMPLES points of [s0, s0 + 1.5 (s_target - s0)]; the chunks are
// dispatched by score bucket, highest first (ORDER_BUCKETS power-of-two buckets from 1/4 up), so the
// expensive ones start with the launch instead of wherever their index puts them.
constexpr int ORDER_SAMPLES = 32;
constexpr int ORDER_BUCKETS = 8;
__device__ inline int order_bucket(const DevRoute& R, const plan_params& P, double s0, double st) {
    double sc = 0.0;
    const double kb = fmax(fabs(P.k_min), fabs(P.k_max));
    for (int i = 0; i < ORDER_SAMPLES; ++i) {
        const double s = s0 + (1.5 * (st - s0)) * ((double)i / (ORDER_SAMPLES - 1));
        const double k = fabs(route_kappa(R, s, nullptr, nullptr)), vm = route_vmax(R, s);
        sc = fmax(sc, fmax(k / kb, k * vm * vm / P.a_max));
    }
    // bucket 0 = highest: score >= 16; then [8, 16), ..., [0.25, 0.5); the last bucket holds the rest
    int q = 0;
    for (double th = 16.0; q < ORDER_BUCKETS - 1 && !(sc >= th); th *= 0.5) ++q;
    return q;
}
__global__ void plan_order_count_kernel(DevRoute R, plan_params P, int B, const double* x0, const double* st,
                                        int* bucket, int* cnt) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int q = order_bucket(R, P, x0[5 * (size_t)b], st[b]);
    bucket[b] = q;
    atomicAdd(&cnt[q], 1);
}
__global__ void plan_order_scatter_kernel(int B, const int* bucket, const int* cnt, int* cur, int* order) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int q = bucket[b];
    int off = 0;
    for (int i = 0; i < q; ++i) off += cnt[i];
    order[off + atomicAdd(&cur[q], 1)] = b;
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

}  // namespace

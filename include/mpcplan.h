/* mpcplan.h — C ABI of the MI355X batched offline planner (libmpcplan.so).
 *
 * Replaces the chunk solve of the reference's offline planner:
 *   TrajectoryOptimizer.optimize(x0, s_target, s_total, k_ref_fun, v_min_fun, v_max_fun, is_final_chunk)
 *   (/root/reference/trajectory_planning.py:351-390): a Hermite-Simpson collocation NLP over
 *   z = [X (N+1)x5, U Nx2, S N] (:91-126) with the cost of :128-170 and the constraints of :172-349, solved
 *   by scipy SLSQP (maxiter 500, ftol 1e-4, :381-387).
 * and the route functions it is called with (optimize_full_trajectory, :437-477): k_ref_fun (curvature of
 * the route's parametric CubicSpline at t = s_to_t(s), :439-459) and v_max_fun (interp1d kind='previous'
 * over the route's speed-limit array, :463-473); v_min_fun = 0 (:476-477).
 *
 * Here B independent chunks (any mix of routes' positions, intermediate or final) are solved in one call:
 * a Gauss-Newton SQP on the same NLP, each QP by a Mehrotra primal-dual interior point on the stage-wise
 * Riccati recursion, FP64.  One 64-lane wavefront (one workgroup) per chunk, the chunk's whole working set
 * in that workgroup's LDS; stage-parallel work runs lane k on stage k ("Offline planner").
 *
 * Reference quirks restated:
 *   - the defect rule.  The committed source computes x_pred = x_k - dt/6 (f_k + 4 f_mid + f_{k+1})
 *     (:205); the committed planner outputs (the trajectories JSON files) satisfy x_{k+1} = x_k + dt/6 (...)
 *     instead (v_{k+1} - v_k = +dt u2_k to 1e-10 on all three).  defect_sign = +1 (default) is the rule the
 *     outputs obey, -1 the source's literal sign;
 *   - the intermediate-chunk terminal row is s_N >= s_target / 2 (:238-246), half of the ABSOLUTE target;
 *   - the slack only relaxes the speed bounds' lower side in effect (v + S >= v_min, v + S <= v_max, S >= 0);
 *     the last state has no slack (:253-256);
 *   - v_max(s) below the first route knot is NaN in the reference (interp1d 'previous' extrapolation); here
 *     it is the first knot's limit.
 * The final chunk's terminal equalities (s_N = s_target, v_N = 0, :221-236) are solved exactly; there the
 * speed and lateral-acceleration rows of x_N, which v_N = 0 satisfies, are left out.  The rows of x_0 alone
 * (curvature, lateral acceleration) are constants fixed by x0 and are left out (x_0 = x0 is exact).
 */
#ifndef MPCPLAN_H
#define MPCPLAN_H

#ifdef __cplusplus
extern "C" {
#endif

#define MPCPLAN_VERSION 3     /* 3: the host backend (device = -1) */
#define PLAN_MAX_N 64          /* collocation intervals per chunk */

/* status[] codes */
#define PLAN_OK 0              /* SQP converged (a QP moved z by <= sqp_tol)                          */
#define PLAN_NOT_CONVERGED 1   /* sqp_iters QPs ran (or a 2-cycle) without convergence; last iterate   */
#define PLAN_QP_FAILED 2       /* a QP's interior point did not converge (infeasible linearisation)   */
#define PLAN_NUMERICAL 3       /* non-finite values; last finite iterate                               */
#define PLAN_FROZEN_LIMITS 4   /* converged after freezing the speed limits at a band change (a 2-cycle:
                                  the reference NLP has no optimum there), feasible for the reference rows */

/* return codes */
#define PLAN_SUCCESS 0
#define PLAN_E_ARG (-1)
#define PLAN_E_DEVICE (-2)
#define PLAN_E_ALLOC (-3)
#define PLAN_E_LAUNCH (-4)

/* TrajectoryOptimizer.__init__ (trajectory_planning.py:14-47) plus solver knobs. */
typedef struct {
    int N;                 /* intervals, when plan_solve_chunks gets no per-chunk N (reference: :515)   */
    double dt;             /* 0.3 s (:514)                                                             */
    double w_y, w_s, w_u, w_slack;   /* 10, 10, 0.1, 100 (:14)                                         */
    double u_min[2], u_max[2];       /* (-0.6, -5), (0.6, 4) (:35-36)                                  */
    double k_min, k_max;             /* -0.8, 0.8 (:43-44)                                             */
    double a_max;                    /* 6 (:47)                                                        */
    double v_min;                    /* 0 (v_min_fun, :476-477)                                        */
    double defect_sign;              /* +1 (see the header comment)                                    */
    int sqp_iters;                   /* cap on QPs per chunk (reference: SLSQP maxiter 500)             */
    double sqp_tol;                  /* converged when a QP moves z by <= sqp_tol (max norm)            */
    int max_iter;                    /* interior-point iterations per QP                                */
    double tol;                      /* interior-point tolerance (complementarity, row residuals)       */
} plan_params;

typedef struct plan_ctx plan_ctx;

void plan_default_params(plan_params* p);

/* The route (optimize_full_trajectory's reference path, :435-477), copied into the context:
 *   s[M]        cumulative chord length of the detailed way-points (unpack_reference_path, :411-414),
 *               strictly increasing; s_total = s[M-1];
 *   cx, cy      [M-1][4] coefficients of the parametric CubicSpline x(t), y(t) over t = 0..M-1
 *               (path_planning.create_spline), scipy PPoly order: row i holds c[0..3, i], the cubic first;
 *   vmax[M]     speed limit at each way-point in m/s (:464-467).
 * device >= 0: HIP device index.  device = -1: the host backend (csrc/plan_host.h): the same chunk algorithm in
 * IEEE double on std::thread workers (PLAN_CPU_THREADS, default every hardware thread), no HIP call; it serves
 * plan_solve_chunks, plan_optimize (the chunk loop on the CPU, one plan per worker), plan_route_eval,
 * plan_set_params and plan_destroy, and the device-pointer entries (plan_solve_chunks_device,
 * plan_optimize_device, plan_chunks_per_cu) fail on it with PLAN_E_DEVICE.  The reference's planner is CPU
 * code (scipy SLSQP, :381-387); this is the library's CPU path behind the same entries. */
int plan_create(const double* s, int M, const double* cx, const double* cy, const double* vmax,
                const plan_params* p, int device, plan_ctx** out);

/* B chunks, host buffers, synchronous.  Per chunk b: x0[b][5] (current_x0, :486/:548), s_target[b]
 * (:503), is_final[b] (:494-499), N[b] (NULL: params N; each <= PLAN_MAX_N).  s_total is the route's.
 * Outputs with row stride Nmax = max over b of N[b]: X[b][Nmax+1][5], U[b][Nmax][2], S[b][Nmax] (rows past
 * a chunk's own N are zero), status[b], iters[b] (interior-point iterations, all QPs), sqp[b] (QPs run);
 * any output pointer may be NULL.  Never fails because a chunk did not converge (status[]). */
int plan_solve_chunks(plan_ctx* c, int B, const int* N, const double* x0, const double* s_target,
                      const int* is_final, double* X, double* U, double* S, int* status, int* iters,
                      int* sqp);

/* Same with device pointers, asynchronous on `stream` (hipStream_t; NULL = the null stream).  Nmax is the
 * row stride of X, U and S in every case and must bound every N[b]; with N NULL every chunk has the params'
 * horizon N and Nmax < params N is PLAN_E_ARG (rows past a chunk's horizon are written as zero).  A chunk
 * whose N[b] lies outside [1, Nmax] is not solved (zero plan, status PLAN_NUMERICAL).  The kernel needs no
 * scratch memory: each chunk's working set lives in LDS (about 2.1 KB per stage, sized for Nmax; Nmax is
 * limited by the device's LDS per workgroup, 64 at 160 KB).  Batches of 128 .. 2^17 chunks are dispatched
 * longest first through a small per-context pool of order buffers (at most 8, allocated by the first eager
 * calls that need them, freed by plan_destroy); each buffer is reused only after the chunk kernel that last
 * read it has finished (an event, so eager calls on any streams stay correct).  A call made while `stream` is
 * being captured into a HIP graph uses no pool buffer (index order, the same results) and allocates nothing,
 * so graphs and eager calls never share a buffer. */
int plan_solve_chunks_device(plan_ctx* c, int B, int Nmax, const int* N, const double* x0,
                             const double* s_target, const int* is_final, double* X, double* U, double* S,
                             int* status, int* iters, int* sqp, void* stream);

/* Chunks resident per compute unit for a plan_solve_chunks_device launch whose LDS is sized for Nmax (the
 * kernel's registers and Nmax's LDS block; one wavefront per chunk), in *out.  A batch of mixed horizons
 * solves fastest in as few launches as keep this number: every horizon whose own launch would reach the
 * same residency goes into one launch sized for the largest of them, with per-chunk N (a launch lasts as
 * long as its slowest chunk, and the in-launch longest-first order starts that chunk first).  No reference
 * counterpart: the reference solves one chunk at a time (trajectory_planning.py:491). */
int plan_chunks_per_cu(plan_ctx* c, int Nmax, int* out);

/* The chunk loop of optimize_full_trajectory (trajectory_planning.py:491-548) for B plans, on the device,
 * asynchronous on `stream`; device pointers.  Replaces the host loop over chunks (:491) for a batch of start
 * states: each plan advances on its own wavefront, chunk after chunk, with no barrier across plans.
 *   starts[B][5]        first current_x0 of each plan (:486; the reference's is all zeros)
 *   max_chunk_size      :419 (20 m); a chunk is final when the remaining distance is < 2 max_chunk_size
 *   max_chunks          chunks per plan at most (the reference has no cap); also the slot count below
 *   avg[nav]            avg[i] = mean(vmax[i:]) over the route's speed-limit array (:507, np.mean, which
 *                       the caller computes so that N matches the host loop bit for bit)
 *   Nmax                bounds every chunk's N = ceil(size / avg[int(s / 5)] * 2 / 0.3) (:507-515)
 * Outputs per plan b and chunk slot n < max_chunks (slot = b * max_chunks + n): X[slot][Nmax+1][5],
 * U[slot][Nmax][2], S[slot][Nmax] (the chunk's whole plan, rows past its N zero), N[slot], is_final[slot],
 * status[slot], iters[slot], sqp[slot]; nchunks[b] = chunks run, or -(n + 1) when chunk n's N falls outside
 * [1, Nmax] or int(s / 5) past the end of avg (the reference raises there; a negative index counts from the
 * end, as a Python slice does).  The committed trajectory is the first
 * int(N/2) intervals of each non-final chunk and the whole final chunk (:523-541), which the caller
 * concatenates (trajectory_planning.optimize_full_trajectory_batch).  No scratch memory; capturable. */
int plan_optimize_device(plan_ctx* c, int B, int Nmax, const double* starts, double max_chunk_size, int max_chunks,
                         const double* avg, int nav, double* X, double* U, double* S, int* N, int* is_final,
                         int* status, int* iters, int* sqp, int* nchunks, void* stream);

/* plan_optimize_device with host buffers, synchronous (inputs staged, outputs copied back): the same
 * arguments and outputs, slot = b * max_chunks + n.  Lets a host caller run the device chunk loop without a
 * device allocator of its own.  On a host context (device = -1) the loop runs on the CPU, one plan per worker
 * (the same chunk sequence and outputs). */
int plan_optimize(plan_ctx* c, int B, int Nmax, const double* starts, double max_chunk_size, int max_chunks,
                  const double* avg, int nav, double* X, double* U, double* S, int* N, int* is_final, int* status,
                  int* iters, int* sqp, int* nchunks);

/* Route functions, for tests: kappa(s) and dkappa/ds (k_ref_fun, :445-459), v_max(s); on the device, or on the
 * CPU for a host context. */
int plan_route_eval(plan_ctx* c, int n, const double* s, double* kappa, double* dkappa, double* vmax);

int plan_set_params(plan_ctx* c, const plan_params* p);
const char* plan_last_error(void);   /* thread-local */
int plan_version(void);
void plan_destroy(plan_ctx* c);

#ifdef __cplusplus
}
#endif
#endif

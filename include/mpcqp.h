/*
 * mpcqp.h — C ABI of the MI355X batched tracking-MPC solver (libmpcqp.so).
 *
 * Drop-in boundary for the reference's hot path:
 *   TrajectoryTracker.solve(x0, obstacles) -> (u0, pred_X, solve_time)
 *       medinammartin3/Safe-Autonomous-Driving-MPC  trajectory_tracking.py:213-263
 *   with its read-only state: TrajectoryTracker.__init__ params  (trajectory_tracking.py:12-47)
 *   and the reference signal  TrajectoryLoader                  (trajectory_loader.py:13-102).
 *
 * A reference-side binding (ctypes) is shown in INTEGRATION.md; the package's
 * trajectory_tracking.py is that binding.
 *
 * Conventions
 *   - all arrays are plain row-major float64 / int32, caller-owned;
 *   - per-instance solver outcomes go to status[] and never fail the call
 *     (the reference ignores SLSQP's status, trajectory_tracking.py:260-263);
 *   - API misuse returns a negative MPC_E* code and sets mpc_last_error();
 *   - a context is bound to one HIP device, or to the host backend (device = -1), and is not re-entrant.
 *   - Without a GPU, mpc_create with a device index >= 0 fails loudly (MPC_E_DEVICE); device = -1 selects the
 *     host (CPU) backend explicitly (BASELINE config 1, the reference's CPU path): the same solver, outputs
 *     and status codes on host threads (csrc/cpu_backend.h; MPC_CPU_THREADS sets the thread count).
 */
#ifndef MPCQP_H
#define MPCQP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: status[] / hist_status[] may carry the MPC_SQP_UNCONVERGED flag (16) OR-ed onto the code; mask with
 *    MPC_STATUS_MASK before comparing with MPC_OK .. MPC_NUMERICAL (version 1 returned 0-3 only).
 * 3: the ego-shard communicator (mpc_comm_*, mpc_gather*, MPC_E_COMM); nothing else changed. */
#define MPCQP_VERSION 3
#define MPC_MAX_N 63          /* horizon limit (one lane per stage k=0..N in the kernel)   */
#define MPC_MAX_OBS 64        /* obstacle slab limit per instance                            */

/* status[] codes */
#define MPC_OK 0              /* QP solved to tolerance, hard constraints satisfied          */
#define MPC_MAX_ITER 1        /* iteration limit hit; best iterate returned                  */
#define MPC_INFEASIBLE 2      /* solved, but elastic slack active: hard QP(ubar) infeasible  */
#define MPC_NUMERICAL 3       /* numerical breakdown; best iterate returned                  */
/* flag OR-ed onto the last QP's code (status & MPC_STATUS_MASK) when sqp_iters > 1 and sqp_tol > 0 and the
 * SQP stopped without a QP moving U by <= sqp_tol: the sqp_iters cap, a 2-cycle or the elastic-QP streak */
#define MPC_SQP_UNCONVERGED 16
#define MPC_STATUS_MASK 15

/* return codes */
#define MPC_SUCCESS 0
#define MPC_E_ARG (-1)
#define MPC_E_DEVICE (-2)
#define MPC_E_ALLOC (-3)
#define MPC_E_LAUNCH (-4)
#define MPC_E_COMM (-5)       /* RCCL missing or a collective failed (mpc_comm_*, mpc_gather*)   */

/* Mirrors TrajectoryTracker.__init__ (trajectory_tracking.py:17-47) plus solver knobs.
 * Field names follow the reference attributes.  mpc_default_params() fills the reference values. */
typedef struct mpc_params {
    int N;                          /* horizon                      :18 (reference default 5)  */
    int max_obs;                    /* obstacle slab width per instance in the batch arrays    */
    double dt;                      /* control period               :17                        */
    double u_min[2], u_max[2];      /* (u1 curvature rate, u2 accel) bounds   :31-32           */
    double vehicle_radius;          /* :33 */
    double w_d, w_o, w_v, w_u1, w_u2;  /* :36-40 */
    double obstacle_safety_distance;   /* :43 */
    double max_time_2_obs;          /* :44 */
    double wheelbase;               /* :45 */
    double lane_width;              /* :46 */
    double safe_lane_margin;        /* :47 */
    double brake_distance;          /* warm start: obstacle closer than this -> brake (:232, 40.0)  */
    double brake_accel;             /* warm start braking control u2 (:240, -2.0)                    */
    /* solver */
    int linearization;              /* 1 = Gauss-Newton (reference slopes, default), 0 = frozen refs  */
    int sqp_iters;                  /* QP solves per call (at most, see sqp_tol): 1 = single QP at ubar
                                       (the tracking-QP parity gate); > 1 = Gauss-Newton SQP on the
                                       reference's nonlinear problem, re-linearised about each solution;
                                       0 = no solve: U = ubar, Xpred = predict(x0, ubar)              */
    int max_iter;                   /* PDIP iteration cap per QP                                     */
    int polish;                     /* 0 off; 1 active-set polish of the interior-point result;
                                       2 (default) crossover first: the active-set solve from the
                                       unconstrained optimum, the interior point only if it fails       */
    double tol;                     /* relative primal/dual residual tolerance                        */
    double tol_mu;                  /* absolute complementarity tolerance                             */
    double elastic_rho;             /* L1 penalty of the elastic (soft) state rows                    */
    double sqp_tol;                 /* SQP stops early once a re-linearised QP moves U by at most this
                                       (max-norm), and also (sqp_tol > 0) on a 2-cycle, i.e. a QP that
                                       returns U of two QPs back (|U_k - U_k-2| <= 1e-6 |U_k - U_k-1|),
                                       and after 5 elastic (infeasible) QPs in a row; 0 = always run
                                       sqp_iters QPs                                                  */
} mpc_params;

typedef struct mpc_ctx mpc_ctx;

/* Fill p with the reference values of trajectory_tracking.py:17-47 (N=5) and solver defaults. */
void mpc_default_params(mpc_params* p);

/* Create a context on HIP device `device` (>= 0), or on the host backend (device = -1).
 * X: T x 5 reference states (s,d,o,k,v), U: Tu x 2
 * reference controls, exactly the arrays of the trajectory JSON (trajectory_loader.py:22-24);
 * the strict-monotone s fix of trajectory_loader.py:26-30 is applied here.  The table is copied
 * to device memory (owned by the context).  Replaces TrajectoryLoader(...) + TrajectoryTracker(X_ref). */
int mpc_create(const double* X, int T, const double* U, int Tu, const mpc_params* p, int device,
               mpc_ctx** out);

/* Batched TrajectoryTracker.solve (trajectory_tracking.py:213-263), host buffers, synchronous.
 *   x0     [B][5]              current states
 *   obs    [B][max_obs][2]     (s, v) of each obstacle, or NULL (no obstacles).  Passing obs with
 *                              params.max_obs == 0 is an error (MPC_E_ARG): it would ignore them.
 *   n_obs  [B]                 obstacles used per instance (<= max_obs); NULL = all max_obs rows
 *   ubar   [B][N][2] or NULL   linearization point; NULL = the reference warm start (:224-246)
 * outputs (any may be NULL):
 *   u0 [B][2], U [B][N][2], Xpred [B][N+1][5] (nonlinear predict(x0,U*), :261),
 *   status [B], iters [B]  */
int mpc_solve_batch(mpc_ctx* c, int B, const double* x0, const double* obs, const int* n_obs,
                    const double* ubar, double* u0, double* U, double* Xpred, int* status, int* iters);

/* Same, with device pointers, launched asynchronously on `stream` (a hipStream_t; 0 = null stream).
 * On a host context (device = -1) the pointers are host memory and the call is synchronous.
 * Same argument contract as mpc_solve_batch (n_obs NULL = all max_obs rows; obs with max_obs == 0 is
 * MPC_E_ARG); the double arrays must be 8-byte aligned (MPC_E_ARG otherwise); u0 and U are written
 * with 16-byte stores when both are 16-byte aligned, else with 8-byte ones.  No host synchronisation and,
 * once warmed up, no allocation (graph-capturable): the
 * two-phase work list is allocated by mpc_create for up to 2^20 instances (a larger B runs the
 * single-kernel path, same results).  The two-phase launch keeps, per deferred instance, its linearisation
 * point, nominal rollout, the crossover's solve (the interior point's start) and the trajectory lookups at
 * its stages (21N+14 doubles for even N, 21N+13 for odd) in a stage cache that grows on the first eager call with a larger B (hipMalloc, which waits for the device; at most
 * 1 GiB, MPC_STAGE_CACHE=0 switches it off); a captured call never uses it (a later eager call may grow it,
 * which would leave the graph with a freed pointer) and recomputes the start bit for bit instead.  The work
 * list belongs to the context: consecutive eager calls on one context are ordered on the device even when
 * they use different streams (a call on a new stream waits for the previous
 * call's kernels), so their results never depend on the streams chosen.  A call made while `stream` is
 * being captured into a HIP graph records no such ordering (it would tie the graph to work outside
 * it): replays of that graph must not overlap eager calls, or replays of another graph, on the same
 * context -- run them on one stream, synchronise between them, or give the graph its own context. */
int mpc_solve_batch_device(mpc_ctx* c, int B, const double* x0, const double* obs, const int* n_obs,
                           const double* ubar, double* u0, double* U, double* Xpred, int* status,
                           int* iters, void* stream);

/* Reference-signal service on the device table: TrajectoryLoader.get_state / get_control
 * (trajectory_loader.py:86-102), batched. Host buffers, synchronous.  out_state [n][5], out_control [n][2]. */
int mpc_lookup(mpc_ctx* c, int n, const double* s, double* out_state, double* out_control);

/* TrajectoryLoader.get_global_pose(s, d) (trajectory_loader.py:104-116), batched: Frenet (s, d) ->
 * global (x, y, psi) of the reference line built at mpc_create (trajectory_loader.py:32-62).
 * Host buffers, synchronous.  out [n][3]. */
int mpc_global_pose(mpc_ctx* c, int n, const double* s, const double* d, double* out);

/* Read a trajectory JSON in the reference's format ({"X": [[s,d,o,k,v],...], "U": [[u1,u2],...]},
 * trajectory_loader.py:13-24; other keys ignored).  Two-call pattern: with X == U == NULL only the
 * sizes T, Tu are returned; then X [T][5] and U [Tu][2] (capacities maxT, maxTu rows) are filled.
 * Host only, no device needed.  A missing file is MPC_E_ARG ("File not found : <path>."). */
int mpc_read_trajectory_json(const char* path, double* X, int maxT, double* U, int maxTu, int* T, int* Tu);

/* mpc_read_trajectory_json + mpc_create: replaces TrajectoryLoader(json_file) + TrajectoryTracker(X_ref). */
int mpc_create_from_json(const char* path, const mpc_params* p, int device, mpc_ctx** out);

/* Change parameters of an existing context (e.g. TrajectoryTracker.N = 20 after construction). */
int mpc_set_params(mpc_ctx* c, const mpc_params* p);
int mpc_get_params(const mpc_ctx* c, mpc_params* p);

/* ObstaclesFSM (trajectory_tracking.py:266-374): one dynamic car and one traffic light per ego.
 * mpc_default_fsm() fills the trajectory2.json preset (:292-308) with both scenarios off. */
typedef struct mpc_fsm {
    int dynamic_obstacle, traffic_light;                        /* :286-288                   */
    double obs_trigger_s, obs_start_s, obs_v, obs_end_s;        /* dynamic obstacle, :293-297 */
    double tl_pos, tl_trigger_s, tl_stop_duration;              /* traffic light, :302-304    */
} mpc_fsm;

void mpc_default_fsm(mpc_fsm* f);

/* Batched closed loop: run_simulation (trajectory_tracking.py:377-443) for B independent egos on the
 * device.  Per step: ObstaclesFSM.update(dt, s, v) per ego, one batched solve, the Euler plant step
 * x <- x + dt*dynamics(x, u0, k_ref(s)) (:403-406).  An ego leaves the loop once s > s_stop (the
 * reference runs while s <= s_max - 1, :395); the call returns when every ego has left or after
 * max_steps.  fsm may be NULL (no obstacles).  Host buffers (any history may be NULL):
 *   x_init [B][5]; hist_x [B][max_steps+1][5] (row 0 = x_init); hist_u [B][max_steps][2];
 *   hist_obs_s [B][max_steps] (car position, NaN if none); hist_tl [B][max_steps] (0 RED, 1 GREEN);
 *   hist_status [B][max_steps] (solver status); n_steps [B] (steps each ego ran; required);
 *   step_ms [max_steps] (wall time of each batched step on the device, NaN for steps not run).
 * Entries past an ego's n_steps are NaN (doubles) / -1 (ints). */
int mpc_closed_loop(mpc_ctx* c, int B, const double* x_init, const mpc_fsm* fsm, int max_steps, double s_stop,
                    double* hist_x, double* hist_u, double* hist_obs_s, int* hist_tl, int* hist_status,
                    int* n_steps, double* step_ms);

/* ---- Multi-GPU: ego shards, one gather ----------------------------------------------------
 * Every ego is independent; a batch splits into contiguous per-rank shards (one process per GPU) with no
 * per-step exchange.  The one collective returns what the reference's run_simulation returns
 * (trajectory_tracking.py:443: the closed-loop histories) to rank 0: ncclGather (RCCL over xGMI,
 * rccl.h:745) of a fixed-size payload per rank.  RCCL is loaded (dlopen librccl.so.1) by the first
 * mpc_comm_unique_id / mpc_comm_create; without it they fail with MPC_E_COMM.
 *   - rank 0 calls mpc_comm_unique_id and hands the MPC_COMM_UID_BYTES bytes to every rank out of band (the
 *     package's shard.py uses a TCP rendezvous on MASTER_ADDR); every rank then calls mpc_comm_create
 *     (collective: it returns once all nranks ranks joined);
 *   - mpc_gather: device buffers, asynchronous on `stream` (hipStream_t, 0 = null stream): rank i's `bytes`
 *     land at recv + i*bytes on the root (recv holds nranks*bytes there; may be NULL elsewhere);
 *   - mpc_gather_host: the same from host buffers, staged through the communicator's device buffer on its
 *     own stream, synchronous (returns when the root's recv is filled);
 *   - mpc_comm_allreduce_max: in-place max of one double over all ranks (the measurement's max-over-ranks
 *     time), synchronous; mpc_comm_barrier: returns on every rank once all ranks entered it;
 *   - one communicator per process and device; not re-entrant. */
#define MPC_COMM_UID_BYTES 128
typedef struct mpc_comm mpc_comm;
int mpc_comm_unique_id(char* uid /* [MPC_COMM_UID_BYTES] */);
int mpc_comm_create(const char* uid, int nranks, int rank, int device, mpc_comm** out);
int mpc_comm_info(const mpc_comm* c, int* nranks, int* rank, int* device);
int mpc_gather(mpc_comm* c, const void* send, size_t bytes, void* recv, int root, void* stream);
int mpc_gather_host(mpc_comm* c, const void* send, size_t bytes, void* recv, int root);
int mpc_comm_allreduce_max(mpc_comm* c, double* value);
int mpc_comm_barrier(mpc_comm* c);
void mpc_comm_destroy(mpc_comm* c);

/* Thread-local description of the last API error on this thread. */
const char* mpc_last_error(void);
int mpc_version(void);
void mpc_destroy(mpc_ctx* c);

#ifdef __cplusplus
}
#endif
#endif /* MPCQP_H */

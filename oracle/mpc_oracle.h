/*
 * mpc_oracle.h — CPU restatement of the reference tracking-MPC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liborcmpc.so, and only as the checker / the timed CPU
 * baseline ("port").  The product (libmpcqp.so) never links or calls it.
 *
 * Parity pins (tests/golden, captured from the reference by tests/golden/make_goldens.py):
 *   orc_get_state/orc_get_control  == TrajectoryLoader.get_state/get_control  bit-exact
 *   orc_predict                     == TrajectoryTracker.predict               bit-exact
 *   orc_cost / orc_constraints      == TrajectoryTracker.cost / constraints   <= 1e-12 rel
 *   orc_warm_start                  == u_init of TrajectoryTracker.solve      bit-exact
 *   orc_build_qp                    == the golden QP(ubar) matrices           <= 1e-10 rel
 *   orc_solve                       == golden KKT-certified U*                <= 1e-8 abs
 */
#ifndef MPC_ORACLE_H
#define MPC_ORACLE_H
#include "../include/mpcqp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_table orc_table;

void orc_default_params(mpc_params* p);
orc_table* orc_table_create(const double* X, int T, const double* U, int Tu);
void orc_table_destroy(orc_table* t);
double orc_s_max(const orc_table* t);

/* trajectory_loader.py:86-102 */
void orc_get_state(const orc_table* t, double s, double out[5]);
void orc_get_control(const orc_table* t, double s, double out[2]);
/* TrajectoryLoader.get_global_pose (trajectory_loader.py:32-62,104-116) -> (x, y, psi) */
void orc_global_pose(const orc_table* t, double s, double d, double out[3]);
/* the interp1d segment slopes of (d,o,k,v) at s (0 for s >= s_max): Gauss-Newton data */
void orc_state_slopes(const orc_table* t, double s, double out[4]);

/* trajectory_tracking.py:224-246 ; ubar [N][2] */
void orc_warm_start(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs,
                    int nobs, double* ubar);
/* trajectory_tracking.py:87-114 ; X [N+1][5] */
void orc_predict(const orc_table* t, const mpc_params* p, const double x0[5], const double* U, double* X);
/* trajectory_tracking.py:116-152 */
double orc_cost(const orc_table* t, const mpc_params* p, const double x0[5], const double* U);
/* trajectory_tracking.py:164-209, reference row order; returns number of rows written */
int orc_constraints(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs,
                    int nobs, const double* U, double* out);

/* Dense QP(ubar) in deviation coordinates dU = U - ubar:
 *   0.5 dU'H dU + f'dU + c0,   lo <= A dU <= hi (rows: per k=1..N: d, d+(L/2)o, d+Lo, [s, s+T v], v),
 *   blo <= dU <= bhi.   H [n][n], f [n], A [m][n], lo/hi [m] (+-INFINITY when absent), blo/bhi [n].
 * Returns m. */
int orc_build_qp(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs,
                 int nobs, const double* ubar, double* H, double* f, double* c0, double* A, double* lo,
                 double* hi, double* blo, double* bhi);

/* One instance of mpc_solve_batch. ubar may be NULL (reference warm start). Returns status. */
int orc_solve(const orc_table* t, const mpc_params* p, const double x0[5], const double* obs, int nobs,
              const double* ubar, double* u0, double* U, double* Xpred, int* iters);

/* Batched, OpenMP over instances (num_threads <= 0: runtime default).  Same layout as mpc_solve_batch. */
int orc_solve_batch(const orc_table* t, const mpc_params* p, int B, const double* x0, const double* obs,
                    const int* n_obs, const double* ubar, double* u0, double* U, double* Xpred, int* status,
                    int* iters, int num_threads);

#ifdef __cplusplus
}
#endif
#endif

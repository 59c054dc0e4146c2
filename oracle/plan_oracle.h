/* plan_oracle.h — CPU restatement of the offline planner's chunk solve (TEST INFRASTRUCTURE ONLY).
 *
 * Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker of libmpcplan's
 * HIP path; never linked or called by the product.  Parity with the reference NLP is unpinned (the
 * reference module trajectory_planning.py is not importable); see plan_oracle.c. */
#ifndef PLAN_ORACLE_H
#define PLAN_ORACLE_H
#include "../include/mpcplan.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_route orc_route;

void orc_plan_default_params(plan_params* p);
int orc_route_create(const double* s, int M, const double* cx, const double* cy, const double* vmax,
                     orc_route** out);
void orc_route_destroy(orc_route* r);
double orc_route_kappa(const orc_route* r, double s, double* dkds);
double orc_route_vmax(const orc_route* r, double s);
double orc_route_s_total(const orc_route* r);

/* the NLP's functions (trajectory_planning.py:50-89, :128-170, :181-210) on one chunk */
void orc_plan_dynamics(const double x[5], double u1, double u2, double kref, double f[5]);
void orc_plan_defect(const orc_route* r, const plan_params* p, const double xa[5], const double xb[5], double u1,
                     double u2, double def[5]);
double orc_plan_cost(const orc_route* r, const plan_params* p, int N, const double x0[5], const double* X,
                     const double* U, const double* S);

/* one chunk: returns the status code; X[(N+1)*5], U[N*2], S[N]; iters = interior-point iterations, sqp = QPs */
int orc_plan_chunk(const orc_route* r, const plan_params* p, int N, const double x0[5], double s_target,
                   int is_final, double* X, double* U, double* S, int* iters, int* sqp);
/* B chunks (layout of plan_solve_chunks, row stride Nmax), OpenMP */
int orc_plan_batch(const orc_route* r, const plan_params* p, int B, const int* N, const double* x0,
                   const double* s_target, const int* is_final, double* X, double* U, double* S, int* status,
                   int* iters, int* sqp, int num_threads);

#ifdef __cplusplus
}
#endif
#endif

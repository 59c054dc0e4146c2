/* Sanitizer driver for the CPU oracle (oracle/mpc_oracle.c), built by tests/asan/Makefile with
 * -fsanitize=address,undefined and run by tests/test_asan.py.
 *
 *   oracle_driver <in.bin> <out.bin>
 * in.bin : int32 T, Tu, N, B, max_obs, sqp_iters; f64 X[T][5], U[Tu][2], x0[B][5], obs[B][max_obs][2];
 *          int32 n_obs[B]
 * out.bin: f64 U[B][N][2], Xpred[B][N+1][5]; int32 status[B], iters[B]
 * The test compares out.bin with the regular (unsanitized) oracle build on the same inputs. */
#include <stdio.h>
#include <stdlib.h>

#include "../../oracle/mpc_oracle.h"

static void* rd(FILE* f, size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p || fread(p, 1, n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
    return p;
}

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int hdr[6];
    if (fread(hdr, sizeof(int), 6, f) != 6) return 2;
    const int T = hdr[0], Tu = hdr[1], N = hdr[2], B = hdr[3], mo = hdr[4];
    double* X = rd(f, sizeof(double) * 5 * (size_t)T);
    double* U = rd(f, sizeof(double) * 2 * (size_t)Tu);
    double* x0 = rd(f, sizeof(double) * 5 * (size_t)B);
    double* obs = rd(f, sizeof(double) * 2 * (size_t)B * mo);
    int* nobs = rd(f, sizeof(int) * (size_t)B);
    fclose(f);
    orc_table* t = orc_table_create(X, T, U, Tu);
    if (!t) return 3;
    mpc_params p;
    orc_default_params(&p);
    p.N = N;
    p.max_obs = mo;
    p.sqp_iters = hdr[5];
    double* Uo = calloc((size_t)B * 2 * N, sizeof(double));
    double* Xo = calloc((size_t)B * 5 * (N + 1), sizeof(double));
    int* st = calloc((size_t)B, sizeof(int));
    int* it = calloc((size_t)B, sizeof(int));
    int rc = orc_solve_batch(t, &p, B, x0, mo ? obs : NULL, mo ? nobs : NULL, NULL, NULL, Uo, Xo, st, it, 1);
    if (rc) return 4;
    FILE* o = fopen(argv[2], "wb");
    if (!o) return 2;
    fwrite(Uo, sizeof(double), (size_t)B * 2 * N, o);
    fwrite(Xo, sizeof(double), (size_t)B * 5 * (N + 1), o);
    fwrite(st, sizeof(int), (size_t)B, o);
    fwrite(it, sizeof(int), (size_t)B, o);
    fclose(o);
    orc_table_destroy(t);
    free(X); free(U); free(x0); free(obs); free(nobs); free(Uo); free(Xo); free(st); free(it);
    return 0;
}

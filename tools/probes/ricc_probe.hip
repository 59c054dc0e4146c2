// Micro-benchmark of the stage recursions of the solver kernel (riccati_factor, riccati_solve) in
// isolation: one wavefront, G = 64 / GL instances, synthetic SPD stage data in LDS.  Prints shader
// cycles per stage for each recursion; one kernel per recursion, so rocprofv3 --pmc can separate
// them.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off.
#include "../../safe-autonomous-driving-mpc_amd/csrc/mpcqp.hip"

// candidate: horizon fixed at compile time, loops fully unrolled (no loop control, immediate LDS
// offsets, no per-step address arithmetic)
template <int NT>
__device__ void riccati_solve_fixed(const Lds& S, double dt, int ln) {
    constexpr int N = NT;
    double p5[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < 4; ++a) p5[st4(a)] = S.qh[4 * N + a];
    {
        BwdBuf buf[2];
        load_bwd(S, N - 1, buf[0]);
#pragma unroll
        for (int t = N - 1; t >= 0; --t) {
            lds_fence();
            load_bwd(S, t >= 1 ? t - 1 : 0, buf[(N - t) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            bwd_step(S, t, dt, buf[(N - 1 - t) & 1], p5, ln);
        }
    }
    wave_sync();
    if (ln == 0)
        for (int a = 0; a < 5; ++a) S.dX[a] = 0.0;
    {
        double x[5] = {0, 0, 0, 0, 0};
        FwdBuf buf[2];
        load_fwd(S, 0, buf[0]);
#pragma unroll
        for (int t = 0; t < N; ++t) {
            lds_fence();
            load_fwd(S, t + 1 < N ? t + 1 : t, buf[(t + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            fwd_step(S, t, dt, buf[t & 1], x, ln);
        }
    }
    wave_sync();
}

// candidate factor: fewer VALU per stage (dt folded into the Cholesky reciprocals, W'W and Q folded
// into fma chains), stage data double-buffered without register copies (2x unrolled)
struct FacBuf { double a[5], r0, r1, q[10]; };
__device__ __forceinline__ void load_fac(const Lds& S, int t, FacBuf& F) {
    ld_a5(S.A5 + A5S * t, F.a);
    ld2(S.Rt + 2 * t, F.r0, F.r1);
#pragma unroll
    for (int a = 0; a < 10; a += 2) ld2(S.Qt + 10 * t + a, F.q[a], F.q[a + 1]);
}
struct FacOut { double K[10], si[3]; };
__device__ __forceinline__ void store_fac(const Lds& S, int t, const FacOut& O, int ln) {
    if (ln == 0) {
#pragma unroll
        for (int j = 0; j < 10; ++j) S.Kf[10 * t + j] = O.K[j];
        S.Si[SIS * t] = O.si[0];
        S.Si[SIS * t + 1] = O.si[1];
        S.Si[SIS * t + 2] = O.si[2];
    }
}
__device__ __forceinline__ void fac_step(int t, double dt, double dt2, const FacBuf& F, double P[15], FacOut& O) {
    const double a12 = F.a[0], a14 = F.a[1], a20 = F.a[2], a23 = F.a[3], a24 = F.a[4];
    const double* q = F.q;
    double s00 = fma(dt2, P[s5(3, 3)], F.r0), s01 = dt2 * P[s5(3, 4)], s11 = fma(dt2, P[s5(4, 4)], F.r1);
    if (!(s00 > 0.0)) s00 = 1e-300 + fabs(s00);
    const double il00 = frsqrt(s00), l10 = s01 * il00;
    double r11 = s11 - l10 * l10;
    if (!(r11 > 1e-14 * s11)) r11 = 1e-14 * fabs(s11) + 1e-300;
    const double il11 = frsqrt(r11);
    const double c0 = dt * il00, c1 = dt * il11, c2 = -l10 * il11;
    double M[5][5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double pi0 = P[s5(i, 0)], pi1 = P[s5(i, 1)], pi2 = P[s5(i, 2)], pi3 = P[s5(i, 3)], pi4 = P[s5(i, 4)];
        M[i][0] = fma(pi2, a20, pi0);
        M[i][1] = pi1;
        M[i][2] = fma(pi1, a12, pi2);
        M[i][3] = fma(pi2, a23, pi3);
        M[i][4] = fma(pi0, dt, fma(pi1, a14, fma(pi2, a24, pi4)));
    }
    double W0[5], W1[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        W0[j] = M[3][j] * c0;
        W1[j] = fma(M[4][j], c1, c2 * W0[j]);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const double K1 = -W1[j] * il11;
        O.K[5 + j] = K1;
        O.K[j] = -(W0[j] + l10 * K1) * il00;
    }
    O.si[0] = il00;
    O.si[1] = l10;
    O.si[2] = il11;
    if (t >= 1) {
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = i; j < 5; ++j) {
                double v = (i != 3 && j != 3) ? M[i][j] + q[p4(i == 4 ? 3 : i, j == 4 ? 3 : j)] : M[i][j];
                if (i == 0) v = fma(a20, M[2][j], v);
                else if (i == 2) v = fma(a12, M[1][j], v);
                else if (i == 3) v = fma(a23, M[2][j], v);
                else if (i == 4) v = fma(dt, M[0][j], fma(a14, M[1][j], fma(a24, M[2][j], v)));
                v = fma(-W0[i], W0[j], fma(-W1[i], W1[j], v));
                P[s5(i, j)] = v;
            }
    }
}
// stores of stage t are issued right after the next stage's fence, so no fence waits on them
__device__ void riccati_factor2(const Lds& S, int N, double dt, int ln) {
    double P[15];
#pragma unroll
    for (int i = 0; i < 15; ++i) P[i] = 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = a; c < 4; ++c) P[s5(st4(a), st4(c))] = S.Qt[10 * N + p4(a, c)];
    const double dt2 = dt * dt;
    FacBuf A, B;
    FacOut O;
    load_fac(S, N - 1, A);
    lds_fence();
    load_fac(S, N >= 2 ? N - 2 : 0, B);
    fac_step(N - 1, dt, dt2, A, P, O);
    int t = N - 2;
    while (t >= 0) {
        lds_fence();
        store_fac(S, t + 1, O, ln);
        load_fac(S, t >= 1 ? t - 1 : 0, A);
        __builtin_amdgcn_sched_barrier(0);
        fac_step(t, dt, dt2, B, P, O);
        if (--t < 0) break;
        lds_fence();
        store_fac(S, t + 1, O, ln);
        load_fac(S, t >= 1 ? t - 1 : 0, B);
        __builtin_amdgcn_sched_barrier(0);
        fac_step(t, dt, dt2, A, P, O);
        --t;
    }
    store_fac(S, 0, O, ln);
    wave_sync();
}

template <int GL, int WHAT>
__global__ void __launch_bounds__(WAVE) ricc_probe(int N, int reps, double dt, unsigned long long* cyc, double* sink) {
    constexpr int G = WAVE / GL;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int ln = threadIdx.x, grp = ln / GL, gl = ln % GL;
    Lds S = carve(smem + (size_t)grp * lds_doubles(N), N);
    for (int i = gl; i < lds_doubles(N); i += GL) smem[(size_t)grp * lds_doubles(N) + i] = 0.0;
    wave_sync();
    for (int t = gl; t <= N; t += GL) {
        double* q = S.Qt + 10 * t;
        q[p4(0, 0)] = 1.0 + 0.01 * t; q[p4(1, 1)] = 20.0; q[p4(2, 2)] = 20.0 + grp; q[p4(3, 3)] = 10.0;
        q[p4(0, 1)] = 0.1; q[p4(0, 3)] = 0.2;
        for (int a = 0; a < 4; ++a) S.qh[4 * t + a] = 0.1 * (a + 1);
        if (t < N) {
            S.A5[A5S * t + 0] = dt * 10.0; S.A5[A5S * t + 1] = dt * 0.01; S.A5[A5S * t + 2] = -dt * 0.001;
            S.A5[A5S * t + 3] = dt * 10.0; S.A5[A5S * t + 4] = dt * 0.002;
            S.Rt[2 * t] = 1.0; S.Rt[2 * t + 1] = 1.0 + 1e3 * (t & 1);
            S.gh[2 * t] = 0.3; S.gh[2 * t + 1] = -0.2;
        }
    }
    wave_sync();
    riccati_factor(S, N, dt, gl);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (WHAT == 0) riccati_factor(S, N, dt, gl);
        if (WHAT == 1) riccati_solve(S, N, dt, gl);
        if (WHAT == 2) riccati_solve_fixed<20>(S, dt, gl);
        if (WHAT == 3) riccati_factor2(S, N, dt, gl);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) cyc[WHAT] = t1 - t0;
    if (gl == 0) sink[grp] = S.dud[0] + S.Kf[0] + S.dX[5 * N];
}

int main() {
    const int N = 20, reps = 50;
    unsigned long long* dc; double* ds;
    hipMalloc(&dc, 16 * 8); hipMalloc(&ds, 64 * 8);
    size_t lds = sizeof(double) * lds_doubles(N) * 2;
    for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL((ricc_probe<32, 0>), dim3(1), dim3(64), lds, 0, N, reps, 0.2, dc, ds);
        hipLaunchKernelGGL((ricc_probe<32, 1>), dim3(1), dim3(64), lds, 0, N, reps, 0.2, dc, ds);
        hipLaunchKernelGGL((ricc_probe<32, 2>), dim3(1), dim3(64), lds, 0, N, reps, 0.2, dc, ds);
        hipLaunchKernelGGL((ricc_probe<32, 3>), dim3(1), dim3(64), lds, 0, N, reps, 0.2, dc, ds);
    }
    unsigned long long c[4]; double sk[2];
    hipMemcpy(c, dc, 32, hipMemcpyDeviceToHost);
    hipMemcpy(sk, ds, 16, hipMemcpyDeviceToHost);
    printf("N=%d GL=32: factor %.0f cyc/stage, solve %.0f cyc/stage-step (bwd+fwd = 2N steps), fixed-N solve %.0f, factor2 %.0f  sink %.6e %.6e\n", N,
           (double)c[0] / reps / N, (double)c[1] / reps / (2 * N), (double)c[2] / reps / (2 * N), (double)c[3] / reps / N, sk[0], sk[1]);
    return 0;
}

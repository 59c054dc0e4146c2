// Latency / issue micro-benchmark of the planner recursions' instruction mix on one wave (gfx950): cycles per
// instruction of dependent and independent chains of v_fmac_f64 (plain and DPP row_newbcast), FP64
// division (IEEE, as the compiler emits it), an LDS read round trip, under a full and an 8-lane exec mask.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/dpp_lat tools/micro/dpp_lat.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256
#define PF(d, s, c, L) "v_fmac_f64_dpp " d ", " s ", " c " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"

__global__ void bench(unsigned long long* out, double* sink, int narrow) {
    __shared__ double lds[256];
    const int ln = threadIdx.x;
    lds[ln] = 1.0 + ln * 1e-9;
    __syncthreads();
    if (narrow && ln >= 8) return;
    double a = 1.0 + ln * 1e-7, b = 0.999999, c = 1e-9;
    double x0 = a, x1 = a, x2 = a, x3 = a, x4 = a;
    unsigned long long t0, t1;
    // 1: dependent plain fma chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2"
                     : "+v"(x0) : "v"(b), "v"(c));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[0] = t1 - t0;
    // 2: five independent plain fma chains (issue rate)
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_fmac_f64 %0, %5, %6\n\tv_fmac_f64 %1, %5, %6\n\tv_fmac_f64 %2, %5, %6\n\tv_fmac_f64 %3, %5, %6\n\t"
                     "v_fmac_f64 %4, %5, %6"
                     : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4) : "v"(b), "v"(c));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[1] = t1 - t0;
    // 3: dependent DPP chain (the accumulator is the destination; the broadcast source is another register)
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) {
        asm volatile("s_nop 1\n\t" PF("%0", "%1", "%2", 0) PF("%0", "%1", "%2", 1) PF("%0", "%1", "%2", 2) PF("%0", "%1", "%2", 3)
                     : "+v"(x1) : "v"(a), "v"(c));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[2] = t1 - t0;
    // 4: five independent DPP chains
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) {
        asm volatile("s_nop 1\n\t" PF("%0", "%5", "%6", 0) PF("%1", "%5", "%6", 1) PF("%2", "%5", "%6", 2) PF("%3", "%5", "%6", 3)
                     PF("%4", "%5", "%6", 4)
                     : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4) : "v"(a), "v"(c));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[3] = t1 - t0;
    // 5: DPP broadcast of the chain value itself (the solve's p / x recursions: source = previous result)
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) {
        double y = 0.0;
        asm volatile("s_nop 1\n\t" PF("%0", "%1", "%2", 0) : "+v"(y) : "v"(x2), "v"(c));
        x2 = y + b;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[4] = t1 - t0;
    // 6: dependent IEEE division chain
    t0 = __builtin_amdgcn_s_memtime();
    double d = x3;
    for (int i = 0; i < REP; ++i) d = 1.0 / (d + 0.5);
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[5] = t1 - t0;
    // 7: dependent LDS read chain (address from the previous value)
    t0 = __builtin_amdgcn_s_memtime();
    int idx = ln;
    double acc = 0.0;
    for (int i = 0; i < REP; ++i) {
        const double v = lds[idx & 255];
        acc += v;
        idx = (int)v + ln + i;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[6] = t1 - t0;
    // 8: dependent v_mul_f64 / v_add_f64 chain
    t0 = __builtin_amdgcn_s_memtime();
    double e = x4;
    for (int i = 0; i < REP; ++i) {
        asm volatile("v_add_f64 %0, %0, %1\n\tv_mul_f64 %0, %0, %2\n\tv_add_f64 %0, %0, %1\n\tv_mul_f64 %0, %0, %2"
                     : "+v"(e) : "v"(c), "v"(b));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (ln == 0) out[7] = t1 - t0;
    sink[ln] = x0 + x1 + x2 + x3 + x4 + d + acc + e;
}

int main() {
    unsigned long long* o;
    double* s;
    hipMalloc(&o, 16 * sizeof(unsigned long long));
    hipMalloc(&s, 64 * sizeof(double));
    const char* names[8] = {"dependent v_fmac_f64 (per fma)", "5 independent v_fmac_f64 chains (per fma)",
                            "dependent v_fmac_f64_dpp (per fma)", "5 independent dpp chains (per fma)",
                            "dpp broadcast of the chain value + add (per step)", "dependent 1/(d+0.5) (per step)",
                            "dependent LDS read + add + cvt (per step)", "dependent v_add/v_mul f64 (per op)"};
    const double per[8] = {4.0 * REP, 5.0 * REP, 4.0 * REP, 5.0 * REP, REP, REP, REP, 4.0 * REP};
    for (int narrow = 0; narrow < 2; ++narrow) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(bench, dim3(1), dim3(64), 0, 0, o, s, narrow);
            hipDeviceSynchronize();
        }
        unsigned long long h[16];
        hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
        printf("exec %s:\n", narrow ? "lanes 0..7" : "64 lanes");
        for (int i = 0; i < 8; ++i) printf("  %-52s %7.1f cycles\n", names[i], h[i] / per[i]);
    }
    return 0;
}

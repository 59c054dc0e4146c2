// Micro-latencies on gfx950 for the stage recursions: dependent v_fma_f64 chain, dependent LDS
// round trip (ds_write + ds_read of the same value), DPP row_newbcast hop, __shfl (ds_bpermute) hop,
// v_rcp_f64, sqrt.  One wave; s_memtime cycles per link.
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP 256
__global__ void k(double* out, long long* cyc, double a, double b) {
    __shared__ double sh[64];
    double x = a + threadIdx.x;
    long long t0, t1;
    // 1. FMA chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) x = fma(x, b, a);
    t1 = __builtin_amdgcn_s_memtime();
    cyc[0] = t1 - t0;
    // 2. LDS round trip chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) {
        sh[threadIdx.x] = x;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        x = sh[threadIdx.x ^ 1] + 1e-300;
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[1] = t1 - t0;
    // 3. DPP hop chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) x = __builtin_amdgcn_update_dpp(0.0, x, 0x153, 0xf, 0xf, false) * b;
    t1 = __builtin_amdgcn_s_memtime();
    cyc[2] = t1 - t0;
    // 4. shfl hop chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) x = __shfl(x, (threadIdx.x + 1) & 63, 64) * b;
    t1 = __builtin_amdgcn_s_memtime();
    cyc[3] = t1 - t0;
    // 5. rcp chain (v_rcp_f64 only)
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) x = __builtin_amdgcn_rcp(x) + a;
    t1 = __builtin_amdgcn_s_memtime();
    cyc[4] = t1 - t0;
    // 6. sqrt chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) x = sqrt(x) + a;
    t1 = __builtin_amdgcn_s_memtime();
    cyc[5] = t1 - t0;
    // 7. independent FMAs (8 chains interleaved) -> issue rate
    double y[8];
    for (int j = 0; j < 8; ++j) y[j] = x + j;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = fma(y[j], b, a);
    t1 = __builtin_amdgcn_s_memtime();
    cyc[6] = t1 - t0;
    // 8. uniform LDS read chain (address depends on previous value)
    sh[threadIdx.x] = 0.0;
    __syncthreads();
    int idx = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP; ++i) idx = (int)sh[idx] + (i & 1);
    t1 = __builtin_amdgcn_s_memtime();
    cyc[7] = t1 - t0;
    double s = x + idx;
    for (int j = 0; j < 8; ++j) s += y[j];
    out[threadIdx.x] = s;
}
int main() {
    double* o; long long* c;
    hipMalloc(&o, 64 * 8); hipMalloc(&c, 16 * 8);
    long long h[16];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, 1e-3, 0.999);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, c, 16 * 8, hipMemcpyDeviceToHost);
    const char* nm[8] = {"fma_f64 dep", "lds write+read", "dpp bcast+mul", "shfl+mul", "rcp_f64+add", "sqrt+add",
                         "8 indep fma_f64 (per fma)", "lds read dep (addr)"};
    for (int i = 0; i < 8; ++i) printf("%-28s %8.1f cycles/link\n", nm[i], (double)h[i] / (i == 6 ? REP * 8 : REP));
    return 0;
}

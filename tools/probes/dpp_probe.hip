// Checks the gfx950 DPP row_newbcast semantics the Riccati kernels rely on:
// out[lane] must be in[(lane & ~15) + n] for v_mov_b64_dpp row_newbcast:n.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* o, const double* in) {
    double x = in[threadIdx.x];
    o[threadIdx.x] = __builtin_amdgcn_update_dpp(0.0, x, 0x153, 0xf, 0xf, false);
    o[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(0.0, x, 0x150, 0xf, 0xf, false);
}
int main() {
    double h[64], r[128];
    for (int i = 0; i < 64; ++i) h[i] = 1000.0 + i;
    double *di, *dout;
    hipMalloc(&di, 64 * 8);
    hipMalloc(&dout, 128 * 8);
    hipMemcpy(di, h, 64 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dout, di);
    hipMemcpy(r, dout, 128 * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; ++i) {
        if (r[i] != 1000.0 + (i & ~15) + 3) bad++;
        if (r[64 + i] != 1000.0 + (i & ~15)) bad++;
    }
    printf("row_newbcast check: %s (lane 17 -> %.0f, lane 40 -> %.0f)\n", bad ? "FAIL" : "ok", r[17], r[40]);
    return bad ? 1 : 0;
}

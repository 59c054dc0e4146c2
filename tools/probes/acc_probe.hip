// Accuracy of v_rsq_f64 / v_rcp_f64 (raw, and with 1 or 2 Newton steps) on gfx950 against IEEE
// 1/sqrt and 1/x computed in long double on the host.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
__global__ void k(const double* x, double* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double y = __builtin_amdgcn_rsq(v);
    const double h = 0.5 * v;
    o[6 * i + 0] = y;
    double y1 = y * fma(-h * y, y, 1.5);
    o[6 * i + 1] = y1;
    o[6 * i + 2] = y1 * fma(-h * y1, y1, 1.5);
    double r = __builtin_amdgcn_rcp(v);
    o[6 * i + 3] = r;
    double e = fma(-v, r, 1.0);
    double r1 = fma(r, e, r);
    o[6 * i + 4] = r1;
    e = fma(-v, r1, 1.0);
    o[6 * i + 5] = fma(r1, e, r1);
}
int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), o(6 * n);
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-30.0, 30.0), m(1.0, 2.0);
    for (int i = 0; i < n; ++i) x[i] = m(g) * std::pow(2.0, std::floor(u(g)));
    double *dx, *dox;
    hipMalloc(&dx, n * 8); hipMalloc(&dox, 6 * n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dox, n);
    hipMemcpy(o.data(), dox, 6 * n * 8, hipMemcpyDeviceToHost);
    double err[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        long double rs = 1.0L / sqrtl((long double)x[i]), rc = 1.0L / (long double)x[i];
        for (int j = 0; j < 3; ++j) err[j] = fmax(err[j], (double)fabsl((o[6 * i + j] - rs) / rs));
        for (int j = 3; j < 6; ++j) err[j] = fmax(err[j], (double)fabsl((o[6 * i + j] - rc) / rc));
    }
    printf("max rel err: rsq raw %.3e, +1 Newton %.3e, +2 Newton %.3e; rcp raw %.3e, +1 %.3e, +2 %.3e (eps %.3e)\n", err[0],
           err[1], err[2], err[3], err[4], err[5], 2.220446e-16);
    return 0;
}

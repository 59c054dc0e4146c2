// LDS instruction costs for one wavefront on gfx950 with exec narrowed as in the recursions
// (lanes 0..4 of each 32-lane group = 10 lanes) and with all 64 lanes: independent ds_read_b64,
// ds_read_b128, ds_read2_b64, ds_write_b64 back to back (s_memtime cycles per instruction,
// including the final wait).
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_probe lds_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP 32

template <int KIND>
__device__ long long run(double* sh, int ln, double& sink) {
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    const unsigned base = (unsigned)(size_t)(sh + 16 * (ln % 32));
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REP; ++r) {
        if (KIND == 0) {
            asm volatile("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:1024\n\tds_read_b64 %2, %4 offset:2048\n\t"
                         "ds_read_b64 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3) : "v"(base));
        } else if (KIND == 1) {
            typedef double v2d __attribute__((ext_vector_type(2)));
            v2d b0, b1, b2, b3;
            asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\tds_read_b128 %2, %4 offset:2048\n\t"
                         "ds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3) : "v"(base));
            a0 = b0.x + b1.y; a1 = b2.x; a2 = b3.y; a3 = b0.y;
        } else if (KIND == 2) {
            asm volatile("ds_write_b64 %0, %1\n\tds_write_b64 %0, %1 offset:1024\n\tds_write_b64 %0, %1 offset:2048\n\t"
                         "ds_write_b64 %0, %1 offset:3072\n\ts_waitcnt lgkmcnt(0)" :: "v"(base), "v"(sink) : "memory");
        } else {
            // one dependent read-after-read chain (latency)
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(a0) : "v"(base));
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(a1) : "v"(base));
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(a2) : "v"(base));
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(a3) : "v"(base));
        }
        sink += a0 + a1 + a2 + a3;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    return t1 - t0;
}

__global__ void __launch_bounds__(64) k(long long* cyc, double* out) {
    __shared__ double sh[4096];
    const int ln = threadIdx.x;
    for (int i = ln; i < 4096; i += 64) sh[i] = 1e-3 * i;
    __syncthreads();
    double sink = 0;
    long long c[8];
    c[0] = run<0>(sh, ln, sink);
    c[1] = run<1>(sh, ln, sink);
    c[2] = run<2>(sh, ln, sink);
    c[3] = run<3>(sh, ln, sink);
    __syncthreads();
    if (ln % 32 < 5) {
        c[4] = run<0>(sh, ln, sink);
        c[5] = run<1>(sh, ln, sink);
        c[6] = run<2>(sh, ln, sink);
        c[7] = run<3>(sh, ln, sink);
    }
    __syncthreads();
    if (ln == 0)
        for (int i = 0; i < 8; ++i) cyc[i] = c[i];
    out[ln] = sink;
}

int main() {
    long long* c;
    double* o;
    (void)hipMalloc(&c, 8 * sizeof(long long));
    (void)hipMalloc(&o, 64 * sizeof(double));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, c, o);
    (void)hipDeviceSynchronize();
    long long h[8];
    (void)hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[4] = {"ds_read_b64 x4 + wait", "ds_read_b128 x4 + wait", "ds_write_b64 x4 + wait", "dependent ds_read_b64"};
    for (int i = 0; i < 4; ++i)
        printf("%-24s 64 lanes %6.1f   10 lanes %6.1f  cycles per instruction\n", nm[i], (double)h[i] / (REP * 4),
               (double)h[4 + i] / (REP * 4));
    return 0;
}

// Issue costs on gfx950 for the solver's recursion design (one wave, s_memtime cycles):
//   - independent v_fma_f64 (8 chains) per instruction;
//   - ds_read_b128 of one LDS address by all lanes (broadcast) per instruction, with 64 / 32 / 16 / 2
//     active lanes;
//   - ds_read_b128 of per-lane addresses (no bank conflicts) per instruction;
//   - v_mov_b32 DPP row_newbcast per instruction (independent);
//   - dependent chains: v_rsq_f64 + 2 Newton steps (the kernel's frsqrt), v_rcp_f64 + 2 Newton steps.
// Build: hipcc --offload-arch=gfx950 -O3 -o cost_probe cost_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP 64

__device__ __forceinline__ double frsqrt(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}
__device__ __forceinline__ double frcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

template <int ACTIVE>
__device__ long long lds_bcast(const double* sh, double& acc) {
    long long t0 = 0, t1 = 0;
    if ((int)threadIdx.x < ACTIVE) {
        double2 v[16];
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = *reinterpret_cast<const double2*>(sh + 2 * i + (r & 1) * 32);
            __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
            for (int i = 0; i < 16; ++i) acc += v[i].x;
        }
        t1 = __builtin_amdgcn_s_memtime();
    }
    return t1 - t0;
}

__global__ void k(double* out, long long* cyc, double a, double b) {
    __shared__ __attribute__((aligned(16))) double sh[64 * 4];
    const int ln = threadIdx.x;
    for (int i = ln; i < 64 * 4; i += 64) sh[i] = 1e-3 * i;
    __syncthreads();
    double x = a + ln, acc = 0.0;
    long long t0, t1;
    // 0. independent FMAs: 8 chains
    double y[8];
    for (int j = 0; j < 8; ++j) y[j] = x + j;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < REP * 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = fma(y[j], b, a);
    t1 = __builtin_amdgcn_s_memtime();
    cyc[0] = t1 - t0;
    for (int j = 0; j < 8; ++j) acc += y[j];
    // 1-4. broadcast LDS reads (16 x ds_read_b128 + 16 adds per round) with 64/32/16/2 active lanes
    cyc[1] = lds_bcast<64>(sh, acc);
    cyc[2] = lds_bcast<32>(sh, acc);
    cyc[3] = lds_bcast<16>(sh, acc);
    cyc[4] = lds_bcast<2>(sh, acc);
    // 5. per-lane LDS reads (lane-strided, conflict-free)
    {
        double2 v[16];
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = *reinterpret_cast<const double2*>(sh + ((2 * ln + 2 * i + r) & 255 & ~1));
            __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
            for (int i = 0; i < 16; ++i) acc += v[i].x;
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[5] = t1 - t0;
    }
    // 6. 16 adds alone (the consumer of 1-5)
    {
        double v[16];
        for (int i = 0; i < 16; ++i) v[i] = x * i;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
#pragma unroll
            for (int i = 0; i < 16; ++i) acc += v[i];
            asm volatile("" : "+v"(acc));
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[6] = t1 - t0;
    }
    // 7. DPP row_newbcast movs: 16 independent 64-bit values (32 v_mov_b32_dpp) per round
    {
        double v[16];
        for (int i = 0; i < 16; ++i) v[i] = x * (i + 1);
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_update_dpp(0.0, v[i], 0x153, 0xf, 0xf, false);
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(v[i]));
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[7] = t1 - t0;
        for (int i = 0; i < 16; ++i) acc += v[i];
    }
    // 8. dependent frsqrt chain
    {
        double z = 2.0 + x;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) z = frsqrt(z) + 2.0;
        t1 = __builtin_amdgcn_s_memtime();
        cyc[8] = t1 - t0;
        acc += z;
    }
    // 9. dependent frcp chain
    {
        double z = 2.0 + x;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) z = frcp(z) + 2.0;
        t1 = __builtin_amdgcn_s_memtime();
        cyc[9] = t1 - t0;
        acc += z;
    }
    // 10. dependent fma chain
    {
        double z = x;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP * 4; ++r) z = fma(z, b, a);
        t1 = __builtin_amdgcn_s_memtime();
        cyc[10] = t1 - t0;
        acc += z;
    }
    // 11. LDS write -> wave-local read round trip (other lane's value)
    {
        double z = x;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
            sh[ln] = z;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            z = sh[ln ^ 5] + 1e-300;
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[11] = t1 - t0;
        acc += z;
    }
    // 12. 16 independent v_fmac_f64_dpp row_newbcast per round (one s_nop per block of 8)
    {
        double d[16], src = x * 3.0, c = b;
        for (int i = 0; i < 16; ++i) d[i] = x * (i + 2);
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
            asm volatile("s_nop 1\n\t"
                "v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %4, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %5, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %6, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %7, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf"
                : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7])
                : "v"(src), "v"(c));
            asm volatile("s_nop 1\n\t"
                "v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %4, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %5, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %6, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %7, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf"
                : "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13]), "+v"(d[14]), "+v"(d[15])
                : "v"(src), "v"(c));
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[12] = t1 - t0;
        for (int i = 0; i < 16; ++i) acc += d[i];
    }
    // 13. same with plain v_fmac_f64 (no DPP)
    {
        double d[16], src = x * 3.0, c = b;
        for (int i = 0; i < 16; ++i) d[i] = x * (i + 2);
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
            asm volatile("s_nop 1\n\t"
                "v_fmac_f64 %0, %8, %9\n\tv_fmac_f64 %1, %8, %9\n\tv_fmac_f64 %2, %8, %9\n\tv_fmac_f64 %3, %8, %9\n\t"
                "v_fmac_f64 %4, %8, %9\n\tv_fmac_f64 %5, %8, %9\n\tv_fmac_f64 %6, %8, %9\n\tv_fmac_f64 %7, %8, %9"
                : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7])
                : "v"(src), "v"(c));
            asm volatile("s_nop 1\n\t"
                "v_fmac_f64 %0, %8, %9\n\tv_fmac_f64 %1, %8, %9\n\tv_fmac_f64 %2, %8, %9\n\tv_fmac_f64 %3, %8, %9\n\t"
                "v_fmac_f64 %4, %8, %9\n\tv_fmac_f64 %5, %8, %9\n\tv_fmac_f64 %6, %8, %9\n\tv_fmac_f64 %7, %8, %9"
                : "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13]), "+v"(d[14]), "+v"(d[15])
                : "v"(src), "v"(c));
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[13] = t1 - t0;
        for (int i = 0; i < 16; ++i) acc += d[i];
    }
    // 14. dependent chain of v_fmac_f64_dpp on the accumulator
    {
        double d0 = x, src = x * 3.0, c = b;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
            asm volatile("s_nop 1\n\t"
                "v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f64_dpp %0, %1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf"
                : "+v"(d0) : "v"(src), "v"(c));
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[14] = t1 - t0;
        acc += d0;
    }
    // 15. recursion pattern: each link's DPP source is the previous link's result (ping-pong a <-> b)
    {
        double a0 = x, b0 = x * 0.5, c = b;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
            asm volatile("s_nop 1\n\t"
                "v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\t"
                "v_fmac_f64_dpp %1, %0, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\t"
                "v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\t"
                "v_fmac_f64_dpp %1, %0, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf"
                : "+v"(a0), "+v"(b0) : "v"(c));
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[15] = t1 - t0;
        acc += a0 + b0;
    }
    // 16. dependent v_add_f64 chain
    {
        double z = x;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP * 4; ++r) { z = z + b; asm volatile("" : "+v"(z)); }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[16] = t1 - t0;
        acc += z;
    }
    // 17. dependent v_fmac_f64 chain through the multiplicand (x <- c + x * d), plain VALU
    {
        double z = x, c = a, d = b;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) {
            asm volatile("v_fma_f64 %0, %0, %2, %1\n\tv_fma_f64 %0, %0, %2, %1\n\t"
                         "v_fma_f64 %0, %0, %2, %1\n\tv_fma_f64 %0, %0, %2, %1"
                         : "+v"(z) : "v"(c), "v"(d));
        }
        t1 = __builtin_amdgcn_s_memtime();
        cyc[17] = t1 - t0;
        acc += z;
    }
    // 18. s_memtime reference: 4 * REP dependent v_add_f64 vs s_sleep-free empty loop
    {
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < REP; ++r) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7");
        t1 = __builtin_amdgcn_s_memtime();
        cyc[18] = t1 - t0;
    }
    out[ln] = acc;
}

int main() {
    double* o;
    long long* c;
    hipMalloc(&o, 64 * 8);
    hipMalloc(&c, 32 * 8);
    hipMemset(c, 0, 32 * 8);
    long long h[32];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, 1e-3, 0.999);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, c, 32 * 8, hipMemcpyDeviceToHost);
    // s_memtime ticks; per unit below
    printf("indep v_fma_f64            %7.2f per instr\n", (double)h[0] / (REP * 4 * 8));
    printf("ds_read_b128 bcast, 64 ln  %7.2f per read (incl. 1 add)\n", (double)h[1] / (REP * 16));
    printf("ds_read_b128 bcast, 32 ln  %7.2f per read\n", (double)h[2] / (REP * 16));
    printf("ds_read_b128 bcast, 16 ln  %7.2f per read\n", (double)h[3] / (REP * 16));
    printf("ds_read_b128 bcast,  2 ln  %7.2f per read\n", (double)h[4] / (REP * 16));
    printf("ds_read_b128 per-lane, 64  %7.2f per read\n", (double)h[5] / (REP * 16));
    printf("dependent add (consumer)   %7.2f per add\n", (double)h[6] / (REP * 16));
    printf("dpp row_newbcast b64       %7.2f per double (2 v_mov_dpp)\n", (double)h[7] / (REP * 16));
    printf("frsqrt dependent           %7.2f per link\n", (double)h[8] / REP);
    printf("frcp dependent             %7.2f per link\n", (double)h[9] / REP);
    printf("fma dependent              %7.2f per link\n", (double)h[10] / (REP * 4));
    printf("lds write+read round trip  %7.2f per link\n", (double)h[11] / REP);
    printf("indep v_fmac_f64_dpp       %7.2f per instr (incl. s_nop 1 per 8)\n", (double)h[12] / (REP * 16));
    printf("indep v_fmac_f64 (asm)     %7.2f per instr (incl. s_nop 1 per 8)\n", (double)h[13] / (REP * 16));
    printf("dependent v_fmac_f64_dpp   %7.2f per link\n", (double)h[14] / (REP * 4));
    printf("dpp source chain (+nop 1)  %7.2f per link\n", (double)h[15] / (REP * 4));
    printf("dependent v_add_f64        %7.2f per link\n", (double)h[16] / (REP * 4));
    printf("dependent v_fma_f64 (asm)  %7.2f per link\n", (double)h[17] / (REP * 4));
    printf("s_nop 7 (8 cycles?)        %7.2f per nop\n", (double)h[18] / (REP * 4));
    return 0;
}

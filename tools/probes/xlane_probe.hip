// Checks the gfx950 v_permlane16_swap / v_permlane32_swap semantics the group reductions rely on.
// Called with the same value in both operands, each swap must return the pair (own-side value,
// partner-side value) up to order: {x[lane & ~16], x[lane | 16]} (16) and {x[lane & ~32], x[lane | 32]}
// (32), i.e. the two outputs together hold both halves on every lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o, const unsigned* in) {
    const unsigned x = in[threadIdx.x];
    auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    o[threadIdx.x] = a[0];
    o[64 + threadIdx.x] = a[1];
    o[128 + threadIdx.x] = b[0];
    o[192 + threadIdx.x] = b[1];
}
int main() {
    unsigned h[64], r[256];
    for (int i = 0; i < 64; ++i) h[i] = 1000 + i;
    unsigned *di, *dout;
    hipMalloc(&di, sizeof(h));
    hipMalloc(&dout, sizeof(r));
    hipMemcpy(di, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dout, di);
    hipMemcpy(r, dout, sizeof(r), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; ++i) {
        const unsigned e16 = 1000 + (i & ~16), o16 = 1000 + (i | 16), e32 = 1000 + (i & ~32), o32 = 1000 + (i | 32);
        if (!((r[i] == e16 && r[64 + i] == o16) || (r[i] == o16 && r[64 + i] == e16))) bad++;
        if (!((r[128 + i] == e32 && r[192 + i] == o32) || (r[128 + i] == o32 && r[192 + i] == e32))) bad++;
    }
    printf("permlane16_swap lane 5 -> (%u, %u), lane 21 -> (%u, %u)\n", r[5], r[69], r[21], r[85]);
    printf("permlane32_swap lane 5 -> (%u, %u), lane 37 -> (%u, %u)\n", r[133], r[197], r[165], r[229]);
    printf("permlane swap check: %s\n", bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}

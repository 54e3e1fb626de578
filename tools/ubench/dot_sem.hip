// Semantics check: v_dot4_i32_i8 (VOP3P, asm) vs __builtin_amdgcn_sdot4 (v_dot4c_i32_i8) vs the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t *a, const uint32_t *b, const uint32_t *c, uint32_t *o1, uint32_t *o2) {
    const int t = threadIdx.x;
    uint32_t r, q;
    // the dot's result read by the very next VALU op (a hazard the compiler cannot see through inline asm)
    asm volatile("v_dot4_i32_i8 %0, %2, %3, %4\n\tv_max3_u32 %1, %0, 0, 0" : "=&v"(r), "=v"(q) : "v"(a[t]), "v"(b[t]), "v"(c[t]));
    o1[t] = q;
    o2[t] = (uint32_t)__builtin_amdgcn_sdot4((int)a[t], (int)b[t], (int)c[t], false);
}
int main() {
    const int N = 64;
    uint32_t ha[N], hb[N], hc[N], h1[N], h2[N];
    uint32_t s = 12345;
    for (int i = 0; i < N; ++i) {
        s = s * 1664525u + 1013904223u; ha[i] = s;
        s = s * 1664525u + 1013904223u; hb[i] = s;
        s = s * 1664525u + 1013904223u; hc[i] = s >> 4;
    }
    uint32_t *da, *db, *dc, *d1, *d2;
    hipMalloc(&da, 4 * N); hipMalloc(&db, 4 * N); hipMalloc(&dc, 4 * N); hipMalloc(&d1, 4 * N); hipMalloc(&d2, 4 * N);
    hipMemcpy(da, ha, 4 * N, hipMemcpyHostToDevice); hipMemcpy(db, hb, 4 * N, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc, 4 * N, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(N), 0, 0, da, db, dc, d1, d2);
    hipMemcpy(h1, d1, 4 * N, hipMemcpyDeviceToHost); hipMemcpy(h2, d2, 4 * N, hipMemcpyDeviceToHost);
    int bad1 = 0, bad2 = 0;
    for (int i = 0; i < N; ++i) {
        int32_t ref = (int32_t)hc[i];
        for (int k = 0; k < 4; ++k) ref += (int32_t)(int8_t)(ha[i] >> (8 * k)) * (int32_t)(int8_t)(hb[i] >> (8 * k));
        bad1 += (uint32_t)ref != h1[i];
        bad2 += (uint32_t)ref != h2[i];
        if (i < 4) printf("%08x %08x %08x -> ref %08x asm %08x builtin %08x\n", ha[i], hb[i], hc[i], (uint32_t)ref, h1[i], h2[i]);
    }
    printf("mismatches: asm v_dot4_i32_i8 + dependent v_max3 %d, builtin %d (of %d)\n", bad1, bad2, N);
    return 0;
}

// How many wait states must separate a v_dot4_i32_i8 (VOP3P, inline asm) from a VALU op reading its result?
// For k = 0..5 the reader follows the dot after k wait states, made either of s_nop (s_nop k-1) or of k
// independent VALU ops (v_mov of an unrelated register).  Each variant is checked against the host's dot
// product on 64 lanes x 64 workgroups.  The static check (tools/dot_hazard.py, tests/test_dot_hazard.py)
// asserts the kernels keep at least the distance this shows to be safe, with LLVM's own gfx940-family
// hazard table value (3, "DotWriteDifferentVALURead") as the floor.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define NOPS(k)                                                                                   \
    __global__ void k_nop##k(const uint32_t *a, const uint32_t *b, const uint32_t *c, uint32_t *o) { \
        const int t = blockIdx.x * 64 + threadIdx.x;                                                 \
        uint32_t r, q;                                                                               \
        asm volatile("v_dot4_i32_i8 %0, %2, %3, %4\n\t" NOPSTR##k "v_max3_u32 %1, %0, 0, 0"          \
                     : "=&v"(r), "=v"(q)                                                             \
                     : "v"(a[t]), "v"(b[t]), "v"(c[t]));                                              \
        o[t] = q;                                                                                    \
    }
#define NOPSTR0 ""
#define NOPSTR1 "s_nop 0\n\t"
#define NOPSTR2 "s_nop 1\n\t"
#define NOPSTR3 "s_nop 2\n\t"
#define NOPSTR4 "s_nop 3\n\t"
#define NOPSTR5 "s_nop 4\n\t"
NOPS(0)
NOPS(1)
NOPS(2)
NOPS(3)
NOPS(4)
NOPS(5)

#define VAL(k)                                                                                    \
    __global__ void k_val##k(const uint32_t *a, const uint32_t *b, const uint32_t *c, uint32_t *o) { \
        const int t = blockIdx.x * 64 + threadIdx.x;                                                 \
        uint32_t r, q, f = t;                                                                        \
        asm volatile("v_dot4_i32_i8 %0, %3, %4, %5\n\t" VALSTR##k "v_max3_u32 %1, %0, 0, 0"          \
                     : "=&v"(r), "=v"(q), "+v"(f)                                                    \
                     : "v"(a[t]), "v"(b[t]), "v"(c[t]));                                              \
        o[t] = q + (f & 0u);                                                                         \
    }
#define VALSTR0 ""
#define VALSTR1 "v_add_u32 %2, 1, %2\n\t"
#define VALSTR2 VALSTR1 VALSTR1
#define VALSTR3 VALSTR2 VALSTR1
#define VALSTR4 VALSTR3 VALSTR1
#define VALSTR5 VALSTR4 VALSTR1
VAL(0)
VAL(1)
VAL(2)
VAL(3)
VAL(4)
VAL(5)

typedef void (*kfn)(const uint32_t *, const uint32_t *, const uint32_t *, uint32_t *);

int main() {
    const int N = 64 * 64;
    static uint32_t ha[N], hb[N], hc[N], ho[N];
    uint32_t s = 12345;
    for (int i = 0; i < N; ++i) {
        s = s * 1664525u + 1013904223u; ha[i] = s;
        s = s * 1664525u + 1013904223u; hb[i] = s;
        s = s * 1664525u + 1013904223u; hc[i] = s >> 4;
    }
    uint32_t *da, *db, *dc, *dout;
    hipMalloc(&da, 4 * N); hipMalloc(&db, 4 * N); hipMalloc(&dc, 4 * N); hipMalloc(&dout, 4 * N);
    hipMemcpy(da, ha, 4 * N, hipMemcpyHostToDevice); hipMemcpy(db, hb, 4 * N, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc, 4 * N, hipMemcpyHostToDevice);
    kfn nops[6] = {k_nop0, k_nop1, k_nop2, k_nop3, k_nop4, k_nop5};
    kfn vals[6] = {k_val0, k_val1, k_val2, k_val3, k_val4, k_val5};
    for (int kind = 0; kind < 2; ++kind) {
        for (int k = 0; k < 6; ++k) {
            hipMemset(dout, 0, 4 * N);
            hipLaunchKernelGGL(kind ? vals[k] : nops[k], dim3(64), dim3(64), 0, 0, da, db, dc, dout);
            hipMemcpy(ho, dout, 4 * N, hipMemcpyDeviceToHost);
            int bad = 0;
            for (int i = 0; i < N; ++i) {
                int32_t ref = (int32_t)hc[i];
                for (int b = 0; b < 4; ++b) ref += (int32_t)(int8_t)(ha[i] >> (8 * b)) * (int32_t)(int8_t)(hb[i] >> (8 * b));
                bad += (uint32_t)ref != ho[i];
            }
            printf("%s wait states %d: %d of %d lanes stale\n", kind ? "valu" : "s_nop", k, bad, N);
        }
    }
    return 0;
}

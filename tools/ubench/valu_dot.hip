// Microbenchmark: can a byte dot product (v_dot4_u32_u8 / v_dot4c_i32_i8) replace the cost lookup + add of the
// DP cell (v_perm_b32 + v_add_u32), and at what issue rate does it interleave with v_max3_u32 / v_min3_u32?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 1024
#define A8(M) M("%0") M("%1") M("%2") M("%3") M("%4") M("%5") M("%6") M("%7")
#define DOT(x) "v_dot4_u32_u8 " x ", %8, %9, " x "\n"
#define DOTC(x) "v_dot4c_i32_i8 " x ", %8, %9\n"
#define MAX3(x) "v_max3_u32 " x ", " x ", %8, %9\n"
// DP row, dot form: t = dot4(r, c, old_up); V = max3(V, new_up, t); old_up kept in t-rotation
#define RDOT(up, me, t) "v_dot4_u32_u8 " t ", %10, %11, " up "\n" "v_max3_u32 " me ", " me ", " up ", " t "\n"
// DP row, perm form: t = perm(cv, k, sel); t = t + old_up; V = min3(V, new_up, t)
#define RPERM(up, me, t) "v_perm_b32 " t ", %10, -3, %11\n" "v_add_u32 " t ", " t ", " up "\n" "v_min3_u32 " me ", " me ", " up ", " t "\n"
#define ROWS8(M) M("%7", "%0", "%8") M("%0", "%1", "%9") M("%1", "%2", "%8") M("%2", "%3", "%9") \
                 M("%3", "%4", "%8") M("%4", "%5", "%9") M("%5", "%6", "%8") M("%6", "%7", "%9")
template <int V> __device__ __forceinline__ void body(uint32_t (&a)[8], uint32_t c1, uint32_t c2, uint32_t (&t)[2]) {
#define REGS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
    if constexpr (V == 0) asm volatile(A8(DOT) : REGS : "v"(c1), "v"(c2));
    if constexpr (V == 1) asm volatile(A8(DOTC) : REGS : "v"(c1), "v"(c2));
    if constexpr (V == 2) asm volatile(A8(MAX3) : REGS : "v"(c1), "v"(c2));
    if constexpr (V == 3) asm volatile(DOT("%0") MAX3("%1") DOT("%2") MAX3("%3") DOT("%4") MAX3("%5") DOT("%6") MAX3("%7") : REGS : "v"(c1), "v"(c2));
    if constexpr (V == 4) asm volatile(DOTC("%0") MAX3("%1") DOTC("%2") MAX3("%3") DOTC("%4") MAX3("%5") DOTC("%6") MAX3("%7") : REGS : "v"(c1), "v"(c2));
    if constexpr (V == 5) asm volatile(ROWS8(RDOT) : REGS, "+v"(t[0]), "+v"(t[1]) : "v"(c1), "v"(c2));
    if constexpr (V == 6) asm volatile(ROWS8(RPERM) : REGS, "+v"(t[0]), "+v"(t[1]) : "v"(c1), "v"(c2));
}
static const int NINSTR[] = {8, 8, 8, 8, 8, 16, 24};
static const char *NAMES[] = {"8 dot4_u32_u8", "8 dot4c_i32_i8", "8 max3_u32", "dot4/max3 alt", "dot4c/max3 alt",
                              "DP row x8 dot4+max3", "DP row x8 perm+add+min3"};
template <int V> __global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    uint32_t c1 = seed * 3 + threadIdx.x, c2 = seed ^ threadIdx.x;
    uint32_t t[2] = {seed, seed + 1};
    for (int it = 0; it < ITERS; ++it) body<V>(a, c1, c2, t);
    uint32_t x = t[0] ^ t[1];
    for (int i = 0; i < 8; ++i) x ^= a[i];
    if (x == 0x12345678u) out[0] = 1;
}
typedef void (*kfn)(uint32_t *, uint32_t);
template <int... I> struct L { static constexpr kfn f[] = {k<I>...}; };
int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    using LL = L<0, 1, 2, 3, 4, 5, 6>;
    const int nops = sizeof(NINSTR) / sizeof(NINSTR[0]);
    for (int wps : {8, 5}) {
        const int blocks = 256 * wps;
        for (int op = 0; op < nops; ++op) {
            hipLaunchKernelGGL(LL::f[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(LL::f[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double winstr = 5.0 * blocks * 4.0 * ITERS * NINSTR[op];
            const double cyc = (ms * 1e6) * 2.4 / (winstr / 1024.0);
            printf("waves/SIMD %d  %-26s %.2f cycles/instr  %.2f cycles/body\n", wps, NAMES[op], cyc, cyc * NINSTR[op]);
        }
    }
    return 0;
}

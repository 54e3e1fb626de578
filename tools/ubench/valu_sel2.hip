// Microbenchmark 5: per-lane selects as a DP kernel would issue them: a compare writes the lane
// mask once (VCC or an SGPR pair), then R selects read it, interleaved with adds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 1024
#define REGS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
#define ADD8 "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n" \
             "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
#define SEL8_VCC "v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n" \
                 "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n"
#define SEL8_S(m) "v_cndmask_b32_e64 %0, %0, %8, " m "\n v_cndmask_b32_e64 %1, %1, %8, " m "\n v_cndmask_b32_e64 %2, %2, %8, " m "\n v_cndmask_b32_e64 %3, %3, %8, " m "\n" \
                  "v_cndmask_b32_e64 %4, %4, %8, " m "\n v_cndmask_b32_e64 %5, %5, %8, " m "\n v_cndmask_b32_e64 %6, %6, %8, " m "\n v_cndmask_b32_e64 %7, %7, %8, " m "\n"
#define BFI8 "v_bfi_b32 %0, %10, %8, %0\n v_bfi_b32 %1, %10, %8, %1\n v_bfi_b32 %2, %10, %8, %2\n v_bfi_b32 %3, %10, %8, %3\n" \
             "v_bfi_b32 %4, %10, %8, %4\n v_bfi_b32 %5, %10, %8, %5\n v_bfi_b32 %6, %10, %8, %6\n v_bfi_b32 %7, %10, %8, %7\n"
template <int V> __global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    uint32_t c1 = seed * 3 + threadIdx.x, lane = threadIdx.x & 63, msk = 0;
    uint64_t sm = 0;
    for (int it = 0; it < ITERS; ++it) {
        // per "step": a compare producing the mask, then 8 adds (the DP work stand-in) and 8 selects
        if constexpr (V == 0) asm volatile(ADD8 ADD8 : REGS : "v"(c1), "v"(lane), "v"(msk));
        if constexpr (V == 1) asm volatile("v_cmp_eq_u32 vcc, %9, %8\n" ADD8 SEL8_VCC : REGS : "v"(c1), "v"(lane), "v"(msk) : "vcc");
        if constexpr (V == 2) asm volatile("v_cmp_eq_u32_e64 %11, %9, %8\n" ADD8 SEL8_S("%11") : REGS : "v"(c1), "v"(lane), "v"(msk), "s"(sm));
        if constexpr (V == 3) asm volatile("v_cmp_eq_u32 vcc, %9, %8\n v_cndmask_b32 %10, 0, -1, vcc\n" ADD8 BFI8 : REGS : "v"(c1), "v"(lane), "v"(msk) : "vcc");
        if constexpr (V == 4) asm volatile("v_cmp_eq_u32 vcc, %9, %8\n" SEL8_VCC ADD8 : REGS : "v"(c1), "v"(lane), "v"(msk) : "vcc");
        if constexpr (V == 5) asm volatile("s_mov_b64 vcc, %11\n" ADD8 SEL8_VCC : REGS : "v"(c1), "v"(lane), "v"(msk), "s"(sm) : "vcc");
        c1 += 1;
    }
    uint32_t x = msk;
    for (int i = 0; i < 8; ++i) x ^= a[i];
    if (x == 0x12345678u) out[0] = 1;
}
static const char *NM[] = {"16 add (reference)", "v_cmp vcc + 8 add + 8 cndmask e32 vcc",
                           "v_cmp sgpr + 8 add + 8 cndmask e64 sgpr", "v_cmp + mask + 8 add + 8 bfi",
                           "v_cmp vcc + 8 cndmask vcc + 8 add", "s_mov vcc + 8 add + 8 cndmask vcc"};
static const int NI[] = {16, 17, 17, 18, 17, 16};
typedef void (*kfn)(uint32_t *, uint32_t);
static kfn F[] = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>};
int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int op = 0; op < 6; ++op) {
        const int blocks = 256 * 8;
        hipLaunchKernelGGL(F[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(F[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double steps = 5.0 * blocks * 4.0 * ITERS / 1024.0;
        const double cyc = (ms * 1e6) * 2.4 / steps;
        printf("%-44s %.1f cycles per step (%d VALU) = %.2f cycles/instr\n", NM[op], cyc, NI[op], cyc / NI[op]);
    }
    return 0;
}

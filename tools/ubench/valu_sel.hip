// Microbenchmark 4: cost of per-lane selects on gfx950 (v_cndmask with VCC vs an SGPR pair,
// with and without an SALU write of the mask right before, and v_bfi with a VGPR lane mask).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 1024
#define R8(X) X("%0") X("%1") X("%2") X("%3") X("%4") X("%5") X("%6") X("%7")
#define CND_VCC(x) "v_cndmask_b32 " x ", " x ", %8, vcc\n"
#define CND_E64VCC(x) "v_cndmask_b32_e64 " x ", " x ", %8, vcc\n"
#define CND_S(x) "v_cndmask_b32_e64 " x ", " x ", %8, %10\n"
#define SALU_VCC(x) "s_and_b64 vcc, %10, %11\n v_cndmask_b32 " x ", " x ", %8, vcc\n"
#define SALU_S(x) "s_and_b64 %8, %11, %12\n v_cndmask_b32_e64 " x ", " x ", %9, %8\n"
#define BFI(x) "v_bfi_b32 " x ", %9, %8, " x "\n"
#define ADD(x) "v_add_u32 " x ", " x ", %8\n"
#define MIXS(x) "v_add_u32 " x ", " x ", %8\n v_cndmask_b32_e64 " x ", " x ", %8, %10\n"
#define MIXV(x) "v_add_u32 " x ", " x ", %8\n v_cndmask_b32 " x ", " x ", %8, vcc\n"
#define REGS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
template <int V> __global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
    uint32_t c1 = seed * 3 + threadIdx.x, msk = (threadIdx.x & 1) ? 0xFFFFFFFFu : 0u;
    uint64_t sm1 = ~0ull, sm2 = 0x5555555555555555ull, st = 0;
    asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
    asm volatile("" : "+s"(sm1), "+s"(sm2));
    for (int it = 0; it < ITERS; ++it) {
        if constexpr (V == 0) asm volatile(R8(CND_VCC) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2) : "vcc");
        if constexpr (V == 1) asm volatile(R8(CND_E64VCC) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2) : "vcc");
        if constexpr (V == 2) asm volatile(R8(CND_S) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2));
        if constexpr (V == 3) asm volatile(R8(SALU_VCC) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2) : "vcc");
        if constexpr (V == 4) asm volatile(R8(SALU_S) : REGS, "+s"(st) : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2));
        if constexpr (V == 5) asm volatile(R8(BFI) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2));
        if constexpr (V == 6) asm volatile(R8(ADD) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2));
        if constexpr (V == 7) asm volatile(R8(MIXS) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2));
        if constexpr (V == 8) asm volatile(R8(MIXV) : REGS : "v"(c1), "v"(msk), "s"(sm1), "s"(sm2) : "vcc");
    }
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x ^= a[i];
    if (x == 0x12345678u) out[0] = 1;
}
static const char *NM[] = {"cndmask e32 vcc", "cndmask e64 vcc", "cndmask e64 s[20:21]", "s_and vcc + cndmask vcc",
                           "s_and s + cndmask e64 s", "bfi with VGPR mask", "add (reference)", "add + cndmask e64 s",
                           "add + cndmask e32 vcc"};
static const int NI[] = {8, 8, 8, 8, 8, 8, 8, 16, 16};
typedef void (*kfn)(uint32_t *, uint32_t);
static kfn F[] = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>};
int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int wps : {8, 2})
        for (int op = 0; op < 9; ++op) {
            const int blocks = 256 * wps;
            hipLaunchKernelGGL(F[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(F[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double winstr = 5.0 * blocks * 4.0 * ITERS * NI[op];
            printf("waves/SIMD %d  %-28s %.2f cycles per VALU instr\n", wps, NM[op], (ms * 1e6) * 2.4 / (winstr / 1024.0));
        }
    return 0;
}

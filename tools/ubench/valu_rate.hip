// Microbenchmark: VALU issue rate of the integer ops the DP kernel uses (gfx950).
// Each lane runs 8 independent chains of ONE instruction, written as inline asm
// so nothing folds; reports cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
#define BODY(INSTR)                                                                      \
    for (int it = 0; it < ITERS; ++it) {                                                 \
        asm volatile(INSTR : "+v"(a0) : "v"(c1), "v"(c2));                               \
        asm volatile(INSTR : "+v"(a1) : "v"(c1), "v"(c2));                               \
        asm volatile(INSTR : "+v"(a2) : "v"(c1), "v"(c2));                               \
        asm volatile(INSTR : "+v"(a3) : "v"(c1), "v"(c2));                               \
        asm volatile(INSTR : "+v"(a4) : "v"(c1), "v"(c2));                               \
        asm volatile(INSTR : "+v"(a5) : "v"(c1), "v"(c2));                               \
        asm volatile(INSTR : "+v"(a6) : "v"(c1), "v"(c2));                               \
        asm volatile(INSTR : "+v"(a7) : "v"(c1), "v"(c2));                               \
    }
template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    uint32_t c1 = seed * 3 + threadIdx.x, c2 = seed ^ threadIdx.x;
    if constexpr (OP == 0) BODY("v_add_u32 %0, %0, %1")
    if constexpr (OP == 1) BODY("v_min3_u32 %0, %0, %1, %2")
    if constexpr (OP == 2) BODY("v_perm_b32 %0, %0, %1, %2")
    if constexpr (OP == 3) BODY("v_alignbit_b32 %0, %0, %1, 2")
    if constexpr (OP == 4) BODY("v_lshl_add_u32 %0, %0, 2, %1")
    if constexpr (OP == 5) BODY("v_pk_add_u16 %0, %0, %1")
    if constexpr (OP == 6) BODY("v_and_b32 %0, %0, %1")
    if constexpr (OP == 7) BODY("v_pk_min_u16 %0, %0, %1")
    if constexpr (OP == 8) BODY("v_add3_u32 %0, %0, %1, %2")
    if constexpr (OP == 9) BODY("v_cndmask_b32 %0, %0, %1, vcc")
    if constexpr (OP == 10) BODY("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf")
    if constexpr (OP == 11) BODY("v_min_u32 %0, %0, %1")
    if constexpr (OP == 12) BODY("v_fma_f32 %0, %0, %1, %2")
    if constexpr (OP == 13) BODY("v_pk_fma_f32 %0, %0, %1, %2")
    if (((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345678u)) out[0] = 1;
}
typedef void (*kfn)(uint32_t *, uint32_t);
int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[] = {"v_add_u32", "v_min3_u32", "v_perm_b32", "v_alignbit_b32", "v_lshl_add_u32",
                           "v_pk_add_u16", "v_and_b32", "v_pk_min_u16", "v_add3_u32", "v_cndmask_b32",
                           "v_mov_dpp(shr)", "v_min_u32", "v_fma_f32", "v_pk_fma_f32(64b regs!)"};
    kfn fns[] = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>, k<11>, k<12>};
    for (int waves_per_simd : {1, 2, 4, 8}) {
        const int blocks = 256 * waves_per_simd;
        for (int op = 0; op < 13; ++op) {
            hipLaunchKernelGGL(fns[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(fns[op], dim3(blocks), dim3(256), 0, 0, d, 1u);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double winstr = 5.0 * blocks * 4.0 * ITERS * 8;
            const double per_ns = winstr / 1024.0 / (ms * 1e6);
            printf("waves/SIMD %d  %-16s %.3f wave-instr/ns/SIMD  (%.2f cycles at 2.4 GHz)\n", waves_per_simd,
                   names[op], per_ns, 2.4 / per_ns);
        }
    }
    return 0;
}

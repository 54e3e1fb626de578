// Microbenchmark 2: issue rate of candidate VALU ops on gfx950 at 8 waves/SIMD.
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
#define OPS(X) \
 X(0,"v_min_f32 %0, %0, %1") X(1,"v_min3_f32 %0, %0, %1, %2") X(2,"v_max3_f32 %0, %0, %1, %2") \
 X(3,"v_med3_f32 %0, %0, %1, %2") X(4,"v_lshlrev_b32 %0, 2, %0") X(5,"v_lshrrev_b32 %0, 2, %0") \
 X(6,"v_or_b32 %0, %0, %1") X(7,"v_xor_b32 %0, %0, %1") X(8,"v_sub_u32 %0, %0, %1") \
 X(9,"v_bfi_b32 %0, %0, %1, %2") X(10,"v_bfe_u32 %0, %0, %1, 8") X(11,"v_and_or_b32 %0, %0, %1, %2") \
 X(12,"v_or3_b32 %0, %0, %1, %2") X(13,"v_cndmask_b32 %0, %0, %1, s[0:1]") X(14,"v_add_f32 %0, %0, %1") \
 X(15,"v_mul_u32_u24 %0, %0, %1") X(16,"v_mad_u32_u24 %0, %0, %1, %2") X(17,"v_mov_b32 %0, %1") \
 X(18,"v_max_u32 %0, %0, %1") X(19,"v_med3_u32 %0, %0, %1, %2") X(20,"v_lshl_or_b32 %0, %0, 2, %1") \
 X(21,"v_add_lshl_u32 %0, %0, %1, 2") X(22,"v_min_i32 %0, %0, %1") X(23,"v_pk_min_i16 %0, %0, %1") \
 X(24,"v_add_u32 %0, %0, %1") X(25,"v_min_u32 %0, %0, %1") X(26,"v_min3_u32 %0, %0, %1, %2") \
 X(27,"v_alignbit_b32 %0, %0, %1, 2") X(28,"v_perm_b32 %0, %0, %1, %2") X(29,"v_max_f32 %0, %0, %1") \
 X(30,"v_add3_u32 %0, %0, %1, %2") X(31,"v_lshl_add_u32 %0, %0, 2, %1") X(32,"v_max_i32 %0, %0, %1") \
 X(33,"v_min_f16 %0, %0, %1") X(34,"v_cvt_f32_u32 %0, %0") X(35,"v_mul_f32 %0, %0, %1")
#define KDEF(N, S) template <> __global__ __launch_bounds__(256) void k<N>(uint32_t *out, uint32_t seed) { \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    uint32_t c1 = seed * 3 + threadIdx.x, c2 = seed ^ threadIdx.x; \
    asm volatile("s_mov_b64 s[0:1], -1" ::: "s0", "s1"); \
    BODY(S) \
    if (((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345678u)) out[0] = 1; }
template <int OP> __global__ void k(uint32_t *, uint32_t);
OPS(KDEF)
typedef void (*kfn)(uint32_t *, uint32_t);
int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
#define NAME(N, S) S,
#define FN(N, S) k<N>,
    const char *names[] = {OPS(NAME)};
    kfn fns[] = {OPS(FN)};
    const int nops = sizeof(fns) / sizeof(fns[0]);
    const int blocks = 256 * 8;
    for (int op = 0; op < nops; ++op) {
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
        printf("%-36s %.3f wave-instr/ns/SIMD  (%.2f cycles at 2.4 GHz)\n", names[op], per_ns, 2.4 / per_ns);
    }
    return 0;
}

// Latency of config 2's SPLIT step on one wave (round 5): R = 4 rows per lane, dot keys (v_dot4 + v_max3 per cell),
// the cell above by DPP wave_shr:1, lane 63's bottom row collected by DPP wave_shl:1, no memory.  One wave per CU
// (the SPLIT compute wave is alone on its SIMD), STEPS steps, cycles per step from s_memtime.
//   CHAINS = 1: the kernel's step;  CHAINS = 2: two independent row chains per lane interleaved (twice the cells per
//   step): if a step costs less than twice as much, the single wave is latency-bound and ILP would pay.
//   COLLECT = 0: without the bottom-row collection (2 of the step's 11 VALU).
// hipcc --offload-arch=gfx950 -O3 split_step.hip -o split_step && ./split_step
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define STEPS 4096

__device__ __forceinline__ uint32_t dot_add(uint32_t rowv, uint32_t colv, uint32_t diag) {
    uint32_t r;
    asm volatile("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r) : "v"(rowv), "v"(colv), "v"(diag));
    return r;
}
__device__ __forceinline__ void fence(uint32_t &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t src) {
    return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ uint32_t shl1(uint32_t old, uint32_t src) {
    return __builtin_amdgcn_update_dpp(old, src, 0x130, 0xF, 0xF, false);  // wave_shl:1
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) { return max(max(a, b), c); }

template <int CHAINS, bool COLLECT>
__global__ __launch_bounds__(64) void k(const uint32_t *in, uint32_t *out, uint64_t *cyc) {
    const int lane = threadIdx.x;
    uint32_t cv[4], V[CHAINS][4], tp[CHAINS], bottom[CHAINS], outc = 0;
    for (int r = 0; r < 4; ++r) cv[r] = in[r];
    for (int c = 0; c < CHAINS; ++c) {
        for (int r = 0; r < 4; ++r) V[c][r] = in[8 + r + 4 * c] + lane;
        tp[c] = in[16 + c];
        bottom[c] = V[c][3];
    }
    const uint32_t sel0 = in[20], top0 = in[21];
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int s = 0; s < STEPS; ++s) {
        const uint32_t selv = sel0 + (uint32_t)s;  // (the step's column vector; in the kernel an LDS read)
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            uint32_t cand[4];
            cand[0] = dot_add(cv[0], selv, tp[c]);
#pragma unroll
            for (int r = 1; r < 4; ++r) cand[r] = dot_add(cv[r], selv, V[c][r - 1]);
            const uint32_t topv = shr1(top0 + (uint32_t)s, bottom[c]);
            uint32_t up = topv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                fence(cand[r]);
                up = umax3(V[c][r], up, cand[r]);
                V[c][r] = up;
            }
            tp[c] = topv;
            bottom[c] = V[c][3];
            if (COLLECT && c == 0) outc = shl1(bottom[c], outc);
        }
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    uint32_t acc = outc;
    for (int c = 0; c < CHAINS; ++c)
        for (int r = 0; r < 4; ++r) acc ^= V[c][r];
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS, bool COLLECT>
void run(const char *name, uint32_t *din, uint32_t *dout, uint64_t *dcyc) {
    hipLaunchKernelGGL((k<CHAINS, COLLECT>), dim3(8), dim3(64), 0, 0, din, dout, dcyc);
    hipLaunchKernelGGL((k<CHAINS, COLLECT>), dim3(8), dim3(64), 0, 0, din, dout, dcyc);
    (void)hipDeviceSynchronize();
    uint64_t h[8];
    (void)hipMemcpy(h, dcyc, sizeof(h), hipMemcpyDeviceToHost);
    uint64_t mn = h[0];
    for (int i = 1; i < 8; ++i) mn = h[i] < mn ? h[i] : mn;
    printf("%-28s %6.1f cycles per step (%d chain%s, %d cells per lane per step)\n", name, (double)mn / STEPS, CHAINS,
           CHAINS > 1 ? "s" : "", 4 * CHAINS);
}

int main() {
    uint32_t hin[32];
    for (int i = 0; i < 32; ++i) hin[i] = 0x01020304u * (uint32_t)(i + 1);
    uint32_t *din, *dout;
    uint64_t *dcyc;
    (void)hipMalloc(&din, sizeof(hin));
    (void)hipMalloc(&dout, 8 * 64 * 4);
    (void)hipMalloc(&dcyc, 8 * 8);
    (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
    run<1, true>("step (kernel)", din, dout, dcyc);
    run<1, false>("step without collection", din, dout, dcyc);
    run<2, true>("two chains interleaved", din, dout, dcyc);
    return 0;
}

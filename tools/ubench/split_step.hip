// Latency of config 2's SPLIT step on one wave (round 5): R = 4 rows per lane, dot keys (v_dot4 + v_max3 per cell),
// the cell above by DPP wave_shr:1, lane 63's bottom row collected by DPP wave_shl:1, no memory.  One wave per CU
// (the SPLIT compute wave is alone on its SIMD), STEPS steps, cycles per step from s_memtime.
//   CHAINS = 1: the kernel's step;  CHAINS = 2: two independent row chains per lane interleaved (twice the cells per
//   step): if a step costs less than twice as much, the single wave is latency-bound and ILP would pay.
//   COLLECT = 0: without the bottom-row collection (2 of the step's 11 VALU).
//   kp (PIPE): one chain, the next step's dots issued between this step's dependent maxes.
//   kr<RR>: the kernel's step at RR = 1, 2, 4, 8 rows per lane.
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

// PIPE: the next step's dots interleaved with this step's max chain (dot r + 1 of step s + 1 right after max r of
// step s, dot 0 right after the DPP of the cell above), so that the independent dots fill the chain's latency bubbles
template <bool COLLECT>
__global__ __launch_bounds__(64) void kp(const uint32_t *in, uint32_t *out, uint64_t *cyc) {
    const int lane = threadIdx.x;
    uint32_t cv[4], V[4], tp, bottom, outc = 0;
    for (int r = 0; r < 4; ++r) cv[r] = in[r];
    for (int r = 0; r < 4; ++r) V[r] = in[8 + r] + lane;
    tp = in[16];
    bottom = V[3];
    const uint32_t sel0 = in[20], top0 = in[21];
    uint32_t cand[4];
    cand[0] = dot_add(cv[0], sel0, tp);
    for (int r = 1; r < 4; ++r) cand[r] = dot_add(cv[r], sel0, V[r - 1]);
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int s = 0; s < STEPS; ++s) {
        const uint32_t seln = sel0 + (uint32_t)(s + 1);  // the next step's column vector
        const uint32_t topv = shr1(top0 + (uint32_t)s, bottom);
        uint32_t nc[4];
        nc[0] = dot_add(cv[0], seln, topv);
        uint32_t up = topv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            fence(cand[r]);
            up = umax3(V[r], up, cand[r]);
            V[r] = up;
            if (r + 1 < 4) nc[r + 1] = dot_add(cv[r + 1], seln, up);
        }
        bottom = V[3];
        if (COLLECT) outc = shl1(bottom, outc);
#pragma unroll
        for (int r = 0; r < 4; ++r) cand[r] = nc[r];
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    uint32_t acc = outc;
    for (int r = 0; r < 4; ++r) acc ^= V[r] ^ cand[r];
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// rows per lane RR (1, 2, 4, 8): the chain of a step is the DPP move plus RR dependent maxes
template <int RR>
__global__ __launch_bounds__(64) void kr(const uint32_t *in, uint32_t *out, uint64_t *cyc) {
    const int lane = threadIdx.x;
    uint32_t cv[RR], V[RR], tp, bottom, outc = 0;
    for (int r = 0; r < RR; ++r) cv[r] = in[r & 3];
    for (int r = 0; r < RR; ++r) V[r] = in[8 + (r & 3)] + lane + r;
    tp = in[16];
    bottom = V[RR - 1];
    const uint32_t sel0 = in[20], top0 = in[21];
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int s = 0; s < STEPS; ++s) {
        const uint32_t selv = sel0 + (uint32_t)s;
        uint32_t cand[RR];
        cand[0] = dot_add(cv[0], selv, tp);
#pragma unroll
        for (int r = 1; r < RR; ++r) cand[r] = dot_add(cv[r], selv, V[r - 1]);
        const uint32_t topv = shr1(top0 + (uint32_t)s, bottom);
        uint32_t up = topv;
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            fence(cand[r]);
            up = umax3(V[r], up, cand[r]);
            V[r] = up;
        }
        tp = topv;
        bottom = V[RR - 1];
        outc = shl1(bottom, outc);
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    uint32_t acc = outc;
    for (int r = 0; r < RR; ++r) acc ^= V[r];
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int RR>
void runr(uint32_t *din, uint32_t *dout, uint64_t *dcyc) {
    hipLaunchKernelGGL((kr<RR>), dim3(8), dim3(64), 0, 0, din, dout, dcyc);
    hipLaunchKernelGGL((kr<RR>), dim3(8), dim3(64), 0, 0, din, dout, dcyc);
    (void)hipDeviceSynchronize();
    uint64_t h[8];
    (void)hipMemcpy(h, dcyc, sizeof(h), hipMemcpyDeviceToHost);
    uint64_t mn = h[0];
    for (int i = 1; i < 8; ++i) mn = h[i] < mn ? h[i] : mn;
    printf("R = %d rows per lane          %6.1f cycles per step\n", RR, (double)mn / STEPS);
}

template <bool COLLECT>
void runp(const char *name, uint32_t *din, uint32_t *dout, uint64_t *dcyc) {
    hipLaunchKernelGGL((kp<COLLECT>), dim3(8), dim3(64), 0, 0, din, dout, dcyc);
    hipLaunchKernelGGL((kp<COLLECT>), dim3(8), dim3(64), 0, 0, din, dout, dcyc);
    (void)hipDeviceSynchronize();
    uint64_t h[8];
    (void)hipMemcpy(h, dcyc, sizeof(h), hipMemcpyDeviceToHost);
    uint64_t mn = h[0];
    for (int i = 1; i < 8; ++i) mn = h[i] < mn ? h[i] : mn;
    printf("%-28s %6.1f cycles per step (1 chain, 4 cells per lane per step)\n", name, (double)mn / STEPS);
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
    runp<true>("next step's dots interleaved", din, dout, dcyc);
    runp<false>("  ... without collection", din, dout, dcyc);
    runr<1>(din, dout, dcyc);
    runr<2>(din, dout, dcyc);
    runr<4>(din, dout, dcyc);
    runr<8>(din, dout, dcyc);
    return 0;
}

// The c4 forward's step (R = 16 rows per lane, dot keys: 16 v_dot4 + 16 dependent v_max3 + the DPP move of the cell
// above) at full occupancy, against the same work as two independent 8-row chains per step (round 6).
//   chains 1: the kernel's step (sed_kernels.hip i32_step DOT): row r's max needs row r-1's, and row 0 needs the previous
//             step's row 15 of the lane before (DPP), a 17-deep chain per step.
//   chains 2: rows 0-7 at column j and rows 8-15 one column behind (j-1): the lower chain's cell above is the upper
//             chain's row 7 of the previous step, so each step holds two 8-deep chains (+ the DPP) that can interleave.
//             (Its lanes would be 2 steps apart, a 126-step ramp per stripe instead of 63.)
// No memory in the loop; the column vector changes per step.  WAVES waves per SIMD (grid = 256 CUs x WAVES workgroups
// of 4 waves), STEPS steps per wave.  Prints ms, ns per step per wave and the VALU issue fraction (33 VALU per step at 4
// cycles each over 1024 SIMDs at the measured clock).
// hipcc --offload-arch=gfx950 -O3 dot_chain.hip -o dot_chain && ./dot_chain
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define STEPS 8192
#define R 16

__device__ __forceinline__ uint32_t dot_add(uint32_t rowv, uint32_t colv, uint32_t diag) {
    uint32_t r;
    asm volatile("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r) : "v"(rowv), "v"(colv), "v"(diag));
    return r;
}
__device__ __forceinline__ void fence(uint32_t &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t src) {
    return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) { return max(max(a, b), c); }

template <int WAVES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void k1(const uint32_t *in,
                                                                                              uint32_t *out) {
    const int lane = threadIdx.x & 63;
    uint32_t cv[R], V[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        cv[r] = in[r];
        V[r] = in[16 + r] + lane;
    }
    uint32_t top_prev = in[32], bottom = V[R - 1];
    const uint32_t sel0 = in[33], top0 = in[34];
    for (int s = 0; s < STEPS; ++s) {
        const uint32_t selv = sel0 + (uint32_t)s;
        constexpr int AH = 8;
        uint32_t cand[R];
        cand[0] = dot_add(cv[0], selv, top_prev);
#pragma unroll
        for (int r = 1; r < AH; ++r) cand[r] = dot_add(cv[r], selv, V[r - 1]);
        const uint32_t topv = shr1(top0 + (uint32_t)s, bottom);
        uint32_t up = topv;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r + AH < R) cand[r + AH] = dot_add(cv[r + AH], selv, V[r + AH - 1]);
            fence(cand[r]);
            up = umax3(V[r], up, cand[r]);
            V[r] = up;
        }
        top_prev = topv;
        bottom = V[R - 1];
    }
    uint32_t acc = top_prev;
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= V[r];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int WAVES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void k2(const uint32_t *in,
                                                                                              uint32_t *out) {
    const int lane = threadIdx.x & 63;
    constexpr int H = R / 2;
    uint32_t cv[R], V[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        cv[r] = in[r];
        V[r] = in[16 + r] + lane;
    }
    uint32_t top_prev = in[32], bottom = V[R - 1], selL = in[35];
    uint32_t c8 = in[36];  // the lower chain's row-8 candidate, issued a step ahead (its diagonal is 2 steps old)
    const uint32_t sel0 = in[33], top0 = in[34];
    for (int s = 0; s < STEPS; ++s) {
        const uint32_t selU = sel0 + (uint32_t)s;
        uint32_t cu[H], cl[H];
        cu[0] = dot_add(cv[0], selU, top_prev);
        cl[0] = c8;
#pragma unroll
        for (int r = 1; r < H; ++r) {
            cu[r] = dot_add(cv[r], selU, V[r - 1]);
            cl[r] = dot_add(cv[H + r], selL, V[H + r - 1]);
        }
        const uint32_t c8n = dot_add(cv[H], selU, V[H - 1]);  // next step's row 8: diagonal = row 7 at this column - 1
        const uint32_t topv = shr1(top0 + (uint32_t)s, bottom);
        uint32_t upU = topv, upL = V[H - 1];  // the lower chain's cell above: row 7 one column back (before this step)
#pragma unroll
        for (int r = 0; r < H; ++r) {
            fence(cu[r]);
            fence(cl[r]);
            upU = umax3(V[r], upU, cu[r]);
            upL = umax3(V[H + r], upL, cl[r]);
            V[r] = upU;
            V[H + r] = upL;
        }
        top_prev = topv;
        bottom = V[R - 1];
        selL = selU;
        c8 = c8n;
    }
    uint32_t acc = top_prev ^ c8;
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= V[r];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <typename K>
static void run(const char *name, K kern, int waves, const uint32_t *din, uint32_t *dout) {
    const int grid = 256 * waves;  // 4 waves per workgroup, one per SIMD
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, din, dout);  // warm-up
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, din, dout);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
    const double cycles = best * 1e-3 * clk * 1e3;
    const double issue = (double)grid * 4 * STEPS * 33 * 4 / (cycles * 1024.0);
    printf("%-8s waves/SIMD %d: %.3f ms, %.1f ns per step per wave, VALU issue %.3f (clock %d MHz)\n", name, waves, best,
           best * 1e6 / STEPS, issue, clk / 1000);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main() {
    uint32_t h[64];
    for (int i = 0; i < 64; ++i) h[i] = 0x01020304u * (i + 1);
    uint32_t *din, *dout;
    hipMalloc(&din, sizeof h);
    hipMalloc(&dout, 256 * 256 * 8 * sizeof(uint32_t));
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    run("chains1", k1<5>, 5, din, dout);
    run("chains2", k2<5>, 5, din, dout);
    run("chains1", k1<4>, 4, din, dout);
    run("chains2", k2<4>, 4, din, dout);
    run("chains1", k1<6>, 6, din, dout);
    run("chains2", k2<6>, 6, din, dout);
    run("chains1", k1<2>, 2, din, dout);
    run("chains2", k2<2>, 2, din, dout);
    run("chains1", k1<1>, 1, din, dout);
    run("chains2", k2<1>, 1, din, dout);
    hipFree(din);
    hipFree(dout);
    return 0;
}

// sed_internal.h — structures shared by the kernels and the runtime (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SED_MAX_K 32

// Per-pair descriptor in device memory (64 bytes).
struct sed_pair_desc {
    uint64_t a_off;    // str1: word offset (integer kernel, 2-bit packed) or byte offset (fp64 kernel)
    uint64_t b_off;    // str2: same
    uint64_t tb_off;   // traceback codes: uint32 word offset
    uint64_t bnd_off;  // stripe bottom-row buffer: uint32 word offset
    uint64_t ops_off;  // packed script: uint32 word offset
    int32_t n, m;
    int32_t lane;      // 1: computed by the lane-per-pair kernel (short str2), the wave kernels skip it
    int32_t map_off;   // stripe-parallel traceback: word offset of the pair's stripe exit map
    int32_t pad[2];
};

// Per-pair result (16 bytes).
struct sed_result {
    double dist;     // dp[n][m].value
    int32_t len;     // ops in the canonical script (L at the sink)
    uint8_t is_int;  // 1 when the reference's value is a Python int
    uint8_t err;     // SED_ERR_* (0 = ok); nonzero: the pair's results are invalid
    uint16_t seq;    // CHAIN mode: ordinal of the pair within the wave that computed it (diagnostics)
};

// sed_result.err codes (sed_runtime.cpp: fetch_results maps them to SED_E_DEVICE with the pair index)
#define SED_ERR_SPLIT_TIMEOUT 1  // SPLIT: an inter-workgroup hand-off wait timed out
#define SED_ERR_TB_CHECK 2       // CK traceback: a recomputed tile disagrees with the path length (bad checkpoint)
#define SED_ERR_TB_STALL 3       // traceback: a tile visit made no progress
#define SED_ERR_TB_GUARD 4       // traceback: more tile visits than any path can need
#define SED_ERR_TB_LENGTH 5      // traceback: the walk's op count differs from the sink's L

#ifdef __HIPCC__  // (device helpers: the runtime, compiled by g++, does not see them)
// Script padding.  A pair's script region holds ceil((n+m)/16) words; its ops fill ceil(len/16) of them.  Every walk
// starts its op accumulator at 0, so the bits past the last op inside the last op word are 0 already; this zeroes the
// spare words after it (lanes lane, lane + stride, ...), so the packed buffer is a function of the scripts alone,
// whatever the buffer held before (sed.h).  Every script-writing kernel calls it once per pair.
#ifndef SED_PAD_ZERO
#define SED_PAD_ZERO 1  // (0: A/B builds only; the padding is then whatever the buffer held)
#endif
__device__ __forceinline__ void zero_script_tail(uint32_t *__restrict__ out, int len, int n, int m, int lane,
                                                 int stride) {
    if (!SED_PAD_ZERO) return;
    const int end = (n + m + 15) >> 4;
    for (int w = ((len > 0 ? len : 0) + 15) / 16 + lane; w < end; w += stride) out[w] = 0u;
}

// The same for the lane-per-pair walks, where each lane owns a pair: the wave stores every active lane's spare words
// [ceil(len/16), ceil((n+m)/16)) pair by pair as one coalesced run, its active lanes side by side.  (Each lane storing
// its own pair's words one after another scattered every store instruction over 64 pairs: config 3's per-cell-code
// traceback took 1.68-1.91 instead of 0.75 ms, profiles/r06/pad_ab.)  Lanes that left the kernel own no pair here.
__device__ __forceinline__ void zero_script_tails_wave(uint32_t *__restrict__ ops, uint64_t off, int len, int n, int m) {
    if (!SED_PAD_ZERO) return;
    const uint64_t act = __ballot(1);
    const int rank = __popcll(act & ((1ull << (threadIdx.x & 63)) - 1ull)), nact = __popcll(act);
    const int w0 = ((len > 0 ? len : 0) + 15) >> 4, w1 = (n + m + 15) >> 4;
    uint64_t todo = __ballot(w0 < w1);
    while (todo) {
        const int l = __builtin_ctzll(todo);
        todo &= todo - 1ull;
        const int a = __builtin_amdgcn_readlane(w0, l), b = __builtin_amdgcn_readlane(w1, l);
        const uint64_t o = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off, l) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(off >> 32), l) << 32);
        for (int w = a + rank; w < b; w += nact) ops[o + (uint64_t)w] = 0u;
    }
}
#endif  // __HIPCC__

// Integer kernel constants (offset-key space, see sed_kernels.hip):
//   costrow[a]   byte b = (cost(a -> b) - insert - delete - 1) & 0xFF  (32-bit keys)
//   costrow16[a] byte b = (cost(a -> b) - insert - delete) & 0xFF      (16-bit packed distance keys)
//   kins = (insert << 16) + 4, kdel = (delete << 16) + 5: the lane kernels' key increments (op included;
//   their offsets per column / row are kins and kdel - 1).  The wave kernels derive their own from ins/del.
#define SED_KB 0xFFFFFFFCu  // bias of the 32-bit distance-only offset keys (sed_kernels.hip)
#define SED_KB_DOT 0u       // border of the dot keys (every border cell is X = U = 0)
struct sed_i32_params {
    uint32_t costrow[4];
    uint32_t costrow16[4];
    uint32_t kins, kdel;
    uint32_t ins, del;
    uint32_t epoch;  // SPLIT hand-off words' tag: 1..32767 per run (sed_kernels.hip: store_tagged)
    // Dot keys (checkpoint batches of the stripe kernel, sed_kernels.hip: i32_step DOT): the update addend
    // A*kappa(a, b) + 1, kappa = insert + delete - cost(a -> b), as a signed byte dot product
    // dot4(dotrow[a], dotcol[b]); keys W = A*X + U (X = sum of kappa on the path, U = its updates), maximised.
    // Decode: X = (k * dotM) >> dotS (= floor(k*kmax / (A*kmax + 1)); dotM includes kmax, dotS >= 32, so the
    // kernels take one v_mul_hi_u32), U = k - A*X.
    uint32_t dot;  // 1: the CK forward kernel runs dot keys, the CK traceback converts them
    uint32_t dotA, dotkmax, dotM, dotS;
    uint32_t dotrow[4], dotcol[4];
    // Ladder dot keys (CHAIN kernel with the L field): V = D*ladA + 8L over the ladder (lad = 1) or D*ladA + 16L over
    // the wide ladder (lad = 2), the update addend of a d = -1 row -(ladA*kappa + 7) (+ 15) = dot4(ladrow[a],
    // ladcol[b]) (sed_kernels.hip: i32_step LDOT)
    uint32_t lad, ladA, ladsent;
    uint32_t ladrow[4], ladcol[4];
};

struct sed_f64_params {
    double ins, del;
    int32_t ins_int, del_int;
    int32_t K;
    uint32_t epoch;  // SPLIT hand-off words' tag, as sed_i32_params::epoch (sed_kernels.hip: sed_wf_f64_split_kernel)
};

// Full-matrix output (dp proxy materialisation): D[i*(m+1)+j], M = edge mask (1 ins, 2 del, 4 upd) | int << 3.
struct sed_full_out {
    double *D;
    uint8_t *M;
    int32_t n, m;
};

// a kernel launch of a sed_launch phase, carrying its events (see sed_launch::ev0 / ev1); the .hip files that
// use it include <hip/hip_ext.h> (the host-compiled runtime does not)
#define SED_LAUNCH(kernel, grid, block, shmem, L, ...) \
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, (L).stream, (L).ev0, (L).ev1, 0, __VA_ARGS__)

struct sed_launch {
    const sed_pair_desc *pd;
    int npairs;
    const void *seqa, *seqb;
    uint32_t *tb;   // nullptr -> distance only
    uint32_t *ops;  // packed scripts (lane kernel writes them itself)
    uint32_t *bnd;
    sed_result *res;
    int R;
    hipStream_t stream;
    bool tb_ladder;     // traceback codes of the integer kernels carry the row's ladder rung (sed_kernels.hip)
    bool tb_wide;       // ... of the wide ladder (ladder dot keys, LadderW: the CHAIN kernel's LDOT batches)
    bool ck;            // integer R = 16 wave kernel: tb holds checkpoints, the traceback recomputes tiles
    // timing events carried by the launches themselves (hipExtLaunchKernelGGL: timestamps on the dispatch
    // packet, no marker packet between kernels): the launcher's first kernel records ev0 at its start, its last
    // kernel ev1 at its end; nullptr = none
    hipEvent_t ev0, ev1;
    const int2 *tasks;  // SPLIT mode: (pair, stripe) per workgroup, else nullptr
    int ntasks;         // 0 -> one wave per pair
    // CHAIN mode: chain c runs pairs chain_pairs[chain_off[c] .. chain_off[c+1]) back to back;
    // with chain_counter set, nchains persistent waves take list entries [0, chain_list) from it
    const int32_t *chain_pairs, *chain_off;
    int nchains;
    uint32_t *chain_counter;
    uint32_t chain_base;  // the counter's value when this run starts (it is never reset between runs)
    int chain_list;
};

// len = false (distance only, SED_NO_LEN): keys without the op-count field, out len = -1.
hipError_t sed_launch_i32(const sed_launch &L, const sed_i32_params &prm, bool len);
// CHAIN mode (single-stripe pairs, R in {4, 8, 16}): one wave per chain of pairs.
hipError_t sed_launch_i32_chain(const sed_launch &L, const sed_i32_params &prm, bool len);
hipError_t sed_launch_f64(const sed_launch &L, const double *gtab, const sed_f64_params &prm, bool typed);
// fp64 wave kernel in 16-lane segments, four pairs per wave (pairs idx[0 .. nidx), pd.pad[1] = 1; the SW = 64 kernel and
// traceback skip them), and their per-cell-code traceback
hipError_t sed_launch_f64_seg(const sed_launch &L, const double *gtab, const sed_f64_params &prm, bool typed,
                              const int32_t *idx, int nidx);
hipError_t sed_launch_traceback_seg(const sed_launch &L, uint32_t *ops, const int32_t *idx, int nidx);
hipError_t sed_launch_f64_full(const sed_launch &L, const double *gtab, const sed_f64_params &prm, bool typed,
                               const sed_full_out &fo);
// Lane-per-pair integer kernel (sed_lane.hip): pairs idx[0..nidx) with 1 <= m <= SED_LANE_MAXM.
// len = false: distance only, no op-count field (3 VALU per cell).
#define SED_LANE_MAXM 32
#define SED_LANE_MAXN 512
hipError_t sed_launch_lane_i32(const sed_launch &L, const int32_t *idx, int nidx, const sed_i32_params &prm, bool len);
// distance only, two pairs of equal shape per wave (packed 16-bit cells); list holds 2 * nwaves pair indices
hipError_t sed_launch_i32x2(const sed_launch &L, const int32_t *list, int nwaves, const sed_i32_params &prm);
// distance only, two pairs of equal n per lane (packed 16-bit cells); idx holds 2 * nlanes pair indices
hipError_t sed_launch_lane_i32x2(const sed_launch &L, const int32_t *idx, int nlanes, const sed_i32_params &prm);
// distance only under unit costs, one pair per lane, bit-parallel (str2 as the bit dimension, m <= 32)
hipError_t sed_launch_lane_bitpar(const sed_launch &L, const int32_t *idx, int nidx);
// fp64 distance-only lane kernel (SED_MODE_F64 with SED_NO_LEN): gtab = the {value, flag} table.  Pairs with
// pd.pad[0] = 1 (every symbol in the unit-cost code set umask, at most 4 codes) run bit-parallel.
hipError_t sed_launch_lane_f64(const sed_launch &L, const int32_t *idx, int nidx, const double *gtab, double ins,
                               double del, int K, uint32_t umask);
// Scaled-integer lane kernel for fp64 distance-only batches whose costs are dyadic over at most 8 symbols (costs.json
// with N: multiples of 1/4): every cost times S = 2^shift is an integer, and the reference's fp64 sums of such values
// are exact, so an integer DP of the scaled costs gives D * S exactly (sed_lane.hip: sed_lane_scaled_kernel).
// row[a] = the 8 bytes (cost(a -> b) * S - ins - del - 1) & 0xFF for b = 0..7 (b = 0..3 in row[a][0]); ins / del
// scaled; pairs with pd.pad[0] run bit-parallel as in sed_lane_f64_kernel (umap: the 2-bit unit-subset code of every
// code < 8 at bits 2c).  Byte-coded sequences start 16-byte aligned (fill_batch).
struct sed_scaled_params {
    uint32_t row[8][2];
    uint32_t ins, del;
    double inv_scale;  // 2^-shift
    uint32_t umask, umap;
};
hipError_t sed_launch_lane_scaled(const sed_launch &L, const int32_t *idx, int nidx, const sed_scaled_params &sp);
hipError_t sed_launch_traceback(const sed_launch &L, uint32_t *ops);
// stripe-parallel traceback of few long pairs (per-cell codes): map[pd.map_off ...] per pair, ops zeroed first
hipError_t sed_launch_traceback_stripes(const sed_launch &L, uint32_t *ops, uint32_t *map, int items, int kmax);
// Checkpoint layout of the CK forward kernels (R = 4, 8 or 16 rows per lane, G = 64/R steps per group):
//   column checkpoints, per stripe [nchunks][R + 1][64 lanes]: each lane's R row values and its top_prev
//   at every 64-step chunk end;
//   then row checkpoints, per stripe [SG/G groups][64/G lanes t = G-1 (mod G)][G steps]: the bottom row of
//   every G-th lane at every step (the row above each 64-row traceback tile).
__host__ __device__ inline uint64_t sed_ck_col_word(int R, int stripe, int nchunks, int c, int r, int t) {
    return (((uint64_t)stripe * (uint64_t)nchunks + (uint64_t)c) * (uint64_t)(R + 1) + (uint64_t)r) * 64u +
           (uint64_t)t;
}
__host__ __device__ inline uint64_t sed_ck_col_words(int R, int nstripes, int nchunks) {
    return (uint64_t)nstripes * (uint64_t)nchunks * (uint64_t)(R + 1) * 64u;
}
// Row checkpoints: every step, the bottom row of the forward lanes t = GH-1 (mod GH), GH = SED_CK_TILE / R, i.e.
// of every SED_CK_TILE-th matrix row (the traceback's tile height, 64).  Per stripe and G-step group (G = 64/R):
// SED_CK_RW = 64 * 64 / SED_CK_TILE words, [group][t / GH][step % G].  SED_CK_TILE = 32 (twice the row checkpoints)
// served a two-pairs-per-wave traceback of 32-row tiles, measured and dropped in round 3: the forward kernel took
// 9.87 instead of 9.18-9.32 ms and that traceback 2.43 instead of 2.20 ms (profiles/r03/ab_tb_tiles.jsonl).
#ifndef SED_CK_HALVES_DEFAULT
#define SED_CK_HALVES_DEFAULT 2  // checkpoint batches: parts on as many streams, >= 1024 wave pairs each (sed_runtime.cpp)
#endif
#ifndef SED_CK_TILE
#define SED_CK_TILE 64
#endif
#define SED_CK_RW (64 * 64 / SED_CK_TILE)
// row checkpoint of forward lane t (t = GH-1 mod GH) at step s of stripe k
__host__ __device__ inline uint64_t sed_ck_row_word(int R, int k, int ngroups, int s, int t) {
    const int G = 64 / R, GH = SED_CK_TILE / R;
    return ((uint64_t)k * (uint64_t)ngroups + (uint64_t)(s / G)) * (uint64_t)SED_CK_RW + (uint64_t)(t / GH) * (uint64_t)G +
           (uint64_t)(s % G);
}
// CK batches (L.ck): the traceback that recomputes tiles from the forward kernel's checkpoints
hipError_t sed_launch_traceback_ck(const sed_launch &L, uint32_t *ops, const sed_i32_params &prm);
// SPLIT batches with checkpoints: every tile's op codes from the checkpoints, into the per-cell code layout (one wave
// per tile of each pair: grid max_tiles x npairs)
hipError_t sed_launch_ck_codes(const sed_launch &L, int max_tiles, const sed_i32_params &prm);
hipError_t sed_launch_selftest(uint32_t *d_out, hipStream_t stream);

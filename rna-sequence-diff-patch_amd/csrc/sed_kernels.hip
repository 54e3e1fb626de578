// sed_kernels.hip — gfx950 (MI355X / CDNA4) kernels for the weighted
// Wagner–Fischer DP and its canonical traceback.
//
// Reference semantics (plsakr/rna-sequence-diff-patch, StringEditDistance.py):
//   border cells :146-182, recurrence min_cost :92-128 (candidates insert,
//   delete, update; one fp64 add each; first minimal value), canonical path =
//   create_paths(dp)[0] :228-271 (shortest co-optimal path, ties
//   insert < delete < update read from the sink), script ops :274-334.
//
// Work decomposition: one wave64 per sequence pair.  A pair's
// rows are cut into stripes of 64*R rows; lane t of the wave owns R
// consecutive rows and sweeps the columns one step behind lane t-1
// (a systolic anti-diagonal wavefront).  Per step a lane receives the cell
// above its band from lane t-1 through a DPP wave_shr:1 move, so there is no
// barrier in the inner loop.  Lane 0 takes its "above" value (the stripe's top
// row) and every lane its str2 selector from small per-wave LDS rings, read as
// broadcasts; lane 63's bottom row is collected by DPP wave_shl:1 and stored as
// the next stripe's top row (per 64-step chunk in one wave, per 16-step group
// through tagged words between SPLIT workgroups, below).
//
// Integer kernels (the exact fast path).  When every cost is
// an integral positive Python float (or the int 0 of a match), the reference's
// fp64 values are exact integers and the per-cell decision
//    (distance, path length, op)   lexicographically minimal
// is one unsigned v_min3_u32 over packed keys.  Three key formats, all kept in
// an offset space where the insert candidate needs no add and every border is a
// constant (details at "Integer (packed-key) kernels" below):
//  - ladder keys V = D << 16 + L << 3 + op (per-cell traceback codes): v_perm,
//    v_add, v_min3, v_and_or (clears the op), v_alignbit (packs the 2-bit op)
//    = 5 VALU per cell, plus a delete add on 3 of 16 rows;
//  - distance keys D << 16 - U (U = updates on the path, so at a fixed cell the
//    low half orders by the path length L = i + j - U): v_perm, v_add, v_min3
//    = 3 VALU.  Distance-only batches and the checkpoint forward kernel (CK),
//    whose traceback recomputes tiles in traceback keys (D << 16 | L << 2 | op
//    in offset space) converted from them;
//  - 16-bit packed distance keys, two pairs per word (distance only).
//
// fp64 kernel (the general path): fp64 candidates added exactly as the
// reference does, equality ties, L tie-break on an integer key, and an
// optional int/float typing bit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>
#include <hip/hip_ext.h>
#include "sed_internal.h"

#define DPP_WAVE_SHL1 0x130  // lane i <- lane i+1, lane 63 keeps `old`
#define DPP_WAVE_ROL1 0x134  // lane i <- lane i+1, lane 63 <- lane 0
#define DPP_WAVE_SHR1 0x138  // lane i <- lane i-1, lane 0 keeps `old`

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, DPP_WAVE_SHR1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, DPP_WAVE_SHL1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_rol1(uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)src, (int)src, DPP_WAVE_ROL1, 0xf, 0xf, false);
}
// lane i <- lane i-1's src + addv, lane 0 keeps `old`: one v_add_u32_dpp (the s_nop covers the DPP read of
// a VGPR written by the previous VALU instruction)
__device__ __forceinline__ uint32_t dpp_shr1_add(uint32_t old, uint32_t src, uint32_t addv) {
    asm("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(old) : "v"(src), "v"(addv));
    return old;
}
__device__ __forceinline__ double dpp_shr1_f64(double old, double src) {
    const uint64_t o = __double_as_longlong(old), s = __double_as_longlong(src);
    const uint32_t lo = dpp_shr1((uint32_t)o, (uint32_t)s);
    const uint32_t hi = dpp_shr1((uint32_t)(o >> 32), (uint32_t)(s >> 32));
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double dpp_shl1_f64(double old, double src) {
    const uint64_t o = __double_as_longlong(old), s = __double_as_longlong(src);
    const uint32_t lo = dpp_shl1((uint32_t)o, (uint32_t)s);
    const uint32_t hi = dpp_shl1((uint32_t)(o >> 32), (uint32_t)(s >> 32));
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double dpp_rol1_f64(double src) {
    const uint64_t s = __double_as_longlong(src);
    const uint32_t lo = dpp_rol1((uint32_t)s), hi = dpp_rol1((uint32_t)(s >> 32));
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// The same moves inside segments of SW lanes (SW = 64: the whole wave; SW = 16: each DPP row, so a wave runs four
// independent segments, the fp64 kernel's short pairs): shr = lane i <- lane i-1 (the segment's lane 0 keeps `old`,
// row_shr:1), shl = lane i <- lane i+1 (the segment's last lane keeps `old`, row_shl:1), rol = lane i <- lane i+1
// mod SW (row_ror:15).
#define DPP_ROW_SHL1 0x101
#define DPP_ROW_SHR1 0x111
#define DPP_ROW_ROR15 0x12F
template <int SW> __device__ __forceinline__ uint32_t seg_shr1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, SW == 64 ? DPP_WAVE_SHR1 : DPP_ROW_SHR1, 0xf, 0xf,
                                                 false);
}
template <int SW> __device__ __forceinline__ uint32_t seg_shl1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, SW == 64 ? DPP_WAVE_SHL1 : DPP_ROW_SHL1, 0xf, 0xf,
                                                 false);
}
template <int SW> __device__ __forceinline__ uint32_t seg_rol1(uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)src, (int)src, SW == 64 ? DPP_WAVE_ROL1 : DPP_ROW_ROR15, 0xf, 0xf,
                                                 false);
}
template <int SW> __device__ __forceinline__ double seg_shr1_f64(double old, double src) {
    const uint64_t o = __double_as_longlong(old), s = __double_as_longlong(src);
    const uint32_t lo = seg_shr1<SW>((uint32_t)o, (uint32_t)s), hi = seg_shr1<SW>((uint32_t)(o >> 32), (uint32_t)(s >> 32));
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
template <int SW> __device__ __forceinline__ double seg_shl1_f64(double old, double src) {
    const uint64_t o = __double_as_longlong(old), s = __double_as_longlong(src);
    const uint32_t lo = seg_shl1<SW>((uint32_t)o, (uint32_t)s), hi = seg_shl1<SW>((uint32_t)(o >> 32), (uint32_t)(s >> 32));
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}
template <int SW> __device__ __forceinline__ double seg_rol1_f64(double src) {
    const uint64_t s = __double_as_longlong(src);
    const uint32_t lo = seg_rol1<SW>((uint32_t)s), hi = seg_rol1<SW>((uint32_t)(s >> 32));
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) { return min(min(a, b), c); }
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) { return max(max(a, b), c); }
// the dot keys' update candidate: diag + dot4(row vector, column vector) over signed bytes (v_dot4_i32_i8)
// (the VOP3P form with its own destination: the builtin picks v_dot4c_i32_i8, which accumulates in place and made
// the register allocator copy every diagonal first, 186 instead of 111 v_mov per 256 cells).  The hardware needs
// wait states between a v_dot4 and a VALU op reading its result, which the compiler cannot see through the asm
// (tools/ubench/dot_sem.hip: the next op reads a stale value), so the asm is volatile (issued in program order)
// and the caller keeps every consumer 4 dots behind its producer (dot_fence).
__device__ __forceinline__ uint32_t dot_add(uint32_t rowv, uint32_t colv, uint32_t diag) {
    uint32_t r;
    asm volatile("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r) : "v"(rowv), "v"(colv), "v"(diag));
    return r;
}
// dots issued ahead of the max / min chain (>= 4: tools/ubench/dot_sem.hip shows the next op reading stale data;
// the fence then leaves 3 or more instructions between a dot and its reader).  A/B on config 4's forward kernel
// (tools/ab.sh, profiles/r02_dot/ab_ahead.jsonl): 4 -> 9.24-9.33 ms, 6 same, 8 -> 9.16-9.23 ms, 12 9.29, 16 9.18.
#ifndef SED_DOT_AHEAD
#define SED_DOT_AHEAD 8
#endif
// an empty volatile asm on a dot result, placed after the dots that must separate it from its consumer: the
// consumer cannot be scheduled above it.  (The compiler treats the asm as a write of x and puts an s_nop 0 between
// it and the max reading x, 50 per 64-cell group.  Fencing one row earlier drops that to 29 but lets the compiler
// pair up dependent maxes back to back: config 4's forward 9.19 -> 9.49 ms, so the fence stays next to its max.)
__device__ __forceinline__ void dot_fence(uint32_t &x) { asm volatile("" : "+v"(x)); }
// An opaque v_min3_u32: over three selects (tie keys of the fp64 kernel) the compiler rewrites
// min(min(a, b), c) into select-of-min chains that cost one op more per cell.
__device__ __forceinline__ uint32_t umin3_op(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// relaxed agent-scope load = global_load sc1: bypasses this CU's L1 so a
// stripe reads the bottom row its own wave stored during the previous stripe.
__device__ __forceinline__ uint32_t load_sc1(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_sc1_u64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Traceback codes are stored per "group" of G = 64/R steps: G steps x R rows x 2 bits
// = 16 bytes per lane, one dwordx4 store; the wave writes 1 KiB contiguous.
template <int R> struct Grp { static constexpr int G = 64 / R; };

__device__ __forceinline__ void store_tb(uint32_t *p, const uint32_t (&w)[4]) {
    *reinterpret_cast<uint4 *>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
// G (a multiple of 4) consecutive words, 16-byte aligned
template <int G> __device__ __forceinline__ void store_words(uint32_t *p, const uint32_t (&w)[G]) {
#pragma unroll
    for (int k = 0; k < G; k += 4) *reinterpret_cast<uint4 *>(p + k) = make_uint4(w[k], w[k + 1], w[k + 2], w[k + 3]);
}

// ---------------------------------------------------------------------------
// Integer (packed-key) kernels.  The reference's decision per cell is the
// lexicographic minimum of (distance, path length, op) over its candidates, i.e.
// one unsigned min over the keys
//     V = D << 16 + L << 3 + op        (op 0 insert, 1 delete, 2 update)
// with candidates V_left + Ki, V_up + Kd + 1, V_diag + (cost << 16) + 10, where
// Ki = (insert << 16) + 8 and Kd = (delete << 16) + 8.  The L field may run past
// its 13 bits: the three candidates of cell (i, j) have L in [max(i,j), i+j],
// so 8 * |L difference| <= 8 * min(n, m) < 2^16 and any distance difference
// still dominates (the host keeps min(n, m) < 8192); at the sink L is read
// modulo 8192 inside that window.
//
// Offset keys.  Subtracting the same amount from the three candidates of a cell
// keeps their order, so cells are stored as
//     W(i, j) = V(i, j) - i*Kd - j*Ki + B + c(i)        (B = SED_KB3)
// where i*Kd + j*Ki bounds V from above (the all-delete-then-insert path) and
// the host checks that it stays below B, so W never wraps.  c(i) in 0..5 is a
// per-row residue ("ladder") that steps down by one from row to row and jumps
// back up on a few rows (Ladder<R> below, periodic in i with a period dividing
// R, so every lane row has a compile-time rung).  With d = c(i) - c(i-1):
//     insert candidate = W_left,
//     delete candidate = W_up + (d + 1)          (no add on the d = -1 rows),
//     update candidate = W_diag + ((cost - delete - insert) << 16) - 6 + d.
// The update constant is one v_perm_b32 of a per-row byte vector (cost - delete
// - insert - 1; the bytes below it 0xFF / (d - 6) from the inline constant d - 6;
// the host requires cost <= insert + delete).  mm = min3 is a clean value (low 3
// bits = c(i)) plus the winning op, which never leaves the 8-block because
// c(i) + 2 <= 7, so clearing the op is one v_and_or: (mm & ~7) | c(i).  A cell
// therefore costs v_perm, v_add, v_min3, v_and_or, v_alignbit = 5 VALU, plus the
// delete add on 3 of 16 rows.  The traceback codes are mm's low 2 bits
// (c(i) + op) & 3; the traceback kernels subtract the rung of the row they are on.
// Every border is a constant: W(0, j) = B, W(i, 0) = B + c(i).
//
// Distance keys (!LEN): V = D << 16 - U without an op field, W = V -
// i*(delete << 16) - j*(insert << 16) + SED_KB, update constant ((cost - delete -
// insert) << 16) - 1: an update also subtracts 1 from the low half, which never
// borrows (fewer than 2^16 updates on any path), so D = (V + 0xFFFF) >> 16 and
// U = (D << 16) - V.  At equal D the smaller key has more updates, i.e. the
// shorter path (L = i + j - U), so the min is the (D, L) minimum; only the op
// tie-break is missing, which the CK traceback recomputes.  That is v_perm,
// v_add, v_min3 = 3 VALU per cell; every border is SED_KB.
// Lanes run unmasked all the time, and a lane past column m computes columns
// that nothing reads.
// ---------------------------------------------------------------------------
#define SED_KB3 0xFFFFFE00u  // bias of the ladder keys (= 0 mod 8, 512 below 2^32 for the ramp sentinel)

// The ladder: rung c(i) of row i by i mod P, 4 bits per rung; runs of 5,4,3,2,1,0 as long as the
// period allows (P = 16: jumps at i = 1, 7, 11 (mod 16); P = 8: at 1, 7; P = 4: at 1).
template <int R> struct Ladder {
    static constexpr int P = R >= 16 ? 16 : R;
    static constexpr uint64_t pat = P == 16 ? 0x1234501230123450ull : (P == 8 ? 0x10123450ull : 0x1230ull);
    static constexpr int rung(int i) { return (int)((pat >> (4 * (i & (P - 1)))) & 0xF); }
};
// The wide ladder of the ladder dot keys (LDOT = 2, the CHAIN kernel): rung + op in the low 4 bits (V = D*A + 16L + op,
// the host keeps 16 min(n, m) + 15 < A and A a multiple of 16), rungs up to 13, so the rung runs down through a whole period
// with one jump (P = 8: rows 1..7 on rungs 7..1; P = 16: 13..0 and two jumps): 1 jump row in 8 instead of 2, each a
// delete add and an update add fewer.  Same P, so the tracebacks read it through their runtime pattern alone.
template <int R> struct LadderW {
    static constexpr int P = R >= 16 ? 16 : R;
    static constexpr uint64_t pat = P == 16 ? 0x10123456789ABCD0ull : (P == 8 ? 0x12345670ull : 0x1230ull);
    static constexpr int rung(int i) { return (int)((pat >> (4 * (i & (P - 1)))) & 0xF); }
};

// One column step of a lane's R rows.  tv = {top, sel} of this step's column
// for lane 0 (the stripe's top row and str2 symbol): every lane reads the same
// LDS word, only lane 0 keeps it (the DPP move's `old` operand).  Lane rows are
// i = (multiple of P) + r + 1, so row r sits on rung Ladder::rung(r + 1).
// SELL: the lane's own selector arrives in tv.y (read from the wave's LDS selector ring, see
// sed_wf_i32_kernel), instead of flowing from lane 0 through a DPP move (one DPP + one copy per step).
// TOPC: lane 0's top is the row-0 constant, which its top_prev already holds (single-stripe pairs: the CHAIN
// kernel), so the DPP move writes over top_prev in place instead of over a copy of tv.x.
template <int R, bool TB, bool LEN, bool COLLECT = true, bool SELL = false, bool TOPC = false, bool DOT = false,
          int LDOT = 0>
__device__ __forceinline__ void i32_step(uint32_t (&V)[R], const uint32_t (&cv)[R], uint32_t &top_prev,
                                         uint32_t &bottom, uint32_t &selv, const uint2 tv, uint32_t &outc,
                                         uint32_t (&W)[4], const int u, const uint32_t jv = 0u) {
    using Lad = Ladder<R>;
    if constexpr (SELL) selv = tv.y;
    else selv = dpp_shr1(tv.y, selv);  // perm selector of this column's str2 symbol
    constexpr int d0 = Lad::rung(1) - Lad::rung(0);
    // row 0's update candidate from top_prev, before the DPP move overwrites top_prev in place (TOPC): the
    // empty asm makes the move's `old` depend on it, so top_prev needs no copy
    if constexpr (LEN && LDOT) {
        // ladder keys with the update addend as one v_dot4 (ladder dot keys, sed_runtime.cpp): the addend of a row
        // whose rung steps down by one (d = -1) is -(A*kappa + 7) over the 3-bit ladder (LDOT = 1: V = D*A + 8L) or
        // -(A*kappa + 15) over the wide one (LDOT = 2: V = D*A + 16L, LadderW) = the dot of the row's and the column's
        // byte vectors (column vectors negated by the host); a row with another step adds d + 1 to it, which is where
        // the perm took its inline constant d - 6.  Candidates run 4 rows ahead of the min chain (dot_add).  Per cell:
        // v_dot4, v_min3, v_and_or, v_alignbit = 4 VALU (5 with the perm), plus two adds on a jump row.
        using Lad = std::conditional_t<LDOT == 2, LadderW<R>, Ladder<R>>;
        constexpr uint32_t LOW = LDOT == 2 ? 15u : 7u;  // the rung + op field
        // the wide ladder's jump is row 0 of every lane (i = 1 mod P): its delete and update inputs, the cell above
        // the band and the diagonal, both take d + 1 = J0, which the DPP move from lane t - 1 adds itself (one
        // v_add_u32_dpp with jv = J0 instead of v_mov_b32_dpp), so top_prev carries it too (i32_reset: tpb)
        constexpr bool BIAS = LDOT == 2;
        constexpr uint32_t J0 = (uint32_t)(Lad::rung(1) - Lad::rung(0) + 1);
        constexpr int AH = R < 4 ? R : 4;
        uint32_t cand[R];
        cand[0] = dot_add(cv[0], selv, top_prev);
#pragma unroll
        for (int r = 1; r < AH; ++r) cand[r] = dot_add(cv[r], selv, V[r - 1]);
        const uint32_t topv = BIAS ? dpp_shr1_add(TOPC ? top_prev : tv.x + J0, bottom, jv)
                                   : dpp_shr1(TOPC ? top_prev : tv.x, bottom);
        uint32_t up = topv;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r + AH < R) cand[r + AH] = dot_add(cv[r + AH], selv, V[r + AH - 1]);
            dot_fence(cand[r]);
            const int c = Lad::rung(r + 1), d = c - Lad::rung(r);  // compile-time after unrolling
            const bool plain = d == -1 || (BIAS && r == 0);          // (BIAS: row 0's inputs carry d + 1)
            const uint32_t upd = plain ? cand[r] : cand[r] + (uint32_t)(d + 1);
            const uint32_t mm = umin3(V[r], plain ? up : up + (uint32_t)(d + 1), upd);
            if constexpr (TB) {
                const int k = u * R + r;
                W[k >> 4] = __builtin_amdgcn_alignbit(mm, W[k >> 4], 2);
            }
            up = (mm & ~LOW) | (uint32_t)c;
            V[r] = up;
        }
        top_prev = topv;
        bottom = V[R - 1];
        if constexpr (COLLECT) outc = dpp_shl1(bottom, outc);
        return;
    }
    if constexpr (DOT) {  // dot keys: maximise, the update addend is one v_dot4 of signed bytes
        // candidates run 4 rows ahead of the max chain (the dot's result hazard, dot_add): row r + 4's diagonal is
        // still the old value of row r + 3 when row r is updated
        constexpr int AH = R < SED_DOT_AHEAD ? R : SED_DOT_AHEAD;
        uint32_t cand[R];
        cand[0] = dot_add(cv[0], selv, top_prev);
#pragma unroll
        for (int r = 1; r < AH; ++r) cand[r] = dot_add(cv[r], selv, V[r - 1]);
        const uint32_t topv = dpp_shr1(TOPC ? top_prev : tv.x, bottom);
        uint32_t up = topv;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r + AH < R) cand[r + AH] = dot_add(cv[r + AH], selv, V[r + AH - 1]);
            dot_fence(cand[r]);  // row r's candidate was issued AH dots ago
            up = umax3(V[r], up, cand[r]);
            V[r] = up;
        }
        top_prev = topv;
        bottom = V[R - 1];
        if constexpr (COLLECT) outc = dpp_shl1(bottom, outc);
        return;
    }
    uint32_t dg0 = top_prev + __builtin_amdgcn_perm(cv[0], LEN ? (uint32_t)(d0 - 6) : 0xFFFFFFFFu, selv);
    if constexpr (TOPC) asm("" : "+v"(top_prev) : "v"(dg0));
    const uint32_t topv = dpp_shr1(TOPC ? top_prev : tv.x, bottom);  // cell above the band, this column
    uint32_t up = topv, diag = top_prev;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t left = V[r];
        uint32_t mm;
        if constexpr (LEN) {
            const int c = Lad::rung(r + 1), d = c - Lad::rung(r);  // compile-time after unrolling
            // insert (op 0) = left, delete (op 1) = up + d + 1, update (op 2) = diag + offset constant
            // (perm bytes 1:0 from the inline constant d - 6)
            mm = umin3(left, d == -1 ? up : up + (uint32_t)(d + 1),
                       r == 0 ? dg0 : diag + __builtin_amdgcn_perm(cv[r], (uint32_t)(d - 6), selv));
            if constexpr (TB) {
                const int k = u * R + r;
                W[k >> 4] = __builtin_amdgcn_alignbit(mm, W[k >> 4], 2);
            }
            up = (mm & ~7u) | (uint32_t)c;
        } else {
            mm = umin3(left, up, r == 0 ? dg0 : diag + __builtin_amdgcn_perm(cv[r], 0xFFFFFFFFu, selv));
            up = mm;
        }
        diag = left;
        V[r] = up;
    }
    top_prev = topv;
    bottom = V[R - 1];
    if constexpr (COLLECT) outc = dpp_shl1(bottom, outc);  // lane 63's bottom row (CK: the row checkpoints)
}

// Column-0 state of rows row0+1 .. row0+R (row0 = multiple of P) and of row0, the diagonal of the
// first column.
template <int R, bool LEN, bool DOT = false, bool WIDE = false>
__device__ __forceinline__ void i32_reset(uint32_t (&V)[R], uint32_t &top_prev) {
    // (WIDE: top_prev carries row 0's jump, i32_step LDOT = 2)
    top_prev = LEN ? SED_KB3 + (WIDE ? (uint32_t)(LadderW<R>::rung(1) - LadderW<R>::rung(0) + 1) : 0u)
                   : DOT ? SED_KB_DOT : SED_KB;
#pragma unroll
    for (int r = 0; r < R; ++r)
        V[r] = LEN ? SED_KB3 + (uint32_t)(WIDE ? LadderW<R>::rung(r + 1) : Ladder<R>::rung(r + 1)) : DOT ? SED_KB_DOT : SED_KB;
}
// row 0 (D = j*insert, L = j) in offset keys
template <bool LEN, bool DOT = false> __device__ __forceinline__ uint32_t i32_row0() {
    return LEN ? SED_KB3 : DOT ? SED_KB_DOT : SED_KB;
}

// The sink cell (n, m) back to V space; returns {D, L} (without LEN, L = n + m - U when WANT_L, else -1).
// Dot key k = A*X + U -> {X, U}: X = floor(k*kmax / (A*kmax + 1)) by a multiply-shift (the host checks k*kmax
// < 2^29 and picks dotM, dotS so the product is exact), U = k - A*X.
__device__ __forceinline__ uint2 dot_split(uint32_t w, const sed_i32_params &prm) {
    const uint32_t k = w - SED_KB_DOT;
    const uint32_t X = __umulhi(k, prm.dotM) >> (prm.dotS - 32u);  // dotM carries kmax (one v_mul_hi, full-rate rest)
    return make_uint2(X, k - __umul24(prm.dotA, X));
}
template <int R, bool LEN, bool WANT_L = false, bool DOT = false, int LDOT = 0>
__device__ __forceinline__ int2 i32_decode(uint32_t w, int n, int m, const sed_i32_params &prm) {
    if constexpr (LEN && LDOT) {  // V = D*A + uL: one division per pair
        // u = 8: the host keeps 8 (n + m) + 7 < A; u = 16 (the wide ladder): 16 min(n, m) + 15 < A, and L is read inside
        // its window [max(n, m), n + m] (the candidates of a cell differ in L by at most min(n, m), so that bound keeps
        // their order)
        constexpr uint32_t U = LDOT == 2 ? 16u : 8u;
        const uint32_t rg = (uint32_t)(LDOT == 2 ? LadderW<R>::rung(n) : Ladder<R>::rung(n));
        const uint32_t v = w - SED_KB3 - rg + (uint32_t)n * (prm.del * prm.ladA + U) + (uint32_t)m * (prm.ins * prm.ladA + U);
        const uint32_t lo = LDOT == 2 ? U * (uint32_t)max(n, m) : 0u;
        const uint32_t D = (v - lo) / prm.ladA;
        return make_int2((int)D, (int)((v - D * prm.ladA) / U));
    } else if constexpr (DOT) {  // D = n*delete + m*insert - X, L = n + m - U
        const uint2 xu = dot_split(w, prm);
        return make_int2((int)((uint32_t)n * prm.del + (uint32_t)m * prm.ins - xu.x), n + m - (int)xu.y);
    } else if constexpr (LEN) {
        const uint32_t v = w - SED_KB3 - (uint32_t)Ladder<R>::rung(n) + (uint32_t)n * ((prm.del << 16) + 8u) +
                           (uint32_t)m * ((prm.ins << 16) + 8u);
        const uint32_t lo = (uint32_t)max(n, m);
        const uint32_t L = lo + ((((v >> 3) & 0x1FFFu) - lo) & 0x1FFFu);  // L in [max(n,m), n+m]
        return make_int2((int)((v - 8u * L) >> 16), (int)L);
    } else {
        const uint32_t v = w - SED_KB + (((uint32_t)n * prm.del + (uint32_t)m * prm.ins) << 16);
        const uint32_t D = (v + 0xFFFFu) >> 16;
        return make_int2((int)D, WANT_L ? n + m - (int)((D << 16) - v) : -1);
    }
}

// Distance key (!LEN) of a cell -> the traceback key of the same (D, L) (clean, op 0).  Traceback keys
// (sed_traceback_ck_kernel) are T = V - i*((delete << 16) + 4) - j*((insert << 16) + 4) + SED_KB over
// V = D << 16 | L << 2 | op: the insert candidate is the left cell, the delete candidate the cell above
// + 1, the update candidate the diagonal + ((cost - delete - insert) << 16) - 2, and the winner's low 2
// bits are the op itself.  With U = (SED_KB - w) & 0xFFFF (updates on the path) both keys share
// (D - i*delete - j*insert) << 16, and T = w - 3U; independent of the cell's position.
__device__ __forceinline__ uint32_t i32_dist_to_tb(uint32_t w) {
    const uint32_t U = (SED_KB - w) & 0xFFFFu;
    return w - 3u * U;
}
// either forward key format -> traceback key: T = SED_KB - (X << 16) - 4U (X = i*delete + j*insert - D)
__device__ __forceinline__ uint32_t ck_to_tb(uint32_t w, const sed_i32_params &prm) {
    if (prm.dot) {  // = SED_KB - 4k + 4A X - (X << 16)
        const uint32_t k = w - SED_KB_DOT;
        const uint32_t X = __umulhi(k, prm.dotM) >> (prm.dotS - 32u);
        return SED_KB - 4u * k + __umul24(4u * prm.dotA, X) - (X << 16);
    }
    return i32_dist_to_tb(w);
}

// Ramp for free.  Every lane starts a stripe at its column-0 state and lane t begins real work
// at step t.  Before that it runs "virtual" columns, which leave its state unchanged: their str2
// selector is a sentinel, so with every neighbour at its column-0 value the insert candidate
// (the border itself) is the minimum and keeps the border:
//   ladder keys: insert B + c(i), delete B + c(i) + 1, update B + c(i-1) + 255 (SED_SEL_SENT3:
//   update constant 0xFF >= any jump d);
//   distance keys (and the 16-bit packed ones): insert = delete = border, update border + 0.
// The lane's first real column then sees exactly D[row][0], D[row-1][0] and the cell above.
#define SED_SEL_SENT 0x0C0C0C0Cu
#define SED_SEL_SENT3 0x0C0C0C0Du
template <bool LEN, bool DOT = false> __device__ __forceinline__ uint32_t i32_sent() {
    return LEN ? SED_SEL_SENT3 : DOT ? 0u : SED_SEL_SENT;  // dot keys: the zero column vector adds 0
}
// perm selector of str2 symbol b: byte3 <- 0xFF, byte2 <- cost byte b, bytes 1:0 <- the constant
__device__ __forceinline__ uint32_t i32_sel(uint32_t b) { return 0x0D000100u | ((4u + b) << 16); }

template <bool B> struct BoolTag { static constexpr bool value = B; };

// CAP: the group that produces the sink cell (captured on its lane); every extra variant is
// another merge point where the register allocator may insert copies of the whole state.
// The stripe kernel's group: lane 0's top values from the chunk's LDS slots (ltop, broadcast reads),
// each lane's str2 selectors from the wave's LDS selector ring at its own column (lsel: this group's
// first step for this lane, doubled ring so the G reads never wrap).
// PF (SED_CK_TVPF, the CK forward's unrolled chunk loop): the group's first {top, selector} pair arrives in tvpf, read
// at the previous group's start, and this group reads the next group's first pair with its own, so its first step's
// dots start without waiting on an LDS round trip (the last group of a chunk reads one entry past it, unused).
template <int R, bool TB, bool LEN, bool CAP, bool CK = false, bool DOT = false, bool COLLECT = !CK, bool PF = false>
__device__ __forceinline__ void i32_group(uint32_t (&V)[R], const uint32_t (&cv)[R], uint32_t &top_prev,
                                          uint32_t &bottom, uint32_t &selv, const uint32_t *__restrict__ ltop,
                                          const uint32_t *__restrict__ lsel, uint32_t &outc, uint32_t (&W)[4],
                                          const int s0, const int lane, const int cap_step, const int cap_lane,
                                          const int cap_row, uint32_t &cap, uint32_t (&rcv)[Grp<R>::G],
                                          uint2 *tvpf = nullptr) {
    constexpr int G = Grp<R>::G;
    uint2 tv[G];
    const uint32_t *lp = ltop + (s0 & 63);  // G divides 64: a group never wraps the chunk
    if constexpr (PF) {
        tv[0] = *tvpf;
#pragma unroll
        for (int u = 1; u < G; ++u) tv[u] = make_uint2(lp[u], lsel[u]);
        *tvpf = make_uint2(lp[G], lsel[G]);
    } else {
#pragma unroll
        for (int u = 0; u < G; ++u) tv[u] = make_uint2(lp[u], lsel[u]);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
        const int s = s0 + u;
        i32_step<R, TB, LEN, COLLECT, true, false, DOT>(V, cv, top_prev, bottom, selv, tv[u], outc, W, u);
        if constexpr (CK) rcv[u] = V[R - 1];  // the band's bottom row, step s (row checkpoints)
        if constexpr (CAP) {
            const bool hit = (s == cap_step) && (lane == cap_lane);
#pragma unroll
            for (int r = 0; r < R; ++r) cap = (hit && r == cap_row) ? V[r] : cap;
        }
    }
}

// Minimum waves per SIMD the register allocator must leave room for, per R: the budget at which
// the hot loop does not spill (R=16: 96 VGPRs / 5 waves; the 80-VGPR budget of 6 waves spills the
// cost rows and ran 2.5x slower; R=4/8: 72 / 7; R=32: 128 / 4, which still spills: never chosen).
template <int R> struct I32Waves { static constexpr int value = R >= 32 ? 4 : (R == 16 ? 5 : 7); };
#ifndef SED_SPLIT_BWORDS
#define SED_SPLIT_BWORDS 1024  // SPLIT: str2 words staged in LDS (m <= 16384)
#endif
#ifndef SED_CK_WAVES
#define SED_CK_WAVES 5
#endif
#ifndef SED_CK_GUNROLL
#define SED_CK_GUNROLL 2  // groups per iteration of the CK chunk loop
#endif
#ifndef SED_CK_TVPF
#define SED_CK_TVPF 0  // CK forward: each group's first LDS pair read a group ahead (i32_group PF; A/B)
#endif
#ifdef SED_I32_WAVES_PER_EU
#define SED_I32_WAVES(R) SED_I32_WAVES_PER_EU
#else
#define SED_I32_WAVES(R) I32Waves<R>::value
#endif
// Inter-workgroup hand-off of stripe bottom rows (SPLIT mode), per 16-step group and self-validating: every
// bottom-row cell travels as one 64-bit word {tag, value}, stored with a relaxed agent-scope 64-bit atomic
// (single-copy atomic, so a reader sees the tag and the value of one store together), tag = the run's epoch
// (1..32767, prm.epoch) | poison << 31.  The consumer's feeder wave (split_feed) polls the words and re-polls any
// whose tag is not this run's.  No counter, fence or s_waitcnt on the producer side:
// with the per-chunk counter hand-off (stores, s_waitcnt, release fence, counter; the consumer prefetching a
// chunk ahead) each stripe ran 3 chunks (192 steps) behind the one above.
// The previous run's words carry another epoch; the host zeroes the buffer on a batch's first run and when the
// epoch wraps.  A stripe that gave up waiting publishes with the poison bit, so its consumer stops waiting too,
// and the last stripe reports err.
#define SED_PROG_POISON 0x80000000u
__device__ __forceinline__ void store_tagged(uint64_t *p, uint32_t tag, uint32_t v) {
    __hip_atomic_store(p, ((uint64_t)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SPLIT: the ring of lane 0's top values (one per step) and the hand-off feeder.  Each stripe below the first runs
// as two waves: the compute wave, which never waits on a global load (any such wait with its own stores in flight is
// an s_waitcnt vmcnt(0): the compiler counts mixed reads and writes as out of order, and the store round trip then
// sat in every group), and this feeder.  The feeder polls the stripe above's tagged words 64 columns at a time (sc1,
// past its L1), moves the longest valid prefix into the LDS ring and publishes how many steps are ready (flag[0]);
// the compute wave publishes how many it has consumed (flag[1]), which bounds how far the feeder may run ahead.
// A poisoned word upstream, or no progress for ~2^22 polls, poisons flag[0] (bit 31) with every step ready, so the
// compute wave never waits again and the last stripe reports err.
#define SED_SPLIT_RING 256
// the flags are relaxed workgroup-scope atomics: a volatile LDS access is followed by s_waitcnt vmcnt(0) lgkmcnt(0)
__device__ __forceinline__ uint32_t lds_flag_get(uint32_t *f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_set(uint32_t *f, uint32_t v) {
    __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <int G>
__device__ __forceinline__ void split_feed(const uint64_t *__restrict__ bin64, const int m, const int SG,
                                           const uint32_t epoch, uint32_t *ring, uint32_t *flag,
                                           const int lane) {
    uint32_t poison = 0, idle = 0;
    int have = 0;  // steps whose top values are in the ring
    while (have < SG) {
        if (have + 64 > (int)lds_flag_get(flag + 1) + SED_SPLIT_RING) {  // ring full: the compute wave is behind
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        const int t = have + lane, col = t + 1;
        const bool need = t < SG && col <= m;  // columns past m are never stored nor waited for
        const uint64_t w = need ? load_sc1_u64(bin64 + (uint32_t)(col + 64)) : 0ull;
        const bool good = !need || (((uint32_t)(w >> 32) & ~SED_PROG_POISON) == epoch);
        const uint64_t bad = __ballot(!good);
        const int nv = min(bad ? (int)__builtin_ctzll(bad) : 64, SG - have);  // the valid prefix
        if (__any(lane < nv && need && (w >> 63))) poison = SED_PROG_POISON;  // poisoned upstream
        if (nv > 0) {
            if (lane < nv) ring[t & (SED_SPLIT_RING - 1)] = (uint32_t)w;
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the values before the count
            have += nv;
            idle = 0;
        } else if (++idle > (1u << 22)) {  // the stripe above stopped: give up, let the compute wave drain
            poison = SED_PROG_POISON;
            have = SG;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0 && (nv > 0 || poison)) lds_flag_set(flag, (uint32_t)have | poison);
    }
}

// SPLIT = false: one wave per pair walks all of its stripes (batches).
// SPLIT = true : one 128-thread workgroup per stripe (the compute wave and its
//                feeder, split_feed), all stripes of a pair run concurrently,
//                each a few groups behind the stripe above it (single long
//                pairs: config 2, the GUI; hand-off above).
// CK (not SPLIT): instead of per-cell codes, tb receives checkpoints for the recompute traceback
// (sed_traceback_ck_kernel; layout in sed_internal.h): per stripe, at every chunk end each lane's R row values
// and its top_prev ("column checkpoints", [chunk][R+1][64 lanes]), and every step the bottom row of the lanes
// t = G-1 (mod G) ("row checkpoints", [group][64/G][G steps]) -- ~0.13 B per cell instead of 0.25.  The CK
// kernel runs distance keys (LEN = false, 3 VALU per cell instead of the ladder keys' 5.19): they carry
// (D, L), which is all the checkpoints need; the traceback recomputes the op tie-break.
// The CK kernel (distance keys, no codes) would fit 80 VGPRs (6 waves per SIMD, spills per chunk only) but
// ran slower: 12.45 against 12.11 ms at 5 waves (profiles/r02/ab_ck_waves.txt).
// issue priority of SPLIT's stripe waves (SED_SPLIT_PRIO): a single pair's stripe chain is latency-bound, and the
// previous run's traceback kernels may share its SIMDs.  Config 2 at 100 steps: 0.2974-0.3008 against 0.2984-0.3039
// ms per step at 0, 3 interleaved rounds (profiles/r05/s17)
#ifndef SED_SPLIT_PRIO
#define SED_SPLIT_PRIO 2
#endif
template <int R, bool TB, bool SPLIT, bool LEN = true, bool CK = false, bool DOT = false>
__global__ __launch_bounds__(SPLIT ? 128 : 256) __attribute__((amdgpu_waves_per_eu(CK ? SED_CK_WAVES : SED_I32_WAVES(R))))
void sed_wf_i32_kernel(const sed_pair_desc *__restrict__ pd, int npairs, const int2 *__restrict__ tasks,
                  const uint32_t *__restrict__ seqa, const uint32_t *__restrict__ seqb,
                  uint32_t *__restrict__ tb, uint32_t *__restrict__ bnd, sed_result *__restrict__ res,
                  sed_i32_params prm) {
    constexpr int ROWS = 64 * R;
    constexpr int G = Grp<R>::G;
    static_assert(!CK || (R <= 16 && !TB && !LEN), "checkpoints: R <= 16, distance keys");
    static_assert(!(CK && SPLIT) || R == 4, "SPLIT checkpoints (sed_ck_codes_kernel): R = 4");
    static_assert(!DOT || CK, "dot keys: checkpoint batches only");
    if constexpr (SPLIT && SED_SPLIT_PRIO > 0) __builtin_amdgcn_s_setprio(SED_SPLIT_PRIO);
    const int lane = threadIdx.x & 63;
    int pair, kfirst = 0;
    if constexpr (SPLIT) {
        const int2 t = tasks[blockIdx.x];
        pair = __builtin_amdgcn_readfirstlane(t.x);
        kfirst = __builtin_amdgcn_readfirstlane(t.y);
    } else {
        pair = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
        if (pair >= npairs) return;
    }
    const sed_pair_desc d = pd[pair];
    if (d.lane) return;  // short str2: sed_lane.hip
    const int n = d.n, m = d.m;
    if (n == 0 || m == 0) {
        if (lane == 0) {
            const uint32_t D = (n == 0) ? (uint32_t)m * prm.ins : (uint32_t)n * prm.del;
            res[pair].dist = (double)D;
            res[pair].len = n + m;
            res[pair].is_int = (D == 0);
            res[pair].err = 0;
        }
        return;
    }
    const int nstripes = (n + ROWS - 1) / ROWS;
    const int klast = SPLIT ? kfirst : nstripes - 1;
    const int SG = (m + 63 + G - 1) / G * G;  // steps per stripe, rounded to whole groups
    const int nchunks = (SG + 63) >> 6;
    const uint32_t bstride = (uint32_t)(nchunks + 2) * 64u;  // bottom-row buffer of one stripe (SPLIT: 64-bit words)
    const uint32_t *pa = seqa + d.a_off;
    const uint32_t *pb = seqb + d.b_off;
    // the sink cell (n, m): last stripe, lane (n-1)%ROWS / R, row (n-1)%R, computed at step m-1+lane
    const int wsink = (n - 1) % ROWS;
    const int cap_lane = wsink / R, cap_row = wsink % R;
    uint32_t cap = 0;
    bool ok = true;
    // per wave: lane 0's top values of the current 64-step chunk, and a ring of str2 selectors by column
    // (column ci at slots ci & 127 and (ci & 127) + 128; the 64 columns before 0 hold the virtual-column
    // sentinel), from which lane t reads column s - t at step s
    __shared__ uint32_t lds_top[SPLIT ? SED_SPLIT_RING / 64 : 4][64];
    __shared__ uint32_t lds_sel[SPLIT ? 1 : 4][256];
    __shared__ uint32_t split_flag[2];
    uint32_t *lch = lds_top[SPLIT ? 0 : (threadIdx.x >> 6)];  // SPLIT: the whole array is the feeder's ring
    uint32_t *ring = lds_sel[SPLIT ? 0 : (threadIdx.x >> 6)];
    // SPLIT: str2's packed words in LDS (m <= 16 * SED_SPLIT_BWORDS), so the chunk loop issues no global load of its
    // own: a wait for one with the group's stores in flight is a vmcnt(0), i.e. a store round trip per chunk.  (The
    // same per wave in the one-wave-per-pair kernels made the checkpoint kernel spill.)
    constexpr int BW = SPLIT ? SED_SPLIT_BWORDS : 1;
    __shared__ uint32_t lds_b[BW];
    const int bwords = (m + 15) >> 4;
    const bool bl = SPLIT && bwords <= BW;  // (uniform)
    if (bl && threadIdx.x < 64) {
        for (int x = lane; x < bwords; x += 64) lds_b[x] = pb[x];
    }
    if constexpr (SPLIT) {
        if (threadIdx.x < 2) split_flag[threadIdx.x] = 0u;
        __syncthreads();
    }

    for (int k = kfirst; k <= klast; ++k) {
        // in-place single buffer per pair when one wave does all stripes; one buffer per stripe otherwise
        const uint32_t *bnd_in = bnd + d.bnd_off;
        uint32_t *bnd_out = bnd + d.bnd_off;
        const uint64_t *bin64 = reinterpret_cast<const uint64_t *>(bnd + d.bnd_off) + (uint32_t)(k - 1) * bstride;
        uint64_t *bout64 = reinterpret_cast<uint64_t *>(bnd + d.bnd_off) + (uint32_t)k * bstride;
        if constexpr (SPLIT) {
            if (threadIdx.x >= 64) {  // the feeder wave
                if (k > 0) split_feed<G>(bin64, m, SG, prm.epoch, lch, split_flag, lane);
                return;
            }
        }
        const int row0 = k * ROWS + lane * R;  // 0-based str1 index of this lane's first row
        uint32_t cv[R], V[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ri = row0 + r;
            const uint32_t a = (pa[ri >> 4] >> ((ri & 15) * 2)) & 3u;
            if constexpr (DOT) cv[r] = a == 0 ? prm.dotrow[0] : a == 1 ? prm.dotrow[1] : a == 2 ? prm.dotrow[2] : prm.dotrow[3];
            else cv[r] = a == 0 ? prm.costrow[0] : a == 1 ? prm.costrow[1] : a == 2 ? prm.costrow[2] : prm.costrow[3];
        }
        uint32_t top_prev;
        i32_reset<R, LEN, DOT>(V, top_prev);
        // column-0 state for every lane; virtual columns until the lane's first real one (see above)
        uint32_t bottom = V[R - 1], selv = i32_sent<LEN, DOT>(), outc = 0;
        uint32_t W[4] = {0, 0, 0, 0};

        // CK: the previous stripe's lane 63 stored its bottom row contiguously by step into the pair's
        // bottom-row buffer (column j at step j + 62, in place: this stripe writes step s while it reads
        // steps >= s + 64; past SG the columns are beyond m and never read)
        auto load_top = [&](int c) -> uint32_t {
            const int j = 64 * c + lane + 1;
            if (k == 0) return i32_row0<LEN, DOT>();
            if constexpr (CK) return load_sc1(bnd + d.bnd_off + (uint32_t)(j + 62));
            return load_sc1(bnd_in + j + 64);
        };
        auto load_sel = [&](int c) -> uint32_t {
            const int ci = 64 * c + lane;
            const uint32_t wb = bl ? lds_b[min(ci >> 4, bwords - 1)] : pb[ci >> 4];  // (past m: never read)
            const uint32_t b = (wb >> ((ci & 15) * 2)) & 3u;
            if constexpr (DOT) return b == 0 ? prm.dotcol[0] : b == 1 ? prm.dotcol[1] : b == 2 ? prm.dotcol[2] : prm.dotcol[3];
            return i32_sel(b);
        };
        uint32_t tch = (SPLIT && k > 0) ? 0u : load_top(0), sch = load_sel(0);
        if constexpr (SPLIT) {  // stripe 0's constant row in the whole ring; the feeder fills the others'
            if (k == 0) {
#pragma unroll
                for (int x = 0; x < SED_SPLIT_RING; x += 64) lch[x + lane] = tch;
            }
        } else {
            lch[lane] = tch;
        }
        ring[lane] = ring[lane + 128] = sch;
        ring[lane + 64] = ring[lane + 192] = i32_sent<LEN, DOT>();
        uint32_t *tbk = tb + d.tb_off + (uint64_t)k * (uint64_t)(SG / G) * 256u;
        // CK: column checkpoints of stripe k at ccb[(chunk * (R+1) + v) * 64 + lane], row checkpoints at
        // rcb[group * 64 + (lane / G) * G + step % G] (sed_ck_*_word, the layout sed_traceback_ck_kernel reads)
        // (SPLIT: the checkpoints follow the pair's per-cell code region, which sed_ck_codes_kernel fills from them)
        const uint64_t ckoff = (SPLIT && CK) ? (uint64_t)nstripes * (uint64_t)(SG / G) * 256u : 0u;
        uint32_t *ccb = tb + d.tb_off + ckoff + sed_ck_col_word(R, k, nchunks, 0, 0, 0);
        uint32_t *rcb = tb + d.tb_off + ckoff + sed_ck_col_words(R, nstripes, nchunks) + (uint64_t)k * (uint64_t)(SG / G) * SED_CK_RW;
        uint32_t rcv[G];
        const bool last = (k == nstripes - 1);
        const int cap_step = last ? m - 1 + cap_lane : -1;
        // CK: a chunk is 64/G groups (unrolled by 2) and always whole: the last chunk's steps past SG compute
        // columns beyond m that nothing reads, and only their stores are skipped.  The chunk holding the sink
        // runs the rolled loop below, so the others have no merge point: a CAP/plain choice per group made the
        // register allocator move the whole row state every group (3.30 -> 3.11 VALU per cell).  The per-cell-code
        // kernels keep the rolled loop for every chunk: split the same way, their hot loop spills.  (Fully
        // unrolled chunks take the compiler > 15 min.)
        const int c_cap = last ? cap_step >> 6 : -1;
        int s = 0;
        int ready = 0;  // SPLIT: steps the feeder has published as ready (last read)
        // CK (not SPLIT): the chunks before the sink's run the unrolled group loop, the sink's chunk and any after it the
        // rolled one, as two loops: one loop choosing per chunk merged the paths, and the register allocator moved the
        // row state in and out of the unrolled loop's registers every chunk (24 VALU per 2112)
        auto chunk = [&](auto fast_tag, const int c) {
            constexpr bool FASTC = decltype(fast_tag)::value;
            uint32_t tnx = 0, snx = 0;
            if (c + 1 < nchunks) {
                if (!SPLIT) tnx = load_top(c + 1);
                snx = load_sel(c + 1);
            }
            const uint32_t *lsel = ring + ((64 * c - lane) & 127);  // this lane's column at the chunk's first step
            auto stores = [&](const int s0) {
                if constexpr (TB) {
                    uint32_t *gp = tbk + (uint64_t)(s0 / G) * 256u;  // wave-uniform base, per-lane 16-byte offset
                    store_tb(gp + lane * 4, W);
                }
                if constexpr (CK) {
                    constexpr int GH = SED_CK_TILE / R;  // forward lanes per traceback tile
                    if ((lane & (GH - 1)) == GH - 1)
                        store_words<G>(rcb + (uint64_t)(s0 / G) * SED_CK_RW + (uint32_t)(lane / GH) * G, rcv);
                    if (!SPLIT && lane == 63 && !last) store_words<G>(bnd + d.bnd_off + (uint32_t)s0, rcv);  // next stripe's top row
                }
            };
            if constexpr (FASTC) {
                uint2 tvpf = make_uint2(lch[0], lsel[0]);  // (SED_CK_TVPF: the first group's first pair)
#pragma unroll SED_CK_GUNROLL
                for (int g = 0; g < 64 / G; ++g) {
                    const int s0 = 64 * c + g * G;  // (s0 & 63 folds to g * G)
                    i32_group<R, TB, LEN, false, CK, DOT, !CK, (bool)SED_CK_TVPF>(V, cv, top_prev, bottom, selv, lch,
                                                     lsel + g * G, outc, W, s0, lane, cap_step, cap_lane, cap_row, cap,
                                                     rcv, &tvpf);
                    if (s0 < SG) stores(s0);
                }
                s = 64 * (c + 1);  // lane 63's bottom cells of the whole chunk are in outc (!CK)
            } else {
                for (int g = 0; g < 64 / G && s < SG; ++g, s += G, lsel += G) {
                    const uint32_t *ltop = lch;
                    if constexpr (SPLIT) {
                        ltop = lch + (s & (SED_SPLIT_RING - 64));
                        // the feeder has this group's top values in the ring (LDS only: no vmcnt).  The ready count
                        // is re-read only when the groups it covered are used up (the feeder publishes up to 64 steps
                        // at a time), so most groups start without an LDS round trip.
                        if (k > 0 && ready < s + G) {
                            uint32_t f = lds_flag_get(split_flag), spins = 0;
                            while (ok && (int)(f & ~SED_PROG_POISON) < s + G) {
                                if (++spins > (1u << 24)) ok = false;
                                __builtin_amdgcn_s_sleep(1);
                                f = lds_flag_get(split_flag);
                            }
                            if (f & SED_PROG_POISON) ok = false;
                            ready = (int)(f & ~SED_PROG_POISON);
                            asm volatile("" ::: "memory");
                        }
                    }
                    const bool capg = cap_step >= s && cap_step < s + G;
                    if (capg)
                        i32_group<R, TB, LEN, true, CK, DOT, !CK || SPLIT>(V, cv, top_prev, bottom, selv, ltop, lsel, outc, W,
                                                                          s, lane, cap_step, cap_lane, cap_row, cap, rcv);
                    else
                        i32_group<R, TB, LEN, false, CK, DOT, !CK || SPLIT>(V, cv, top_prev, bottom, selv, ltop, lsel, outc, W,
                                                                           s, lane, cap_step, cap_lane, cap_row, cap, rcv);
                    stores(s);
                    if constexpr (SPLIT) {
                        // lanes 64-G+u hold lane 63's bottom cell of step s+u, column s+u-62 (word col + 64)
                        if (!last && lane >= 64 - G)
                            store_tagged(bout64 + (uint32_t)(s + lane - (64 - G) - 62 + 64),
                                         prm.epoch | (ok ? 0u : SED_PROG_POISON), outc);
                        if (k > 0) {  // this group's ring slots are free again
                            asm volatile("" ::: "memory");
                            if (lane == 0) lds_flag_set(split_flag + 1, (uint32_t)(s + G));
                        }
                    }
                }
            }
            if constexpr (CK) {  // column checkpoint: state after the chunk's last step
                uint32_t *cp = ccb + (uint64_t)c * (uint64_t)(R + 1) * 64u + lane;
#pragma unroll
                for (int r = 0; r < R; ++r) cp[r * 64] = V[r];
                cp[R * 64] = top_prev;
            }
            // lane i holds lane 63's bottom cell of step s-64+i, i.e. column s-126+i at bnd index col+64
            if (!CK && !SPLIT && !last) bnd_out[s - 62 + lane] = outc;
            tch = tnx;
            sch = snx;
            if (!SPLIT) lch[lane] = tch;  // after the chunk's last LDS read (in order)
            const uint32_t slot = (uint32_t)(64 * (c + 1) + lane) & 127u;  // replaces column 64(c-1) + lane
            ring[slot] = ring[slot + 128] = sch;
        };
        int cfast = 0;
        if constexpr (CK && !SPLIT) {
            cfast = c_cap >= 0 ? c_cap : nchunks;
            for (int c = 0; c < cfast; ++c) chunk(BoolTag<true>{}, c);
        }
        for (int c = cfast; c < nchunks; ++c) chunk(BoolTag<false>{}, c);
        if (!last) __builtin_amdgcn_s_waitcnt(0);  // own bottom-row stores done before the next stripe reads them
    }
    if (klast == nstripes - 1 && lane == cap_lane) {
        const int2 dl = i32_decode<R, LEN, CK, DOT>(cap, n, m, prm);
        res[pair].dist = (double)dl.x;
        res[pair].len = dl.y;
        res[pair].is_int = (dl.x == 0);
        res[pair].err = ok ? 0 : SED_ERR_SPLIT_TIMEOUT;  // SPLIT: a timed-out wait anywhere up the stripe chain poisons the pair
    }
}

// ---------------------------------------------------------------------------
// Distance only, two pairs per wave (SED_NO_LEN batches, pairs of equal n): pair P in the low
// 16 bits of every cell word, pair Q in the high 16 bits.  Each half is a 16-bit offset key
// W = D - i*delete - j*insert + 0xFFFF (the host checks i*delete + j*insert <= 0xFFFF over the
// computed block, so no half wraps), with insert candidate W_left, delete candidate W_up and
// update candidate W_diag + (cost - delete - insert), a 16-bit constant 0xFFxx since the host
// packs only when every substitution is cheaper than delete + insert.  Packed 16-bit ops do two
// cells at once: perm + v_pk_add_u16 + 2 v_pk_min_u16 = 4 VALU / 2 cells.  The rest is the stripe
// kernel's schedule (virtual-column ramp, lane-0 LDS chunk, in-place bottom rows in P's buffer,
// which the host makes the pair with the larger m); both pairs have the same n, so they share
// stripes and rows, and the wave runs max(m) columns, the shorter pair's extra columns being
// don't-care.  Each pair's sink is captured at its own step.
// ---------------------------------------------------------------------------
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
// 16-bit offset key of the sink back to D: D = W - 0xFFFF + n*delete + m*insert (mod 2^16)
__device__ __forceinline__ uint32_t x2_decode(uint32_t half, int n, int m, const sed_i32_params &prm) {
    return (half + 1u + (uint32_t)n * prm.del + (uint32_t)m * prm.ins) & 0xFFFFu;
}

template <int R, bool CAP>
__device__ __forceinline__ void x2_group(uint32_t (&V)[R], const uint32_t (&cP)[R], const uint32_t (&cQ)[R],
                                         uint32_t &top_prev, uint32_t &bottom, uint32_t &selv,
                                         const uint2 *__restrict__ lch, uint32_t &outc, const int s0, const int lane,
                                         const int capP_step, const int capQ_step, const int cap_lane,
                                         const int cap_row, uint32_t &capP, uint32_t &capQ) {
    constexpr int G = Grp<R>::G;
    uint2 tv[G];
    const uint2 *lp = lch + (s0 & 63);
#pragma unroll
    for (int u = 0; u < G; ++u) tv[u] = lp[u];
#pragma unroll
    for (int u = 0; u < G; ++u) {
        const int s = s0 + u;
        const uint32_t topv = dpp_shr1(tv[u].x, bottom);
        selv = dpp_shr1(tv[u].y, selv);
        uint32_t up = topv, diag = top_prev;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t left = V[r];
            // the row above (up) enters last: one dependent op per row on the column's chain
            const uint32_t mm = pk_min(pk_min(left, pk_add(diag, __builtin_amdgcn_perm(cQ[r], cP[r], selv))), up);
            diag = left;
            up = mm;
            V[r] = mm;
        }
        top_prev = topv;
        bottom = V[R - 1];
        outc = dpp_shl1(bottom, outc);
        if constexpr (CAP) {
            const bool hP = (s == capP_step) && (lane == cap_lane), hQ = (s == capQ_step) && (lane == cap_lane);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                capP = (hP && r == cap_row) ? V[r] : capP;
                capQ = (hQ && r == cap_row) ? V[r] : capQ;
            }
        }
    }
}

// occupancy targets with room for both pairs' cost rows (2R) next to the packed row values (R)
template <int R> struct X2Waves { static constexpr int value = R >= 32 ? 3 : (R == 16 ? 5 : (R == 8 ? 7 : 8)); };
template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(X2Waves<R>::value))) void
sed_wf_i32x2_kernel(const sed_pair_desc *__restrict__ pd, const int32_t *__restrict__ list, int nwaves,
                    const uint32_t *__restrict__ seqa, const uint32_t *__restrict__ seqb,
                    uint32_t *__restrict__ bnd, sed_result *__restrict__ res, sed_i32_params prm) {
    constexpr int ROWS = 64 * R;
    constexpr int G = Grp<R>::G;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (w >= nwaves) return;
    const int P = __builtin_amdgcn_readfirstlane(list[2 * w]), Q = __builtin_amdgcn_readfirstlane(list[2 * w + 1]);
    const sed_pair_desc dP = pd[P], dQ = pd[Q];
    const int n = dP.n, m = dP.m, mQ = dQ.m;  // host: dQ.n == n, 1 <= mQ <= m
    const int nstripes = (n + ROWS - 1) / ROWS;
    const int SG = (m + 63 + G - 1) / G * G;
    const int nchunks = (SG + 63) >> 6;
    const uint32_t *paP = seqa + dP.a_off, *paQ = seqa + dQ.a_off;
    const uint32_t *pbP = seqb + dP.b_off, *pbQ = seqb + dQ.b_off;
    const int wsink = (n - 1) % ROWS;
    const int cap_lane = wsink / R, cap_row = wsink % R;
    uint32_t capP = 0, capQ = 0;
    __shared__ uint2 lds_chunk[4][64];
    uint2 *lch = lds_chunk[threadIdx.x >> 6];
    uint32_t *bnd_io = bnd + dP.bnd_off;  // in place, as in the stripe kernel

    for (int k = 0; k < nstripes; ++k) {
        const int row0 = k * ROWS + lane * R;
        uint32_t cP[R], cQ[R], V[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ri = row0 + r;
            const uint32_t aP = (paP[ri >> 4] >> ((ri & 15) * 2)) & 3u, aQ = (paQ[ri >> 4] >> ((ri & 15) * 2)) & 3u;
            cP[r] = aP == 0 ? prm.costrow16[0] : aP == 1 ? prm.costrow16[1] : aP == 2 ? prm.costrow16[2] : prm.costrow16[3];
            cQ[r] = aQ == 0 ? prm.costrow16[0] : aQ == 1 ? prm.costrow16[1] : aQ == 2 ? prm.costrow16[2] : prm.costrow16[3];
        }
        uint32_t top_prev = 0xFFFFFFFFu;  // column 0 and row 0 are the offset key 0xFFFF in both halves
#pragma unroll
        for (int r = 0; r < R; ++r) V[r] = 0xFFFFFFFFu;
        uint32_t bottom = V[R - 1], selv = SED_SEL_SENT, outc = 0;
        auto load_top = [&](int c) -> uint32_t {
            const int j = 64 * c + lane + 1;
            if (k == 0) return 0xFFFFFFFFu;
            return load_sc1(bnd_io + j + 64);
        };
        auto load_sel = [&](int c) -> uint32_t {
            const int ci = 64 * c + lane;
            const uint32_t bp = (pbP[ci >> 4] >> ((ci & 15) * 2)) & 3u;
            const uint32_t bq = ci < mQ ? (pbQ[ci >> 4] >> ((ci & 15) * 2)) & 3u : 0u;  // Q may be far shorter
            return 0x0D000D00u | bp | ((4u + bq) << 16);  // byte0 <- cP byte bP, byte2 <- cQ byte bQ, 1 and 3 <- 0xFF
        };
        uint32_t tch = load_top(0), sch = load_sel(0);
        lch[lane] = make_uint2(tch, sch);
        const bool last = (k == nstripes - 1);
        const int capP_step = last ? m - 1 + cap_lane : -1, capQ_step = last ? mQ - 1 + cap_lane : -1;
        int s = 0;
        for (int c = 0; c < nchunks; ++c) {
            uint32_t tnx = 0, snx = 0;
            if (c + 1 < nchunks) { tnx = load_top(c + 1); snx = load_sel(c + 1); }
            for (int g = 0; g < 64 / G && s < SG; ++g, s += G) {
                const bool capg = (capP_step >= s && capP_step < s + G) || (capQ_step >= s && capQ_step < s + G);
                if (capg)
                    x2_group<R, true>(V, cP, cQ, top_prev, bottom, selv, lch, outc, s, lane, capP_step, capQ_step,
                                      cap_lane, cap_row, capP, capQ);
                else
                    x2_group<R, false>(V, cP, cQ, top_prev, bottom, selv, lch, outc, s, lane, capP_step, capQ_step,
                                       cap_lane, cap_row, capP, capQ);
            }
            if (!last) bnd_io[s - 62 + lane] = outc;
            lch[lane] = make_uint2(tnx, snx);
        }
        if (!last) __builtin_amdgcn_s_waitcnt(0);
    }
    if (lane == cap_lane) {
        sed_result r;
        r.len = -1;
        r.err = 0;
        r.seq = 0;
        const uint32_t DP = x2_decode(capP & 0xFFFFu, n, m, prm), DQ = x2_decode(capQ >> 16, n, mQ, prm);
        r.dist = (double)DP;
        r.is_int = (DP == 0);
        res[P] = r;
        r.dist = (double)DQ;
        r.is_int = (DQ == 0);
        res[Q] = r;
    }
}

// ---------------------------------------------------------------------------
// CHAIN mode (integer keys, single-stripe pairs: n <= 64R).  One wave runs a chain of pairs
// back to back so that a pair's 63-step wavefront ramp overlaps the previous pair's drain.
// Pair q of the chain owns global steps [T_q, T_q + S_q) for lane 0, S_q = m_q rounded up to
// 64 (whole LDS chunks); lane t runs it at [T_q + t, T_q + S_q + t).  Lane t therefore
// switches pairs right after global step T_q + t - 1: its V / cost rows / diagonal are set
// to the new pair's column-0 state with per-lane selects (rows are the same for every pair
// of the chain: row0 = 64R * 0 + t*R, so the column-0 borders are per-lane constants).
// The cell above a lane's band keeps arriving by DPP from lane t-1, which switched one step
// earlier, and the str2 selectors flow from lane 0 as in the stripe kernel.  The first pair
// starts with the virtual-column ramp.  Per-pair traceback layout, results and captures are
// exactly the stripe kernel's (one stripe), so the traceback kernel is shared.
// ---------------------------------------------------------------------------
struct chain_pair_state {
    int pair, n, m, T, S, end;         // end: first global step after its last real column (T + m + 63)
    int cap_step, cap_lane, cap_row;   // the sink cell (n, m)
    uint64_t tb_off;
    int sg;                            // traceback groups allocated per stripe
    int nchunks;                       // CK: 64-step chunks of the pair's stripe (column checkpoints)
    const uint32_t *pb;                // str2 codes
};

template <int R>
__device__ __forceinline__ chain_pair_state chain_load(const sed_pair_desc *__restrict__ pd,
                                                       const uint32_t *__restrict__ seqb, int pair, int T) {
    constexpr int G = Grp<R>::G;
    const sed_pair_desc d = pd[pair];
    chain_pair_state c;
    c.pair = pair;
    c.n = d.n;
    c.m = d.m;
    c.T = T;
    c.S = (d.m + 63) & ~63;
    c.end = T + d.m + 63;
    const int wsink = d.n - 1;
    c.cap_lane = wsink / R;
    c.cap_row = wsink % R;
    c.cap_step = T + d.m - 1 + c.cap_lane;
    c.tb_off = d.tb_off;
    c.sg = (d.m + 63 + G - 1) / G;
    c.nchunks = (c.sg * G + 63) >> 6;
    c.pb = seqb + d.b_off;
    return c;
}

// One group of G steps.  SW: lanes switch from the previous pair to the pair starting at
// `Tcur` after the step at which lane == s + 1 - Tcur.  GEN (rare groups: sink captures of the
// previous (A) and current (B) pair, and any switch in those groups) additionally captures.
// Lane 0's top value is row 0 (single-stripe pairs); every lane reads its str2 selector from the wave's
// selector ring by global column s - t (lsel: this lane's column at the group's first step), which always
// belongs to the pair the lane is working on: lane t is on the pair starting at T exactly when s - t >= T.
template <int R, bool TB, bool LEN, bool SW, bool GEN, bool CK, int LDOT = 0>
__device__ __forceinline__ void i32_chain_group(uint32_t (&V)[R], uint32_t (&cv)[R], const uint32_t (&cvn)[R],
                                                const uint32_t (&Vb)[R], const uint32_t tpb, uint32_t &top_prev,
                                                uint32_t &bottom, uint32_t &selv, const uint32_t *__restrict__ lsel,
                                                uint32_t &outc, uint32_t (&W)[4], const int s0, const int lane,
                                                const int Tcur, const int csA, const int clA, const int crA,
                                                uint32_t &capA, const int csB, const int clB, const int crB,
                                                uint32_t &capB, uint32_t (&rcv)[Grp<R>::G], const uint32_t jv) {
    constexpr int G = Grp<R>::G;
    uint2 tv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) tv[u] = make_uint2(i32_row0<LEN>(), lsel[u]);
#pragma unroll
    for (int u = 0; u < G; ++u) {
        const int s = s0 + u;
        i32_step<R, TB, LEN, false, true, true, false, LDOT>(V, cv, top_prev, bottom, selv, tv[u], outc, W, u, jv);
        if constexpr (CK) rcv[u] = V[R - 1];  // the band's bottom row (row checkpoints), before any switch
        if constexpr (GEN) {
            const bool hA = (s == csA) && (lane == clA), hB = (s == csB) && (lane == clB);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                capA = (hA && r == crA) ? V[r] : capA;
                capB = (hB && r == crB) ? V[r] : capB;
            }
        }
        if constexpr (SW || GEN) {
            const bool sw = (lane == s + 1 - Tcur);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                V[r] = sw ? Vb[r] : V[r];
                cv[r] = sw ? cvn[r] : cv[r];
            }
            top_prev = sw ? tpb : top_prev;
        }
    }
}

template <int R, bool TB, bool LEN, bool CK, int LDOT = 0>
__device__ __forceinline__ void chain_store_result(sed_result *__restrict__ res, int pair, uint32_t cap, int n,
                                                   int m, int seq, const sed_i32_params &prm) {
    const int2 dl = i32_decode<R, LEN, CK, false, LDOT>(cap, n, m, prm);
    res[pair].dist = (double)dl.x;
    res[pair].len = dl.y;
    res[pair].is_int = (dl.x == 0);
    res[pair].err = 0;
    res[pair].seq = (uint16_t)min(seq, 65535);  // the pair's ordinal in its wave (dynamic-CHAIN diagnostics)
}

// the chain kernel also holds the next pair's cost rows and the column-0 constants
#ifndef SED_CHAIN_WAVES
#define SED_CHAIN_WAVES 5
#endif
template <int R> struct ChainWaves { static constexpr int value = R >= 16 ? 4 : SED_CHAIN_WAVES; };

// CK: distance keys, and checkpoints instead of codes (the stripe kernel's layout, one stripe per pair).  At every
// chunk end all lanes are on the pair lane 0 is on (a lane switches at most 63 steps after lane 0), so the column
// checkpoints go to that pair; a row-checkpoint group of a switch window goes to both pairs, like the codes.
template <int R, bool TB, bool LEN, bool CK = false, int LDOT = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ChainWaves<R>::value))) void
sed_wf_i32_chain_kernel(const sed_pair_desc *__restrict__ pd, const int32_t *__restrict__ chain_pairs,
                        const int32_t *__restrict__ chain_off, int nchains, uint32_t *__restrict__ counter,
                        uint32_t cbase, int nlist, const uint32_t *__restrict__ seqa, const uint32_t *__restrict__ seqb,
                        uint32_t *__restrict__ tb, sed_result *__restrict__ res, sed_i32_params prm) {
    constexpr int G = Grp<R>::G;
    static_assert(!CK || (!TB && !LEN), "checkpoints: distance keys, no codes");
    const int lane = threadIdx.x & 63;
    const int chain = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (chain >= nchains) return;
    // Static chains: list entries [chain_off[c], chain_off[c+1]).  Dynamic (counter != null):
    // persistent waves take the next list entry from a device counter whenever lane 0 reaches
    // the end of a pair, so every wave stays busy until the list is exhausted.  A run takes exactly
    // nlist + nchains values (every wave ends with one failed grab), so the counter is never reset:
    // this run's values start at cbase (no fill kernel per run).
    auto grab = [&]() -> int {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(counter, 1u) - cbase;
        return (int)__builtin_amdgcn_readfirstlane(v);
    };
    int c0, c1;
    if (counter) {
        c0 = grab();
        c1 = nlist;
        if (c0 >= nlist) return;
    } else {
        c0 = chain_off[chain];
        c1 = chain_off[chain + 1];
    }
    // per wave: str2 selectors by global column (column g at slots g & 127 and (g & 127) + 128; the 64 columns
    // before the chain's first pair hold the virtual-column sentinel)
    __shared__ uint32_t lds_sel[4][256];
    uint32_t *ring = lds_sel[threadIdx.x >> 6];
    const int row0 = lane * R;

    // per-lane constants: column-0 state of this lane's rows (the same for every pair)
    uint32_t Vb[R], tpb;
    i32_reset<R, LEN, false, LDOT == 2>(Vb, tpb);
    uint32_t jv = (uint32_t)(LadderW<R>::rung(1) - LadderW<R>::rung(0) + 1);  // (LDOT = 2: the DPP move's add, a VGPR)
    asm volatile("" : "+v"(jv));
    auto rows_of = [&](int pair, uint32_t (&out)[R]) {
        const uint32_t *pa = seqa + pd[pair].a_off;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ri = row0 + r;
            const uint32_t a = (pa[ri >> 4] >> ((ri & 15) * 2)) & 3u;
            if constexpr (LDOT) out[r] = a == 0 ? prm.ladrow[0] : a == 1 ? prm.ladrow[1] : a == 2 ? prm.ladrow[2] : prm.ladrow[3];
            else out[r] = a == 0 ? prm.costrow[0] : a == 1 ? prm.costrow[1] : a == 2 ? prm.costrow[2] : prm.costrow[3];
        }
    };
    auto chunk_of = [&](const chain_pair_state &c, int cl) -> uint2 {  // lane 0's inputs, local chunk cl
        const int j = 64 * cl + lane;
        const uint32_t b = (c.pb[j >> 4] >> ((j & 15) * 2)) & 3u;
        if constexpr (LDOT)
            return make_uint2(i32_row0<LEN>(), b == 0 ? prm.ladcol[0] : b == 1 ? prm.ladcol[1] : b == 2 ? prm.ladcol[2] : prm.ladcol[3]);
        return make_uint2(i32_row0<LEN>(), i32_sel(b));  // row 0, str2 selector
    };
    // ladder dot keys: the host's column vector {s, 0, 0, 0} adds s*x in [8, 490] (above any jump, and the border
    // SED_KB3 + c(i) plus it stays below 2^32)
    const uint32_t sent = LDOT ? prm.ladsent : i32_sent<LEN>();

    chain_pair_state cur = chain_load<R>(pd, seqb, chain_pairs[c0], 0), prv = cur;
    bool have_cur = true, have_prv = false;
    int q = c0;
    int ord = 0, ord_prv = 0;  // ordinals of cur and prv among this wave's pairs
    uint32_t cv[R], cvn[R], V[R];
    rows_of(cur.pair, cv);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        V[r] = Vb[r];
        cvn[r] = cv[r];
    }
    uint32_t top_prev = tpb, bottom = V[R - 1], selv = sent, outc = 0, capA = 0, capB = 0;
    uint32_t W[4] = {0, 0, 0, 0};
    uint32_t rcv[G];
    ring[lane] = ring[lane + 128] = chunk_of(cur, 0).y;
    ring[lane + 64] = ring[lane + 192] = sent;

    for (int s0 = 0;; s0 += 64) {
        // prefetch the next chunk's lane-0 inputs (this pair's next chunk, or the next pair's first)
        uint2 nx = make_uint2(0, 0);
        chain_pair_state nxt = cur;
        bool have_nxt = false;
        if (have_cur && s0 + 64 < cur.T + cur.S) {
            nx = chunk_of(cur, (s0 + 64 - cur.T) >> 6);
        } else if (have_cur) {
            const int qn = counter ? grab() : q + 1;
            if (qn < c1) {
                nxt = chain_load<R>(pd, seqb, chain_pairs[qn], cur.T + cur.S);
                have_nxt = true;
                nx = chunk_of(nxt, 0);
                q = qn - 1;  // advanced below when nxt becomes cur
            }
        }
        const uint32_t *lsel0 = ring + ((s0 - lane) & 127);  // this lane's global column at the chunk's first step
        // A chunk with every lane on cur, no switch window and no sink capture runs its own loop of plain groups:
        // with the three group variants in one loop, the register allocator copied the row state (18 v_mov) after
        // every plain group at the merge point (5.6 % of its VALU).  Pairs start on chunk boundaries (T is a
        // multiple of 64), so a window is always a whole chunk.
        const bool plain = have_cur && s0 >= cur.T && !(have_prv && s0 < cur.T + 64) &&
                           !(have_prv && prv.cap_step >= s0 && prv.cap_step < s0 + 64) &&
                           !(cur.cap_step >= s0 && cur.cap_step < s0 + 64);
        if (plain) {
            for (int g = 0; g < 64 / G; ++g) {
                const int s = s0 + g * G;
                i32_chain_group<R, TB, LEN, false, false, CK, LDOT>(
                    V, cv, cvn, Vb, tpb, top_prev, bottom, selv, lsel0 + g * G, outc, W, s, lane, -(1 << 30), prv.cap_step,
                    prv.cap_lane, prv.cap_row, capA, cur.cap_step, cur.cap_lane, cur.cap_row, capB, rcv, jv);
                if constexpr (TB) {
                    uint32_t lo = (uint32_t)lane * 16u;
                    asm volatile("" : "+v"(lo));
                    char *gp = reinterpret_cast<char *>(tb + cur.tb_off + (uint64_t)((s - cur.T) / G) * 256u);
                    *reinterpret_cast<uint4 *>(gp + lo) = make_uint4(W[0], W[1], W[2], W[3]);
                }
                if constexpr (CK) {
                    constexpr int GH = SED_CK_TILE / R;
                    if ((lane & (GH - 1)) == GH - 1)
                        store_words<G>(tb + cur.tb_off + sed_ck_col_words(R, 1, cur.nchunks) +
                                           (uint64_t)((s - cur.T) / G) * SED_CK_RW + (uint32_t)(lane / GH) * G, rcv);
                }
            }
        } else
        for (int g = 0; g < 64 / G; ++g) {
            const int s = s0 + g * G;
            const uint32_t *lsel = lsel0 + g * G;
            const bool win = have_cur && have_prv && s < cur.T + 64;  // lanes switch from prv to cur
            const bool capg = (have_prv && prv.cap_step >= s && prv.cap_step < s + G) ||
                              (have_cur && cur.cap_step >= s && cur.cap_step < s + G);
            // wave-uniform: which body; Tsw never matches a lane outside a switch window
            const int Tsw = win ? cur.T : -(1 << 30);
#define SED_CGROUP(SW, GEN)                                                                               \
    i32_chain_group<R, TB, LEN, SW, GEN, CK, LDOT>(V, cv, cvn, Vb, tpb, top_prev, bottom, selv, lsel, outc, W, s, lane, \
                                             Tsw, prv.cap_step, prv.cap_lane, prv.cap_row, capA, cur.cap_step,    \
                                             cur.cap_lane, cur.cap_row, capB, rcv, jv)
            if (capg) SED_CGROUP(false, true);
            else if (win) SED_CGROUP(true, false);
            else SED_CGROUP(false, false);
#undef SED_CGROUP
            if constexpr (TB) {
                // a lane's 16 bytes go to the pair it worked on; in the switch window a group holds
                // steps of both pairs, so it is stored to both (each slot's unused part is never read).
                // Uniform base + 32-bit lane offset: saddr stores, no per-lane 64-bit address kept live.
                uint32_t lo = (uint32_t)lane * 16u;
                asm volatile("" : "+v"(lo));
                if (have_cur && s >= cur.T) {
                    char *gp = reinterpret_cast<char *>(tb + cur.tb_off + (uint64_t)((s - cur.T) / G) * 256u);
                    *reinterpret_cast<uint4 *>(gp + lo) = make_uint4(W[0], W[1], W[2], W[3]);
                }
                // lanes still on prv: the switch window, or the final drain after the chain's last pair
                if (have_prv && s < (have_cur ? cur.T + 64 : prv.end) && (s - prv.T) / G < prv.sg) {
                    char *gp = reinterpret_cast<char *>(tb + prv.tb_off + (uint64_t)((s - prv.T) / G) * 256u);
                    *reinterpret_cast<uint4 *>(gp + lo) = make_uint4(W[0], W[1], W[2], W[3]);
                }
            }
            if constexpr (CK) {  // row checkpoints of lanes t = G-1 (mod G), to the pair(s) the group's steps belong to
                constexpr int GH = SED_CK_TILE / R;
                if ((lane & (GH - 1)) == GH - 1) {
                    const uint32_t lo = (uint32_t)(lane / GH) * G;
                    if (have_cur && s >= cur.T)
                        store_words<G>(tb + cur.tb_off + sed_ck_col_words(R, 1, cur.nchunks) +
                                           (uint64_t)((s - cur.T) / G) * SED_CK_RW + lo, rcv);
                    if (have_prv && s < (have_cur ? cur.T + 64 : prv.end) && (s - prv.T) / G < prv.sg)
                        store_words<G>(tb + prv.tb_off + sed_ck_col_words(R, 1, prv.nchunks) +
                                           (uint64_t)((s - prv.T) / G) * SED_CK_RW + lo, rcv);
                }
            }
            if (capg) {
                if (have_prv && prv.cap_step >= s && prv.cap_step < s + G && lane == prv.cap_lane)
                    chain_store_result<R, TB, LEN, CK, LDOT>(res, prv.pair, capA, prv.n, prv.m, ord_prv, prm);
                if (have_cur && cur.cap_step >= s && cur.cap_step < s + G && lane == cur.cap_lane)
                    chain_store_result<R, TB, LEN, CK, LDOT>(res, cur.pair, capB, cur.n, cur.m, ord, prm);
            }
        }
        if constexpr (CK) {  // column checkpoint of cur's local chunk: every lane is on cur at a chunk end
            if (have_cur) {
                const int lc = (s0 - cur.T) >> 6;
                if (lc < cur.nchunks) {
                    uint32_t *cp = tb + cur.tb_off + sed_ck_col_word(R, 0, cur.nchunks, lc, 0, lane);
#pragma unroll
                    for (int r = 0; r < R; ++r) cp[r * 64] = V[r];
                    cp[R * 64] = top_prev;
                }
            }
        }
        {  // global columns s0 + 64 .. s0 + 127, after the chunk's last LDS read (in order)
            const uint32_t slot = (uint32_t)(s0 + 64 + lane) & 127u;
            ring[slot] = ring[slot + 128] = nx.y;
        }
        const int s1 = s0 + 64;
        if (have_cur && s1 == cur.T + cur.S) {  // lane 0 is done with cur: it becomes the draining pair
            prv = cur;
            ord_prv = ord;
            have_prv = true;
            capA = capB;
            if (have_nxt) {
                cur = nxt;
                ++q;
                ++ord;
                rows_of(cur.pair, cvn);
                // lane 0 switches before the next pair's first step
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    V[r] = lane == 0 ? Vb[r] : V[r];
                    cv[r] = lane == 0 ? cvn[r] : cv[r];
                }
                top_prev = lane == 0 ? tpb : top_prev;
            } else {
                have_cur = false;
            }
        }
        if (have_prv && s1 >= prv.end && (!have_cur || s1 >= cur.T + 64)) have_prv = false;  // drained
        if (!have_cur && !have_prv) break;
    }
}

// ---------------------------------------------------------------------------
// fp64 kernel (general costs).  State per row: D (fp64), Lk = L << 2,
// optional int-typing bit T (TYPED).  Cost table in LDS:
//   tab[a*K + b] = {cost value, is-int flag}
// ---------------------------------------------------------------------------
// Path-length keys of the fp64 kernel in U-space: LK = SED_F64_LB - 4U (U = updates on the canonical path to the
// cell, so L = i + j - U) with the op in the low 2 bits of a candidate.  At a cell every candidate's L is the cell's
// i + j - U, so comparing B - 4U orders candidates exactly as L does, and the borders are all B: the insert
// candidate is LK_left (op 0), the delete candidate LK_up + 1, the update candidate LK_diag - 4 + 2.  (L << 2 keys
// took an add per candidate, +4, +5, +6: 21.25 against 20.25 VALU per cell on the R = 8 group loop's unmasked path.)
#define SED_F64_LB 0x80000000u
struct f64_cell_in {
    double d;
    uint32_t lk;
    uint32_t t;
};

// PF: the caller has moved this step's column symbol (bsel) and read its table entries (epf) a step ahead (the
// SPLIT kernel's lone waves, whose LDS reads would otherwise stall every step)
template <int R, bool TB, bool TYPED, bool MASKED, bool FULL, int SW = 64, bool PF = false>
__device__ __forceinline__ void f64_step(double (&D)[R], uint32_t (&LK)[R], uint32_t (&T)[R],
                                         const uint32_t (&rowbase)[R], const double2 *__restrict__ tab,
                                         double &dtop_prev, uint32_t &ltop_prev, uint32_t &ttop_prev,
                                         double &dbot, uint32_t &lbot, uint32_t &tbot, uint32_t &bsel,
                                         const double dtin, const uint32_t ltin, const uint32_t ttin,
                                         const uint32_t stin, uint32_t (&W)[4], const int u,
                                         const double cins, const double cdel, const uint32_t tins,
                                         const uint32_t tdel, const bool active, const sed_full_out &fo,
                                         const int i0, const int j, const double2 *epf = nullptr) {
    // the segment's first lane takes this step's top-row cell and column symbol (dtin .. stin, broadcast LDS reads of
    // the chunk), the others the lane above's bottom cell and previous symbol
    const double dtop = seg_shr1_f64<SW>(dtin, dbot);
    const uint32_t ltop = seg_shr1<SW>(ltin, lbot);
    uint32_t ttop = 0;
    if constexpr (TYPED) ttop = seg_shr1<SW>(ttin, tbot);
    if constexpr (!PF) bsel = seg_shr1<SW>(stin, bsel);
    double dup = dtop, ddiag = dtop_prev;
    uint32_t lup = ltop, ldiag = ltop_prev, tup = ttop, tdiag = ttop_prev;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double2 e = PF ? epf[r] : tab[rowbase[r] + bsel];  // x = cost, y = int flag (as double bits)
        const double dl = D[r];
        const double ca = dl + cins;
        const double cb = dup + cdel;
        const double cc = ddiag + e.x;
        const double mn = fmin(ca, fmin(cb, cc));
        const bool ea = (ca == mn), eb = (cb == mn), ec = (cc == mn);
        const uint32_t ka = ea ? LK[r] : 0xFFFFFFFFu;  // (U-space keys: the insert candidate needs no add)
        const uint32_t kb = eb ? lup + 1u : 0xFFFFFFFFu;
        const uint32_t kc = ec ? ldiag - 2u : 0xFFFFFFFFu;
        const uint32_t km = umin3_op(ka, kb, kc);
        const uint32_t ln = km & ~3u;
        uint32_t tn = 0;
        if constexpr (TYPED) {
            const uint32_t tc = (uint32_t)__double_as_longlong(e.y);
            tn = ea ? (T[r] & tins) : (eb ? (tup & tdel) : (tdiag & tc));
        }
        if constexpr (TB) {
            const int c = u * R + r;
            W[c >> 4] = __builtin_amdgcn_alignbit(km, W[c >> 4], 2);
        }
        if constexpr (FULL) {  // full-matrix materialisation (dp proxy, GUI path): value, edge mask, typing
            if (active && i0 + r <= fo.n) {
                const uint64_t o = (uint64_t)(i0 + r) * (uint64_t)(fo.m + 1) + (uint64_t)j;
                const uint32_t t = TYPED ? tn : (uint32_t)(mn == 0.0);
                fo.D[o] = mn;
                fo.M[o] = (uint8_t)((ea ? 1u : 0u) | (eb ? 2u : 0u) | (ec ? 4u : 0u) | (t << 3));
            }
        }
        ddiag = dl;
        ldiag = LK[r];
        if constexpr (TYPED) tdiag = T[r];
        dup = mn;
        lup = ln;
        if constexpr (TYPED) tup = tn;
        if constexpr (MASKED) {
            D[r] = active ? mn : dl;
            LK[r] = active ? ln : LK[r];
            if constexpr (TYPED) T[r] = active ? tn : T[r];
        } else {
            D[r] = mn;
            LK[r] = ln;
            if constexpr (TYPED) T[r] = tn;
        }
    }
    if constexpr (MASKED) {
        dtop_prev = active ? dtop : dtop_prev;
        ltop_prev = active ? ltop : ltop_prev;
        if constexpr (TYPED) ttop_prev = active ? ttop : ttop_prev;
    } else {
        dtop_prev = dtop;
        ltop_prev = ltop;
        if constexpr (TYPED) ttop_prev = ttop;
    }
    dbot = D[R - 1];
    lbot = LK[R - 1];
    if constexpr (TYPED) tbot = T[R - 1];
}

// Per wave: the current chunk's top row (cell values, L keys, typing) and str2 symbols, which the segment's first lane
// reads one per step, and the segment's last lane's bottom cells of the chunk, which it writes one per step (the
// next stripe's top row, stored to global memory at the chunk's end).  These replace DPP rotations of the chunk
// values and a DPP collection of the bottom cells: 8-11 VALU per step.
struct f64_chunk_lds {
    double d[64], od[64];
    uint32_t l[64], t[64], s[64], ol[64], ot[64];
};

// SW = 64: one wave per pair (pairs with d.seg set are skipped: they run in segments).  SW = 16 (short pairs of
// large batches): each DPP row of 16 lanes runs its own pair (items idx[0 .. nidx), four per wave, the
// host sorts them so a wave's four pairs have similar shapes): stripes of 16 R rows, 16-step chunks, a 15-step ramp
// instead of 63, and every lane move a row DPP (seg_*), so the four segments never exchange data.  The loop bounds
// are then per lane (uniform within a segment), and a segment whose pair is done sits out with its lanes masked.
// issue priority of the fp64 DP's waves (SED_F64_PRIO): pipelined fp64 script batches run the traceback of run k
// beside the DP of run k+1, which now issues first.  iupac 4.83-4.85 against 4.87-4.89 ms per step at 0, timing within
// noise, 3 interleaved rounds (profiles/r05/s17)
#ifndef SED_F64_PRIO
#define SED_F64_PRIO 1
#endif
template <int R, bool TB, bool TYPED, bool FULL, int SW = 64>
__global__ __launch_bounds__(256) void sed_wf_f64_kernel(const sed_pair_desc *__restrict__ pd, int npairs,
                                                         const uint8_t *__restrict__ seqa,
                                                         const uint8_t *__restrict__ seqb,
                                                         uint32_t *__restrict__ tb, uint32_t *__restrict__ bnd,
                                                         sed_result *__restrict__ res,
                                                         const double *__restrict__ gtab, sed_f64_params prm,
                                                         sed_full_out fo, const int32_t *__restrict__ idx) {
    if constexpr (SED_F64_PRIO > 0) __builtin_amdgcn_s_setprio(SED_F64_PRIO);
    static_assert(SW == 64 || (SW == 16 && !FULL), "segments of 16 lanes: no full-matrix output");
    constexpr int ROWS = SW * R;
    constexpr int G = Grp<R>::G;
    static_assert(SW % G == 0, "a group of G steps never crosses a chunk");
    __shared__ double2 tab[SED_MAX_K * SED_MAX_K];
    __shared__ f64_chunk_lds chx[4];
    const int K = prm.K;
    for (int e = threadIdx.x; e < K * K; e += blockDim.x)
        tab[e] = make_double2(gtab[2 * e], gtab[2 * e + 1]);
    __syncthreads();

    const int lane = SW == 64 ? (threadIdx.x & 63) : (threadIdx.x & (SW - 1));  // lane within the segment
    int pair;
    if constexpr (SW == 64) {
        pair = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
        if (pair >= npairs) return;
    } else {
        const int item = (blockIdx.x * 256 + threadIdx.x) / SW;
        if (item >= npairs) return;  // (npairs = the item count)
        pair = idx[item];
    }
    const sed_pair_desc d = pd[pair];
    if (d.lane || (SW == 64 && d.pad[1])) return;  // short str2, distance only: sed_lane.hip; segments: the SW = 16 launch
    const int n = d.n, m = d.m;
    if constexpr (FULL) {  // border cells: row 0 (insert edges) and column 0 (delete edges)
        for (int j = lane; j <= m; j += 64) {
            const double v = (double)j * prm.ins;
            const uint32_t t = (j == 0) ? 1u : (TYPED ? (uint32_t)prm.ins_int : (uint32_t)(v == 0.0));
            fo.D[j] = v;
            fo.M[j] = (uint8_t)((j == 0 ? 0u : 1u) | (t << 3));
        }
        for (int i = 1 + lane; i <= n; i += 64) {
            const double v = (double)i * prm.del;
            const uint32_t t = TYPED ? (uint32_t)prm.del_int : (uint32_t)(v == 0.0);
            fo.D[(uint64_t)i * (m + 1)] = v;
            fo.M[(uint64_t)i * (m + 1)] = (uint8_t)(2u | (t << 3));
        }
    }
    if (n == 0 || m == 0) {
        if (lane == 0) {
            res[pair].dist = (n == 0) ? (double)m * prm.ins : (double)n * prm.del;
            res[pair].len = n + m;
            res[pair].is_int = (n == 0 && m == 0) ? 1 : (n == 0 ? prm.ins_int : prm.del_int);
            res[pair].err = 0;
        }
        return;
    }
    const int nstripes = (n + ROWS - 1) / ROWS;
    const int SG = (m + SW - 1 + G - 1) / G * G;
    const int nchunks = (SG + SW - 1) / SW;
    // bottom-row buffer of a pair: [D as u64 | L as u32 | T as u32] planes; column j at index j + SW
    const uint64_t bwords = (uint64_t)(nchunks + 2) * SW;
    uint64_t *bndD = reinterpret_cast<uint64_t *>(bnd + d.bnd_off);
    uint32_t *bndL = bnd + d.bnd_off + 2 * bwords;
    uint32_t *bndT = bndL + bwords;
    const uint8_t *pa = seqa + d.a_off;
    const uint8_t *pb = seqb + d.b_off;
    const uint32_t tins = (uint32_t)prm.ins_int, tdel = (uint32_t)prm.del_int;

    for (int k = 0; k < nstripes; ++k) {
        const int row0 = k * ROWS + lane * R;
        double D[R];
        uint32_t LK[R], T[R], rowbase[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ri = row0 + r;
            const uint32_t a = (ri < n) ? pa[ri] : 0u;
            rowbase[r] = a * (uint32_t)K;
            D[r] = (double)(ri + 1) * prm.del;
            LK[r] = SED_F64_LB;
            T[r] = tdel;
        }
        double dtop_prev = (double)row0 * prm.del;
        uint32_t ltop_prev = SED_F64_LB;
        uint32_t ttop_prev = (row0 == 0) ? 1u : tdel;
        double dbot = 0.0;
        uint32_t lbot = 0, tbot = 0, bsel = 0;
        uint32_t W[4] = {0, 0, 0, 0};

        auto load_d = [&](int c) -> double {
            const int j = SW * c + lane + 1;
            if (k == 0) return (double)j * prm.ins;
            return __longlong_as_double((long long)load_sc1_u64(bndD + j + SW));
        };
        auto load_l = [&](int c) -> uint32_t {
            const int j = SW * c + lane + 1;
            if (k == 0) return SED_F64_LB;
            return load_sc1(bndL + j + SW);
        };
        auto load_t = [&](int c) -> uint32_t {
            if (k == 0) return tins;
            return load_sc1(bndT + SW * c + lane + SW + 1);
        };
        auto load_sel = [&](int c) -> uint32_t {
            const int ci = SW * c + lane;
            return (ci < m) ? (uint32_t)pb[ci] : 0u;
        };
        double dch = load_d(0);
        uint32_t lch = load_l(0), tch = TYPED ? load_t(0) : 0u, sch = load_sel(0);
        f64_chunk_lds &cx = chx[threadIdx.x >> 6];
        const int sb = (threadIdx.x & 63) - lane;  // the segment's first slot
        const bool lastlane = lane == SW - 1;
        uint32_t *tbk = tb + d.tb_off + (uint64_t)k * (uint64_t)(SG / G) * (SW * 4u);
        const bool last = (k == nstripes - 1);
        int s = 0;
        for (int c = 0; c < nchunks; ++c) {
            double dnx = 0.0;
            uint32_t lnx = 0, tnx = 0, snx = 0;
            if (c + 1 < nchunks) {
                dnx = load_d(c + 1);
                lnx = load_l(c + 1);
                if (TYPED) tnx = load_t(c + 1);
                snx = load_sel(c + 1);
            }
            // this chunk's top row and symbols (after the previous chunk's last reads: a wave's LDS accesses run in
            // order)
            cx.d[sb + lane] = dch;
            cx.l[sb + lane] = lch;
            if (TYPED) cx.t[sb + lane] = tch;
            cx.s[sb + lane] = sch;
            // (A separate loop for chunks of unmasked steps, as in the integer kernels, measured slower: iupac DP
            // 4.89 against 4.81 ms, timing 4.60 against 4.47 ms; profiles/r03/f64_plain_dropped.)
            for (int g = 0; g < SW / G && s < SG; ++g, s += G) {
                const bool full = (s >= SW - 1) && (s + G - 1 < m);
                const int cu0 = sb + g * G;
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    const int j = s + u - lane + 1;
                    const bool active = (j >= 1) && (j <= m);
                    const double dtin = cx.d[cu0 + u];
                    const uint32_t ltin = cx.l[cu0 + u], ttin = TYPED ? cx.t[cu0 + u] : 0u, stin = cx.s[cu0 + u];
                    if (full)
                        f64_step<R, TB, TYPED, false, FULL, SW>(D, LK, T, rowbase, tab, dtop_prev, ltop_prev, ttop_prev,
                                                                dbot, lbot, tbot, bsel, dtin, ltin, ttin, stin, W, u,
                                                                prm.ins, prm.del, tins, tdel, active, fo, row0 + 1, j);
                    else
                        f64_step<R, TB, TYPED, true, FULL, SW>(D, LK, T, rowbase, tab, dtop_prev, ltop_prev, ttop_prev,
                                                               dbot, lbot, tbot, bsel, dtin, ltin, ttin, stin, W, u,
                                                               prm.ins, prm.del, tins, tdel, active, fo, row0 + 1, j);
                    if (!last && lastlane) {  // the next stripe's top row
                        cx.od[cu0 + u] = dbot;
                        cx.ol[cu0 + u] = lbot;
                        if (TYPED) cx.ot[cu0 + u] = tbot;
                    }
                }
                if constexpr (TB) store_tb(tbk + ((uint64_t)(s / G) * SW + lane) * 4u, W);
            }
            // slot i holds the segment's last lane's bottom cell of the chunk's step SW c + i, i.e. column
            // SW (c - 1) + 2 + i at index SW c + 2 + i (a short last chunk: only its steps' slots)
            if (!last && lane < s - SW * c) {
                bndD[SW * c + 2 + lane] = (uint64_t)__double_as_longlong(cx.od[sb + lane]);
                bndL[SW * c + 2 + lane] = cx.ol[sb + lane];
                if (TYPED) bndT[SW * c + 2 + lane] = cx.ot[sb + lane];
            }
            dch = dnx;
            lch = lnx;
            tch = tnx;
            sch = snx;
        }
        if (!last) __builtin_amdgcn_s_waitcnt(0);
        else {
            const int w = (n - 1) % ROWS;
            if (lane == w / R) {
                const int rf = w % R;
                double dv = 0.0;
                uint32_t lv = 0, tv = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    dv = (r == rf) ? D[r] : dv;
                    lv = (r == rf) ? LK[r] : lv;
                    tv = (r == rf) ? T[r] : tv;
                }
                res[pair].dist = dv;
                res[pair].len = n + m - (int32_t)((SED_F64_LB - lv) >> 2);
                res[pair].is_int = TYPED ? (uint8_t)tv : (uint8_t)(dv == 0.0);
                res[pair].err = 0;
            }
        }
    }
}

// SPLIT fp64 (few long pairs: timing.py's one-call loop, GUI calls over IUPAC symbols).  A lone fp64 wave issues
// ~20 dependent VALU per cell on one SIMD (a 2000^2 pair took 3.5 ms), so, as in the integer SPLIT kernel, each
// stripe of 64 R rows (R = 2 by default, 4 on request) is a 128-thread workgroup of its own: all stripes of a pair
// run at once, each ~63 steps (its lanes' systolic depth) plus a 16-step block and the hand-off's latency behind the
// stripe above.  The hand-off is the integer kernel's tagged words: lane 63's bottom cell of column j
// travels as three relaxed agent-scope 64-bit stores {tag, D low}, {tag, D high}, {tag, L key | T} (the L key is a
// multiple of 4, so its bit 0 carries the typing bit), each single-copy atomic and validated on its own, tag = the
// run's epoch | poison << 31.  The feeder wave (f64_split_feed) polls the stripe above's words, writes the steps'
// top-row cells and str2 symbols into an LDS ring and publishes how many steps are ready; stripe 0's feeder writes
// the row-0 border.  The compute wave is sed_wf_f64_kernel's stripe loop (SW = 64) reading the ring, with each step's
// column symbol and table entries read a step ahead (f64_step PF).  Codes, their layout and the result are the
// one-wave kernel's, so the tracebacks read them unchanged.
#define SED_F64_RING 256
template <int G> struct f64_split_lds {
    double d[SED_F64_RING];
    uint32_t l[SED_F64_RING], t[SED_F64_RING], s[SED_F64_RING];
    double od[G][64];  // every lane's bottom cell of the group's steps (lane 63's are handed off)
    uint32_t ol[G][64], ot[G][64];
};
// the three hand-off planes of stripe k: words [plane][column + 64], (nchunks + 2) * 64 per plane
__device__ __forceinline__ uint64_t *f64_split_words(uint32_t *bnd, const sed_pair_desc &d, int k, uint32_t plane_words) {
    return reinterpret_cast<uint64_t *>(bnd + d.bnd_off) + (uint64_t)k * 3u * plane_words;
}
template <int G>
__device__ void f64_split_feed(const uint64_t *__restrict__ hin, const uint32_t plane_words, const bool top, const int m,
                               const int SG, const uint32_t epoch, const uint8_t *__restrict__ pb, const double ins,
                               const uint32_t tins, f64_split_lds<G> &rg, uint32_t *flag, const int lane) {
    uint32_t poison = 0, idle = 0;
    int have = 0;  // steps whose top-row cells are in the ring
    while (have < SG) {
        if (have + 64 > (int)lds_flag_get(flag + 1) + SED_F64_RING) {  // ring full: the compute wave is behind
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        const int t = have + lane, col = t + 1;
        const bool need = !top && t < SG && col <= m;  // columns past m are never stored nor waited for
        uint64_t w0 = 0, w1 = 0, w2 = 0;
        if (need) {
            w0 = load_sc1_u64(hin + (uint32_t)(col + 64));
            w1 = load_sc1_u64(hin + plane_words + (uint32_t)(col + 64));
            w2 = load_sc1_u64(hin + 2u * plane_words + (uint32_t)(col + 64));
        }
        const uint32_t g0 = (uint32_t)(w0 >> 32), g1 = (uint32_t)(w1 >> 32), g2 = (uint32_t)(w2 >> 32);
        const bool good = !need || (((g0 & ~SED_PROG_POISON) == epoch) && ((g1 & ~SED_PROG_POISON) == epoch) &&
                                    ((g2 & ~SED_PROG_POISON) == epoch));
        const uint64_t bad = __ballot(!good);
        const int nv = min(bad ? (int)__builtin_ctzll(bad) : 64, SG - have);  // the valid prefix
        if (__any(lane < nv && need && ((g0 | g1 | g2) & SED_PROG_POISON))) poison = SED_PROG_POISON;
        if (nv > 0) {
            if (lane < nv) {
                const int slot = t & (SED_F64_RING - 1);
                if (top) {  // row 0: D = j * insert, L key B, typing of insert
                    rg.d[slot] = (double)col * ins;
                    rg.l[slot] = SED_F64_LB;
                    rg.t[slot] = tins;
                } else {
                    rg.d[slot] = __longlong_as_double((long long)(((w1 & 0xFFFFFFFFull) << 32) | (w0 & 0xFFFFFFFFull)));
                    rg.l[slot] = (uint32_t)w2 & ~3u;
                    rg.t[slot] = (uint32_t)w2 & 1u;
                }
                rg.s[slot] = t < m ? (uint32_t)pb[t] : 0u;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the values before the count
            have += nv;
            idle = 0;
        } else if (++idle > (1u << 22)) {  // the stripe above stopped: give up, let the compute wave drain
            poison = SED_PROG_POISON;
            have = SG;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0 && (nv > 0 || poison)) lds_flag_set(flag, (uint32_t)have | poison);
    }
}

template <int R, bool TB, bool TYPED, bool FULL>
__global__ __launch_bounds__(128) void sed_wf_f64_split_kernel(const sed_pair_desc *__restrict__ pd,
                                                               const int2 *__restrict__ tasks,
                                                               const uint8_t *__restrict__ seqa,
                                                               const uint8_t *__restrict__ seqb,
                                                               uint32_t *__restrict__ tb, uint32_t *__restrict__ bnd,
                                                               sed_result *__restrict__ res,
                                                               const double *__restrict__ gtab, sed_f64_params prm,
                                                               sed_full_out fo) {
    if constexpr (SED_SPLIT_PRIO > 0) __builtin_amdgcn_s_setprio(SED_SPLIT_PRIO);
    static_assert(!(FULL && TB), "full-matrix output: distance kernel");
    constexpr int ROWS = 64 * R;
    constexpr int G = Grp<R>::G;
    __shared__ double2 tab[SED_MAX_K * SED_MAX_K];
    __shared__ f64_split_lds<Grp<R>::G> rg;
    __shared__ uint32_t split_flag[2];
    const int K = prm.K;
    for (int e = threadIdx.x; e < K * K; e += blockDim.x) tab[e] = make_double2(gtab[2 * e], gtab[2 * e + 1]);
    if (threadIdx.x < 2) split_flag[threadIdx.x] = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int2 task = tasks[blockIdx.x];
    const int pair = __builtin_amdgcn_readfirstlane(task.x), k = __builtin_amdgcn_readfirstlane(task.y);
    const sed_pair_desc d = pd[pair];
    const int n = d.n, m = d.m;
    if constexpr (FULL) {  // border cells (stripe 0's compute wave): row 0 (insert edges) and column 0 (delete edges)
        if (k == 0 && threadIdx.x < 64) {
            for (int j = lane; j <= m; j += 64) {
                const double v = (double)j * prm.ins;
                const uint32_t t = (j == 0) ? 1u : (TYPED ? (uint32_t)prm.ins_int : (uint32_t)(v == 0.0));
                fo.D[j] = v;
                fo.M[j] = (uint8_t)((j == 0 ? 0u : 1u) | (t << 3));
            }
            for (int i = 1 + lane; i <= n; i += 64) {
                const double v = (double)i * prm.del;
                const uint32_t t = TYPED ? (uint32_t)prm.del_int : (uint32_t)(v == 0.0);
                fo.D[(uint64_t)i * (m + 1)] = v;
                fo.M[(uint64_t)i * (m + 1)] = (uint8_t)(2u | (t << 3));
            }
        }
    }
    if (n == 0 || m == 0) {
        if (threadIdx.x == 0) {
            res[pair].dist = (n == 0) ? (double)m * prm.ins : (double)n * prm.del;
            res[pair].len = n + m;
            res[pair].is_int = (n == 0 && m == 0) ? 1 : (n == 0 ? prm.ins_int : prm.del_int);
            res[pair].err = 0;
        }
        return;
    }
    const int nstripes = (n + ROWS - 1) / ROWS;
    const int SG = (m + 63 + G - 1) / G * G;
    const int nchunks = (SG + 63) >> 6;
    const uint32_t plane_words = (uint32_t)(nchunks + 2) * 64u;
    const uint8_t *pa = seqa + d.a_off;
    const uint8_t *pb = seqb + d.b_off;
    const uint32_t tins = (uint32_t)prm.ins_int, tdel = (uint32_t)prm.del_int;
    if (threadIdx.x >= 64) {  // the feeder wave
        f64_split_feed<G>(k > 0 ? f64_split_words(bnd, d, k - 1, plane_words) : nullptr, plane_words, k == 0, m, SG,
                       prm.epoch, pb, prm.ins, tins, rg, split_flag, lane);
        return;
    }
    uint64_t *hout = f64_split_words(bnd, d, k, plane_words);
    const int row0 = k * ROWS + lane * R;
    double D[R];
    uint32_t LK[R], T[R], rowbase[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int ri = row0 + r;
        const uint32_t a = (ri < n) ? pa[ri] : 0u;
        rowbase[r] = a * (uint32_t)K;
        D[r] = (double)(ri + 1) * prm.del;
        LK[r] = SED_F64_LB;
        T[r] = tdel;
    }
    double dtop_prev = (double)row0 * prm.del;
    uint32_t ltop_prev = SED_F64_LB;
    uint32_t ttop_prev = (row0 == 0) ? 1u : tdel;
    double dbot = 0.0;
    uint32_t lbot = 0, tbot = 0, bsel = 0;
    uint32_t W[4] = {0, 0, 0, 0};
    uint32_t *tbk = TB ? tb + d.tb_off + (uint64_t)k * (uint64_t)(SG / G) * 256u : nullptr;
    const bool last = (k == nstripes - 1);
    const uint32_t tag = prm.epoch;
    bool ok = true;
    int ready = 0;  // steps the feeder has published as ready (last read)
    constexpr int HB = G < 16 ? G : 16;  // steps per block of ring reads, waits and hand-offs
    // until the ring holds the top-row cells of steps < upto (LDS only)
    auto wait_ready = [&](int upto) {
        upto = min(upto, SG);  // (the feeder publishes SG steps in all)
        if (ready < upto) {
            uint32_t f = lds_flag_get(split_flag), spins = 0;
            while (ok && (int)(f & ~SED_PROG_POISON) < upto) {
                if (++spins > (1u << 24)) ok = false;
                __builtin_amdgcn_s_sleep(1);
                f = lds_flag_get(split_flag);
            }
            if (f & SED_PROG_POISON) ok = false;
            ready = (int)(f & ~SED_PROG_POISON);
            asm volatile("" ::: "memory");
        }
    };
    // lane u < HB hands off column s0 + u - 62 (lane 63's cell of step s0 + u, staged at rg.od[u0 + u]), then the
    // block's ring slots are free again
    auto handoff = [&](const int s0, const int u0) {
        if (!last && lane < HB) {
            const int col = s0 + lane - 62;
            if (col >= 1 && col <= m) {
                const uint32_t tg = tag | (ok ? 0u : SED_PROG_POISON);
                const uint64_t bits = (uint64_t)__double_as_longlong(rg.od[u0 + lane][63]);
                const uint32_t lt = rg.ol[u0 + lane][63] | (TYPED ? rg.ot[u0 + lane][63] : 0u);
                store_tagged(hout + (uint32_t)(col + 64), tg, (uint32_t)bits);
                store_tagged(hout + plane_words + (uint32_t)(col + 64), tg, (uint32_t)(bits >> 32));
                store_tagged(hout + 2u * plane_words + (uint32_t)(col + 64), tg, lt);
            }
        }
        asm volatile("" ::: "memory");
        if (lane == 0) lds_flag_set(split_flag + 1, (uint32_t)(s0 + HB));
    };
    for (int s = 0; s < SG; s += G) {
        // a block needs its own steps and the next block's first symbol (the table reads a step ahead)
        wait_ready(s + (HB < G ? HB + 1 : HB));
        // the group's steps as one straight-line block per variant (a lone wave is latency-bound: a branch per step
        // kept the compiler from overlapping one step's table reads with the previous step's arithmetic)
        // The group's top-row cells and symbols are read from the ring at its start, and each step's column symbol
        // and table entries are fetched one step ahead (PF).
        // (ring entries in blocks of 16 steps: the R = 2 group's 32 would take ~160 VGPRs at once; each block waits
        // for its own steps and hands its bottom cells off, so the stripe below trails by 16 steps, not 32)
        auto group = [&](auto masked_tag) {
            constexpr bool MASKED = decltype(masked_tag)::value;
            double2 en[R];
            uint32_t bn = dpp_shr1(rg.s[s & (SED_F64_RING - 1)], bsel);
#pragma unroll
            for (int r = 0; r < R; ++r) en[r] = tab[rowbase[r] + bn];
#pragma unroll
            for (int h = 0; h < G; h += HB) {
                if (h > 0) wait_ready(s + h + (h + HB < G ? HB + 1 : HB));
                double dg[HB];
                uint32_t lg[HB], tg[HB], sg[HB + 1];
#pragma unroll
                for (int v = 0; v <= HB; ++v) {
                    const int slot = (s + h + v) & (SED_F64_RING - 1);
                    if (v < HB) {
                        dg[v] = rg.d[slot];
                        lg[v] = rg.l[slot];
                        tg[v] = TYPED ? rg.t[slot] : 0u;
                    }
                    if (v > 0) sg[v] = rg.s[slot];  // (sg[0]: in bn already)
                }
#pragma unroll
                for (int v = 0; v < HB; ++v) {
                    const int u = h + v;
                    const int j = s + u - lane + 1;
                    const bool active = (j >= 1) && (j <= m);
                    double2 e[R];
#pragma unroll
                    for (int r = 0; r < R; ++r) e[r] = en[r];
                    bsel = bn;
                    if (u + 1 < G) {
                        bn = dpp_shr1(sg[v + 1], bsel);
#pragma unroll
                        for (int r = 0; r < R; ++r) en[r] = tab[rowbase[r] + bn];
                    }
                    f64_step<R, TB, TYPED, MASKED, FULL, 64, true>(D, LK, T, rowbase, tab, dtop_prev, ltop_prev,
                                                                   ttop_prev, dbot, lbot, tbot, bsel, dg[v], lg[v],
                                                                   tg[v], 0u, W, u, prm.ins, prm.del, tins, tdel,
                                                                   active, fo, row0 + 1, j, e);
                    // every lane's bottom cell, lane 63's read back below: a write under lane == 63 put a branch
                    // (exec skip) between every two steps
                    rg.od[u][lane] = dbot;
                    rg.ol[u][lane] = lbot;
                    if (TYPED) rg.ot[u][lane] = tbot;
                    __builtin_amdgcn_sched_barrier(0);  // (the next step's table reads stay a step ahead of their use)
                }
                handoff(s + h, h);
            }
        };
        if ((s >= 63) && (s + G - 1 < m))
            group(BoolTag<false>{});
        else
            group(BoolTag<true>{});
        if constexpr (TB) store_tb(tbk + ((uint64_t)(s / G) * 64u + lane) * 4u, W);
    }
    if (last) {
        const int w = (n - 1) % ROWS;
        if (lane == w / R) {
            const int rf = w % R;
            double dv = 0.0;
            uint32_t lv = 0, tv = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                dv = (r == rf) ? D[r] : dv;
                lv = (r == rf) ? LK[r] : lv;
                tv = (r == rf) ? T[r] : tv;
            }
            res[pair].dist = dv;
            res[pair].len = n + m - (int32_t)((SED_F64_LB - lv) >> 2);
            res[pair].is_int = TYPED ? (uint8_t)tv : (uint8_t)(dv == 0.0);
            res[pair].err = ok ? 0 : SED_ERR_SPLIT_TIMEOUT;  // a timed-out wait anywhere up the chain poisons the pair
        }
    }
}

// ---------------------------------------------------------------------------
// Traceback: one lane per pair walks the 2-bit choices from (n, m) to (0, 0)
// and writes the op codes origin->sink, 16 per word.  Position bookkeeping is
// incremental (stripe k, lane t, row r, step s) with power-of-two R, and the
// 16-byte aligned block of codes last read is kept in registers: a diagonal
// run stays in it for up to four steps.
// ---------------------------------------------------------------------------
// SW = 16: the fp64 kernel's segment pairs (idx[0 .. npairs)), whose codes have the stripe layout of 16 lanes; SW = 64
// skips them (d.pad[1]).
// issue priority of the per-cell-code traceback's waves on integer (ladder-code) batches (SED_TB_PRIO, s_setprio):
// pipelined batches run the traceback of run k beside the DP of run k+1, and at priority 1 it no longer trails it.
// Config 3 (CHAIN): 2.50-2.51 against 2.62-2.72 ms per step at 10 steps (traceback span 0.71 against 1.85-1.95 ms),
// the last run's unoverlapped traceback; 2.38 ms at 20 steps either way.  The fp64 workloads (pat = 0) stay at
// priority 0: iupac 4.89-4.90 against 4.83-4.89 ms (profiles/r05/s16)
#ifndef SED_TB_PRIO
#define SED_TB_PRIO 1
#endif
template <int R, int SW = 64>
__global__ __launch_bounds__(64) void sed_traceback_kernel(const sed_pair_desc *__restrict__ pd, int npairs,
                                                           const uint32_t *__restrict__ tb,
                                                           sed_result *__restrict__ res,
                                                           uint32_t *__restrict__ ops, const uint64_t pat,
                                                           const int32_t *__restrict__ idx) {
    constexpr int G = Grp<R>::G, P = Ladder<R>::P;
    if (SED_TB_PRIO > 0 && pat != 0) __builtin_amdgcn_s_setprio(SED_TB_PRIO);
    const int item = blockIdx.x * blockDim.x + threadIdx.x;
    if (item >= npairs) return;
    const int pair = SW == 64 ? item : idx[item];
    const sed_pair_desc d = pd[pair];
    if (d.lane || (SW == 64 && d.pad[1])) return;  // scripted by sed_lane.hip / by the SW = 16 launch
    const int n = d.n, m = d.m;
    const int SG = (m + SW - 1 + G - 1) / G * G;
    const uint64_t stripe_words = (uint64_t)(SG / G) * (SW * 4u);
    uint32_t *out = ops + d.ops_off;
    const int L0 = res[pair].len;
    int q = L0;  // ops in the script; written from position q-1 down to 0
    int i = n, j = m;
    // the padding past the script first: zeroed after the walk instead, config 3's traceback span is 1.65-1.90 against
    // 0.70-0.76 ms (step 2.60-2.76 against 2.57-2.58 ms; none at all: 2.56-2.57 ms, profiles/r06/pad_ab)
    zero_script_tails_wave(ops, d.ops_off, L0, n, m);
    uint32_t acc = 0, bad = 0;
    auto emit = [&](uint32_t op) {
        if (q <= 0) {  // the walk is longer than the sink's L: never write below the pair's script
            bad = 1;
            return;
        }
        --q;
        acc |= op << (2 * (q & 15));
        if ((q & 15) == 0) {
            out[q >> 4] = acc;
            acc = 0;
        }
    };
    if (i > 0 && j > 0) {
        const int rr = i - 1;
        int k = rr / (SW * R);
        int t = (rr >> __builtin_ctz(R)) & (SW - 1);
        int r = rr & (R - 1);
        const uint32_t *base = tb + d.tb_off + (uint64_t)k * stripe_words;
        uint64_t cached = ~0ull;
        uint4 cw = make_uint4(0, 0, 0, 0);
        while (true) {
            const int s = j - 1 + t;
            const int c = (s % G) * R + r;  // code index inside the lane's 16-byte group block
            const uint64_t blk = ((uint64_t)(s / G) * SW + t) * 4u;
            if (blk != cached) {
                cached = blk;
                cw = *reinterpret_cast<const uint4 *>(base + blk);
            }
            const int wsel = c >> 4;
            const uint32_t wv = (wsel & 2) ? ((wsel & 1) ? cw.w : cw.z) : ((wsel & 1) ? cw.y : cw.x);
            // integer codes are (rung(i) + op) & 3 (pat = the ladder), fp64 codes op (pat = 0)
            const uint32_t op = ((wv >> (2 * (c & 15))) - (uint32_t)(pat >> (4 * (i & (P - 1))))) & 3u;
            emit(op);
            if (op != 1) --j;
            if (op != 0) {  // move up one row
                --i;
                if (--r < 0) {
                    r = R - 1;
                    if (--t < 0) {
                        t = SW - 1;
                        --k;
                        base -= stripe_words;
                        cached = ~0ull;
                    }
                }
            }
            if (i == 0 || j == 0) break;
        }
    }
    while (j > 0) { emit(0u); --j; }
    while (i > 0) { emit(1u); --i; }
    if (bad || q != 0) res[pair].err = SED_ERR_TB_LENGTH;
}


// Few pairs (config 2, the GUI): one pair per wave, the walk itself wave-uniform (scalar unit),
// and the wave's 64 lanes fetch a window of 64 code blocks at once.  A lone walk is bound by the
// latency of its dependent block loads (a new 16-byte block every ~R steps of a diagonal path);
// the window covers NT = G lanes x NS = R step-groups, i.e. the next ~50-64 steps of any path
// direction, so one load latency serves them all.  Blocks move from the window's VGPRs to SGPRs
// with v_readlane when the walk enters them.
// The window walk of one pair from cell (i, j), emitting script positions q-1 down, until it reaches row istop
// (0: the origin, with the trailing border runs).  SEG: one segment of the stripe-parallel traceback, whose
// script words go through atomicOr (the buffer is zeroed; the first and last words are shared with the
// neighbouring segments), the last partial word included.  Returns the final q.
template <int R, bool SEG>
__device__ __forceinline__ uint32_t window_walk(const sed_pair_desc &d, int i, int j, const int istop, uint32_t q,
                                                const int lane, const uint32_t *__restrict__ tb,
                                                uint32_t *__restrict__ out, const uint64_t pat, uint32_t &bad) {
    constexpr int G = Grp<R>::G, NT = G, NS = R;  // NT * NS = 64 blocks
    constexpr int P = Ladder<R>::P;
    constexpr int LR = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : 5, LG = 6 - LR;
    static_assert((1 << LR) == R, "R must be a power of two in 2..32");
    const int m = d.m;
    const int SG = (m + 63 + G - 1) / G * G;
    const uint64_t stripe_words = (uint64_t)(SG / G) * 256u;
    // ops are emitted sink -> origin, i.e. from position q-1 down; acc = acc<<2 | op leaves the op of
    // position q in bits 1:0 and position q+p in bits 2p+1:2p when a word [q, q+16) completes
    uint32_t acc = 0;
    auto emit = [&](uint32_t op) {
        if (q == 0) {  // longer than the sink's L (integer flag: a wave-uniform walk)
            bad = 1;
            return;
        }
        acc = (acc << 2) | op;
        if ((--q & 15u) == 0) {
            if constexpr (SEG) {
                if (lane == 0) atomicOr(out + (q >> 4), acc);
            } else {
                out[q >> 4] = acc;  // every lane stores the same word (no exec switching)
            }
        }
    };
    if (i > istop && j > 0) {
        const int rr = i - 1;
        int k = rr >> (6 + LR);
        int t = (rr >> LR) & 63;
        uint32_t r = (uint32_t)rr & (R - 1);
        int s = j - 1 + t;  // the step at which lane t computed column j
        const uint32_t *base = tb + d.tb_off + (uint64_t)k * stripe_words;
        int wt = -1, wsg = -1;  // window corner (highest lane, highest step-group); -1: none loaded
        uint4 wv = make_uint4(0, 0, 0, 0);
        uint64_t lo = 0, hi = 0;  // codes 0..31 and 32..63 of the block being walked
        uint32_t fresh = 1;  // integer flags throughout: bools of uniform values round-trip through VALU masks
        while (true) {
            if (fresh) {  // entered another block: from the window, reloading it first if needed
                const int sg = s >> LG;
                if (!(t <= wt && t > wt - NT && sg <= wsg && sg > wsg - NS)) {
                    wt = t;
                    wsg = sg;
                    const int lt = t - lane / NS, ls = sg - lane % NS;
                    wv = (lt >= 0 && ls >= 0) ? *reinterpret_cast<const uint4 *>(base + ((uint64_t)ls * 64u + lt) * 4u)
                                              : make_uint4(0, 0, 0, 0);
                }
                const int L = (wt - t) * NS + (wsg - sg);
                lo = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(wv.x, L) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(wv.y, L) << 32);
                hi = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(wv.z, L) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(wv.w, L) << 32);
            }
            const uint32_t c = ((uint32_t)(s & (G - 1)) << LR) | r;  // code index inside the block
            const uint32_t op =  // minus the ladder rung of row i (sed_traceback_kernel)
                ((uint32_t)(((c & 32u) ? hi : lo) >> (2u * c & 63u)) - (uint32_t)(pat >> (4 * (i & (P - 1))))) & 3u;
            emit(op);
            const uint32_t di = (op + 1u) >> 1, dj = (5u >> op) & 1u;  // row move (del, upd), column move (ins, upd)
            i -= (int)di;
            j -= (int)dj;
            if (i == istop || j == 0) break;
            const uint32_t wrap = di & ((r - 1u) >> 31);  // moved up out of the lane's rows (r was 0)
            r = (r - di) & (R - 1);
            const int s_old = s;
            s -= (int)(dj + wrap);
            fresh = wrap | ((uint32_t)(s ^ s_old) >> LG);
            if (wrap) {
                if (--t < 0) {  // the stripe above
                    t = 63;
                    --k;
                    base -= stripe_words;
                    s = j - 1 + t;
                    wt = -1;
                }
            }
        }
    }
    if (istop == 0) {
        while (j > 0) { emit(0u); --j; }
        while (i > 0) { emit(1u); --i; }
    } else {
        while (i > istop) { emit(1u); --i; }  // the column-0 border inside the segment
    }
    if constexpr (SEG) {
        if ((q & 15u) != 0 && lane == 0) atomicOr(out + (q >> 4), acc << (2u * (q & 15u)));  // last partial word
    }
    return q;
}

template <int R>
__global__ __launch_bounds__(64) void sed_traceback_window_kernel(const sed_pair_desc *__restrict__ pd,
                                                                  int npairs, const uint32_t *__restrict__ tb,
                                                                  sed_result *__restrict__ res,
                                                                  uint32_t *__restrict__ ops, const uint64_t pat) {
    const int lane = threadIdx.x;
    const int pair = __builtin_amdgcn_readfirstlane(blockIdx.x);
    if (pair >= npairs) return;
    const sed_pair_desc d = pd[pair];
    if (d.lane) return;  // scripted by sed_lane.hip
    const uint32_t q0 = (uint32_t)__builtin_amdgcn_readfirstlane(res[pair].len);
    uint32_t bad = 0;
    zero_script_tail(ops + d.ops_off, (int)q0, d.n, d.m, lane, 64);  // (before the walk, as sed_traceback_kernel)
    const uint32_t q = window_walk<R, false>(d, d.n, d.m, 0, q0, lane, tb, ops + d.ops_off, pat, bad);
    if ((bad | q) && lane == 0) res[pair].err = SED_ERR_TB_LENGTH;
}


// ---------------------------------------------------------------------------
// Stripe-parallel traceback for few pairs (per-cell codes; config 2, the GUI: one 4096^2 pair, SPLIT at
// R = 4, 16 stripes).  The window walk above is one dependent chain of ~4200 steps.  Instead:
//   map kernel: one lane per (stripe k in 1 .. K-2, column x): walk the codes from cell (last row of stripe
//     k, x) until the path steps into stripe k-1; record that column and the ops taken.  One more lane walks
//     the sink's stripe from the sink.  A path through a cell continues the same way whatever led to it (each
//     code is the cell's canonical op), so these maps compose;
//   emit kernel: one wave per (pair, stripe): compose the maps from the sink down to its stripe (its entry
//     column and the script positions of its segment), then walk that segment with the window walk, storing
//     script words with atomicOr (the two words a segment shares with its neighbours; the buffer is zeroed).
// ---------------------------------------------------------------------------
template <int R> struct CodeCursor {  // per-lane reader of one pair's per-cell codes, one 16-byte block cached
    static constexpr int G = Grp<R>::G, LR = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : 5, LG = 6 - LR;
    static constexpr int P = Ladder<R>::P;
    const uint32_t *base;
    uint64_t stripe_words;
    uint4 blk;
    uint64_t key;
    __device__ CodeCursor(const uint32_t *b, uint64_t sw) : base(b), stripe_words(sw), blk(make_uint4(0, 0, 0, 0)), key(~0ull) {}
    // canonical op (0 insert, 1 delete, 2 update) of cell (i, j), 1 <= i, 1 <= j
    __device__ __forceinline__ uint32_t op(int i, int j, uint64_t pat) {
        const int rr = i - 1, k = rr >> (6 + LR), t = (rr >> LR) & 63, r = rr & (R - 1);
        const int s = j - 1 + t;  // the step at which lane t computed column j
        const uint64_t kk = ((uint64_t)k << 40) | ((uint64_t)(s >> LG) << 6) | (uint64_t)t;
        if (kk != key) {
            key = kk;
            blk = *reinterpret_cast<const uint4 *>(base + (uint64_t)k * stripe_words + ((uint64_t)(s >> LG) * 64u + t) * 4u);
        }
        const uint32_t c = ((uint32_t)(s & (G - 1)) << LR) | (uint32_t)r;
        const uint32_t w = (c & 32u) ? ((c & 16u) ? blk.w : blk.z) : ((c & 16u) ? blk.y : blk.x);
        return ((w >> (2u * (c & 15u))) - (uint32_t)(pat >> (4 * (i & (P - 1))))) & 3u;
    }
};

// map[pd.map_off + 2 * (k * (m + 1) + x)] = {exit column, ops} for stripes 1 .. K-2; the sink's stripe at x = 0.
// A workgroup takes 256 consecutive columns x0 .. x0+255 of one stripe.  Paths near the diagonal stay in the
// stripe's 64R rows and within SED_TBMAP_LEFT (R = 2: SED_TBMAP_LEFT_R2) columns left of x0: the code groups of those steps are one
// contiguous run of 1 KiB groups (layout [group][64 lanes][16 B]), copied to LDS once, so a step reads LDS
// instead of waiting on a global load (a wave's lanes need new blocks at different steps: with global loads
// nearly every step waited on one).  A path that leaves the staged steps (cells far from the diagonal insert
// first, since ties prefer insert, and can run along the row for thousands of columns) stops: its entry is
// marked unknown (exit 0xFFFFFFFF) and the emit kernel walks that stripe itself if the real path needs it.
// The last workgroup of a pair walks the sink's stripe from the sink.  Every workgroup also zeroes its share
// of the pair's script words, which the emit kernel's segments OR into (lane-kernel pairs wrote theirs already).
#ifndef SED_TBMAP_LEFT
#define SED_TBMAP_LEFT 512
#endif
// R = 2 (the fp64 SPLIT route's 128-row stripes): a path crosses its stripe within fewer columns, and the map's time is
// its longest walks (lanes far from the path, running left through the staged columns): 1000^2 per call 400 -> 360 us,
// 2000^2 629 -> 587 us at 192 (tools/script_calls.py, profiles/r05/s47); the 256-row stripes of config 2 keep 512
// (at 192 its path needed columns past the staged ones, and the emit kernel's fallback walks took 187 against 53 us)
// With the band maps (64-row walks) 128 staged columns serve R = 2 better still: 1000^2 343 -> 335 us, 2000^2 572 -> 563 us
// per call (96: 335 / 562; profiles/r05/s57)
#ifndef SED_TBMAP_LEFT_R2
#define SED_TBMAP_LEFT_R2 128
#endif
#ifndef SED_TBMAP_BANDS  // 1: band maps + compose (sed_tb_bandmap_kernel), 0: one lane per stripe (A/B)
#define SED_TBMAP_BANDS 1
#endif
#ifndef SED_TBMAP_RUN
#define SED_TBMAP_RUN 96
#endif
// Band-map walks stop (entry unknown, left to the emit kernel's fallback walk) after 64 + 64 ceil(m / n) steps: the
// canonical path crosses a 64-row band in 64 steps plus its inserts, while a wave's time is its longest lane, and the
// lanes far from the path run left for 200-340 steps (config 2's pair: median walk 65 steps, 99th percentile 283,
// tools/tbmap_walks.py).  SED_TBMAP_CAP: the base (96: map 36.3 against 33.9 us at R = 4, 32.7 against 26.8 at R = 2,
// profiles/r06/tbmap_cap/step23); 0: no step limit (A/B)
#ifndef SED_TBMAP_CAP
#define SED_TBMAP_CAP 64
#endif
template <int R>
__global__ __launch_bounds__(256) void sed_tb_stripemap_kernel(const sed_pair_desc *__restrict__ pd,
                                                               const uint32_t *__restrict__ tb,
                                                               uint32_t *__restrict__ map,
                                                               uint32_t *__restrict__ ops, const uint64_t pat) {
    constexpr int ROWS = 64 * R, G = Grp<R>::G, LG = CodeCursor<R>::LG, LR = CodeCursor<R>::LR;
    constexpr int P = Ladder<R>::P;
    constexpr int LEFT = R == 2 ? SED_TBMAP_LEFT_R2 : SED_TBMAP_LEFT;
    constexpr int NSG = (LEFT + 256 + 64 + 2 * G) / G + 1;  // staged step groups
    constexpr int NIT = (NSG * 64 + 255) / 256;  // staging trips of the 256 threads
    __shared__ uint4 stage[NIT * 256];
    const __attribute__((address_space(3))) uint32_t *stage32 =
        (const __attribute__((address_space(3))) uint32_t *)(stage);
    const int p = blockIdx.y;
    const sed_pair_desc d = pd[p];
    const int n = d.n, m = d.m;
    if (d.lane) return;
    const int tid = threadIdx.x, idx = blockIdx.x * 256 + tid;
    if (idx < (n + m + 15) / 16) ops[d.ops_off + idx] = 0u;
    if (n == 0 || m == 0) return;
    const int K = (n + ROWS - 1) / ROWS;
    if (K < 3) return;  // walked whole by the emit kernel
    const int nx = m + 1, nxc = (nx + 255) / 256;
    const int blk = blockIdx.x;
    if (blk > (K - 2) * nxc) return;
    const int SG = (m + 63 + G - 1) / G * G;
    const uint64_t stripe_words = (uint64_t)(SG / G) * 256u;
    int k, i, j, slot, x0;
    bool live;
    if (blk == (K - 2) * nxc) {  // the sink's stripe, from the sink: the last lane of a block ending at m
        k = K - 1;
        x0 = max(0, m - 255);
        i = n;
        j = m;
        slot = k * nx;
        live = tid == m - x0;
    } else {
        k = 1 + blk / nxc;
        x0 = (blk % nxc) * 256;
        j = x0 + tid;
        i = (k + 1) * ROWS;
        slot = k * nx + j;
        live = j <= m;
    }
    // stage the groups of steps s = j' - 1 + t, j' in [x0 - LEFT, x0 + 255], t in [0, 63]
    const uint32_t *tbk = tb + d.tb_off + (uint64_t)k * stripe_words;
    const int s_lo = max(0, x0 - LEFT - 1), s_hi = min(SG - 1, x0 + 255 + 63);
    const int sg_lo = s_lo >> LG, nsg = min(NSG, (s_hi >> LG) - sg_lo + 1);
    const uint4 *src = reinterpret_cast<const uint4 *>(tbk) + (uint64_t)sg_lo * 64u;
    {  // fixed trip count, unguarded stores (clamped loads fill the tail): every load is in flight before the first
       // wait (guarded stores split the blocks, and the copy ran load, wait, store per trip)
        uint4 v[NIT];
#pragma unroll
        for (int u = 0; u < NIT; ++u) {
            const int e = tid + 256 * u;
            v[u] = src[e < nsg * 64 ? e : 0];
        }
#pragma unroll
        for (int u = 0; u < NIT; ++u) stage[tid + 256 * u] = v[u];
    }
    __syncthreads();
    if (!live) return;
    const int top = k * ROWS;  // row top belongs to stripe k - 1
    uint32_t cnt = 0, run = 0;  // run: consecutive inserts
    for (;;) {  // one exit per step (separate exits became nested exec-mask regions); reason decided after
        const int rr = i - 1, t = (rr >> LR) & 63, r = rr & (R - 1);
        const int s = j - 1 + t;
        const uint32_t c = ((uint32_t)(s & (G - 1)) << LR) | (uint32_t)r;
        // one unconditional ds_read_b32 per step (an LDS-qualified pointer: a generic one became a flat load, and
        // a uint4 read was split into two branch-guarded halves)
        const uint32_t rel = (uint32_t)((s >> LG) - sg_lo);
        const bool inside = rel < (uint32_t)nsg;
        const uint32_t word = stage32[(inside ? rel : 0u) * 256u + (uint32_t)t * 4u + (c >> 4)];
        if (!((i > top) & (j > 0) & inside & (run <= SED_TBMAP_RUN))) break;
        const uint32_t op = ((word >> (2u * (c & 15u))) - (uint32_t)(pat >> (4 * (i & (P - 1))))) & 3u;
        ++cnt;
        run = op == 0u ? run + 1u : 0u;
        i -= (int)(op != 0u);
        j -= (int)(op != 1u);
    }
    if (i > top) {
        if (j == 0) {  // the column-0 border: deletes up to the stripe above
            cnt += (uint32_t)(i - top);
        } else {  // left of the staged steps, or a long run of inserts (a cell far from the diagonal): unknown,
            j = -1;  // walked by the emit kernel if the real path needs it; the run limit bounds such walks
            cnt = 0;
        }
    }
    uint32_t *mp = map + (uint32_t)d.map_off + 2u * (uint32_t)slot;
    mp[0] = (uint32_t)j;  // 0xFFFFFFFF: unknown
    mp[1] = cnt;
}

// Band maps (round 5, SED_TBMAP_BANDS = 1, the default): the map kernel above gives one lane a whole stripe, a
// chain of up to ~700 dependent LDS steps at about one wave per SIMD (config 2: 104 us).  Here a lane walks one
// 64-row band (band g: rows 64g + 1 .. 64g + 64, from its last row, or from the sink in the sink's band) for every
// band 1 .. nbt-1 (stripe 0's upper bands too, for the banded emit) and every column: 4x (R = 4) the lanes at 1/4 the
// chain, each workgroup staging only its band's 64/R forward lanes of the code groups (1/4 the LDS, so many
// workgroups per CU).  band map entry bm[(g - 1) * (m + 1) + x] = {exit column at row 64g, ops}, or unknown; it
// follows the stripe map's K (m + 1) entries.  sed_tb_bandcompose_kernel then chains a stripe's NB bands into the
// stripe map, and the emit kernel composes both.
template <int R>
__global__ __launch_bounds__(256) void sed_tb_bandmap_kernel(const sed_pair_desc *__restrict__ pd,
                                                             const uint32_t *__restrict__ tb,
                                                             uint32_t *__restrict__ map,
                                                             uint32_t *__restrict__ ops, const uint64_t pat) {
    constexpr int ROWS = 64 * R, NB = R, NL = 64 / R, G = Grp<R>::G, LG = CodeCursor<R>::LG, LR = CodeCursor<R>::LR;
    constexpr int P = Ladder<R>::P;
    constexpr int LEFT = R == 2 ? SED_TBMAP_LEFT_R2 : SED_TBMAP_LEFT;
    constexpr int NSG = (LEFT + 256 + 64 + 2 * G) / G + 1;  // staged step groups
    constexpr int NIT = (NSG * NL + 255) / 256;  // staging trips of the 256 threads
    __shared__ uint4 stage[NIT * 256];
    const __attribute__((address_space(3))) uint32_t *stage32 =
        (const __attribute__((address_space(3))) uint32_t *)(stage);
    const int p = blockIdx.y;
    const sed_pair_desc d = pd[p];
    const int n = d.n, m = d.m;
    if (d.lane) return;
    const int tid = threadIdx.x, idx = blockIdx.x * 256 + tid;
    if (idx < (n + m + 15) / 16) ops[d.ops_off + idx] = 0u;
    if (n == 0 || m == 0) return;
    const int K = (n + ROWS - 1) / ROWS;
    if (K < 3) return;  // walked whole by the emit kernel
    const int nx = m + 1, nxc = (nx + 255) / 256, nbt = (n + 63) / 64;  // bands 1 .. nbt-1 are mapped
    const int blk = blockIdx.x;
    if (blk >= (nbt - 1) * nxc) return;
    const int g = 1 + blk / nxc, x0 = (blk % nxc) * 256;
    const int k = g / NB, t0 = (g % NB) * NL;  // the band's stripe and first forward lane
    const int SG = (m + 63 + G - 1) / G * G;
    const uint64_t stripe_words = (uint64_t)(SG / G) * 256u;
    int j = x0 + tid, i = min(64 * (g + 1), n);
    const bool live = j <= m;
    // stage the band's lanes of the groups of steps s = j' - 1 + t, j' in [x0 - LEFT, x0 + 255], t in [0, 63]
    const uint32_t *tbk = tb + d.tb_off + (uint64_t)k * stripe_words;
    const int s_lo = max(0, x0 - LEFT - 1), s_hi = min(SG - 1, x0 + 255 + 63);
    const int sg_lo = s_lo >> LG, nsg = min(NSG, (s_hi >> LG) - sg_lo + 1);
    const uint4 *src = reinterpret_cast<const uint4 *>(tbk) + (uint64_t)sg_lo * 64u + t0;
    {  // as in the stripe map kernel: every load in flight before the first wait
        uint4 v[NIT];
#pragma unroll
        for (int u = 0; u < NIT; ++u) {
            const int e = tid + 256 * u;
            v[u] = src[e < nsg * NL ? (e / NL) * 64 + (e % NL) : 0];
        }
#pragma unroll
        for (int u = 0; u < NIT; ++u) stage[tid + 256 * u] = v[u];
    }
    __syncthreads();
    if (!live) return;
    const int top = 64 * g;  // row top belongs to band g - 1
    uint32_t cnt = 0, run = 0;  // run: consecutive inserts
    const uint32_t cap = SED_TBMAP_CAP ? (uint32_t)SED_TBMAP_CAP + 64u * (uint32_t)((m + n - 1) / n) : 0xFFFFFFFFu;
    for (;;) {  // the stripe map kernel's loop on the band's staged lanes
        const int rr = i - 1, t = (rr >> LR) & 63, r = rr & (R - 1);
        const int s = j - 1 + t;
        const uint32_t c = ((uint32_t)(s & (G - 1)) << LR) | (uint32_t)r;
        const uint32_t rel = (uint32_t)((s >> LG) - sg_lo);
        const bool inside = rel < (uint32_t)nsg;
        // (t - t0) & (NL - 1): the read after the exit row (t outside the band) stays inside the staged lanes
        const uint32_t word = stage32[(inside ? rel : 0u) * (NL * 4u) + ((uint32_t)(t - t0) & (NL - 1u)) * 4u + (c >> 4)];
        if (!((i > top) & (j > 0) & inside & (run <= SED_TBMAP_RUN) & (cnt < cap))) break;
        const uint32_t op = ((word >> (2u * (c & 15u))) - (uint32_t)(pat >> (4 * (i & (P - 1))))) & 3u;
        ++cnt;
        run = op == 0u ? run + 1u : 0u;
        i -= (int)(op != 0u);
        j -= (int)(op != 1u);
    }
    if (i > top) {
        if (j == 0) {  // the column-0 border: deletes up to the band above
            cnt += (uint32_t)(i - top);
        } else {  // unknown (see the stripe map kernel)
            j = -1;
            cnt = 0;
        }
    }
    uint32_t *mp = map + (uint32_t)d.map_off + 2u * ((uint32_t)K * (uint32_t)nx + (uint32_t)(g - 1) * (uint32_t)nx + (uint32_t)(x0 + tid));
    mp[0] = (uint32_t)j;
    mp[1] = cnt;
}

// The stripe map from the band maps: one thread per (stripe k in 1 .. K-2, column x), chaining the stripe's NB
// bands from its last row, and one for the sink's stripe, from the sink (stored at x = 0, as the stripe map kernel
// does).  Unknown if any band on the chain is.
template <int R>
__global__ __launch_bounds__(256) void sed_tb_bandcompose_kernel(const sed_pair_desc *__restrict__ pd,
                                                                 uint32_t *__restrict__ map) {
    constexpr int ROWS = 64 * R, NB = R;
    const int p = blockIdx.y;
    const sed_pair_desc d = pd[p];
    const int n = d.n, m = d.m;
    if (d.lane || n == 0 || m == 0) return;
    const int K = (n + ROWS - 1) / ROWS;
    if (K < 3) return;
    const int nx = m + 1, idx = blockIdx.x * 256 + threadIdx.x;
    if (idx > (K - 2) * nx) return;
    int k, g, x;
    uint32_t slot;
    if (idx == (K - 2) * nx) {  // the sink: from (n, m) in the band holding row n
        k = K - 1;
        g = (n - 1) / 64;
        x = m;
        slot = (uint32_t)k * nx;
    } else {
        k = 1 + idx / nx;
        x = idx % nx;
        g = (k + 1) * NB - 1;
        slot = (uint32_t)k * nx + x;
    }
    uint32_t *mp = map + (uint32_t)d.map_off;
    const uint32_t *bm = mp + 2u * (uint32_t)K * nx;
    uint32_t cnt = 0;
    for (; g >= k * NB; --g) {
        const uint32_t e = 2u * ((uint32_t)(g - 1) * nx + (uint32_t)x);
        const uint32_t xn = bm[e];
        if (xn == 0xFFFFFFFFu) {
            x = -1;
            cnt = 0;
            break;
        }
        cnt += bm[e + 1u];
        x = (int)xn;
    }
    mp[2u * slot] = (uint32_t)x;
    mp[2u * slot + 1u] = cnt;
}

// The exit column and op count of stripe k's segment from cell (i, j), walked here (entries the map kernel left
// unknown); wave-uniform, codes read one word per step
template <int R>
__device__ __forceinline__ uint2 ck_count_walk(const sed_pair_desc &d, const uint32_t *__restrict__ tb, const uint64_t pat,
                                               const int k, int i, int j, int top = -1) {
    constexpr int ROWS = 64 * R, G = Grp<R>::G, LG = CodeCursor<R>::LG, LR = CodeCursor<R>::LR, P = Ladder<R>::P;
    const int SG = (d.m + 63 + G - 1) / G * G;
    const uint32_t *tbk = tb + d.tb_off + (uint64_t)k * (uint64_t)(SG / G) * 256u;
    if (top < 0) top = k * ROWS;  // (else a band's top row inside stripe k)
    uint32_t cnt = 0;
    while (i > top) {
        if (j == 0) {
            cnt += (uint32_t)(i - top);
            break;
        }
        const int rr = i - 1, t = (rr >> LR) & 63, r = rr & (R - 1);
        const int s = j - 1 + t;
        const uint32_t c = ((uint32_t)(s & (G - 1)) << LR) | (uint32_t)r;
        const uint32_t word = tbk[((uint64_t)(s >> LG) * 64u + t) * 4u + (c >> 4)];
        const uint32_t op = ((word >> (2u * (c & 15u))) - (uint32_t)(pat >> (4 * (i & (P - 1))))) & 3u;
        ++cnt;
        i -= (int)(op != 0u);
        j -= (int)(op != 1u);
    }
    return make_uint2((uint32_t)j, cnt);
}

// One wave per (pair, stripe): its segment of the canonical path, from the composed maps (see above; entries the map left unknown are walked here)
template <int R>
__global__ __launch_bounds__(64) void sed_tb_stripeemit_kernel(const sed_pair_desc *__restrict__ pd,
                                                               const uint32_t *__restrict__ tb,
                                                               sed_result *__restrict__ res,
                                                               uint32_t *__restrict__ ops,
                                                               const uint32_t *__restrict__ map, const uint64_t pat) {
    constexpr int ROWS = 64 * R;
    const int lane = threadIdx.x;
    const int pair = __builtin_amdgcn_readfirstlane(blockIdx.x), kme = __builtin_amdgcn_readfirstlane(blockIdx.y);
    const sed_pair_desc d = pd[pair];
    if (d.lane) return;
    const int n = d.n, m = d.m;
    const int K = n > 0 ? (n + ROWS - 1) / ROWS : 1;
    const int Keff = (K >= 3 && m > 0) ? K : 1;  // pairs of one or two stripes: one segment, the whole walk
    if (kme >= Keff) return;
    const uint32_t L = (uint32_t)__builtin_amdgcn_readfirstlane(res[pair].len);
    int i0 = n, j0 = m;
    uint32_t qhi = L, cnt = L;  // cnt: the ops of this segment
    if (Keff > 1) {
        const uint32_t nx = (uint32_t)m + 1u;
        const uint32_t *mp = map + (uint32_t)d.map_off;
        uint32_t x = mp[2u * ((uint32_t)(K - 1) * nx)];
        cnt = mp[2u * ((uint32_t)(K - 1) * nx) + 1u];
        if (x == 0xFFFFFFFFu) {  // the sink's walk left its staged columns
            const uint2 w = ck_count_walk<R>(d, tb, pat, K - 1, n, m);
            x = w.x;
            cnt = w.y;
        }
        for (int kk = K - 2; kk >= kme; --kk) {  // down to this stripe: its entry column and script positions
            qhi -= cnt;
            const uint32_t e = 2u * ((uint32_t)kk * nx + x);
            if (kk > 0) {
                i0 = (kk + 1) * ROWS;
                j0 = (int)x;
                uint32_t xn = mp[e];
                cnt = mp[e + 1u];
                if (xn == 0xFFFFFFFFu) {
                    const uint2 w = ck_count_walk<R>(d, tb, pat, kk, i0, j0);
                    xn = w.x;
                    cnt = w.y;
                }
                x = xn;
            } else {  // stripe 0: to the origin, whatever is left
                cnt = qhi;
                i0 = ROWS;
                j0 = (int)x;
            }
        }
    }
    const int istop = (Keff == 1 || kme == 0) ? 0 : kme * ROWS;
    uint32_t bad = 0;
    const uint32_t q = window_walk<R, true>(d, i0, j0, istop, qhi, lane, tb, ops + d.ops_off, pat, bad);
    if ((bad || q != qhi - cnt) && lane == 0) res[pair].err = SED_ERR_TB_LENGTH;
}

// Banded emit (round 6, SED_TB_BANDEMIT = 1, the default): one wave per (pair, 64-row band) instead of per stripe, so
// a wave walks one band's segment of the path (~1/R of a stripe's).  The wave composes the stripe maps from the sink
// down to its band's stripe, then that stripe's band maps down to its band (entries the maps left unknown are walked
// here, ck_count_walk), and walks its segment to the band's top row (band 0: to the origin) with the window walk,
// ORing its script words into the zeroed buffer as the stripe emit does.
#ifndef SED_TB_BANDEMIT
#define SED_TB_BANDEMIT 1
#endif
template <int R>
__global__ __launch_bounds__(64) void sed_tb_bandemit_kernel(const sed_pair_desc *__restrict__ pd,
                                                             const uint32_t *__restrict__ tb,
                                                             sed_result *__restrict__ res,
                                                             uint32_t *__restrict__ ops,
                                                             const uint32_t *__restrict__ map, const uint64_t pat) {
    constexpr int ROWS = 64 * R, NB = R;
    const int lane = threadIdx.x;
    const int pair = __builtin_amdgcn_readfirstlane(blockIdx.x), gme = __builtin_amdgcn_readfirstlane(blockIdx.y);
    const sed_pair_desc d = pd[pair];
    if (d.lane) return;
    const int n = d.n, m = d.m;
    const int K = n > 0 ? (n + ROWS - 1) / ROWS : 1;
    const bool multi = K >= 3 && m > 0;  // pairs of one or two stripes: one segment, the whole walk (band 0's wave)
    const int nbt = multi ? (n + 63) / 64 : 1;
    if (gme >= nbt) return;
    const uint32_t L = (uint32_t)__builtin_amdgcn_readfirstlane(res[pair].len);
    int i0 = n, j0 = m;
    uint32_t qhi = L, cnt = L;  // cnt: the ops of this segment
    if (multi) {
        const uint32_t nx = (uint32_t)m + 1u;
        const uint32_t *mp = map + (uint32_t)d.map_off;
        const uint32_t *bm = mp + 2u * (uint32_t)K * nx;
        const int kme = gme / NB;
        uint32_t x = (uint32_t)m;
        for (int kk = K - 1; kk > kme; --kk) {  // whole stripes above this band's: from the sink's
            const uint32_t e = kk == K - 1 ? 2u * ((uint32_t)(K - 1) * nx) : 2u * ((uint32_t)kk * nx + x);
            uint32_t xn = mp[e], c = mp[e + 1u];
            if (xn == 0xFFFFFFFFu) {
                const uint2 w = ck_count_walk<R>(d, tb, pat, kk, i0, (int)x);
                xn = w.x;
                c = w.y;
            }
            qhi -= c;
            x = xn;
            i0 = kk * ROWS;
        }
        for (int g = (i0 - 1) / 64; g >= gme; --g) {  // bands of this stripe from its entry: the last one is this band's
            uint32_t xn, c;
            if (g == 0) {  // band 0: to the origin, whatever is left
                xn = 0u;
                c = qhi;
            } else {
                const uint32_t e = 2u * ((uint32_t)(g - 1) * nx + x);
                xn = bm[e];
                c = bm[e + 1u];
                if (xn == 0xFFFFFFFFu) {
                    const uint2 w = ck_count_walk<R>(d, tb, pat, kme, i0, (int)x, 64 * g);
                    xn = w.x;
                    c = w.y;
                }
            }
            if (g == gme) {
                cnt = c;
                break;
            }
            qhi -= c;
            x = xn;
            i0 = 64 * g;
        }
        j0 = (int)x;
    }
    const int istop = multi ? 64 * gme : 0;
    uint32_t bad = 0;
    const uint32_t q = window_walk<R, true>(d, i0, j0, istop, qhi, lane, tb, ops + d.ops_off, pat, bad);
    if ((bad || q != qhi - cnt) && lane == 0) res[pair].err = SED_ERR_TB_LENGTH;
}


// ---------------------------------------------------------------------------
// Traceback from checkpoints (CK: script batches of the stripe and CHAIN kernels with R = 4, 8 or 16 rows
// per lane, G = 64/R).  One wave per pair walks the canonical path back from (n, m) tile by tile.  A tile
// is 64 rows (forward lanes GQ .. GQ+G-1 of a stripe, the tile's G bands of R rows) x the 64 columns those
// lanes processed in one chunk c, a staircase: band t = GQ + b covers columns 64c - t + 1 .. 64c - t + 64.
// Entering a tile, the wave recomputes it from
//   - the column checkpoints of chunk c-1 (each band's R row values at column 64c - t, and the value
//     above the band at that column), or the column-0 borders for c = 0;
//   - the row above the tile: the row checkpoints of lane GQ-1 (or lane 63 of the stripe above, or
//     row 0), read through LDS by lane 0;
// with one lane per row (row r at sweep step sigma is at column J0 - (G-1) + sigma - r, J0 = 64c - GQ + 1;
// the cell above arrives through the DPP chain from lane r - 1, the str2 selector from LDS).  The forward kernel
// stores distance keys (D, L without the op); every checkpoint value is converted on load to the
// traceback key of the same (D, L) (i32_dist_to_tb), whose min carries the canonical op in its low two
// bits: 6 VALU per cell (v_add_u32_dpp for the cell above + 1, perm, add, min3, and, alignbit).  Lanes of
// band b hold their checkpoint until their first column (step r - b + G - 1: one v_cndmask on a scalar
// mask) and read code 3 there (outside the band's window, OR-ed in per word); the first row of bands
// 1..G-1 takes its first diagonal from the checkpoint; columns < 1 get the sentinel selector, so they keep
// the column-0 border.  The sweep stops after the 16-step word holding the entry cell's step (the path only
// goes up and left), and the entry cell's key must carry the path length still to emit: a mismatch (a
// corrupted checkpoint, SED_OPT_DEBUG_CORRUPT) sets res.err instead of writing a wrong script.  Codes stay
// in registers, 16 steps per word.  The walk is scalar: one v_readlane per step and the state packed as
// S = row + (step << 7), 10 SALU per step (a step moves S by 128 / 129 / 257 for insert / delete /
// update; one masked compare catches leaving the word, the tile (bit 6 = above it) and the window (code
// 3)), one unrolled copy per code word since the step only decreases.
// ---------------------------------------------------------------------------
// S decrement per code: insert 128, delete 129, update 257 (S = row | step << 7); the marker 3 (left of the
// band's window) moves S by 0x8000, out of every word, and is taken back at the exit.  Only the low 16 bits of S
// are kept: a move subtracts the next code's field << 16 as well.
#define SED_TB_MOVES (128ull | (129ull << 16) | (257ull << 32) | (0x8000ull << 48))
#define SED_TB_WORD 0xF840u  // S bits that change when the walk leaves a 16-step word or the tile (bit 6: above it)
// The walk of one tile from state S; returns the state of the first cell it did not take (outside the
// tile: above it, left of its band's window, or at column 0 for C0), low 16 bits.  One loop per code word with a
// single exit test: the next state's word bits (S & SED_TB_WORD) must still be the word's tag.
template <bool C0, int NW>  // C0: chunk-0 tile, whose window reaches the column-0 border: stop at j = 0
__device__ __forceinline__ uint32_t ck_walk(const uint32_t (&W)[NW], uint32_t S, uint32_t &q, uint64_t &acc,
                                            uint32_t &err, uint32_t *__restrict__ out, int jcol) {
    static_assert(NW <= 15, "the step field (S bits 7..14) and the word tags need a free bit 15");
#pragma unroll
    for (int w = NW - 1; w >= 0; --w) {
        const uint32_t tag = (uint32_t)w << 11;
        if ((S & SED_TB_WORD) == tag) {
            // Every op moves the walk at least one step left, so one word yields at most 16 ops.  Inside the loop
            // the state is carried as T = S - tag (same low 11 bits: lane and shift), so leaving the word, the tile or
            // the window is (T & SED_TB_WORD) != 0, one s_and that sets SCC; the codes collect in a 32-bit lo
            // (s_lshl2_add_u32), which holds all of them, and go onto the 64-bit acc (the last 32 ops) after the
            // loop, where the script word completed in it, if any, is stored.  A step is one v_readlane and 10 SALU.
            const uint32_t qs = q;
            uint32_t T = S - tag, lo = 0, code;
            do {
                // s_lshr takes the low 5 bits of T >> 6: 2 * (step & 15), bit 6 being clear inside the tile
                code = ((uint32_t)__builtin_amdgcn_readlane((int)W[w], (int)T) >> ((T >> 6) & 31u)) & 3u;
                if (C0 && jcol == 0) code = 3u;
                // the marker too: taken back below (asm: the compiler emits s_lshl + s_or; the op writes SCC)
                asm("s_lshl2_add_u32 %0, %1, %2" : "=s"(lo) : "s"(lo), "s"(code) : "scc");
                if constexpr (C0) jcol -= (int)((5u >> code) & 1u);
                T -= (uint32_t)(SED_TB_MOVES >> (code << 4));
                --q;
            } while ((T & SED_TB_WORD) == 0u);
            S = T + tag;
            const bool marker = code == 3u;
            // opaque: otherwise the compiler keeps the previous lo and q alive through the loop for the undo
            asm volatile("" : "+s"(lo), "+s"(q));
            if (marker) {  // not an op: the walk stays at the cell before it
                lo >>= 2;
                ++q;
            }
            // lo started at 0 and holds exactly this word's ops (at most 16)
            const uint32_t nw = qs - q;
            acc = (acc << (2u * nw)) | lo;
            // the script word [p, p + 16) completed in this word, if any: [q, qs) holds at most 16 positions, so at most
            // one p = 16k with q <= p < qs
            const uint32_t p = (q + 15u) & ~15u;
            if ((int32_t)nw < 0) err = SED_ERR_TB_LENGTH;  // ran past the sink's L (q wrapped; the tile bounds the walk)
            else if (p < qs) out[p >> 4] = (uint32_t)(acc >> (2u * (p - q)));
            if (marker) return (S + 0x8000u) & 0xFFFFu;
        }
    }
    return S & 0xFFFFu;
}

// SED_CK_VHOLD (default on; -DSED_CK_VHOLD=0 restores the select): at R = 16 lanes left of their window hold
// their key without a select (per-band selector copies carry the sentinel, and each band's first row takes a
// compensated delete addend until its band starts).  6 VALU per swept cell instead of 7; profiles/r03/vhold:
// traceback 3.78 against 3.91 ms beside the forward parts, step within noise
#ifndef SED_CK_VHOLD
#define SED_CK_VHOLD 1
#endif
// NW code words per lane cover sweep steps 0 .. 16 NW - 1: 8 for one chunk's tile (127 steps), 12 for a wide window
// of two chunks (191 steps); topb holds 16 NW + 4 words, each band's selector copy 64 more
#define SED_CK_NX(NW) (16 * (NW) + 4)
#define SED_CK_SELB(NW) (64 + SED_CK_NX(NW))
template <int R> struct CkVHold { static constexpr bool value = SED_CK_VHOLD && R == 16; };
// lanes 0 .. n-1 have reached their window at sweep step sig (sig0(r) = r - r/R + G - 1 is nondecreasing)
template <int R> constexpr int ck_active_lanes(int sig) {
    constexpr int G = 64 / R;
    int n = 0;
    for (int r = 0; r < 64; ++r)
        if (r - r / R + G - 1 <= sig) n = r + 1;
    return n;
}
// lanes >= act keep v, the others take vn: the mask is built on the scalar unit inside the asm, so the
// compiler can neither hoist the 60-odd constant masks (they spill) nor turn them into a VALU compare
__device__ __forceinline__ uint32_t ck_hold(uint32_t vn, uint32_t v, const int act) {
    uint32_t r;
    uint64_t m;
    // (s_lshl_b64 writes SCC: without the clobber a compare's SCC could be read across the asm)
    asm("s_lshl_b64 %1, -1, %4\n\tv_cndmask_b32 %0, %2, %3, %1" : "=v"(r), "=&s"(m) : "v"(vn), "v"(v), "i"(act) : "scc");
    return r;
}

// band b >= 1 of a tile starts (its first row takes the checkpoint's top_prev as diagonal) at sweep step
// (R - 1) b + G - 1; returns b, or 0 when `sig` starts no band
template <int R> constexpr int ck_band_start(int sig) {
    constexpr int G = 64 / R;
    for (int b = 1; b < G; ++b)
        if (sig == (R - 1) * b + G - 1) return b;
    return 0;
}

// f(integral_constant<int, I>) for I = B .. E-1, expanded at compile time
template <int B, int E, class F> __device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// a word at a 32-bit byte offset from a uniform base: the scalar-base (saddr) load form, no 64-bit lane address
__device__ __forceinline__ uint32_t ld_byte_off(const uint32_t *__restrict__ base, const uint32_t off) {
    return *(const uint32_t *)((const char *)base + off);
}

// LDS ordering inside the traceback: a workgroup barrier for the one-wave traceback kernel; WAVE: a wave-local
// wait, for a traceback run by a wave of a larger workgroup (LDS accesses of one wave execute in order; the
// clobber keeps the compiler from moving them across).  Fusing the traceback into the CK forward kernel this way
// (each wave walks its pair after its forward pass) measured 13.9-14.0 ms per config-4 step against 13.87 ms
// for the separate kernel (profiles/r02/abfuse), so the traceback stays a kernel of its own.
template <bool WAVE> __device__ __forceinline__ void ck_sync() {
    if constexpr (WAVE) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else __syncthreads();
}

// topb[x] (132 words): the row above the tile at lane 0's column of step x, plus 1 (lane 0's delete candidate);
// selb[64 + x] (196 words): str2 selector of lane 0's column at step x; lane r reads selb[64 + sigma - r] itself
// (its column at step sigma), so no selector travels through the DPP chain.  q0: the sink's L.
// Per-pair constants of the checkpoint tiles.  ckoff: word offset of the checkpoints past d.tb_off (SPLIT batches keep
// them after the pair's per-cell code region, sed_ck_codes_kernel).
struct CkPairCtx {
    int n, m, SG, nchunks, ngroups, band;
    const uint32_t *ccp, *rcp, *pa, *pb;
    uint32_t cko0, cko1, hm[4];
};
template <int R>
__device__ __forceinline__ CkPairCtx ck_pair_ctx(const sed_pair_desc &d, const int lane, const uint32_t *__restrict__ seqa,
                                                 const uint32_t *__restrict__ seqb, const uint32_t *__restrict__ ck,
                                                 const uint64_t ckoff) {
    constexpr int ROWS = 64 * R, G = Grp<R>::G;
    constexpr int LR = R == 4 ? 2 : R == 8 ? 3 : 4;
    CkPairCtx px;
    px.n = d.n;
    px.m = d.m;
    const int nstripes = (d.n + ROWS - 1) / ROWS;
    px.SG = (d.m + 63 + G - 1) / G * G;
    px.nchunks = (px.SG + 63) >> 6;
    px.ngroups = px.SG / G;
    px.ccp = ck + d.tb_off + ckoff;
    px.rcp = px.ccp + sed_ck_col_words(R, nstripes, px.nchunks);
    px.pa = seqa + d.a_off;
    px.pb = seqb + d.b_off;
    px.band = lane >> LR;
    px.cko0 = ((uint32_t)(lane & (R - 1)) * 64u + (uint32_t)px.band) * 4u;
    px.cko1 = (uint32_t)(R * 64 + px.band) * 4u;
    const int sig0 = lane - px.band + G - 1;  // first real sweep step of this lane (<= 63)
    // code 3 (outside the window) for the steps before sig0, OR-ed into words 0..3 once they are complete
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int h = min(max(sig0 - 16 * w, 0), 16);
        px.hm[w] = h >= 16 ? ~0u : (1u << (2 * h)) - 1u;
    }
    return px;
}

// One tile visit: tile (stripe k, band group Q, chunk c) recomputed from its checkpoints up to sweep step sig_end (FULL:
// all 128 steps), the codes in W (lane r's code of step sigma in W[sigma >> 4], bits 2 (sigma & 15)); returns the lanes'
// keys after the last step (the entry keys).
template <int R, bool WAVE, bool FULL, int NW>
__device__ __forceinline__ uint32_t ck_tile_sweep(const CkPairCtx &px, const int lane, const sed_i32_params &prm,
                                                  uint32_t *__restrict__ topb, uint32_t *__restrict__ selb, const int k,
                                                  const int Q, const int c, const int sig_end, uint32_t &one,
                                                  uint32_t (&W)[NW], uint32_t &vinit) {
    constexpr int NX = SED_CK_NX(NW), SELB = SED_CK_SELB(NW), NH = (NX + 63) / 64;
    constexpr int ROWS = 64 * R, G = Grp<R>::G;  // a tile: G forward lanes (bands) of R rows
    constexpr int LR = R == 4 ? 2 : R == 8 ? 3 : 4;
    constexpr bool VHOLD = CkVHold<R>::value;
    const int n = px.n, m = px.m, SG = px.SG, nchunks = px.nchunks, ngroups = px.ngroups, band = px.band;
    const int J0 = 64 * c - G * Q + 1, rowbase = k * ROWS + 64 * Q;
    // ---- boundaries (distance keys -> traceback keys) ----
    // Every load of the tile is issued before the first use (one memory round trip per tile visit): addresses
    // are clamped to valid words and the border cases are selects afterwards.
    const int ir = min(rowbase + lane, n - 1);  // 0-based str1 index of this lane's row (clamped)
    const uint32_t wa = px.pa[ir >> 4];
    // (uniform 64-bit bases + 32-bit lane offsets: the loads take the scalar-base form and the address
    // arithmetic stays on the scalar unit)
    uint32_t ck0 = 0, ck1 = 0;
    if (c >= 1) {  // (uniform)
        const uint32_t *cp = px.ccp + sed_ck_col_word(R, k, nchunks, c - 1, 0, G * Q);
        uint32_t o0 = px.cko0, o1 = px.cko1;
        asm volatile("" : "+v"(o0), "+v"(o1));  // (else the zero-extended offsets are hoisted as 64-bit pairs)
        ck0 = ld_byte_off(cp, o0);
        ck1 = ld_byte_off(cp, o1);
    }
    // the row above the tile at column J0 - G + x (x = lane, lane + 64, lane + 128 < 132): row checkpoints of
    // forward lane G*Q - 1 (or lane 63 of the stripe above); steps clamped: past SG the columns are beyond m and
    // never read by the walk; columns < 1 are the column-0 border (a CHAIN wave's lanes still hold the
    // previous pair there)
    const bool above = Q >= 1 || k >= 1;  // (uniform) else row 0: the border
    const int kr = Q >= 1 ? k : k - 1, tr = Q >= 1 ? G * Q - 1 : 63, s0r = Q >= 1 ? 64 * c - G - 1 : 64 * c + 63 - G;
    uint32_t rk[NH], wb[NH];
    const uint32_t *rbase = px.rcp + sed_ck_row_word(R, max(kr, 0), ngroups, 0, tr);  // (uniform; read when above)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int x = lane + 64 * h;
        rk[h] = 0u;
        // (a visit reads the top row and selectors of steps <= sig_end + 1 only: the blocks past it are skipped, a
        // uniform branch; the entry word's reads past sig_end see unused words)
        if ((FULL || 64 * h <= sig_end + 1) && (64 * (h + 1) <= NX || x < NX)) {
            if (above) {
                const uint32_t s = (uint32_t)min(max(s0r + x, 0), SG - 1);
                rk[h] = ld_byte_off(rbase, ((s >> (6 - LR)) * (uint32_t)SED_CK_RW + (s & (uint32_t)(G - 1))) * 4u);
            }
            const int ci = min(max(J0 - (G - 1) + x - 1, 0), m - 1);
            wb[h] = px.pb[ci >> 4];
        }
    }
    const uint32_t a = (wa >> ((ir & 15) * 2)) & 3u;
    const uint32_t clo = (a & 1u) ? prm.costrow[1] : prm.costrow[0];
    const uint32_t chi = (a & 1u) ? prm.costrow[3] : prm.costrow[2];
    const uint32_t cv = (a & 2u) ? chi : clo;
    uint32_t V = SED_KB, tp = SED_KB;  // c = 0: the column-0 borders
    if (c >= 1) {
        V = ck_to_tb(ck0, prm);
        tp = ck_to_tb(ck1, prm);
        if (VHOLD && J0 - band - 1 > m) V = 0u;  // (forward garbage past m: key 0 holds under the recurrence)
    }
    tp += 1u;  // diagonals carry the +1 of the delete candidate they were taken from
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int x = lane + 64 * h;
        if ((FULL || 64 * h <= sig_end + 1) && (64 * (h + 1) <= NX || x < NX)) {
            const uint32_t v = (above && J0 - G + x >= 1) ? ck_to_tb(rk[h], prm) : SED_KB;
            topb[x] = v + 1u;
            const int col = J0 - (G - 1) + x;  // column of lane 0 at step x
            const int ci = min(max(col - 1, 0), m - 1);
            const uint32_t sv = col < 1 ? SED_SEL_SENT : i32_sel((wb[h] >> ((ci & 15) * 2)) & 3u);
            if constexpr (VHOLD) {  // band b's copy: the sentinel left of its window (x < G - 1 - b)
#pragma unroll
                for (int b = 0; b < G; ++b) selb[b * SELB + 64 + x] = x < G - 1 - b ? SED_SEL_SENT : sv;
            } else {
                selb[64 + x] = sv;
            }
        }
    }
    ck_sync<WAVE>();
    // ---- sweep: lane r at step sigma computes (row rowbase + r + 1, column J0 - (G-1) + sigma - r) ----
    // Whole 16-step words (a branch per step would keep the LDS reads from running ahead), except the
    // word holding the entry step, which stops at it: the lanes' keys are then the entry keys.  The cell above and the diagonal
    // carry the delete candidate's +1 (one v_add_u32_dpp: lane r - 1's key + 1, or topb for lane 0), so
    // the update constant is one less.  Lanes still left of their window (sigma < sig0: lanes
    // ck_active_lanes(sigma) .. 63, a compile-time count) keep their checkpoint through one v_cndmask on a
    // scalar mask; their codes become 3 through hm.  Steps 0 .. G-2 hold every lane and are skipped.
    W[0] = 0u;  // steps 0 .. G-2 are skipped: their bits are OR-ed to 3 from a defined word
    if constexpr (VHOLD) {  // a band's first row: V - V_above + 1 until the band starts
        // (through the asm DPP add: with the builtin, the compiler folded V - dpp(V) into one
        // v_subrev_u32_dpp ... bound_ctrl:1, which returned V_above - V on the device)
        uint32_t zero = 0u;
        asm volatile("" : "+v"(zero));
        const uint32_t vabove = dpp_shr1_add(0u, V, zero);
        one = ((lane & (R - 1)) == 0 && lane > 0) ? V - vabove + 1u : 1u;
    }
#ifdef SED_TB_DEBUG
    vinit = V;
#endif
    uint32_t tprev = dpp_shr1_add(topb[G - 1], V, one);  // diagonal of step G-1 (+1)
    // the top row's reads through one opaque base register and immediate offsets (else every constant address became a
    // VGPR of its own: 28 preloaded at the kernel's start, one more v_mov per two steps of an entry word)
    const uint32_t *topr = topb;
    {
        uint32_t z = 0u;
        asm volatile("" : "+v"(z));
        topr += z;
    }
    const uint32_t *selp = selb + (VHOLD ? band * SELB : 0) + 64 - lane;  // lane r's selector at step sigma
    const int w_end = FULL ? NW - 1 : sig_end >> 4;  // FULL: every word, whole
    auto step = [&](const int sig, uint32_t &wv, const uint32_t topin, const uint32_t selv) {
        if (sig < G - 1) return;  // every lane holds
        const int bs = ck_band_start<R>(sig);  // folds to a constant in the unrolled sweep
        if (VHOLD && bs > 0) one = lane == R * bs ? 1u : one;  // the band starts: its first row's real delete
        const uint32_t topv = dpp_shr1_add(topin, V, one);
        // (selv: steps before the lane's first column read don't-care)
        uint32_t diag = tprev;
        if (bs > 0) diag = lane == R * bs ? tp : diag;
        const uint32_t mm = umin3(V, topv, diag + __builtin_amdgcn_perm(cv, 0xFFFFFFFDu, selv));
        const uint32_t vn = mm & ~3u;
        if constexpr (VHOLD) {
            V = vn;
        } else {
            const int act = ck_active_lanes<R>(sig);  // lanes 0 .. act-1 are inside their window
            V = act >= 64 ? vn : ck_hold(vn, V, act);
        }
        wv = __builtin_amdgcn_alignbit(mm, wv, 2);
        tprev = topv;
    };
    // (the words expand through static_for: a #pragma unroll over 12 words gives up, and the steps' constants with it)
    static_for<0, NW>([&](auto wc) {
        constexpr int w = decltype(wc)::value;
        if (w > w_end) return;  // the path never needs later steps
        if (!FULL && w == w_end) {  // up to the entry step exactly: the lanes then hold the entry keys
            // the word's LDS inputs first (the compiler sinks them into the steps anyway; pinning them ahead of the exits
            // with an asm use measured the same, profiles/r06/ck_wide)
            uint32_t tw[16], sw[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                tw[u] = topr[16 * w + u + 1];
                sw[u] = selp[16 * w + u];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                if (16 * w + u > sig_end) break;
                step(16 * w + u, W[w], tw[u], sw[u]);
            }
            W[w] >>= 2u * (15u - ((uint32_t)sig_end & 15u));  // step u's code to bits 2u, 2u+1
        } else {
#pragma unroll
            for (int u = 0; u < 16; ++u) step(16 * w + u, W[w], topr[16 * w + u + 1], selp[16 * w + u]);
        }
        if (w < 4) W[w] |= px.hm[w];
    });
    return V;
}

template <int R, bool WAVE, int NW>
__device__ __forceinline__ void ck_traceback_pair(const sed_pair_desc &d, const int pair, const uint32_t q0,
                                                  const int lane, const uint32_t *__restrict__ seqa,
                                                  const uint32_t *__restrict__ seqb, const uint32_t *__restrict__ ck,
                                                  sed_result *__restrict__ res, uint32_t *__restrict__ ops,
                                                  const sed_i32_params &prm, uint32_t *__restrict__ topb,
                                                  uint32_t *__restrict__ selb) {
    constexpr int ROWS = 64 * R, G = Grp<R>::G;  // a tile: G forward lanes (bands) of R rows
    static_assert(R == 4 || R == 8 || R == 16, "R in {4, 8, 16}");
    const int n = d.n, m = d.m;
#ifdef SED_TB_DEBUG
    int visit = 0;  // debug dumps: 136 words per tile visit (entry keys, initial keys, coordinates)
#endif
    uint32_t *out = ops + d.ops_off;
#ifndef SED_TB_DEBUG
    zero_script_tail(out, (int)q0, n, m, lane, 64);  // (before the walk, as sed_traceback_kernel)
#endif
    uint32_t q = q0, err = 0;
    uint64_t acc = 0;  // the last 32 ops, the latest (position q) in bits 1:0
    auto emit = [&](uint32_t op) {  // sink -> origin (trailing border runs)
        if (q == 0) {
            err = SED_ERR_TB_LENGTH;
            return;
        }
        acc = (acc << 2) | op;
        if ((--q & 15u) == 0) out[q >> 4] = (uint32_t)acc;
    };
    const uint32_t Kd = (prm.del << 16) + 4u, Ki = (prm.ins << 16) + 4u;
    int i = n, j = m;
    if (i > 0 && j > 0) {
        const CkPairCtx px = ck_pair_ctx<R>(d, lane, seqa, seqb, ck, 0);
        uint32_t one = 1u;  // the delete candidate's +1, a VGPR operand of v_add_u32_dpp
        asm volatile("" : "+v"(one));
        int guard = 2 * (n + m) + 8;       // tiles visited; every visit makes progress
        while (i > 0 && j > 0) {
            if (--guard <= 0) {
                err = SED_ERR_TB_GUARD;
                break;
            }
            const int k = (i - 1) / ROWS, t = ((i - 1) % ROWS) / R, Q = t / G;
            const int ce = (j - 1 + t) >> 6;            // the entry cell's chunk
            const int rowbase = k * ROWS + 64 * Q;
            const int re = i - rowbase - 1;             // the entry cell's tile row
            // NW = 12: a window of two chunks (ce - 1, ce) when the entry step x inside its chunk is below re, i.e. when
            // a diagonal path would leave chunk ce through its left edge before the tile's top: the path then crosses
            // the row group in one visit instead of two, 151 against 93 sweep steps per visit but half the visits
            // (22.3 -> 17.1 VALU per emitted op on config 4's pairs, tools/tb_window_model.py)
            const int c = (NW > 8 && ce >= 1 && ((j - 1 + t) & 63) < re) ? ce - 1 : ce;
            const int J0 = 64 * c - G * Q + 1;
            const int sig_end = (j - J0 + G - 1) + re;  // the entry cell's sweep step (<= 16 NW - 2)
            uint32_t W[NW], vinit = 0;
            const uint32_t ent = ck_tile_sweep<R, WAVE, false, NW>(px, lane, prm, topb, selb, k, Q, c, sig_end, one, W, vinit);
            (void)vinit;
#ifdef SED_TB_DEBUG
            if (visit < 32) {  // debug builds only (pair 0; its script words, 64 spare, then 136 words per visit v)
                uint32_t *dv = out + ((n + m + 15) >> 4) + 64 + 136 * visit;
                dv[lane] = ent;
                dv[64 + lane] = vinit;
                if (lane == 0) {
                    dv[128] = (uint32_t)i; dv[129] = (uint32_t)j; dv[130] = (uint32_t)c; dv[131] = (uint32_t)Q;
                    dv[132] = (uint32_t)k; dv[133] = (uint32_t)sig_end; dv[134] = (uint32_t)re; dv[135] = q;
                }
            }
            ++visit;
#endif
            // ---- the entry cell's key must carry the ops still to emit (L of a canonical-path cell) ----
            {
                const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)ent, re) - SED_KB + (uint32_t)i * Kd +
                                   (uint32_t)j * Ki;
                if (((v >> 2) & 0x3FFFu) != q) {
                    err = SED_ERR_TB_CHECK;
                    break;
                }
            }
            // ---- walk inside the tile ----
            const uint32_t qin = q;
            const uint32_t S0 = (uint32_t)re | ((uint32_t)sig_end << 7);
            const uint32_t S = c == 0 ? ck_walk<true, NW>(W, S0, q, acc, err, out, j)
                                      : ck_walk<false, NW>(W, S0, q, acc, err, out, j);
            if (err) break;
            if (q == qin) {  // no progress: give up rather than spin
                err = SED_ERR_TB_STALL;
                break;
            }
            const int sg = (int)((S + 64u) >> 7), r = (int)((S + 64u) & 127u) - 64;
            i = rowbase + r + 1;
            j = J0 - (G - 1) + sg - r;
            ck_sync<WAVE>();  // topb / selb are rewritten for the next tile
        }
    }
    if (!err) {
        while (j > 0) { emit(0u); --j; }
        while (i > 0) { emit(1u); --i; }
        if (q != 0) err = SED_ERR_TB_LENGTH;
    }
#ifdef SED_TB_DEBUG
    if (lane == 0) out[((n + m + 15) >> 4) + 63] = err | ((uint32_t)visit << 8);  // (debug: no error, the dumps stay)
#else
    if (err && lane == 0) res[pair].err = (uint8_t)err;
#endif
}

// waves per SIMD the checkpoint traceback is compiled for (A/B: SED_CKTB_WAVES; 1 = the compiler's choice: 128 VGPRs and
// 4 waves with the two-chunk windows, whose c4 traceback span was 3.2-3.3 against 2.06 ms at 5 waves / 96 VGPRs, no
// spills; profiles/r06/ck_wide), and its
// waves' issue priority against the other part's forward waves on the same SIMD (SED_CKTB_PRIO, s_setprio).  At
// priority 1 the traceback's waves issue ahead of the forward's when both are ready, so a part's traceback ends
// sooner beside the other part's forward and the step's tracebacks-only tail shrinks from ~0.5 to ~0.13 ms: c4
// 9.74-9.79 against 9.91-9.98 ms at 0, 3 interleaved rounds (profiles/r05/s15; 3 is no different from 1).  With the
// two-chunk windows: 0 9.70-9.74 against 9.55-9.60 ms; 2 and 3 within noise of 1 over 4 rounds (profiles/r06/ckprio)
#ifndef SED_CKTB_WAVES
#define SED_CKTB_WAVES 5
#endif
#ifndef SED_CKTB_PRIO
#define SED_CKTB_PRIO 1
#endif
// code words per lane of the checkpoint traceback's sweep: 12 = two-chunk windows where they pay (ck_traceback_pair), 8 =
// one chunk per visit
#ifndef SED_CKTB_NW
#define SED_CKTB_NW 12
#endif
template <int R>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SED_CKTB_WAVES))) void sed_traceback_ck_kernel(const sed_pair_desc *__restrict__ pd, int npairs,
                                                              const uint32_t *__restrict__ seqa,
                                                              const uint32_t *__restrict__ seqb,
                                                              const uint32_t *__restrict__ ck,
                                                              sed_result *__restrict__ res,
                                                              uint32_t *__restrict__ ops, sed_i32_params prm) {
    if constexpr (SED_CKTB_PRIO > 0) __builtin_amdgcn_s_setprio(SED_CKTB_PRIO);
    const int lane = threadIdx.x;
    const int pair = __builtin_amdgcn_readfirstlane(blockIdx.x);
    if (pair >= npairs) return;
    const sed_pair_desc d = pd[pair];
    if (d.lane) return;  // scripted by sed_lane.hip
#ifdef SED_TB_DEBUG
    if (pair != 0) return;
#endif
    constexpr int NSEL = CkVHold<R>::value ? Grp<R>::G : 1, NW = SED_CKTB_NW;
    __shared__ uint32_t topb[SED_CK_NX(NW)], selb[NSEL * SED_CK_SELB(NW)];
    if constexpr (NSEL > 1) {
        for (int x = lane; x < NSEL * SED_CK_SELB(NW); x += 64) selb[x] = SED_SEL_SENT;  // (entries below 64: before column 1)
        __syncthreads();
    }
    const uint32_t q0 = (uint32_t)__builtin_amdgcn_readfirstlane(res[pair].len);
    ck_traceback_pair<R, false, NW>(d, pair, q0, lane, seqa, seqb, ck, res, ops, prm, topb, selb);
}

// ---------------------------------------------------------------------------
// SPLIT batches with checkpoints (config 2, GUI pairs; sed_runtime.cpp: split_ck).  The SPLIT forward kernel runs the
// distance (or dot) keys, 2-3 VALU per cell instead of the ladder keys' 5.2, and stores checkpoints after the pair's
// per-cell code region; this kernel then recomputes every 64 x 64 tile from them at once (one wave per tile, the
// traceback's whole-tile sweep) and writes the tile's canonical op codes in the per-cell code layout of the TB kernels
// (store_tb: per stripe and G-step group, 4 words per forward lane, code (step u, row rr) at bits 2 (u R + rr)), which
// the stripe-parallel traceback walks (as plain ops: the ladder keys' per-row code offsets are not applied, L.tb_ladder).
// Every tile is written, those below row n too, so the walks only ever read codes of a DP.  R = 4 (G = 16): tile lane r = 4 b + rr is forward lane G Q + b's row rr; its
// codes of the chunk's forward steps 64 c .. 64 c + 63 sit at sweep steps G - 1 + 3 b + rr onwards.
__device__ __forceinline__ uint32_t ck_codes_transpose(uint32_t y) {
    // 4 x 4 transpose of 2-bit elements, byte = row: (row rr, element u) -> (row u, element rr)
    uint32_t t = ((y >> 6) ^ y) & 0x00CC00CCu;
    y ^= t ^ (t << 6);
    t = ((y >> 12) ^ y) & 0x0000F0F0u;
    return y ^ t ^ (t << 12);
}
template <int R>
__global__ __launch_bounds__(64) void sed_ck_codes_kernel(const sed_pair_desc *__restrict__ pd,
                                                          const uint32_t *__restrict__ seqa,
                                                          const uint32_t *__restrict__ seqb, uint32_t *__restrict__ tb,
                                                          sed_i32_params prm) {
    static_assert(R == 4, "the code layout transposition is written for R = 4");
    constexpr int ROWS = 64 * R, G = Grp<R>::G;
    const int lane = threadIdx.x;
    const sed_pair_desc d = pd[blockIdx.y];
    if (d.lane || d.n == 0 || d.m == 0) return;
    const int n = d.n, m = d.m;
    const int nstripes = (n + ROWS - 1) / ROWS, SG = (m + 63 + G - 1) / G * G, nchunks = (SG + 63) >> 6;
    const int tile = (int)blockIdx.x;  // (k R + Q) nchunks + c
    if (tile >= nstripes * R * nchunks) return;
    const int c = tile % nchunks, kq = tile / nchunks, Q = kq % R, k = kq / R;
    const uint64_t codew = (uint64_t)nstripes * (uint64_t)(SG / G) * 256u;  // the pair's per-cell code words
    __shared__ uint32_t topb[SED_CK_NX(8)], selb[SED_CK_SELB(8)], wl[64 * 9], win[64 * 5];
    const CkPairCtx px = ck_pair_ctx<R>(d, lane, seqa, seqb, tb, codew);
    uint32_t one = 1u;
    asm volatile("" : "+v"(one));
    uint32_t W[8], vinit = 0;
    (void)ck_tile_sweep<R, false, true, 8>(px, lane, prm, topb, selb, k, Q, c, 127, one, W, vinit);
    // this lane's window: 64 codes from sweep step s0 (bit 2 s0 of W[0..7])
    const int b = lane >> 2, rr = lane & 3;
    const uint32_t s0 = (uint32_t)(G - 1 + (R - 1) * b + rr);
#pragma unroll
    for (int w = 0; w < 8; ++w) wl[lane * 9 + w] = W[w];
    __syncthreads();
    uint32_t x[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) x[i] = wl[lane * 9 + (int)(s0 >> 4) + i];
#pragma unroll
    for (int i = 0; i < 4; ++i) win[lane * 5 + i] = __builtin_amdgcn_alignbit(x[i + 1], x[i], (2u * s0) & 31u);
    __syncthreads();
    // lane = 4 b' + g writes forward lane G Q + b''s group 4 c + g: rows 4 b' .. 4 b' + 3, window word g
    const int bo = lane >> 2, g = lane & 3;
    const int gg = 4 * c + g;
    if (gg >= SG / G) return;  // past the stripe's last group
    uint32_t y[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) y[q] = win[(4 * bo + q) * 5 + g];
    uint32_t o[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {  // word w: steps 4w .. 4w+3 of the group, byte w of each row's window word
        const uint32_t sel = (uint32_t)w * 0x0101u + 0x0400u;  // bytes w of y[0], w of y[1]
        const uint32_t y01 = __builtin_amdgcn_perm(y[1], y[0], sel | 0x0C0C0000u);
        const uint32_t y23 = __builtin_amdgcn_perm(y[3], y[2], sel | 0x0C0C0000u);
        o[w] = ck_codes_transpose(__builtin_amdgcn_perm(y23, y01, 0x05040100u));
    }
    uint32_t *gp = tb + d.tb_off + (uint64_t)k * (uint64_t)(SG / G) * 256u + (uint64_t)gg * 256u + (uint32_t)(G * Q + bo) * 4u;
    *reinterpret_cast<uint4 *>(gp) = make_uint4(o[0], o[1], o[2], o[3]);
}

#ifndef SED_CKTB_TU  // (sed_cktb.hip compiles this file for the checkpoint traceback's launcher alone)
// ---------------------------------------------------------------------------
// Self-test of the cross-lane primitives the kernels rely on.
// ---------------------------------------------------------------------------
__global__ void sed_selftest_kernel(uint32_t *out) {
    const uint32_t lane = threadIdx.x;
    const uint32_t v = 1000u + lane;
    uint32_t fail = 0;
    const uint32_t shr = dpp_shr1(7u, v);
    if (shr != (lane == 0 ? 7u : 999u + lane)) fail |= 1;
    const uint32_t shl = dpp_shl1(9u, v);
    if (shl != (lane == 63 ? 9u : 1001u + lane)) fail |= 2;
    const uint32_t rol = dpp_rol1(v);
    if (rol != 1000u + ((lane + 1) & 63)) fail |= 4;
    const uint32_t p = __builtin_amdgcn_perm(0x44332211u, 0xFFFFFFFEu, i32_sel(lane & 3));
    if (p != (0xFF00FFFEu | (((0x44332211u >> (8 * (lane & 3))) & 0xFFu) << 16))) fail |= 8;
    const uint32_t ab = __builtin_amdgcn_alignbit(0x3u + (lane << 2), 0x80000000u, 2);
    if (ab != (0xE0000000u | 0x20000000u)) fail |= 16;
    // the 16-lane segment moves of the fp64 kernel's short-pair route (row_shr:1, row_shl:1, row_ror:15)
    const uint32_t sl = lane & 15u;
    if (seg_shr1<16>(7u, v) != (sl == 0 ? 7u : 999u + lane)) fail |= 32;
    if (seg_shl1<16>(9u, v) != (sl == 15 ? 9u : 1001u + lane)) fail |= 64;
    if (seg_rol1<16>(v) != 1000u + (lane & ~15u) + ((sl + 1) & 15u)) fail |= 128;
    atomicOr(out, fail);
}

// ---------------------------------------------------------------------------
// Launchers (host side, called from sed_runtime.cpp)
// ---------------------------------------------------------------------------
template <int R, bool TB, bool LEN = true, bool CK = false, bool DOT = false>
static hipError_t launch_i32_R(const sed_launch &L, const sed_i32_params &prm) {
    if (L.ntasks > 0) {  // SPLIT: one workgroup per (pair, stripe): the compute wave and its feeder
        if constexpr (CK && R != 4) {  // (SPLIT checkpoints: R = 4 only)
            return hipErrorInvalidValue;
        } else {
            SED_LAUNCH((sed_wf_i32_kernel<R, TB, true, LEN, CK, DOT>), dim3(L.ntasks), dim3(128), 0, L, L.pd, L.npairs,
                       L.tasks, (const uint32_t *)L.seqa, (const uint32_t *)L.seqb, L.tb, L.bnd, L.res, prm);
        }
    } else {
        const int grid = (L.npairs + 3) / 4;
        // SED_OCC_LDS (tuning/A-B only): dynamic LDS bytes per workgroup, which caps the resident waves
        static const int occ_lds = [] { const char *e = getenv("SED_OCC_LDS"); return e ? atoi(e) : 0; }();
        SED_LAUNCH((sed_wf_i32_kernel<R, TB, false, LEN, CK, DOT>), dim3(grid), dim3(256), occ_lds, L, L.pd, L.npairs,
                           L.tasks, (const uint32_t *)L.seqa, (const uint32_t *)L.seqb, L.tb, L.bnd, L.res,
                           prm);
    }
    return hipGetLastError();
}

template <int R, bool TB, bool LEN, bool CK = false, int LDOT = 0>
static hipError_t launch_chain_R(const sed_launch &L, const sed_i32_params &prm) {
    SED_LAUNCH((sed_wf_i32_chain_kernel<R, TB, LEN, CK, LDOT>), dim3((L.nchains + 3) / 4), dim3(256), 0, L, L.pd,
                       L.chain_pairs, L.chain_off, L.nchains, L.chain_counter, L.chain_base, L.chain_list,
                       (const uint32_t *)L.seqa, (const uint32_t *)L.seqb, L.tb, L.res, prm);
    return hipGetLastError();
}

hipError_t sed_launch_i32_chain(const sed_launch &L, const sed_i32_params &prm, bool len) {
    const bool tb = L.tb != nullptr;
    if (tb && L.ck) {  // distance keys + checkpoints
        switch (L.R) {
        case 4: return launch_chain_R<4, false, false, true>(L, prm);
        case 8: return launch_chain_R<8, false, false, true>(L, prm);
        case 16: return launch_chain_R<16, false, false, true>(L, prm);
        default: return hipErrorInvalidValue;
        }
    }
    switch (L.R) {
#define CASE(RR)                                                                                   \
    case RR:                                                                                       \
        if (prm.lad == 2 && len)                                                                   \
            return tb ? launch_chain_R<RR, true, true, false, 2>(L, prm)                          \
                      : launch_chain_R<RR, false, true, false, 2>(L, prm);                         \
        if (prm.lad && len)                                                                        \
            return tb ? launch_chain_R<RR, true, true, false, 1>(L, prm)                          \
                      : launch_chain_R<RR, false, true, false, 1>(L, prm);                         \
        return tb ? launch_chain_R<RR, true, true>(L, prm)                                         \
                  : (len ? launch_chain_R<RR, false, true>(L, prm) : launch_chain_R<RR, false, false>(L, prm));
        CASE(4) CASE(8) CASE(16)
#undef CASE
    default: return hipErrorInvalidValue;
    }
}

hipError_t sed_launch_i32x2(const sed_launch &L, const int32_t *list, int nwaves, const sed_i32_params &prm) {
    if (nwaves <= 0) return hipSuccess;
    const dim3 grid((nwaves + 3) / 4), block(256);
    const uint32_t *a = (const uint32_t *)L.seqa, *b = (const uint32_t *)L.seqb;
    switch (L.R) {
    case 4: SED_LAUNCH((sed_wf_i32x2_kernel<4>), grid, block, 0, L, L.pd, list, nwaves, a, b, L.bnd, L.res, prm); break;
    case 8: SED_LAUNCH((sed_wf_i32x2_kernel<8>), grid, block, 0, L, L.pd, list, nwaves, a, b, L.bnd, L.res, prm); break;
    case 16: SED_LAUNCH((sed_wf_i32x2_kernel<16>), grid, block, 0, L, L.pd, list, nwaves, a, b, L.bnd, L.res, prm); break;
    case 32: SED_LAUNCH((sed_wf_i32x2_kernel<32>), grid, block, 0, L, L.pd, list, nwaves, a, b, L.bnd, L.res, prm); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t sed_launch_i32(const sed_launch &L, const sed_i32_params &prm, bool len) {
    const bool tb = L.tb != nullptr;
    if (tb && L.ck) {  // distance keys + checkpoints
        if (L.ntasks > 0) {  // SPLIT: R = 4 (sed_ck_codes_kernel)
            if (L.R != 4) return hipErrorInvalidValue;
            return prm.dot ? launch_i32_R<4, false, false, true, true>(L, prm) : launch_i32_R<4, false, false, true>(L, prm);
        }
        if (prm.dot) {  // dot keys (the host found a byte factorisation of the update addends)
            switch (L.R) {
            case 4: return launch_i32_R<4, false, false, true, true>(L, prm);
            case 8: return launch_i32_R<8, false, false, true, true>(L, prm);
            case 16: return launch_i32_R<16, false, false, true, true>(L, prm);
            default: return hipErrorInvalidValue;
            }
        }
        switch (L.R) {
        case 4: return launch_i32_R<4, false, false, true>(L, prm);
        case 8: return launch_i32_R<8, false, false, true>(L, prm);
        case 16: return launch_i32_R<16, false, false, true>(L, prm);
        default: return hipErrorInvalidValue;
        }
    }
    switch (L.R) {
#define CASE(RR)                                                                                     \
    case RR:                                                                                         \
        return tb ? launch_i32_R<RR, true>(L, prm)                                                   \
                  : (len ? launch_i32_R<RR, false>(L, prm) : launch_i32_R<RR, false, false>(L, prm));
        CASE(4) CASE(8) CASE(16) CASE(32)
#undef CASE
    default: return hipErrorInvalidValue;
    }
}

template <int R, bool TB, bool TYPED, bool FULL = false, int SW = 64>
static hipError_t launch_f64_R(const sed_launch &L, const double *gtab, const sed_f64_params &prm,
                               const sed_full_out &fo = sed_full_out{}, const int32_t *idx = nullptr, int nidx = 0) {
    const int items = SW == 64 ? L.npairs : nidx;
    const int grid = (items * SW + 255) / 256;
    if (items <= 0) return hipSuccess;
    SED_LAUNCH((sed_wf_f64_kernel<R, TB, TYPED, FULL, SW>), dim3(grid), dim3(256), 0, L, L.pd, items,
                       (const uint8_t *)L.seqa, (const uint8_t *)L.seqb, L.tb, L.bnd, L.res, gtab, prm, fo, idx);
    return hipGetLastError();
}

// SPLIT (L.ntasks > 0): one 128-thread workgroup per (pair, stripe) task, R = 2 (the default) or 4
template <bool TB, bool TYPED, bool FULL = false>
static hipError_t launch_f64_split(const sed_launch &L, const double *gtab, const sed_f64_params &prm,
                                   const sed_full_out &fo = sed_full_out{}) {
    if (L.R == 2)
        SED_LAUNCH((sed_wf_f64_split_kernel<2, TB, TYPED, FULL>), dim3(L.ntasks), dim3(128), 0, L, L.pd, L.tasks,
                   (const uint8_t *)L.seqa, (const uint8_t *)L.seqb, L.tb, L.bnd, L.res, gtab, prm, fo);
    else if (L.R == 4)
        SED_LAUNCH((sed_wf_f64_split_kernel<4, TB, TYPED, FULL>), dim3(L.ntasks), dim3(128), 0, L, L.pd, L.tasks,
               (const uint8_t *)L.seqa, (const uint8_t *)L.seqb, L.tb, L.bnd, L.res, gtab, prm, fo);
    return hipGetLastError();
}

hipError_t sed_launch_f64_full(const sed_launch &L, const double *gtab, const sed_f64_params &prm, bool typed,
                               const sed_full_out &fo) {
    if (L.tb || (L.ntasks > 0 ? (L.R != 2 && L.R != 4) : L.R != 4)) return hipErrorInvalidValue;
    if (L.ntasks > 0)
        return typed ? launch_f64_split<false, true, true>(L, gtab, prm, fo)
                     : launch_f64_split<false, false, true>(L, gtab, prm, fo);
    return typed ? launch_f64_R<4, false, true, true>(L, gtab, prm, fo)
                 : launch_f64_R<4, false, false, true>(L, gtab, prm, fo);
}

hipError_t sed_launch_f64(const sed_launch &L, const double *gtab, const sed_f64_params &prm, bool typed) {
    const bool tb = L.tb != nullptr;
    if (L.ntasks > 0) {
        if (L.R != 2 && L.R != 4) return hipErrorInvalidValue;
        if (typed) return tb ? launch_f64_split<true, true>(L, gtab, prm) : launch_f64_split<false, true>(L, gtab, prm);
        return tb ? launch_f64_split<true, false>(L, gtab, prm) : launch_f64_split<false, false>(L, gtab, prm);
    }
    switch (L.R) {
#define CASE(RR)                                                                                    \
    case RR:                                                                                        \
        if (typed) return tb ? launch_f64_R<RR, true, true>(L, gtab, prm)                           \
                             : launch_f64_R<RR, false, true>(L, gtab, prm);                         \
        return tb ? launch_f64_R<RR, true, false>(L, gtab, prm) : launch_f64_R<RR, false, false>(L, gtab, prm);
        CASE(4) CASE(8)  // (R = 16: 206 VGPRs, 2 waves per SIMD, iupac 5.22-5.25 against 5.04-5.06 ms at R = 8)
#undef CASE
    default: return hipErrorInvalidValue;
    }
}

hipError_t sed_launch_f64_seg(const sed_launch &L, const double *gtab, const sed_f64_params &prm, bool typed,
                              const int32_t *idx, int nidx) {
    const bool tb = L.tb != nullptr;
    const sed_full_out none{};
    switch (L.R) {
#define CASE(RR)                                                                                               \
    case RR:                                                                                                   \
        if (typed) return tb ? launch_f64_R<RR, true, true, false, 16>(L, gtab, prm, none, idx, nidx)          \
                             : launch_f64_R<RR, false, true, false, 16>(L, gtab, prm, none, idx, nidx);        \
        return tb ? launch_f64_R<RR, true, false, false, 16>(L, gtab, prm, none, idx, nidx)                    \
                  : launch_f64_R<RR, false, false, false, 16>(L, gtab, prm, none, idx, nidx);
        CASE(4) CASE(8)
#undef CASE
    default: return hipErrorInvalidValue;
    }
}

hipError_t sed_launch_traceback_seg(const sed_launch &L, uint32_t *ops, const int32_t *idx, int nidx) {
    if (nidx <= 0) return hipSuccess;
    const int grid = (nidx + 63) / 64;
    switch (L.R) {
    case 4: SED_LAUNCH((sed_traceback_kernel<4, 16>), dim3(grid), dim3(64), 0, L, L.pd, nidx, L.tb, L.res, ops, 0ull, idx); break;
    case 8: SED_LAUNCH((sed_traceback_kernel<8, 16>), dim3(grid), dim3(64), 0, L, L.pd, nidx, L.tb, L.res, ops, 0ull, idx); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t sed_launch_ck_codes(const sed_launch &L, int max_tiles, const sed_i32_params &prm) {
    if (L.R != 4 || max_tiles <= 0 || L.npairs <= 0) return hipErrorInvalidValue;
    SED_LAUNCH(sed_ck_codes_kernel<4>, dim3(max_tiles, L.npairs), dim3(64), 0, L, L.pd, (const uint32_t *)L.seqa,
               (const uint32_t *)L.seqb, L.tb, prm);
    return hipGetLastError();
}

hipError_t sed_launch_traceback(const sed_launch &L, uint32_t *ops) {
    // up to one pair per CU: a wave-uniform walk per pair over windows of blocks; beyond: one lane per pair
    const bool uni = L.npairs <= 256;
    const int grid = uni ? L.npairs : (L.npairs + 63) / 64;
    switch (L.R) {
#define CASE(RR)                                                                                                 \
    case RR: {                                                                                                   \
        const uint64_t pat = L.tb_ladder ? (L.tb_wide ? LadderW<RR>::pat : Ladder<RR>::pat) : 0ull;                                               \
        if (uni)                                                                                                 \
            SED_LAUNCH((sed_traceback_window_kernel<RR>), dim3(grid), dim3(64), 0, L, L.pd,       \
                               L.npairs, L.tb, L.res, ops, pat);                                                \
        else                                                                                                     \
            SED_LAUNCH((sed_traceback_kernel<RR>), dim3(grid), dim3(64), 0, L, L.pd,              \
                               L.npairs, L.tb, L.res, ops, pat, nullptr);                                       \
        break;                                                                                                   \
    }
        CASE(2) CASE(4) CASE(8) CASE(16) CASE(32)  // (R = 2: the fp64 SPLIT route's codes)
#undef CASE
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// stripe-parallel traceback (few pairs with >= 3 stripes): ops zeroed by the caller; items = the most map lanes
// of a pair ((K-2)(m+1)+1), kmax = the most stripes of a pair
hipError_t sed_launch_traceback_stripes(const sed_launch &L, uint32_t *ops, uint32_t *map, int items, int kmax) {
    // items: map workgroups x 256 of the largest pair, and at least every pair's script words; >= one block
    // (the compose grid: (K-2)(m+1)+1 threads per pair, at most items / 256 / R + 1 blocks, sed_runtime.cpp)
    const bool bandemit = SED_TBMAP_BANDS && SED_TB_BANDEMIT;
    const dim3 gmap((max(items, 1) + 255) / 256, L.npairs), gemit(L.npairs, max(kmax, 1) * (bandemit ? L.R : 1)),
        gcomp((max(items, 1) + 255) / 256 / max(L.R, 1) + 1, L.npairs);
    switch (L.R) {
#define CASE(RR)                                                                                                 \
    case RR: {                                                                                                   \
        const uint64_t pat = L.tb_ladder ? (L.tb_wide ? LadderW<RR>::pat : Ladder<RR>::pat) : 0ull;                                               \
        if (SED_TBMAP_BANDS) {                                                                                   \
            hipExtLaunchKernelGGL((sed_tb_bandmap_kernel<RR>), gmap, dim3(256), 0, L.stream, L.ev0, nullptr, 0, L.pd, L.tb, map, ops, pat); \
            hipLaunchKernelGGL((sed_tb_bandcompose_kernel<RR>), gcomp, dim3(256), 0, L.stream, L.pd, map);          \
        } else {                                                                                                 \
            hipExtLaunchKernelGGL((sed_tb_stripemap_kernel<RR>), gmap, dim3(256), 0, L.stream, L.ev0, nullptr, 0, L.pd, L.tb, map, ops, pat); \
        }                                                                                                        \
        if (bandemit)                                                                                            \
            hipExtLaunchKernelGGL((sed_tb_bandemit_kernel<RR>), gemit, dim3(64), 0, L.stream, nullptr, L.ev1, 0, L.pd, L.tb, L.res, ops, \
                                  map, pat);                                                                     \
        else                                                                                                     \
            hipExtLaunchKernelGGL((sed_tb_stripeemit_kernel<RR>), gemit, dim3(64), 0, L.stream, nullptr, L.ev1, 0, L.pd, L.tb, L.res, ops, \
                                  map, pat);                                                                     \
        break;                                                                                                   \
    }
        CASE(2) CASE(4)
#undef CASE
    default: return hipErrorInvalidValue;  // the runtime takes this route at R = 2 (fp64 SPLIT) and 4 only
    }
    return hipGetLastError();
}

hipError_t sed_launch_selftest(uint32_t *d_out, hipStream_t stream) {
    hipLaunchKernelGGL(sed_selftest_kernel, dim3(1), dim3(64), 0, stream, d_out);
    return hipGetLastError();
}
#else
// the checkpoint traceback, in its own translation unit (sed_cktb.hip: built with private arrays kept out of vector
// registers, so a visit's code words stay separate registers)
hipError_t sed_launch_traceback_ck(const sed_launch &L, uint32_t *ops, const sed_i32_params &prm) {
    const dim3 grid(L.npairs), block(64);
    const uint32_t *a = (const uint32_t *)L.seqa, *b = (const uint32_t *)L.seqb;
    switch (L.R) {
    case 4: SED_LAUNCH(sed_traceback_ck_kernel<4>, grid, block, 0, L, L.pd, L.npairs, a, b, L.tb, L.res, ops, prm); break;
    case 8: SED_LAUNCH(sed_traceback_ck_kernel<8>, grid, block, 0, L, L.pd, L.npairs, a, b, L.tb, L.res, ops, prm); break;
    case 16: SED_LAUNCH(sed_traceback_ck_kernel<16>, grid, block, 0, L, L.pd, L.npairs, a, b, L.tb, L.res, ops, prm); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
#endif

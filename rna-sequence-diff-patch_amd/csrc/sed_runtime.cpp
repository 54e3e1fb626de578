// sed_runtime.cpp — the C-ABI of libsed.so (include/sed.h): contexts, the
// cost model, mode selection, device-resident batches and the launch sequence
//   DP kernel (integer or fp64)  ->  traceback kernel
// on one HIP stream, timed with HIP events recorded on that stream.
#include "../../include/sed.h"
#include "sed_internal.h"

#include <hip/hip_runtime.h>
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    uint64_t gen = 0;  // bumped by every (re)allocation: memory of a new generation may hold anything
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // grow-only; returns false on OOM
    bool reserve(size_t bytes) {
        if (bytes <= cap) return true;
        release();
        size_t want = std::max<size_t>(bytes, 256);
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            (void)hipGetLastError();
            return false;
        }
        cap = want;
        ++gen;
        return true;
    }
};

bool is_integral_small(double v, int lim) { return v == std::floor(v) && v >= 0 && v < lim; }

}  // namespace

// Batches whose input arrays and results fit this many bytes go up as one blob from pinned staging (fill_batch)
#define SED_SMALL_BATCH_BYTES (4u << 20)

struct sed_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // cost model
    bool have_costs = false;
    int K = 0;
    std::vector<double> sub;
    std::vector<uint8_t> sub_int;
    double ins = 1, del = 1;
    int ins_int = 0, del_int = 0;
    DevBuf gtab;  // fp64 kernel table: per entry {value bits, is-int flag}
    // options
    int opt_mode = 0, opt_R = 0, opt_split = 0, opt_lane = 0, opt_chain = 0, opt_pack = 0, opt_tb = 0;
    int opt_chain_waves = 0;
    int opt_bitpar = 0;         // SED_OPT_BITPAR: 0 auto (unit-cost distance-only lane pairs), 2 never
    int opt_scaled = 0;         // SED_OPT_SCALED: 0 auto (fp64 lane pairs under dyadic costs), 2 never
    int opt_seg = 0;            // SED_OPT_SEG: 0 auto (fp64 pairs the cost model prefers in 16-lane segments), 1 every
                                // eligible pair, 2 never
    int opt_splitck = 0;        // SED_OPT_SPLITCK: 0 auto (on), 2 never (SPLIT script batches keep the per-cell-code forward)
    int opt_zc = 0;             // SED_OPT_ZEROCOPY: 0 auto (small batches write results into pinned host memory), 2 never
    int opt_dot = 0;            // SED_OPT_DOT: 0 auto, 2 never (checkpoint batches keep the perm-based distance keys), 3 no wide ladder    // SED_OPT_CHAIN_WAVES: cap on the persistent waves of dynamic CHAIN mode
    int opt_debug_corrupt = 0;  // SED_OPT_DEBUG_CORRUPT: pair + 1 whose sink-tile checkpoint is overwritten
    DevBuf selftest;
    sed_batch *scratch = nullptr;
    // pinned host staging (hipHostMalloc) of small batches: the upload blob, then the results' download
    void *pin = nullptr;
    size_t pin_cap = 0;
    bool pin_busy = false;  // a copy from / to `pin` may still be in flight on `stream`
    bool pair_pending = false;  // sed_pair_submit enqueued the scratch batch; sed_pair_wait has not fetched it

    int fail(int code, const char *fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
    int hipfail(hipError_t e, const char *what) {
        return fail(SED_E_DEVICE, "%s: %s", what, hipGetErrorString(e));
    }
};

struct sed_batch;
namespace {
// grow the context's pinned staging to `bytes` (first waiting for a copy still in flight from it)
hipError_t pin_reserve(sed_ctx *c, size_t bytes) {
    hipError_t e = hipSuccess;
    if (c->pin_busy && (e = hipStreamSynchronize(c->stream)) != hipSuccess) return e;
    c->pin_busy = false;
    if (bytes <= c->pin_cap) return hipSuccess;
    if (c->pin) (void)hipHostFree(c->pin);
    c->pin = nullptr;
    c->pin_cap = 0;
    const size_t want = std::max<size_t>(bytes, 1u << 20);
    if ((e = hipHostMalloc(&c->pin, want, hipHostMallocDefault)) != hipSuccess) {
        c->pin = nullptr;
        return e;
    }
    c->pin_cap = want;
    return hipSuccess;
}
}  // namespace

struct sed_batch {
    sed_ctx *ctx = nullptr;
    int npairs = 0;
    uint32_t flags = 0;
    int mode = 0, R = 0;
    std::vector<sed_pair_desc> pd;
    std::vector<int32_t> n, m;
    uint64_t tb_words = 0, bnd_words = 0, ops_words = 0;
    double cells = 0, algo_bytes = 0;
    DevBuf d_pd, d_seqa, d_seqb, d_bnd, d_ops, d_tasks, d_lane, d_chain, d_x2, d_tbmap, d_seg;
    int nseg = 0;              // fp64 wave pairs in 16-lane segments (pd.pad[1]), listed in d_seg
    // small batches (fill_batch: SED_SMALL_BATCH_BYTES) keep every input array and the results in one blob, d_small;
    // the kernels' pointers (p_*) point into it or at the per-array buffers above
    DevBuf d_small;
    bool small = false;
    size_t o_ops_small = 0;  // small batches: the scripts' offset from the results in d_small
    // small batches whose kernels write their results and scripts with plain stores (not the stripe-parallel walk's
    // atomicOr): the kernels write them straight into this pinned host block, so no download follows the run
    // (sed_run_pair on a 30-nt pair: one copy kernel fewer per call)
    void *h_out = nullptr;
    size_t h_out_cap = 0;
    bool zc = false;
    // a zero-copy run was enqueued on the context's stream and not yet waited for (set before its first launch, so a
    // run that failed halfway counts too): the kernels may still store into h_out
    bool zc_busy = false;
    void *p_pd = nullptr, *p_seqa = nullptr, *p_seqb = nullptr, *p_tasks = nullptr, *p_lane = nullptr,
         *p_chain = nullptr, *p_x2 = nullptr, *p_ops = nullptr, *p_seg = nullptr, *p_res[3] = {nullptr, nullptr, nullptr};
    // timing events: 1 on every run (default), k > 1 on every k-th run, 0 never (sed_batch_set_timing; runs that
    // order buffer reuse through their events always record them)
    int time_every = 1;
    bool tbpar = false;        // stripe-parallel traceback (few long pairs, per-cell codes; sed_tb_stripe*_kernel)
    int tbpar_items = 0, tbpar_kmax = 0;
    // SPLIT script batches at R = 4 (config 2, GUI pairs): the forward runs distance / dot keys and stores checkpoints
    // after each pair's per-cell code region; sed_ck_codes_kernel (ck_tiles waves per pair) recomputes every tile's
    // codes into that region, which the stripe-parallel traceback walks
    bool split_ck = false;
    int ck_tiles = 0;
    bool split = false;
    // SPLIT hand-off words' tag: the last run's epoch (1..32767), kept across fills, so that a refilled batch (the
    // per-call path fills the context's scratch batch every call) needs no memset; the buffer is zeroed when it is
    // (re)allocated (d_bnd.gen differs from bnd_zero_gen: a failed and a later successful reserve may return new
    // memory of the old capacity, so the capacity does not tell) and when the epoch wraps
    uint32_t split_epoch = 0;
    uint64_t bnd_zero_gen = 0;
    bool ck = false;           // traceback from checkpoints + recompute (sed_kernels.hip: CK) instead of codes
    bool dot = false;          // CK forward kernel on dot keys (dot_keys below)
    bool lad = false;          // CHAIN kernel with the L field on ladder dot keys (dot_keys ladder mode)
    int nlane = 0, nwave = 0;  // pairs on the lane-per-pair kernel / on the wave kernels
    int nlane_x2 = 0;          // > 0: lane pairs run two per lane (distance only), in this many lanes
    bool lane_bitpar = false;  // lane pairs run the bit-parallel unit-cost kernel (distance only)
    uint32_t umask = 0;        // fp64 lane kernel: codes of the unit-cost subset; its pairs run bit-parallel
    int nbitpar_f64 = 0;       // fp64 lane pairs flagged for it (pd.pad[0])
    bool scaled = false;       // fp64 lane pairs on the scaled-integer kernel (dyadic costs, scaled_costs)
    sed_scaled_params sp{};
    int nwave_x2 = 0;          // distance-only wave pairs of equal shape run two per wave, in this many waves
    int nchains = 0;           // CHAIN mode: wave pairs run as nchains back-to-back chains (0 = off)
    size_t chain_npairs = 0;   // d_chain = [chain_pairs (chain_npairs) | chain_off (nchains + 1) | counter]
    bool chain_dyn = false;    // persistent waves + device counter instead of static chains
    int ntasks = 0;
    // SED_PIPELINE: run k uses traceback/result buffer k%3 and its traceback runs on a second
    // stream, overlapping the DP of run k+1.  Three buffers, so the DP of run k+3 is the first
    // to wait for that traceback: with two, a traceback starved of CUs during the next DP
    // (it only gets them in that DP's tail) delayed the DP after it (~0.7 ms per 27 ms step).
    int nbuf = 1;
    DevBuf d_tb[3], d_res[3];
    hipStream_t tb_stream = nullptr;
    // Checkpoint batches in parts (SED_CK_HALVES = number of parts): part 0 runs forward then traceback on the
    // context's stream, part i on part_stream[i - 1], so one part's traceback overlaps another part's forward.
    int nparts = 1;
    hipStream_t part_stream[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_start = nullptr;
    // per event-log entry: the {dp start, dp end, tb start, tb end} events of parts 1..3 (created on first use)
    std::vector<std::array<hipEvent_t, 12>> plog;
    // per buffer: the event-log entry of the last run that used it (handles copied from `log`)
    std::array<hipEvent_t, 4> evk[3] = {};
    long runs = 0;
    // dynamic-CHAIN launches since the fill per buffer slot: each slot has its own device counter, whose base is
    // slot launches x (list + waves)
    long chain_launches[3] = {0, 0, 0};
    // pipelined batches whose runs share no scratch (dynamic-CHAIN script batches, distance-only batches of lane
    // pairs): odd runs' DP on dp2_stream, so run k+1's kernels fill the tail of run k's (CHAIN: persistent waves;
    // lane kernels: the launch gap).  CHAIN slots have their own counters; a slot's runs are ordered through the
    // wait of buffer reuse (run_batch)
    bool alt_dp = false;
    hipStream_t dp2_stream = nullptr;
    bool ran = false;
    // per-run event log (sed_batch_times): {dp start, dp end, tb start, tb end}
    std::vector<std::array<hipEvent_t, 4>> log;
    size_t nlog = 0;
    long last_log = -1;  // the event-log entry of the last run (its parts' events: plog[last_log])
    sed_i32_params ip{};
    sed_f64_params fp{};
    std::vector<sed_result> h_res;

    int cur() const { return (int)((runs - 1) % nbuf); }
    ~sed_batch() {
        if (zc_busy) (void)hipStreamSynchronize(ctx->stream);
        if (h_out) (void)hipHostFree(h_out);
        d_pd.release(); d_seqa.release(); d_seqb.release(); d_bnd.release(); d_ops.release(); d_tbmap.release();
        d_tasks.release(); d_lane.release(); d_chain.release(); d_x2.release(); d_small.release(); d_seg.release();
        for (int i = 0; i < 3; ++i) {
            d_tb[i].release();
            d_res[i].release();
        }
        if (tb_stream) (void)hipStreamDestroy(tb_stream);
        if (dp2_stream) (void)hipStreamDestroy(dp2_stream);
        for (hipStream_t &ps : part_stream)
            if (ps) (void)hipStreamDestroy(ps);
        if (ev_start) (void)hipEventDestroy(ev_start);
        for (auto &a : plog)
            for (hipEvent_t e : a)
                if (e) (void)hipEventDestroy(e);
        for (auto &a : log)
            for (hipEvent_t e : a)
                if (e) (void)hipEventDestroy(e);
    }
};

namespace {

// ---- dot keys ----
// The CK forward kernel's update candidate can be one signed-byte dot product v_dot4_i32_i8(row vector of str1's
// symbol a, column vector of str2's symbol b, diagonal) when the addends H(a, b) = A*kappa(a, b) + 1 (kappa =
// insert + delete - cost(a -> b)) factor as sum_k r_k(a) c_k(b) over bytes in [-127, 127]: keys W = A*X + U
// (X = sum of kappa over the path's updates, U = its number of updates) are maximised with v_max3, so the cell is
// v_dot4 + v_max3 (2 VALU) instead of v_perm + v_add + v_min3.  Ordering: at a fixed cell a candidate with a larger
// X must win whatever the U's, i.e. A > the U spread of two candidates, which is below min(i, j) (kmax - kmin) /
// kmin because every update contributes kappa in [kmin, kmax]; the same bound makes X = floor(k kmax / (A kmax +
// 1)) recover X from k = A*X + U.
// Construction (rank 3 + one constant slot): with det/S = num/den (S = 1^T adj(K) 1), N = den*K - num*J has rank 3
// and left null vector v = 1^T adj(K); if some |v_g| = 1, row g of N is an integer combination of the other three.
// Slot 0 is the constant x*y = num*a + 1, slots 1..3 are a*N's rank-3 factorisation (coordinates P0 scaled by a1,
// rows of N scaled by a2, a1*a2 = a), so sum_k r_k c_k = num*a + 1 + a*(den K - num) = A K + 1 with A = den*a.
struct DotKeys {
    bool ok = false;
    uint32_t A = 0, kmax = 0, kmin = 0, M = 0, S = 0;
    uint32_t row[4] = {0, 0, 0, 0}, col[4] = {0, 0, 0, 0};
};
int64_t det3(const int64_t m[3][3]) {
    return m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
           m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
}
int64_t gcd64(int64_t a, int64_t b) {
    a = a < 0 ? -a : a;
    b = b < 0 ? -b : b;
    while (b) {
        const int64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}
// kap: kappa[a][b] (>= 1); maxmin: the largest min(n, m) of the batch's wave pairs.
// Ladder mode (lad_amin > 0, lad_beta): the factorisation of A*K + lad_beta*J for the per-cell-code kernels'
// ladder keys with A >= lad_amin and A < 2^16 (dot_ladder below); no ordering bound or decode constants.
DotKeys dot_keys_search(const int64_t kap[4][4], int64_t maxmin, int64_t lad_amin, int64_t lad_beta) {
    const bool lad = lad_amin > 0;
    const int64_t beta = lad ? lad_beta : 1;
    DotKeys dk;
    int64_t kmax = 0, kmin = INT64_MAX;
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) {
            kmax = std::max(kmax, kap[a][b]);
            kmin = std::min(kmin, kap[a][b]);
        }
    if (kmin < 1 || kmax > 255) return dk;
    // adjugate (adj[b][a] = cofactor(a, b)) and determinant
    int64_t adj[4][4], det = 0;
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) {
            int64_t m3[3][3];
            for (int i = 0, ii = 0; i < 4; ++i) {
                if (i == a) continue;
                for (int j = 0, jj = 0; j < 4; ++j) {
                    if (j == b) continue;
                    m3[ii][jj++] = kap[i][j];
                }
                ++ii;
            }
            adj[b][a] = (((a + b) & 1) ? -1 : 1) * det3(m3);
        }
    for (int b = 0; b < 4; ++b) det += kap[0][b] * adj[b][0];
    int64_t S = 0, v[4] = {0, 0, 0, 0};
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) {
            S += adj[a][b];
            v[b] += adj[a][b];  // v = 1^T adj(K)
        }
    if (S == 0) return dk;
    int64_t num = det, den = S;
    if (den < 0) { num = -num; den = -den; }
    const int64_t gd = gcd64(num, den);
    if (gd > 1) { num /= gd; den /= gd; }
    int64_t gv = 0;
    for (int a = 0; a < 4; ++a) gv = gcd64(gv, v[a]);
    if (gv == 0) return dk;
    for (int a = 0; a < 4; ++a) v[a] /= gv;
    int g = -1;
    for (int a = 0; a < 4; ++a)
        if (v[a] == 1 || v[a] == -1) { g = a; break; }
    if (g < 0) return dk;
    int64_t N[4][4];
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) N[a][b] = den * kap[a][b] - num;
    // slots 1..3 <-> rows s[0..2] != g: P0[a][k] = [a == s_k] (a != g), P0[g][k] = -v[s_k] / v[g]
    int sr[3], ns = 0;
    for (int a = 0; a < 4; ++a)
        if (a != g) sr[ns++] = a;
    int64_t P0[4][3], pmax[3], qmax[3];
    for (int k = 0; k < 3; ++k) {
        pmax[k] = qmax[k] = 0;
        for (int a = 0; a < 4; ++a) {
            P0[a][k] = a == g ? -v[sr[k]] * v[g] : (a == sr[k] ? 1 : 0);  // v[g] = +-1: 1/v[g] = v[g]
            pmax[k] = std::max(pmax[k], P0[a][k] < 0 ? -P0[a][k] : P0[a][k]);
        }
        for (int b = 0; b < 4; ++b) qmax[k] = std::max(qmax[k], N[sr[k]][b] < 0 ? -N[sr[k]][b] : N[sr[k]][b]);
    }
    // the rank-3 identity must hold exactly
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) {
            int64_t t = 0;
            for (int k = 0; k < 3; ++k) t += P0[a][k] * N[sr[k]][b];
            if (t != N[a][b]) return dk;
        }
    // the largest a with every slot within bytes (larger A leaves more room for long pairs)
    const int64_t a_hi = num != 0 ? (127 * 127 + 127) / (num < 0 ? -num : num) : 127 * 127;  // |num a + 1| <= 127^2
    for (int64_t a = a_hi; a >= 1; --a) {
        const int64_t A = den * a;
        if (lad ? A < lad_amin : A * kmin <= maxmin * (kmax - kmin)) break;  // fails for every smaller a too
        // ladder keys keep the rung c(i) and the op in the low 3 (wide: 4) bits of W = A*(D - i*delete - j*insert) +
        // u*(L - i - j) + B + c(i), u = 8 (16): A must be a multiple of u, or the D part leaks into them (a random GUI
        // table found this: insert 2 / delete 1 factored with A = 8835, and its scripts came out wrong)
        if (lad && (A >= 65536 || (A & lad_beta))) continue;  // (lad_beta + 1 = the L unit, 8 or 16)
        const int64_t J = num * a + beta;
        int64_t x = 0, y = 0;
        for (int64_t t = 1; t <= 127 && !x; ++t)
            if (J % t == 0 && (J / t >= -127 && J / t <= 127)) { x = t; y = J / t; }
        if (!x) continue;
        int64_t a1[3], a2[3];
        bool fit = true;
        for (int k = 0; k < 3 && fit; ++k) {
            a1[k] = 0;
            for (int64_t t = 1; t <= 127; ++t)
                if (a % t == 0 && t * pmax[k] <= 127 && (a / t) * qmax[k] <= 127) { a1[k] = t; break; }
            if (!a1[k]) fit = false;
            else a2[k] = a / a1[k];
        }
        if (!fit) continue;
        // decode: k * kmax < 2^29 over every real cell (k <= A * kmax * maxmin + maxmin)
        if (!lad && (A * kmax * maxmin + maxmin) * kmax >= (int64_t)1 << 29) continue;
        int8_t R[4][4], C[4][4];
        for (int i = 0; i < 4; ++i) {
            R[i][0] = (int8_t)x;
            C[i][0] = (int8_t)y;
            for (int k = 0; k < 3; ++k) {
                R[i][k + 1] = (int8_t)(a1[k] * P0[i][k]);
                C[i][k + 1] = (int8_t)(a2[k] * N[sr[k]][i]);
            }
        }
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                int64_t t = 0;
                for (int k = 0; k < 4; ++k) t += (int64_t)R[i][k] * C[j][k];
                if (t != A * kap[i][j] + beta) return dk;
            }
        dk.A = (uint32_t)A;
        dk.kmax = (uint32_t)kmax;
        dk.kmin = (uint32_t)kmin;
        if (lad) {  // min-form ladder keys add -(A*kappa + beta): the column vectors are negated
            for (int i = 0; i < 4; ++i) {
                uint32_t rw = 0, cw = 0;
                for (int k = 0; k < 4; ++k) {
                    rw |= (uint32_t)(uint8_t)R[i][k] << (8 * k);
                    cw |= (uint32_t)(uint8_t)(int8_t)(-C[i][k]) << (8 * k);
                }
                dk.row[i] = rw;
                dk.col[i] = cw;
            }
            // the virtual-column sentinel {s, 0, 0, 0} adds s x in [u, 490] (wide: [16, 480]): above every ladder jump
            // (at most +5, wide +13), and below the 512 the border leaves to 2^32 (sed_kernels.hip: SED_KB3)
            const int64_t lo = lad_beta + 1, hi = lad_beta == 15 ? 480 : 490;
            const int64_t sx = x > 0 ? (lo + x - 1) / x : 0;
            dk.ok = x > 0 && sx * x <= hi;
            dk.S = (uint32_t)sx;
            return dk;
        }
        const uint64_t Dd = (uint64_t)A * kmax + 1;
        int lg = 0;
        while (((uint64_t)1 << lg) < Dd) ++lg;
        dk.S = (uint32_t)(29 + lg);
        const uint64_t M = ((((uint64_t)1 << dk.S) / Dd) + 1) * (uint64_t)kmax;  // the kernels multiply k by M
        if (M >> 32 || dk.S < 32 || 4 * A >= (1 << 24)) return dk;
        dk.M = (uint32_t)M;
        for (int i = 0; i < 4; ++i) {
            uint32_t rw = 0, cw = 0;
            for (int k = 0; k < 4; ++k) {
                rw |= (uint32_t)(uint8_t)R[i][k] << (8 * k);
                cw |= (uint32_t)(uint8_t)C[i][k] << (8 * k);
            }
            dk.row[i] = rw;
            dk.col[i] = cw;
        }
        dk.ok = true;
        return dk;
    }
    return dk;
}
// dot_keys_search walks the factorisation's scale a down from ~16 000 / |num| with byte searches at every step (~75 us
// for user_costs on the build host): per-call batches (the GUI's script calls) would pay it before every launch, so
// the last few results are kept per thread, keyed by the whole input.
DotKeys dot_keys(const int64_t kap[4][4], int64_t maxmin, int64_t lad_amin = 0, int64_t lad_beta = 0) {
    struct Memo {
        int64_t kap[4][4], maxmin, amin, beta;
        DotKeys dk;
        bool used;
    };
    static thread_local Memo memo[4] = {};
    static thread_local int next = 0;
    for (Memo &e : memo)
        if (e.used && e.maxmin == maxmin && e.amin == lad_amin && e.beta == lad_beta &&
            std::memcmp(e.kap, kap, sizeof(e.kap)) == 0)
            return e.dk;
    Memo &e = memo[next];
    next = (next + 1) & 3;
    std::memcpy(e.kap, kap, sizeof(e.kap));
    e.maxmin = maxmin;
    e.amin = lad_amin;
    e.beta = lad_beta;
    e.dk = dot_keys_search(kap, maxmin, lad_amin, lad_beta);
    e.used = true;
    return e.dk;
}

int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Mode selection.  The packed-integer kernel is exact when
// every value a cell can add is an integral positive Python float, or the int
// 0 of a match; then a cell's Python value is an int exactly when it is 0.
bool i32_eligible(const sed_ctx *c) {
    if (c->K > 4) return false;
    if (c->ins_int || c->del_int) return false;
    if (!is_integral_small(c->ins, 256) || !is_integral_small(c->del, 256) || c->ins < 1 || c->del < 1) return false;
    // offset keys (sed_kernels.hip): the update constant cost - insert - delete - 1 is one byte
    // below 0xFF, i.e. 0 <= cost <= insert + delete <= 255
    if (c->ins + c->del > 255) return false;
    for (int e = 0; e < c->K * c->K; ++e) {
        const double v = c->sub[e];
        if (c->sub_int[e]) {
            if (v != 0) return false;
        } else if (!is_integral_small(v, 256) || v < 1 || v > c->ins + c->del) {
            return false;
        }
    }
    return true;
}

// 16-bit packed distance keys (i32x2 kernels) need every substitution strictly cheaper than
// delete + insert: their update constant cost - delete - insert is a 16-bit 0xFFxx.
bool x2_costs_ok(const sed_ctx *c) {
    for (int a = 0; a < c->K; ++a)
        for (int bb = 0; bb < c->K; ++bb)
            if (a != bb && !(c->sub[a * c->K + bb] < c->ins + c->del)) return false;
    return true;
}

// Unit costs (insert = delete = 1, every mismatch 1, every match the int 0): the bit-parallel lane kernel
// (sed_lane.hip: sed_lane_bitpar_kernel) computes exactly the reference's distance.
bool unit_costs(const sed_ctx *c) {
    if (c->K > 4 || c->ins_int || c->del_int || c->ins != 1.0 || c->del != 1.0) return false;
    for (int a = 0; a < c->K; ++a)
        for (int bb = 0; bb < c->K; ++bb) {
            const int e = a * c->K + bb;
            if (a == bb ? !(c->sub_int[e] && c->sub[e] == 0) : (c->sub_int[e] || c->sub[e] != 1.0)) return false;
        }
    return true;
}

// A set of at most 4 codes with unit costs among themselves (insert = delete = 1.0, every mismatch 1.0, every match
// the int 0), as a bit mask, greedily in code order; 0 when insert / delete are not 1.0.  A pair whose symbols all
// lie in it has the unit-cost distance whatever the other symbols cost (config 5 with N: the pairs without N).
uint32_t unit_subset(const sed_ctx *c) {
    if (c->K > SED_MAX_K || c->ins_int || c->del_int || c->ins != 1.0 || c->del != 1.0) return 0;
    uint32_t S = 0;
    int cnt = 0;
    for (int a = 0; a < c->K && cnt < 4; ++a) {
        bool ok = c->sub_int[a * c->K + a] && c->sub[a * c->K + a] == 0;
        for (int bb = 0; bb < c->K && ok; ++bb)
            if ((S >> bb) & 1u) {
                const int e1 = a * c->K + bb, e2 = bb * c->K + a;
                ok = !c->sub_int[e1] && c->sub[e1] == 1.0 && !c->sub_int[e2] && c->sub[e2] == 1.0;
            }
        if (ok) {
            S |= 1u << a;
            ++cnt;
        }
    }
    return cnt >= 2 ? S : 0;
}

// Dyadic costs over at most 8 symbols (sed_lane.hip: sed_lane_scaled_kernel): the smallest S = 2^k (k <= 8) that makes
// insert, delete and every update cost integral, with 1 <= insert * S, delete * S, 0 <= cost * S <= (insert + delete)
// * S <= 255 (the offset keys' update byte) and the lane block's n * delete + 32 * insert within the 16-bit D field.
// Simple typing is the caller's condition (every value a float, or the int 0 of a match).
bool scaled_costs(const sed_ctx *c, sed_scaled_params *sp) {
    if (c->K > 8) return false;
    for (int k = 0; k <= 8; ++k) {
        const double S = std::ldexp(1.0, k);
        auto integral = [&](double v) { const double x = v * S; return x == std::floor(x) && x >= 0 && x <= 255; };
        bool ok = integral(c->ins) && integral(c->del) && c->ins * S >= 1 && c->del * S >= 1 &&
                  (c->ins + c->del) * S <= 255;
        for (int e = 0; e < c->K * c->K && ok; ++e) ok = integral(c->sub[e]) && c->sub[e] <= c->ins + c->del;
        if (!ok) continue;
        const uint32_t ins = (uint32_t)(c->ins * S), del = (uint32_t)(c->del * S);
        if ((double)SED_LANE_MAXN * del + (SED_LANE_MAXM + 1) * (double)ins > 65533.0) return false;
        *sp = sed_scaled_params{};
        sp->ins = ins;
        sp->del = del;
        sp->inv_scale = std::ldexp(1.0, -k);
        for (int a = 0; a < 8; ++a)
            for (int b = 0; b < 8; ++b) {
                const uint32_t v = (a < c->K && b < c->K) ? (uint32_t)(c->sub[a * c->K + b] * S) : 0u;
                sp->row[a][b >> 2] |= ((v - ins - del - 1u) & 0xFFu) << (8 * (b & 3));
            }
        return true;
    }
    return false;
}

// "simple typing": a cell's value is an int exactly when it equals 0.
bool simple_typing(const sed_ctx *c) {
    if (c->ins_int || c->del_int || !(c->ins > 0) || !(c->del > 0)) return false;
    for (int e = 0; e < c->K * c->K; ++e) {
        if (c->sub_int[e] ? c->sub[e] != 0 : !(c->sub[e] > 0)) return false;
    }
    return true;
}

int choose_R(int mode, int max_n, int forced) {
    if (forced) return forced;
    const int want = next_pow2(std::max(1, (max_n + 63) / 64));
    if (mode == SED_MODE_I32) return std::min(16, std::max(4, want));
    return std::min(8, std::max(4, want));
}

// fp64 wave kernel: R = 4 or 8 by a cost model over the batch, not by its longest pair.  A pair costs
// stripes(R) * (m + 63) steps of R rows plus a per-step overhead worth ~0.6 rows (fitted to the iupac workload,
// 1024^2: R = 8 5.01 ms, R = 4 5.34 ms).  The timing workload (lengths 10..500) then takes R = 4: 4.59 against
// 4.82 ms at R = 8 (profiles/r03/fp64_R.jsonl).
// lane: the batch routes short pairs to the fp64 lane kernel (fill_batch: use_lane), which never runs the wave
// kernel, so they are left out of the model.
// seg: pairs may run in 16-lane segments, four per wave (sed_kernels.hip: sed_wf_f64_kernel SW = 16): stripes of 16 R
// rows and a 15-step ramp, at a quarter of a wave: stripes16(R) * (m + 15) * (R + 0.6) / 4, times a penalty for the
// segments' per-lane loop control and stripe changes, fitted to the two fp64 workloads (profiles/r04/seg/ab_seg.jsonl):
// timing (R = 4) ran 3.34 against 4.48 ms where the bare model says 0.71 of it (penalty 1.05), iupac (1024^2, R = 8)
// 5.41 against 4.87 ms where it says 0.96 (penalty 1.16).
double f64_cost(int n, int m, int R, int SW) {
    const double pen = SW == 16 ? (R >= 8 ? 1.16 : 1.05) : 1.0;
    return (double)((n + SW * R - 1) / (SW * R)) * (m + SW - 1) * (R + 0.6) * SW / 64.0 * pen;
}
bool f64_seg_better(int n, int m, int R) { return f64_cost(n, m, R, 16) < f64_cost(n, m, R, 64); }
int choose_R_f64(const int32_t *len_a, const int32_t *len_b, int npairs, bool lane, bool seg) {
    double cost[2] = {0, 0};
    for (int p = 0; p < npairs; ++p) {
        if (lane && len_a[p] >= 1 && len_a[p] <= SED_LANE_MAXN && len_b[p] >= 1 && len_b[p] <= SED_LANE_MAXM) continue;
        for (int k = 0; k < 2; ++k) {
            const int R = 4 << k;
            const double c64 = f64_cost(len_a[p], len_b[p], R, 64);
            cost[k] += seg ? std::min(c64, f64_cost(len_a[p], len_b[p], R, 16)) : c64;
        }
    }
    return cost[1] < cost[0] ? 8 : 4;
}

// fp64 batches of several pairs: does the SPLIT route (R = 2) beat one wave per pair?  A SPLIT workgroup holds its slot
// for its pair's whole stripe chain, m + 63 steps plus ~64 steps of lag per stripe above it, so a batch whose stripes
// outnumber the resident workgroups (~256) runs in rounds, and long narrow pairs (n >> m) spend most of each round
// waiting on the lag.  The lone waves (one per pair, all resident) take the f64_cost units of their stripes.  Fitted to
// 32 batches of 16..256 pairs, 300..4000 rows, 100..2000 columns, scripts and distances (tools/fp64_split_batch.py,
// profiles/r06/fp64_split): the model picks the faster route in all 32; SPLIT lost up to 2.7x on 256 pairs of
// 2000 x 100 (1.34 against 0.49 ms) and won up to 3.8x on 64 pairs of 2000^2 (0.95 against 3.65 ms).
bool f64_split_pays(const int32_t *len_a, const int32_t *len_b, int npairs, bool script) {
    double lone = 0, lat_max = 0, slots = 0;
    for (int p = 0; p < npairs; ++p) {
        const int n = len_a[p], m = len_b[p];
        if (n <= 0 || m <= 0) continue;
        lone = std::max(lone, std::min(f64_cost(n, m, 4, 64), f64_cost(n, m, 8, 64)));
        const double ns = (double)((n + 127) / 128), lat = (double)m + 63.0 + 64.0 * ns;
        lat_max = std::max(lat_max, lat);
        slots += ns * lat;
    }
    const double t_split = (script ? 0.318 : 0.138) + (script ? 7.40e-5 : 6.53e-5) * std::max(lat_max, slots / 256.0);
    const double t_lone = (script ? 0.359 : 0.140) + (script ? 5.44e-5 : 5.09e-5) * lone;
    return t_split < t_lone;
}

// the next run's SPLIT epoch, zeroing the hand-off words first when no word may carry a tag of its own (see split_epoch)
hipError_t next_split_epoch(sed_batch *b, hipStream_t s, uint32_t *epoch) {
    *epoch = b->split_epoch % 32767u + 1u;
    b->split_epoch = *epoch;
    if (!b->split || b->bnd_words == 0) return hipSuccess;
    if (*epoch == 1 || b->d_bnd.gen != b->bnd_zero_gen) {
        hipError_t e = hipMemsetAsync(b->d_bnd.p, 0, b->d_bnd.cap, s);
        if (e != hipSuccess) return e;
        b->bnd_zero_gen = b->d_bnd.gen;
    }
    return hipSuccess;
}

// Event-log entries {DP start, DP end, traceback start, traceback end}, created ahead of the runs
// that use them (outside any timed loop for up to `more` runs).  Batches in parts also get the parts' entries
// (plog), up to the same count, so no event is created while runs are being timed.
hipError_t grow_log(sed_batch *b, size_t more) {
    for (size_t i = 0; i < more; ++i) {
        std::array<hipEvent_t, 4> a{};
        for (auto &x : a) {
            hipError_t e = hipEventCreate(&x);
            if (e != hipSuccess) return e;
        }
        b->log.push_back(a);
    }
    while (b->nparts > 1 && b->plog.size() < b->log.size()) {
        std::array<hipEvent_t, 12> a{};
        for (auto &x : a) {
            hipError_t e = hipEventCreate(&x);
            if (e != hipSuccess) return e;
        }
        b->plog.push_back(a);
    }
    return hipSuccess;
}

int fill_batch(sed_batch *b, const uint8_t *codes_a, const int64_t *off_a, const int32_t *len_a,
               const uint8_t *codes_b, const int64_t *off_b, const int32_t *len_b, int32_t npairs,
               uint32_t flags) {
    sed_ctx *c = b->ctx;
    if (!c->have_costs) return c->fail(SED_E_STATE, "sed_set_costs() was not called");
    {  // a refill must not overwrite a running part; a fault of the previous run is reported as such
        hipError_t e = hipSuccess;
        for (hipStream_t ps : b->part_stream)
            if (e == hipSuccess && ps) e = hipStreamSynchronize(ps);
        if (e == hipSuccess && b->dp2_stream) e = hipStreamSynchronize(b->dp2_stream);
        if (e == hipSuccess && b->tb_stream) e = hipStreamSynchronize(b->tb_stream);
        // zero-copy runs store into h_out from the context's stream, which a refill memsets below
        if (e == hipSuccess && b->zc_busy) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return c->hipfail(e, "previous run");
        b->zc_busy = false;
    }
    if (npairs < 0 || (npairs > 0 && (!codes_a || !off_a || !len_a || !codes_b || !off_b || !len_b)))
        return c->fail(SED_E_ARG, "bad batch arguments");
    b->npairs = npairs;
    b->flags = flags;
    b->ran = false;
    b->runs = 0;
    b->chain_launches[0] = b->chain_launches[1] = b->chain_launches[2] = 0;
    b->nbuf = (flags & SED_PIPELINE) ? 3 : 1;
    b->n.assign(len_a, len_a + npairs);
    b->m.assign(len_b, len_b + npairs);
    int max_n = 0, max_m = 0;
    for (int p = 0; p < npairs; ++p) {
        if (len_a[p] < 0 || len_b[p] < 0) return c->fail(SED_E_ARG, "negative length at pair %d", p);
        max_n = std::max(max_n, len_a[p]);
        max_m = std::max(max_m, len_b[p]);
        const uint8_t *pa = codes_a + off_a[p], *pb = codes_b + off_b[p];
        for (int i = 0; i < len_a[p]; ++i)
            if (pa[i] >= c->K) return c->fail(SED_E_ARG, "code %d >= K at pair %d", pa[i], p);
        for (int j = 0; j < len_b[p]; ++j)
            if (pb[j] >= c->K) return c->fail(SED_E_ARG, "code %d >= K at pair %d", pb[j], p);
    }
    // ---- mode ----
    int mode;
    const bool elig = i32_eligible(c);
    switch (c->opt_mode) {
    case 1:
        if (!elig) return c->fail(SED_E_RANGE, "costs are not eligible for the integer kernel");
        mode = SED_MODE_I32;
        break;
    case 2: mode = simple_typing(c) ? SED_MODE_F64 : SED_MODE_F64_TYPED; break;
    case 3: mode = SED_MODE_F64_TYPED; break;
    default: mode = elig ? SED_MODE_I32 : (simple_typing(c) ? SED_MODE_F64 : SED_MODE_F64_TYPED);
    }
    // fp64 batches whose short pairs go to the lane kernel (use_lane below: distance only, simple typing)
    const bool f64_lane = c->opt_lane != 2 && !(flags & SED_WANT_SCRIPT) && (flags & SED_NO_LEN) && simple_typing(c);
    // fp64 batches of more than 256 wave pairs may run short pairs in 16-lane segments (SED_OPT_SEG; the window
    // traceback of smaller batches reads the 64-lane layout only)
    int nwave_f64 = 0;
    double lane_cells_f64 = 0;  // the largest fp64 lane pair (n m): one lane walks all of it
    for (int p = 0; p < npairs; ++p) {
        if (len_a[p] <= 0 || len_b[p] <= 0) continue;
        if (f64_lane && len_a[p] <= SED_LANE_MAXN && len_b[p] <= SED_LANE_MAXM)
            lane_cells_f64 = std::max(lane_cells_f64, (double)len_a[p] * len_b[p]);
        else
            ++nwave_f64;
    }
    bool seg_ok = c->opt_seg != 2 && nwave_f64 > 256;
    int R = (mode == SED_MODE_I32 || c->opt_R) ? choose_R(mode, max_n, c->opt_R)
                                                : choose_R_f64(len_a, len_b, npairs, f64_lane && mode == SED_MODE_F64, seg_ok);
    if (mode == SED_MODE_I32) {
        const int ROWS = 64 * R;
        bool fits = true;
        for (int p = 0; p < npairs && fits; ++p) {
            // offset keys: i*delete + j*insert over every computed cell (padded rows, the columns
            // the wave or the lane kernel runs past m) must stay below the bias, and L < 2^14
            const double npad = (double)((len_a[p] + ROWS - 1) / ROWS) * ROWS;
            const double cols = (double)std::max(len_b[p] + 64 + 64 / R, SED_LANE_MAXM);
            const double dsum = npad * c->del + cols * c->ins;
            if (dsum > 65533.0 || npad + cols >= 16384.0) fits = false;
        }
        if (!fits) {
            if (c->opt_mode == 1) return c->fail(SED_E_RANGE, "integer key would overflow (D < 2^16, L < 2^14)");
            mode = simple_typing(c) ? SED_MODE_F64 : SED_MODE_F64_TYPED;
            R = c->opt_R ? c->opt_R : choose_R_f64(len_a, len_b, npairs, f64_lane && mode == SED_MODE_F64, seg_ok);
        }
    } else if (c->K > SED_MAX_K) {
        return c->fail(SED_E_ALPHABET, "alphabet of %d symbols exceeds %d", c->K, SED_MAX_K);
    }
    if (mode == SED_MODE_I32 ? !(R == 4 || R == 8 || R == 16 || R == 32) : !(R == 2 || R == 4 || R == 8))
        return c->fail(SED_E_ARG, "unsupported rows-per-lane %d for mode %d", R, mode);
    // SPLIT (integer kernel): one wave per stripe with inter-workgroup hand-offs, for
    // batches too small to fill the GPU with one wave per pair (config 2, GUI calls).
    bool split = false;
    if (mode == SED_MODE_I32 && c->opt_split != 2) {
        split = c->opt_split == 1 || (npairs <= 256 && max_n > 256 && c->opt_chain != 1 && c->opt_chain < 3);
        if (split && !c->opt_R) R = 4;
        if (split && R != 4 && R != 8 && R != 16 && R != 32) split = false;
    } else if (mode != SED_MODE_I32 && c->opt_split != 2 && (!seg_ok || c->opt_split == 1)) {
        // fp64 SPLIT (sed_wf_f64_split_kernel, R = 4): batches of few pairs, whose lone fp64 waves are otherwise one
        // SIMD each.  It also runs the one-stripe pairs (tools/fp64_call_scaling.py, profiles/r05/s25: 30 nt 39.9
        // against 40.6 us per call, 200 nt 72 against 87, 500 nt 151 against 255, 2000 nt 544 against 3497), since
        // its lone wave reads each step's table entries a step ahead; distance-only batches whose pairs all fit the
        // lane kernels keep those
        // R = 2 by default: a lone fp64 wave is issue-bound (~80 VALU per step at R = 4), so halving the rows per
        // step outweighs the twice as many hand-offs (per call, 500^2: 150 us at R = 4, tools/fp64_call_scaling.py)
        // A lane pair past 256 cells also goes SPLIT: 30^2 distance-only took 45 us per call on the lane kernel,
        // 32 us SPLIT (10^2: 27 against 33 us)
        split = (c->opt_split == 1 || (npairs <= 256 && (nwave_f64 > 0 || lane_cells_f64 > 256.0) &&
                                       (npairs == 1 || f64_split_pays(len_a, len_b, npairs, (flags & SED_WANT_SCRIPT) != 0)))) &&
                (!c->opt_R || c->opt_R == 2 || c->opt_R == 4);
        if (split) R = c->opt_R ? c->opt_R : 2;
        // (automatic route: its hand-off words, 24 B per column and stripe, stay under 4 GB)
        if (split && c->opt_split != 1 && !c->opt_R) {
            double words = 0;
            for (int p = 0; p < npairs; ++p) {
                const double st = (double)((len_a[p] + 64 * R - 1) / (64 * R)), ch = (double)((len_b[p] + 127) / 64 + 2);
                if (st > 1) words += st * ch * 64.0 * 6.0;
            }
            if (4.0 * words > 4e9) {
                split = false;
                R = choose_R_f64(len_a, len_b, npairs, f64_lane && mode == SED_MODE_F64, seg_ok);
            }
        }
    }
    if (split && mode != SED_MODE_I32) seg_ok = false;  // (SED_OPT_SPLIT = 1 over the segments of > 256 wave pairs)
    // rows per lane 2 is the fp64 SPLIT route's; an fp64 batch that does not take it runs the automatic R
    if (mode != SED_MODE_I32 && R == 2 && !split) R = choose_R_f64(len_a, len_b, npairs, f64_lane && mode == SED_MODE_F64, seg_ok);
    b->split = split;
    b->mode = mode;
    b->R = R;
    const int ROWS = 64 * R;
    const bool want_tb = (flags & SED_WANT_SCRIPT) != 0;
    // CK traceback (R = 4/8/16 wave kernels, stripe or CHAIN, not SPLIT): distance-key forward kernel +
    // checkpoints, traceback recomputes tiles.  Auto: batches past the window kernel's 256 pairs whose pairs
    // are large enough.  The forward kernel saves ~1.7 VALU per cell (n m), the tile recompute costs per
    // path step (n + m): measured, config 4 (4096^2) step 20.4 -> 15.0 ms, config 3 (512^2) 2.90 -> 4.40 ms;
    // break-even near 1024^2, i.e. sum(n m) / sum(n + m) = 512.
    double sum_nm = 0, sum_len = 0;
    for (int p = 0; p < npairs; ++p) {
        sum_nm += (double)len_a[p] * len_b[p];
        sum_len += (double)len_a[p] + len_b[p];
    }
    b->ck = want_tb && mode == SED_MODE_I32 && !split && (R == 4 || R == 8 || R == 16) && c->opt_tb != 1 &&
            (c->opt_tb == 2 || (npairs > 256 && sum_nm >= 512.0 * sum_len));
    // SED_PIPELINE is a hint: checkpoint batches run their traceback after the DP on one stream (in parts on
    // several, run_batch_parts).  Both kernels are issue-bound, so overlapping a run's traceback with the next run's
    // forward only adds contention (config 4: 20.33 ms sequential against 20.5-20.8 ms pipelined in round 1,
    // profiles/r01_ck/ab_pipeline.jsonl; 11.13 against 9.78 ms for 2 pipelined parts in round 5,
    // profiles/r05/s14/ab.jsonl) and saves two checkpoint buffers.
    if (b->ck) b->nbuf = 1;
    // few pairs with per-cell codes (config 2, the GUI): the traceback walks the stripes of a pair in parallel
    // (a map of every stripe's exits, then one wave per stripe segment) instead of one ~n+m step chain;
    // SED_TBPAR=0/1 overrides (A/B)
    static const int tbpar_env = [] { const char *e = getenv("SED_TBPAR"); return e ? atoi(e) : -1; }();
    // (never with fp64 pairs in 16-lane segments: the stripe kernels read the 64-lane code layout only)
    b->tbpar = want_tb && !b->ck && (R == 4 || R == 2) && (tbpar_env < 0 ? npairs <= 64 : tbpar_env > 0) &&
               !(seg_ok && mode != SED_MODE_I32);
    b->tbpar_items = b->tbpar_kmax = 0;
    // SPLIT script batches: checkpoints + a tile-parallel recompute of the codes (dot or distance keys in the forward:
    // 2-3 VALU per cell against the ladder keys' 5.2 on the latency-bound stripe chain)
    b->split_ck = want_tb && split && mode == SED_MODE_I32 && R == 4 && c->opt_splitck != 2;
    b->ck_tiles = 0;

    // ---- layout ----
    b->pd.assign(npairs, sed_pair_desc{});
    std::vector<int2> tasks;
    std::vector<int32_t> lane_idx, seg_idx;
    // lane-per-pair kernels: integer keys (any flags), or fp64 distance-only in "simple typing" mode
    // a batch of a few pairs (the per-call path) leaves the GPU empty, so one lane walking a pair alone only pays off
    // for a small distance-only pair: a 30-nt script call took 42 us on the lane kernel and 34 us on the wave kernels,
    // a 30-nt distance call 19 against 22 us (tools/zc_ab.py SED_OPT_LANE, profiles/r05/s38)
    const bool few_pairs = npairs <= 16 && c->opt_lane == 0;
    const bool use_lane = !split && c->opt_lane != 2 &&
                          (mode == SED_MODE_I32 || (mode == SED_MODE_F64 && !want_tb && (flags & SED_NO_LEN)));
    uint64_t aw = 0, bw = 0, tbw = 0, bndw = 0, opw = 0, mapw = 0;
    const bool packed = (mode == SED_MODE_I32);
    double cells = 0, in_bytes = 0, tb_bytes = 0, ck_bytes = 0;
    for (int p = 0; p < npairs; ++p) {
        const int nn = len_a[p], mm = len_b[p];
        sed_pair_desc &d = b->pd[p];
        d.n = nn;
        d.m = mm;
        d.a_off = aw;
        d.b_off = bw;
        if (packed) {
            aw += (nn + 15) / 16;
            bw += (mm + 15) / 16;
        } else {  // bytes, each sequence 16-byte aligned (the lane kernels read str2 as two 16-byte words)
            aw += ((uint64_t)nn + 15) & ~(uint64_t)15;
            bw += ((uint64_t)mm + 15) & ~(uint64_t)15;
        }
        d.tb_off = tbw;
        d.bnd_off = bndw;
        d.ops_off = opw;
        d.map_off = (int32_t)mapw;  // stripe-parallel traceback: this pair's exit map
        if (use_lane && nn >= 1 && nn <= SED_LANE_MAXN && mm >= 1 && mm <= SED_LANE_MAXM &&
            !(few_pairs && (want_tb || (double)nn * mm > 1024.0))) {
            d.lane = 1;
            lane_idx.push_back(p);
            if (want_tb) tbw += 2 * (uint64_t)nn;  // one uint2 of 2-bit ops per row
        } else if (nn > 0 && mm > 0) {
            // fp64 pairs the cost model prefers in 16-lane segments (sed_kernels.hip: sed_wf_f64_kernel SW = 16)
            const bool seg = !packed && seg_ok && (c->opt_seg == 1 || f64_seg_better(nn, mm, R));
            const uint64_t SW = seg ? 16 : 64;
            if (seg) {
                d.pad[1] = 1;
                seg_idx.push_back(p);
            }
            const uint64_t G = 64 / R;  // steps per 16-byte traceback group (sed_kernels.hip: Grp)
            const uint64_t nstripes = (nn + SW * R - 1) / (SW * R);
            const uint64_t SG = (mm + SW - 1 + G - 1) / G * G;
            const uint64_t nchunks = (SG + SW - 1) / SW;
            if (want_tb) {  // CK: per stripe nchunks x (R+1) x 64 column checkpoints + (SG/G) x 64 row checkpoints
                const uint64_t wck = nstripes * (nchunks * (R + 1) * 64 + (SG / G) * SED_CK_RW);
                const uint64_t w = b->ck ? wck : nstripes * (SG / G) * SW * 4 + (b->split_ck ? wck : 0);
                tbw += w;
                ck_bytes += 4.0 * (double)w;
                if (b->split_ck) b->ck_tiles = std::max<int>(b->ck_tiles, (int)(nstripes * R * nchunks));
            }
            // SPLIT: 64-bit {epoch tag, value} words per column and stripe (the tagged hand-off, sed_kernels.hip)
            // (fp64: D, L and T planes; SPLIT: three 64-bit {tag, D low | D high | L key and T} words)
            if (nstripes > 1) bndw += (nchunks + 2) * SW * (packed ? (split ? 2 : 1) : (split ? 6 : 4)) * (split ? nstripes : 1);
            if (b->tbpar && nstripes >= 3) {  // {exit column, ops} per stripe and column, then per 64-row band and column
                const uint64_t nbands = ((uint64_t)nn + 63) / 64 - 1;  // bands 1 .. nbt-1 (the banded emit's)
                mapw += (nstripes + nbands) * (uint64_t)(mm + 1) * 2;
                // band map: workgroups of 256 columns per band (a superset of the stripe map kernel's middle
                // stripes + sink; the compose kernel's grid is derived from it, sed_launch_traceback_stripes)
                b->tbpar_items = std::max<int>(b->tbpar_items, (int)(nbands * ((mm + 256) / 256) * 256));
            }
            b->tbpar_kmax = std::max<int>(b->tbpar_kmax, (int)(nstripes >= 3 ? nstripes : 1));
            if (split) {
                for (uint64_t k = 0; k < nstripes; ++k) tasks.push_back(make_int2(p, (int)k));
            }
        } else if (split) {
            tasks.push_back(make_int2(p, 0));
        }
        if (b->tbpar && !d.lane) {
            b->tbpar_items = std::max<int>(b->tbpar_items, (nn + mm + 15) / 16);  // the map kernel zeroes these
            b->tbpar_kmax = std::max(b->tbpar_kmax, 1);
        }
        opw += (uint64_t)(nn + mm + 15) / 16;
        cells += (double)nn * mm;
        in_bytes += packed ? (nn + mm) / 4.0 : (double)(nn + mm);
    }
    // a SPLIT script batch whose pairs all have an empty side has no tile to recompute: plain per-cell codes (the
    // traceback walks only the border)
    if (b->split_ck && b->ck_tiles == 0) b->split_ck = false;
    // no pair with 3 stripes or more: the stripe map has nothing to do and the emit kernel walks every pair in one
    // segment, as the window traceback does without the map launch and the OR into zeroed scripts (so zero-copy
    // results apply)
    if (b->tbpar && b->tbpar_kmax < 3 && tbpar_env < 0) {
        b->tbpar = false;
        b->tbpar_items = b->tbpar_kmax = 0;
    }
    // algorithmic traceback bytes: the 2-bit choice of every cell, or (CK) the checkpoints written
    tb_bytes = b->ck ? ck_bytes : cells * 0.25;
    b->tb_words = tbw;
    b->bnd_words = bndw;
    b->nlane = (int)lane_idx.size();
    b->nwave = npairs - b->nlane;
    // segment pairs by shape, so the four pairs of a wave run alike
    std::stable_sort(seg_idx.begin(), seg_idx.end(), [&](int32_t x, int32_t y) {
        return len_a[x] != len_a[y] ? len_a[x] < len_a[y] : len_b[x] < len_b[y];
    });
    b->nseg = (int)seg_idx.size();
    // distance-only integer lane pairs: two pairs of equal n per lane (sed_lane.hip: i32x2). Stable
    // sort by n, pair neighbours of equal n; a pair without a partner shares its lane with itself.
    b->nlane_x2 = 0;
    // unit costs: one pair per lane, bit-parallel (~18 word ops per str1 symbol instead of 2 per cell)
    b->lane_bitpar = mode == SED_MODE_I32 && !want_tb && (flags & SED_NO_LEN) && c->opt_bitpar != 2 &&
                     !lane_idx.empty() && unit_costs(c);
    // fp64 lane pairs whose symbols all lie in a unit-cost subset: bit-parallel inside the fp64 lane kernel, first
    // in the lane list so that waves stay uniform
    b->umask = 0;
    b->nbitpar_f64 = 0;
    if (mode == SED_MODE_F64 && use_lane && !want_tb && (flags & SED_NO_LEN) && c->opt_bitpar != 2 &&
        !lane_idx.empty() && (b->umask = unit_subset(c)) != 0) {
        auto inside = [&](const uint8_t *s, int len) {
            for (int i = 0; i < len; ++i)
                if (!((b->umask >> s[i]) & 1u)) return false;
            return true;
        };
        for (int32_t x : lane_idx)
            if (inside(codes_a + off_a[x], len_a[x]) && inside(codes_b + off_b[x], len_b[x])) {
                b->pd[x].pad[0] = 1;
                ++b->nbitpar_f64;
            }
        std::stable_partition(lane_idx.begin(), lane_idx.end(), [&](int32_t x) { return b->pd[x].pad[0] != 0; });
    }
    // fp64 lane pairs under dyadic costs over <= 8 symbols: the scaled-integer lane kernel (exact, 3 VALU per cell)
    b->scaled = mode == SED_MODE_F64 && use_lane && !want_tb && (flags & SED_NO_LEN) && c->opt_scaled != 2 &&
                !lane_idx.empty() && scaled_costs(c, &b->sp);
    if (b->scaled) {
        b->sp.umask = b->umask;
        b->sp.umap = 0;  // 2-bit unit-subset code of every code < 8 (the bit-parallel pairs)
        for (uint32_t cc = 0; cc < 8; ++cc)
            if ((b->umask >> cc) & 1u) b->sp.umap |= (uint32_t)__builtin_popcount(b->umask & ((1u << cc) - 1u)) << (2 * cc);
    }
    const bool x2_ok = mode == SED_MODE_I32 && x2_costs_ok(c);
    // 16-bit offset keys: n*delete + 32*insert (the lane kernel's whole block) within 0xFFFF
    bool lane_fit16 = true;
    for (int32_t x : lane_idx)
        if ((double)len_a[x] * c->del + SED_LANE_MAXM * c->ins > 65535.0) lane_fit16 = false;
    if (x2_ok && lane_fit16 && !b->lane_bitpar && !want_tb && (flags & SED_NO_LEN) && c->opt_pack != 2 &&
        !lane_idx.empty()) {
        std::stable_sort(lane_idx.begin(), lane_idx.end(), [&](int32_t x, int32_t y) { return len_a[x] < len_a[y]; });
        std::vector<int32_t> two;
        two.reserve(lane_idx.size() + 1);
        for (size_t q = 0; q < lane_idx.size();) {
            const int32_t x = lane_idx[q];
            const bool partner = q + 1 < lane_idx.size() && len_a[lane_idx[q + 1]] == len_a[x];
            two.push_back(x);
            two.push_back(partner ? lane_idx[q + 1] : x);
            q += partner ? 2 : 1;
        }
        lane_idx.swap(two);
        b->nlane_x2 = (int)(lane_idx.size() / 2);
    }

    // distance-only integer wave pairs: two of equal n per wave (sed_kernels.hip: i32x2), the one with
    // the larger m first (its bottom-row buffer serves both).  Partners come from a (n, m) sort and
    // must have 3 min(m) > max(m): the wave runs max(m) columns at 4 ops per 2 cells, which beats 3 ops
    // per cell of each pair alone while 4 max(m) < 3 (m_P + m_Q).  Packed pairs are marked lane = 2,
    // so the other wave kernels (and CHAIN mode) skip them.
    std::vector<int32_t> x2;
    b->nwave_x2 = 0;
    if (x2_ok && !split && !want_tb && (flags & SED_NO_LEN) && c->opt_pack != 2 && b->nwave > 1) {
        std::vector<int32_t> w;
        for (int p = 0; p < npairs; ++p) {
            // 16-bit offset keys over the wave's block: padded rows x (m + 63 + G) columns within 0xFFFF
            const double npad = (double)((len_a[p] + ROWS - 1) / ROWS) * ROWS;
            const bool fit16 = npad * c->del + (double)(len_b[p] + 64 + 64 / R) * c->ins <= 65535.0;
            if (!b->pd[p].lane && len_a[p] > 0 && len_b[p] > 0 && fit16) w.push_back(p);
        }
        std::stable_sort(w.begin(), w.end(), [&](int32_t x, int32_t y) {
            return len_a[x] != len_a[y] ? len_a[x] < len_a[y] : len_b[x] < len_b[y];
        });
        for (size_t q = 0; q + 1 < w.size();) {
            const int32_t x = w[q], y = w[q + 1];  // len_b[x] <= len_b[y]
            if (len_a[x] == len_a[y] && 3LL * len_b[x] > len_b[y]) {
                x2.push_back(y);
                x2.push_back(x);
                b->pd[x].lane = b->pd[y].lane = 2;
                q += 2;
            } else {
                ++q;
            }
        }
        b->nwave_x2 = (int)(x2.size() / 2);
        b->nwave -= (int)x2.size();
    }

    // ---- CHAIN mode (integer keys): single-stripe wave pairs run back to back, one chain per
    // wave, so each pair's 63-step ramp overlaps the previous pair's drain (sed_kernels.hip) ----
    std::vector<int32_t> chain_pairs, chain_off;
    b->nchains = 0;
    b->chain_dyn = false;
    if (mode == SED_MODE_I32 && !split && c->opt_chain != 2 && (R == 4 || R == 8) && b->nwave > 0) {
        // SIMDs x the chain kernel's waves per SIMD, unless capped (tests: several fetched pairs per wave)
        const int resident = c->opt_chain_waves > 0 ? c->opt_chain_waves : 1024 * 5;
        bool ok = true;
        for (int p = 0; p < npairs && ok; ++p)
            if (!b->pd[p].lane && (len_a[p] < 1 || len_a[p] > ROWS || len_b[p] < 1)) ok = false;
        if (ok && c->opt_chain >= 3) {  // static chains of opt_chain pairs (tests, A/B)
            const int L = c->opt_chain;
            double total = 0;
            for (int p = 0; p < npairs; ++p)
                if (!b->pd[p].lane) total += (double)((len_b[p] + 63) & ~63);
            const int nch = std::max(1, (b->nwave + L - 1) / L);
            const double target = total / nch;
            double acc = 0;
            chain_off.push_back(0);
            for (int p = 0; p < npairs; ++p) {
                if (b->pd[p].lane) continue;
                chain_pairs.push_back(p);
                acc += (double)((len_b[p] + 63) & ~63);
                if (acc >= target * (double)chain_off.size() && (int)chain_off.size() < nch)
                    chain_off.push_back((int32_t)chain_pairs.size());
            }
            if (chain_off.back() != (int32_t)chain_pairs.size()) chain_off.push_back((int32_t)chain_pairs.size());
            b->nchains = (int)chain_off.size() - 1;
        } else if (ok && (c->opt_chain == 1 || b->nwave >= 2 * resident)) {
            // dynamic: `resident` persistent waves take the next pair from a device counter
            for (int p = 0; p < npairs; ++p)
                if (!b->pd[p].lane) chain_pairs.push_back(p);
            b->nchains = std::min(b->nwave, resident);
            b->chain_dyn = true;
        }
    }
    b->ntasks = (int)tasks.size();
    b->ops_words = opw;
    b->cells = cells;
    b->algo_bytes = in_bytes + (want_tb ? tb_bytes : 0) + 16.0 * npairs;

    // ---- pack & upload ----
    const uint64_t pad_words = (uint64_t)ROWS / 16 * 2 + 64;
    std::vector<uint32_t> ha, hb;
    std::vector<uint8_t> ha8, hb8;
    if (packed) {
        ha.assign(aw + pad_words, 0);
        hb.assign(bw + pad_words, 0);
        // 16 codes per word, each word built in a register (an OR into memory per code was ~1 ns per symbol)
        auto pack2 = [](const uint8_t *src, int len, uint32_t *dst) {
            const int full = len >> 4;
            for (int w = 0; w < full; ++w) {
                const uint8_t *q = src + 16 * w;
                uint32_t v = 0;
                for (int k = 0; k < 16; ++k) v |= (uint32_t)q[k] << (2 * k);
                dst[w] = v;
            }
            if (len & 15) {
                uint32_t v = 0;
                for (int k = 0; k < (len & 15); ++k) v |= (uint32_t)src[16 * full + k] << (2 * k);
                dst[full] = v;
            }
        };
        for (int p = 0; p < npairs; ++p) {
            pack2(codes_a + off_a[p], len_a[p], ha.data() + b->pd[p].a_off);
            pack2(codes_b + off_b[p], len_b[p], hb.data() + b->pd[p].b_off);
        }
    } else {
        ha8.assign(aw + 64, 0);
        hb8.assign(bw + 64, 0);
        for (int p = 0; p < npairs; ++p) {
            if (len_a[p]) memcpy(ha8.data() + b->pd[p].a_off, codes_a + off_a[p], len_a[p]);
            if (len_b[p]) memcpy(hb8.data() + b->pd[p].b_off, codes_b + off_b[p], len_b[p]);
        }
    }
    const size_t sa = packed ? ha.size() * 4 : ha8.size(), sb = packed ? hb.size() * 4 : hb8.size();
    const void *hsa = packed ? (const void *)ha.data() : (const void *)ha8.data();
    const void *hsb = packed ? (const void *)hb.data() : (const void *)hb8.data();
    b->chain_npairs = chain_pairs.size();
    // Small batches (the drop-in module's per-call pairs, sed_run_batch): every input array and the zeroed results go
    // up as one blob from the context's pinned staging buffer, with no upload sync (the staging buffer is not
    // rewritten before that copy has completed: pin_busy), instead of one pageable copy per array and a memset.
    const size_t s_pd = sizeof(sed_pair_desc) * std::max(1, npairs), s_tasks = sizeof(int2) * std::max<size_t>(1, tasks.size()),
                 s_chain = 4 * (chain_pairs.size() + chain_off.size() + 4), s_lane = 4 * std::max<size_t>(1, lane_idx.size()),
                 s_x2 = 4 * std::max<size_t>(1, x2.size()), s_res = sizeof(sed_result) * std::max(1, npairs),
                 s_seg = 4 * std::max<size_t>(1, seg_idx.size());
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o_pd = 0, o_sa = o_pd + al(s_pd), o_sb = o_sa + al(sa), o_tasks = o_sb + al(sb), o_chain = o_tasks + al(s_tasks),
           o_lane = o_chain + al(s_chain), o_x2 = o_lane + al(s_lane), o_seg = o_x2 + al(s_x2), o_res = o_seg + al(s_seg),
           o_ops = o_res + al(s_res),
           total = o_ops + al(4 * std::max<uint64_t>(1, opw));  // (results and scripts adjacent: one download)
    b->small = b->nbuf == 1 && total <= SED_SMALL_BATCH_BYTES;
    b->zc = b->small && !b->tbpar && c->opt_zc != 2;
    bool okalloc = b->d_bnd.reserve(4 * std::max<uint64_t>(1, bndw)) && b->d_tbmap.reserve(4 * std::max<uint64_t>(1, mapw));
    if (b->small) {
        okalloc = okalloc && b->d_small.reserve(total);
    } else {
        okalloc = okalloc && b->d_ops.reserve(4 * std::max<uint64_t>(1, opw)) && b->d_pd.reserve(s_pd) && b->d_seqa.reserve(sa) && b->d_seqb.reserve(sb) &&
                  b->d_tasks.reserve(s_tasks) && b->d_lane.reserve(s_lane) && b->d_chain.reserve(s_chain) &&
                  b->d_x2.reserve(s_x2) && b->d_seg.reserve(s_seg);
        for (int i = 0; i < b->nbuf && okalloc; ++i) okalloc = b->d_res[i].reserve(s_res);
    }
    for (int i = 0; i < b->nbuf && okalloc; ++i) okalloc = !want_tb || b->d_tb[i].reserve(4 * std::max<uint64_t>(1, tbw));
    if (!okalloc)
        return c->fail(SED_E_OOM, "device allocation failed (traceback %d x %.3f GB)", b->nbuf, 4.0 * tbw / 1e9);
    hipError_t e;
    if (b->small) {
        if ((e = pin_reserve(c, total)) != hipSuccess) return c->hipfail(e, "pinned staging");
        char *h = (char *)c->pin, *d = (char *)b->d_small.p;
        memcpy(h + o_pd, b->pd.data(), sizeof(sed_pair_desc) * npairs);
        memcpy(h + o_sa, hsa, sa);
        memcpy(h + o_sb, hsb, sb);
        if (!tasks.empty()) memcpy(h + o_tasks, tasks.data(), sizeof(int2) * tasks.size());
        memset(h + o_chain, 0, s_chain);
        if (!chain_pairs.empty()) memcpy(h + o_chain, chain_pairs.data(), 4 * chain_pairs.size());
        if (!chain_off.empty()) memcpy(h + o_chain + 4 * chain_pairs.size(), chain_off.data(), 4 * chain_off.size());
        if (!lane_idx.empty()) memcpy(h + o_lane, lane_idx.data(), 4 * lane_idx.size());
        if (!x2.empty()) memcpy(h + o_x2, x2.data(), 4 * x2.size());
        if (!seg_idx.empty()) memcpy(h + o_seg, seg_idx.data(), 4 * seg_idx.size());
        memset(h + o_res, 0, s_res);
        const size_t up = b->zc ? o_res : total;  // (zero-copy results: the results and scripts stay in h_out)
        if (b->zc) {
            const size_t want = total - o_res;
            if (want > b->h_out_cap) {
                if (b->h_out) (void)hipHostFree(b->h_out);
                b->h_out = nullptr;
                b->h_out_cap = 0;
                if ((e = hipHostMalloc(&b->h_out, std::max<size_t>(want, 1u << 16), hipHostMallocDefault)) != hipSuccess) {
                    b->h_out = nullptr;
                    return c->hipfail(e, "pinned results");
                }
                b->h_out_cap = std::max<size_t>(want, 1u << 16);
            }
            memset(b->h_out, 0, want);  // (no run of this batch is in flight: zc_busy was waited for above)
        }
        if ((e = hipMemcpyAsync(d, h, up, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return c->hipfail(e, "upload");
        c->pin_busy = true;
        b->p_pd = d + o_pd;
        b->p_seqa = d + o_sa;
        b->p_seqb = d + o_sb;
        b->p_tasks = d + o_tasks;
        b->p_chain = d + o_chain;
        b->p_lane = d + o_lane;
        b->p_x2 = d + o_x2;
        b->p_seg = d + o_seg;
        b->p_res[0] = b->zc ? b->h_out : d + o_res;
        b->p_ops = b->zc ? (char *)b->h_out + (o_ops - o_res) : d + o_ops;
        b->o_ops_small = o_ops - o_res;
    } else {
        b->p_ops = b->d_ops.p;
        b->p_pd = b->d_pd.p;
        b->p_seqa = b->d_seqa.p;
        b->p_seqb = b->d_seqb.p;
        b->p_tasks = b->d_tasks.p;
        b->p_chain = b->d_chain.p;
        b->p_lane = b->d_lane.p;
        b->p_x2 = b->d_x2.p;
        b->p_seg = b->d_seg.p;
        for (int i = 0; i < 3; ++i) b->p_res[i] = b->d_res[i].p;
        if ((e = hipMemcpyAsync(b->p_pd, b->pd.data(), sizeof(sed_pair_desc) * npairs, hipMemcpyHostToDevice,
                                c->stream)) != hipSuccess)
            return c->hipfail(e, "upload descriptors");
        if ((e = hipMemcpyAsync(b->p_seqa, hsa, sa, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return c->hipfail(e, "upload str1");
        if ((e = hipMemcpyAsync(b->p_seqb, hsb, sb, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return c->hipfail(e, "upload str2");
        if (!tasks.empty() && (e = hipMemcpyAsync(b->p_tasks, tasks.data(), sizeof(int2) * tasks.size(),
                                                  hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return c->hipfail(e, "upload tasks");
        if (b->nchains &&
            ((e = hipMemcpyAsync(b->p_chain, chain_pairs.data(), 4 * chain_pairs.size(), hipMemcpyHostToDevice,
                                 c->stream)) != hipSuccess ||
             (!chain_off.empty() &&
              (e = hipMemcpyAsync((int32_t *)b->p_chain + chain_pairs.size(), chain_off.data(), 4 * chain_off.size(),
                                  hipMemcpyHostToDevice, c->stream)) != hipSuccess)))
            return c->hipfail(e, "upload chains");
        if (!lane_idx.empty() && (e = hipMemcpyAsync(b->p_lane, lane_idx.data(), 4 * lane_idx.size(),
                                                     hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return c->hipfail(e, "upload lane list");
        if (!x2.empty() &&
            (e = hipMemcpyAsync(b->p_x2, x2.data(), 4 * x2.size(), hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return c->hipfail(e, "upload packed-wave list");
        if (!seg_idx.empty() && (e = hipMemcpyAsync(b->p_seg, seg_idx.data(), 4 * seg_idx.size(), hipMemcpyHostToDevice,
                                                    c->stream)) != hipSuccess)
            return c->hipfail(e, "upload segment list");
        for (int i = 0; i < b->nbuf; ++i)
            if ((e = hipMemsetAsync(b->p_res[i], 0, s_res, c->stream)) != hipSuccess) return c->hipfail(e, "zero results");
        if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hipfail(e, "upload sync");
        c->pin_busy = false;
    }

    // ---- kernel parameters ----
    if (mode == SED_MODE_I32) {
        sed_i32_params ip{};
        ip.ins = (uint32_t)c->ins;
        ip.del = (uint32_t)c->del;
        for (int a = 0; a < 4; ++a) {
            uint32_t row = 0, row16 = 0;
            for (int bb = 0; bb < 4; ++bb) {
                // symbols outside the alphabet never occur in real cells: any cost <= ins + del will do
                const uint32_t v = (a < c->K && bb < c->K) ? (uint32_t)c->sub[a * c->K + bb] : 0u;
                row |= ((v - ip.ins - ip.del - 1u) & 0xFFu) << (8 * bb);
                row16 |= ((v - ip.ins - ip.del) & 0xFFu) << (8 * bb);
            }
            ip.costrow[a] = row;
            ip.costrow16[a] = row16;
        }
        ip.kins = (ip.ins << 16) + 4u;
        ip.kdel = (ip.del << 16) + 5u;
        // dot keys: checkpoint batches of the stripe kernel (CHAIN batches share the traceback's key format)
        b->dot = false;
        if ((b->ck || b->split_ck) && b->nchains == 0 && c->K == 4 && c->opt_dot != 2) {
            int64_t kap[4][4], maxmin = 0;
            for (int a = 0; a < 4; ++a)
                for (int bb = 0; bb < 4; ++bb) kap[a][bb] = (int64_t)ip.ins + ip.del - (int64_t)c->sub[a * 4 + bb];
            for (int p = 0; p < npairs; ++p)
                if (!b->pd[p].lane) maxmin = std::max<int64_t>(maxmin, std::min(len_a[p], len_b[p]));
            const DotKeys dk = dot_keys(kap, maxmin);
            if (dk.ok) {
                ip.dot = 1;
                ip.dotA = dk.A;
                ip.dotkmax = dk.kmax;
                ip.dotM = dk.M;
                ip.dotS = dk.S;
                for (int a = 0; a < 4; ++a) {
                    ip.dotrow[a] = dk.row[a];
                    ip.dotcol[a] = dk.col[a];
                }
                b->dot = true;
            }
        }
        // ladder dot keys: the CHAIN kernel's ladder keys (L field, with or without codes) with the update addend
        // as one v_dot4.  V = D*A + uL needs A < 2^16 and the factorisation of A*K + (u - 1)J (the d = -1 rows'
        // constant) in bytes: u = 16 over the wide ladder (sed_kernels.hip: LadderW, ip.lad = 2) with 16 min(n, m) + 15
        // < A, else u = 8 over the 3-bit one (ip.lad = 1) with 8 (n + m) + 7 < A (the L field below the D unit).
        b->lad = false;
        if (b->nchains > 0 && !b->ck && (want_tb || !(flags & SED_NO_LEN)) && c->K == 4 && c->opt_dot != 2) {
            int64_t kap[4][4], maxsum = 0, maxmin = 0;
            for (int a = 0; a < 4; ++a)
                for (int bb = 0; bb < 4; ++bb) kap[a][bb] = (int64_t)ip.ins + ip.del - (int64_t)c->sub[a * 4 + bb];
            for (int p = 0; p < npairs; ++p)
                if (!b->pd[p].lane) {
                    maxsum = std::max<int64_t>(maxsum, (int64_t)len_a[p] + len_b[p]);
                    maxmin = std::max<int64_t>(maxmin, std::min(len_a[p], len_b[p]));
                }
            // the wide ladder first (one jump row in 8; its sink decode reads L inside [max(n, m), n + m], so A > 16
            // min(n, m) + 15 keeps the keys apart), the 3-bit one where that does not fit bytes
            DotKeys lk = c->opt_dot == 3 ? DotKeys{} : dot_keys(kap, 0, 16 * maxmin + 16, 15);  // (3: tests)
            uint32_t lad = 2;
            if (!lk.ok) {
                lk = dot_keys(kap, 0, 8 * maxsum + 8, 7);
                lad = 1;
            }
            if (lk.ok) {
                ip.lad = lad;
                ip.ladA = lk.A;
                ip.ladsent = lk.S;  // (ladder mode: the sentinel's byte 0)
                for (int a = 0; a < 4; ++a) {
                    ip.ladrow[a] = lk.row[a];
                    ip.ladcol[a] = lk.col[a];
                }
                b->lad = true;
            }
        }
        b->ip = ip;
    } else {
        sed_f64_params fp{};
        fp.ins = c->ins;
        fp.del = c->del;
        fp.ins_int = c->ins_int;
        fp.del_int = c->del_int;
        fp.K = c->K;
        b->fp = fp;
    }
    // the event log is reused across refills (sed_run_batch's scratch batch): entries are created
    // only up to 64 ahead of the runs, and run_batch grows it on demand past that
    b->nlog = 0;
    b->last_log = -1;
    if (b->log.size() < 64 && (e = grow_log(b, 64 - b->log.size())) != hipSuccess)
        return c->hipfail(e, "event create");
    if (b->nbuf > 1 && !b->tb_stream &&
        (e = hipStreamCreateWithFlags(&b->tb_stream, hipStreamNonBlocking)) != hipSuccess)
        return c->hipfail(e, "traceback stream");
    // SED_ALT_DP=0 keeps every DP on the context's stream (A/B)
    static const int alt_env = [] { const char *e = getenv("SED_ALT_DP"); return e ? atoi(e) : 1; }();
    b->alt_dp = alt_env != 0 && b->nbuf > 1 &&
                ((b->chain_dyn && (flags & SED_WANT_SCRIPT)) ||
                 (b->nwave == 0 && b->nwave_x2 == 0 && !(flags & SED_WANT_SCRIPT)));
    if (b->alt_dp && !b->dp2_stream &&
        (e = hipStreamCreateWithFlags(&b->dp2_stream, hipStreamNonBlocking)) != hipSuccess)
        return c->hipfail(e, "second DP stream");
    // distance-only lane batches on two streams use two result slots, one per stream: a slot's runs are then
    // ordered by their stream and need no event query or cross-stream wait
    if (b->alt_dp && !(flags & SED_WANT_SCRIPT)) b->nbuf = 2;
    // SED_CK_HALVES: parts per checkpoint batch of >= 1024 wave pairs per part (1 = off; default
    // SED_CK_HALVES_DEFAULT; at most 4, the hardware queues a process gets)
    static const int parts_env = [] { const char *e = getenv("SED_CK_HALVES"); return e ? atoi(e) : -1; }();
    const int want = std::min(4, std::max(1, parts_env < 0 ? SED_CK_HALVES_DEFAULT : parts_env));
    b->nparts = 1;
    if (b->ck && b->nchains == 0 && b->nbuf == 1 && b->nwave_x2 == 0)
        b->nparts = std::max(1, std::min(want, b->nwave / 1024));
    for (int i = 0; i + 1 < b->nparts; ++i)
        if (!b->part_stream[i] && (e = hipStreamCreateWithFlags(&b->part_stream[i], hipStreamNonBlocking)) != hipSuccess)
            return c->hipfail(e, "part stream");
    if (b->nparts > 1 && !b->ev_start && (e = hipEventCreateWithFlags(&b->ev_start, hipEventDisableTiming)) != hipSuccess)
        return c->hipfail(e, "event create");
    if (b->nparts > 1 && (e = grow_log(b, 0)) != hipSuccess) return c->hipfail(e, "event create");  // the parts' entries
    return SED_OK;
}

// A checkpoint batch in parts on as many streams (b->nparts).  Stream i runs forward(part i) then
// traceback(part i).  The other streams start each run after stream 0's previous work, and nothing joins the
// streams at a run's end, so the parts settle into a stagger: one part's traceback runs beside another part's
// forward (config 4: 11.42-11.47 ms in one part, 10.85-11.0 in two, 10.77-10.83 in three, 11.6-11.8 in four;
// with the select-free hold 9.86-9.93 in two against 10.30-10.54 in three, profiles/r03/parts2/;
// joined at every run's end two halves ran in lockstep and gained nothing; profiles/r03/halves/, parts/).  The
// parts share no buffer region (every pair has its own
// checkpoints, bottom rows, script words and result), and sync_batch waits for every stream.  The run's event
// log keeps every part's kernels, one launch each: sed_batch_times reports the mean launch (sed_batch_dp_launches() =
// nparts).
int run_batch_parts(sed_batch *b, const std::array<hipEvent_t, 4> &lg, sed_launch L, const sed_i32_params &ip,
                    bool len) {
    sed_ctx *c = b->ctx;
    hipError_t e;
    const int P = b->nparts;
    auto stream = [&](int i) { return i == 0 ? c->stream : b->part_stream[i - 1]; };
    auto first = [&](int i) { return (int)((int64_t)b->npairs * i / P); };
    // the other streams start after everything queued before this run (uploads, the previous run's part 0)
    if ((e = hipEventRecord(b->ev_start, c->stream)) != hipSuccess) return c->hipfail(e, "stream fork");
    for (int i = 1; i < P; ++i)
        if ((e = hipStreamWaitEvent(stream(i), b->ev_start, 0)) != hipSuccess) return c->hipfail(e, "stream fork");
    // every part's kernels carry their own events (sed_batch_times averages the parts' launches); grow_log created
    // the parts' entries with the run's own
    std::array<hipEvent_t, 12> pl{};  // (an untimed run: none)
    if (lg[0]) {
        const size_t li = b->nlog - 1;
        if (b->plog.size() <= li) return c->fail(SED_E_STATE, "parts event log not grown");
        pl = b->plog[li];
    }
    auto part = [&](int i, int ph) {  // ph 0: forward, 1: traceback
        sed_launch Li = L;
        Li.pd = L.pd + first(i);
        Li.res = L.res + first(i);
        Li.npairs = first(i + 1) - first(i);
        Li.stream = stream(i);
        Li.ev0 = i == 0 ? lg[2 * ph] : pl[4 * (i - 1) + 2 * ph];
        Li.ev1 = i == 0 ? lg[2 * ph + 1] : pl[4 * (i - 1) + 2 * ph + 1];
        return Li;
    };
    for (int i = 0; i < P; ++i) {
        sed_launch Lp = part(i, 0);
        if (i == 0 && b->nlane > 0) Lp.ev1 = nullptr;  // part 0's DP window ends with the lane kernel below
        if ((e = sed_launch_i32(Lp, ip, len)) != hipSuccess) return c->hipfail(e, "DP kernel launch");
    }
    if (b->nlane > 0) {  // lane pairs (the whole batch's, by index) after part 0's forward, inside its DP window
        sed_launch Ll = L;
        Ll.ev0 = nullptr;
        Ll.ev1 = lg[1];
        if ((e = sed_launch_lane_i32(Ll, (const int32_t *)b->p_lane, b->nlane, ip, len)) != hipSuccess)
            return c->hipfail(e, "lane kernel launch");
    }
    if (c->opt_debug_corrupt > 0 && c->opt_debug_corrupt <= b->npairs) {
        const int p = c->opt_debug_corrupt - 1;
        const sed_pair_desc &d = b->pd[p];
        const int R = b->R, ROWS = R * 64, G = 64 / R;
        int ip_ = 0;
        while (ip_ + 1 < P && p >= first(ip_ + 1)) ++ip_;
        if (!d.lane && d.n > 0 && d.m > 0) {
            const int nstripes = (d.n + ROWS - 1) / ROWS, SG = (d.m + 63 + G - 1) / G * G, nchunks = (SG + 63) >> 6;
            const int t = ((d.n - 1) % ROWS) / R, r = (d.n - 1) % R, cs = (d.m - 1 + t) >> 6;
            if (cs >= 1) {
                uint32_t *w = (uint32_t *)L.tb + d.tb_off + sed_ck_col_word(R, nstripes - 1, nchunks, cs - 1, r, t);
                if ((e = hipMemsetD32Async((hipDeviceptr_t)w, b->dot ? 0x3FFFFFFFu : 0x0000FFFCu, 1, stream(ip_))) !=
                    hipSuccess)
                    return c->hipfail(e, "debug corrupt");
            }
        }
    }
    for (int i = 0; i < P; ++i)
        if ((e = sed_launch_traceback_ck(part(i, 1), (uint32_t *)b->p_ops, ip)) != hipSuccess)
            return c->hipfail(e, "traceback kernel launch");
    b->evk[0] = lg;
    ++b->runs;
    b->ran = true;
    return SED_OK;
}

int run_batch(sed_batch *b) {
    sed_ctx *c = b->ctx;
    if (b->npairs == 0) {
        b->ran = true;
        ++b->runs;
        return SED_OK;
    }
    const int k = (int)(b->runs % b->nbuf);
    const bool want_tb = (b->flags & SED_WANT_SCRIPT) != 0;
    hipError_t e;
    if (b->zc) b->zc_busy = true;
    // The run's events time it (sed_batch_times) and, when buffers rotate, order their reuse (evk below; two-slot lane
    // batches order by stream instead).  Untimed runs (sed_batch_set_timing) launch without them.
    const bool need_ev = b->nbuf > 1 && !(b->alt_dp && b->nbuf == 2 && !want_tb);
    const bool timed = need_ev || b->time_every == 1 || (b->time_every > 1 && b->runs % b->time_every == 0);
    std::array<hipEvent_t, 4> lg{};
    if (timed) {
        if (b->nlog == b->log.size() && (e = grow_log(b, 64)) != hipSuccess) return c->hipfail(e, "event create");
        b->last_log = (long)b->nlog;
        lg = b->log[b->nlog++];
    }
    hipStream_t ts = b->nbuf > 1 ? b->tb_stream : c->stream;
    const hipStream_t ds = b->alt_dp && (b->runs & 1) ? b->dp2_stream : c->stream;  // this run's DP stream
    sed_launch L{};
    L.pd = (const sed_pair_desc *)b->p_pd;
    L.npairs = b->npairs;
    L.seqa = b->p_seqa;
    L.seqb = b->p_seqb;
    L.tb = want_tb ? (uint32_t *)b->d_tb[k].p : nullptr;
    L.ops = (uint32_t *)b->p_ops;
    L.bnd = (uint32_t *)b->d_bnd.p;
    L.res = (sed_result *)b->p_res[k];
    L.R = b->R;
    L.stream = ds;
    L.tb_ladder = b->mode == SED_MODE_I32 && !b->split_ck;  // (split_ck codes are the plain ops)
    L.tb_wide = b->lad && b->ip.lad == 2;  // (a ladder-dot batch is a CHAIN batch: every wave pair's codes come from the LDOT kernel)
    L.ck = b->ck;
    L.tasks = b->split ? (const int2 *)b->p_tasks : nullptr;
    L.ntasks = b->split ? b->ntasks : 0;
    // buffer k was last read by the traceback of run runs-3 (written by its DP, distance only): wait for it unless it
    // has finished already (a cross-queue wait is a barrier packet between this run's kernel and the previous one)
    const int kev = want_tb ? 3 : 1;
    if (b->nbuf > 1 && (want_tb || (b->alt_dp && b->nbuf != 2)) && b->runs >= b->nbuf &&
        hipEventQuery(b->evk[k][kev]) != hipSuccess &&
        (e = hipStreamWaitEvent(ds, b->evk[k][kev], 0)) != hipSuccess)
        return c->hipfail(e, "stream wait");
    // The event log's timestamps ride on the kernels' own dispatch packets (SED_LAUNCH: the DP phase's first
    // kernel records lg[0] at its start and its last kernel lg[1] at its end; the same for the traceback phase
    // with lg[2] / lg[3]).  An event record is a marker packet on the queue: with records around the kernels,
    // consecutive config-2 DP kernels were ~18 us apart, and for the ~25 us lane kernel (config 5) every
    // avoided packet is measurable.  A phase that launches nothing records its events directly.
    const int nw64 = b->nwave - b->nseg;  // wave pairs of the one-wave-per-pair kernels
    const int ndp = (b->nwave_x2 > 0) + (nw64 > 0) + (b->nseg > 0) + (b->nlane > 0);
    int idp = 0;
    auto dp_events = [&]() {
        L.ev0 = idp == 0 ? lg[0] : nullptr;
        L.ev1 = idp == ndp - 1 ? lg[1] : nullptr;
        ++idp;
    };
    if (ndp == 0 && lg[0] && (e = hipEventRecord(lg[0], ds)) != hipSuccess) return c->hipfail(e, "event record");
    // SPLIT hand-off words carry the run's epoch (1..32767, next_split_epoch); every kernel writes all result
    // fields, err included
    sed_i32_params ip = b->ip;
    if ((e = next_split_epoch(b, ds, &ip.epoch)) != hipSuccess) return c->hipfail(e, "memset hand-off words");
    const bool len = want_tb || !(b->flags & SED_NO_LEN);
    if (b->nparts > 1 && want_tb) return run_batch_parts(b, lg, L, ip, len);
    if (b->nwave_x2 > 0) {
        dp_events();
        if ((e = sed_launch_i32x2(L, (const int32_t *)b->p_x2, b->nwave_x2, ip)) != hipSuccess)
            return c->hipfail(e, "packed DP kernel launch");
    }
    if (nw64 > 0) {
        dp_events();
        if (b->mode == SED_MODE_I32 && b->nchains) {
            L.chain_pairs = (const int32_t *)b->p_chain;
            L.chain_off = (const int32_t *)b->p_chain + b->chain_npairs;
            L.nchains = b->nchains;
            L.chain_list = (int)b->chain_npairs;
            L.chain_counter = nullptr;
            if (b->chain_dyn) {  // zeroed on a batch's first launch only: a launch takes list + waves values
                // (counted per launch, not per run: a run that fails after its CHAIN launch has still advanced it)
                L.chain_counter = (uint32_t *)b->p_chain + b->chain_npairs + 1 + k;
                L.chain_base = (uint32_t)((uint64_t)b->chain_launches[k] * (uint64_t)(b->chain_npairs + b->nchains));
                if (b->chain_launches[k] == 0 && (e = hipMemsetAsync(L.chain_counter, 0, 4, ds)) != hipSuccess)
                    return c->hipfail(e, "reset chain counter");
            }
            e = sed_launch_i32_chain(L, ip, len);
            if (e == hipSuccess && b->chain_dyn) ++b->chain_launches[k];
        } else if (b->mode == SED_MODE_I32 && b->split_ck) {  // forward with checkpoints, then every tile's codes
            // (pipelined runs: the codes kernel opens the traceback phase on its stream below, so the next run's
            // forward follows this one directly: config 2 ran 0.297-0.301 ms per step with it on the DP stream)
            sed_launch Lf = L;
            Lf.ck = true;
            if (ts == ds) Lf.ev1 = nullptr;
            e = sed_launch_i32(Lf, ip, len);
            if (e == hipSuccess && ts == ds) {
                sed_launch Lc = L;
                Lc.ev0 = nullptr;
                e = sed_launch_ck_codes(Lc, b->ck_tiles, ip);
            }
        } else if (b->mode == SED_MODE_I32)
            e = sed_launch_i32(L, ip, len);
        else {
            sed_f64_params fp = b->fp;
            fp.epoch = ip.epoch;
            e = sed_launch_f64(L, (const double *)c->gtab.p, fp, b->mode == SED_MODE_F64_TYPED);
        }
        if (e != hipSuccess) return c->hipfail(e, "DP kernel launch");
    }
    if (b->nseg > 0) {  // fp64 pairs in 16-lane segments, four per wave
        dp_events();
        if ((e = sed_launch_f64_seg(L, (const double *)c->gtab.p, b->fp, b->mode == SED_MODE_F64_TYPED,
                                    (const int32_t *)b->p_seg, b->nseg)) != hipSuccess)
            return c->hipfail(e, "segment DP kernel launch");
    }
    if (b->nlane > 0) {
        dp_events();
        if (b->lane_bitpar)
            e = sed_launch_lane_bitpar(L, (const int32_t *)b->p_lane, b->nlane);
        else if (b->nlane_x2 > 0)
            e = sed_launch_lane_i32x2(L, (const int32_t *)b->p_lane, b->nlane_x2, ip);
        else if (b->mode == SED_MODE_I32)
            e = sed_launch_lane_i32(L, (const int32_t *)b->p_lane, b->nlane, ip, len);
        else if (b->scaled)
            e = sed_launch_lane_scaled(L, (const int32_t *)b->p_lane, b->nlane, b->sp);
        else
            e = sed_launch_lane_f64(L, (const int32_t *)b->p_lane, b->nlane, (const double *)c->gtab.p, c->ins,
                                    c->del, c->K, b->umask);
        if (e != hipSuccess) return c->hipfail(e, "lane kernel launch");
    }
    if (ndp == 0 && lg[1] && (e = hipEventRecord(lg[1], ds)) != hipSuccess) return c->hipfail(e, "event record");
    L.ev0 = L.ev1 = nullptr;
    if (want_tb && b->ck && c->opt_debug_corrupt > 0 && c->opt_debug_corrupt <= b->npairs) {
        // SED_OPT_DEBUG_CORRUPT: overwrite the column checkpoint of the sink's row in the chunk before the
        // sink's tile with the smallest distance key (D offset 0, no updates), which the recompute then
        // spreads to the sink (test of the traceback's error path: the pair must come back SED_E_DEVICE)
        const int p = c->opt_debug_corrupt - 1;
        const sed_pair_desc &d = b->pd[p];
        const int R = b->R, ROWS = R * 64, G = 64 / R;
        if (!d.lane && d.n > 0 && d.m > 0) {
            const int nstripes = (d.n + ROWS - 1) / ROWS, SG = (d.m + 63 + G - 1) / G * G, nchunks = (SG + 63) >> 6;
            const int t = ((d.n - 1) % ROWS) / R, r = (d.n - 1) % R, cs = (d.m - 1 + t) >> 6;
            if (cs >= 1) {
                uint32_t *w = (uint32_t *)b->d_tb[k].p + d.tb_off + sed_ck_col_word(R, nstripes - 1, nchunks, cs - 1, r, t);
                // (dot keys are maximised: the largest key there instead)
                if ((e = hipMemsetD32Async((hipDeviceptr_t)w, b->dot ? 0x3FFFFFFFu : 0x0000FFFCu, 1, ds)) !=
                    hipSuccess)
                    return c->hipfail(e, "debug corrupt");
            }
        }
    }
    if (want_tb) {
        if (ts != ds && (e = hipStreamWaitEvent(ts, lg[1], 0)) != hipSuccess) return c->hipfail(e, "stream wait");
        if (b->nwave == 0 && lg[2] && (e = hipEventRecord(lg[2], ts)) != hipSuccess) return c->hipfail(e, "event record");
        if (b->nwave > 0) {
            L.stream = ts;
            L.ev0 = lg[2];
            L.ev1 = lg[3];
            if (b->split_ck && ts != ds) {  // the tile codes of this run's checkpoints (see the DP phase)
                sed_launch Lc = L;
                Lc.ev1 = nullptr;
                if ((e = sed_launch_ck_codes(Lc, b->ck_tiles, ip)) != hipSuccess) return c->hipfail(e, "codes kernel launch");
                L.ev0 = nullptr;
            }
            if (b->tbpar) {  // (the map kernel zeroes the scripts the segments OR into)
                e = sed_launch_traceback_stripes(L, (uint32_t *)b->p_ops, (uint32_t *)b->d_tbmap.p, b->tbpar_items,
                                                 b->tbpar_kmax);
            } else {
                const hipEvent_t tb_end = L.ev1;
                if (b->nseg > 0) L.ev1 = nullptr;  // the segment pairs' traceback below ends the phase
                e = nw64 <= 0 ? hipSuccess
                    : b->ck   ? sed_launch_traceback_ck(L, (uint32_t *)b->p_ops, ip)
                              : sed_launch_traceback(L, (uint32_t *)b->p_ops);
                if (e == hipSuccess && b->nseg > 0) {
                    L.ev0 = nw64 <= 0 ? L.ev0 : nullptr;
                    L.ev1 = tb_end;
                    e = sed_launch_traceback_seg(L, (uint32_t *)b->p_ops, (const int32_t *)b->p_seg, b->nseg);
                }
            }
            if (e != hipSuccess) return c->hipfail(e, "traceback kernel launch");
        }
        if (b->nwave == 0 && lg[3] && (e = hipEventRecord(lg[3], ts)) != hipSuccess) return c->hipfail(e, "event record");
    }
    b->evk[k] = lg;
    ++b->runs;
    b->ran = true;
    return SED_OK;
}

int sync_batch(sed_batch *b) {
    sed_ctx *c = b->ctx;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && b->tb_stream) e = hipStreamSynchronize(b->tb_stream);
    if (e == hipSuccess && b->dp2_stream) e = hipStreamSynchronize(b->dp2_stream);
    for (hipStream_t ps : b->part_stream)
        if (e == hipSuccess && ps) e = hipStreamSynchronize(ps);
    if (e == hipSuccess) b->zc_busy = false;
    return e == hipSuccess ? SED_OK : c->hipfail(e, "kernel execution");
}

int fetch_results(sed_batch *b, double *out_dist, uint8_t *out_is_int, int32_t *out_len, uint32_t *out_ops,
                  const int64_t *ops_off) {
    sed_ctx *c = b->ctx;
    if (!b->ran) return c->fail(SED_E_STATE, "batch has not been run");
    const int np = b->npairs;
    hipError_t e;
    const bool want_ops = out_ops && ops_off && (b->flags & SED_WANT_SCRIPT) && np;
    const sed_result *hr = nullptr;
    const uint32_t *hops = nullptr;
    std::vector<uint32_t> h;
    if (b->small && b->nbuf == 1 && b->nparts == 1 && !b->alt_dp) {
        // every kernel ran on the context's stream: one download of the adjacent results and scripts into the pinned
        // staging, ordered after them, and one wait
        const size_t bytes = b->o_ops_small + (want_ops ? 4 * b->ops_words : 0);
        const char *src = (const char *)b->h_out;
        if (!b->zc) {
            if (bytes > c->pin_cap && (e = pin_reserve(c, bytes)) != hipSuccess) return c->hipfail(e, "pinned staging");
            if (np && (e = hipMemcpyAsync(c->pin, b->p_res[0], bytes, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
                return c->hipfail(e, "download results");
            c->pin_busy = true;
            src = (const char *)c->pin;
        }
        int rc = sync_batch(b);
        if (rc != SED_OK) return rc;
        c->pin_busy = false;
        hr = (const sed_result *)src;
        hops = (const uint32_t *)(src + b->o_ops_small);
    } else {
        int rc = sync_batch(b);
        if (rc != SED_OK) return rc;
        b->h_res.resize(np);
        if (np && (e = hipMemcpy(b->h_res.data(), b->p_res[b->cur()], sizeof(sed_result) * np, hipMemcpyDeviceToHost)) !=
                      hipSuccess)
            return c->hipfail(e, "download results");
        hr = b->h_res.data();
        if (want_ops) {
            h.resize(b->ops_words);
            if ((e = hipMemcpy(h.data(), b->p_ops, 4 * b->ops_words, hipMemcpyDeviceToHost)) != hipSuccess)
                return c->hipfail(e, "download scripts");
            hops = h.data();
        }
    }
    for (int p = 0; p < np; ++p) {
        switch (hr[p].err) {
        case 0: break;
        case SED_ERR_SPLIT_TIMEOUT: return c->fail(SED_E_DEVICE, "pair %d: inter-workgroup hand-off timed out", p);
        case SED_ERR_TB_CHECK:
            return c->fail(SED_E_DEVICE, "pair %d: traceback failed: a recomputed tile contradicts the path length "
                                         "(corrupt checkpoint)", p);
        case SED_ERR_TB_STALL: return c->fail(SED_E_DEVICE, "pair %d: traceback failed: a tile made no progress", p);
        case SED_ERR_TB_GUARD: return c->fail(SED_E_DEVICE, "pair %d: traceback failed: too many tile visits", p);
        case SED_ERR_TB_LENGTH:
            return c->fail(SED_E_DEVICE, "pair %d: traceback failed: script length differs from the sink's", p);
        default: return c->fail(SED_E_DEVICE, "pair %d: device error code %d", p, (int)hr[p].err);
        }
    }
    for (int p = 0; p < np; ++p) {
        if (out_dist) out_dist[p] = hr[p].dist;
        if (out_is_int) out_is_int[p] = hr[p].is_int;
        if (out_len) out_len[p] = hr[p].len;
    }
    if (want_ops)
        for (int p = 0; p < np; ++p) {
            const uint64_t words = (uint64_t)(b->n[p] + b->m[p] + 15) / 16;
            memcpy(out_ops + ops_off[p], hops + b->pd[p].ops_off, 4 * words);
        }
    return SED_OK;
}

}  // namespace

extern "C" {

const char *sed_version(void) { return "libsed 0.1 (gfx950)"; }

sed_ctx *sed_create(int device) {
    if (hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    sed_ctx *c = new sed_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        delete c;
        return nullptr;
    }
    return c;
}

void sed_destroy(sed_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    delete c->scratch;
    if (c->pin) (void)hipHostFree(c->pin);
    c->gtab.release();
    c->selftest.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *sed_last_error(const sed_ctx *c) { return c ? c->err.c_str() : "null context"; }

int sed_set_option(sed_ctx *c, int key, int value) {
    if (!c) return SED_E_ARG;
    if (key == SED_OPT_MODE && value >= 0 && value <= 3) {
        c->opt_mode = value;
        return SED_OK;
    }
    if (key == SED_OPT_SPLIT && value >= 0 && value <= 2) {
        c->opt_split = value;
        return SED_OK;
    }
    if (key == SED_OPT_LANE && value >= 0 && value <= 2) {
        c->opt_lane = value;
        return SED_OK;
    }
    if (key == SED_OPT_TB && value >= 0 && value <= 2) {
        c->opt_tb = value;
        return SED_OK;
    }
    if (key == SED_OPT_PACK && (value == 0 || value == 2)) {
        c->opt_pack = value;
        return SED_OK;
    }
    if (key == SED_OPT_BITPAR && (value == 0 || value == 2)) {
        c->opt_bitpar = value;
        return SED_OK;
    }
    if (key == SED_OPT_SEG && value >= 0 && value <= 2) {
        c->opt_seg = value;
        return SED_OK;
    }
    if (key == SED_OPT_SPLITCK && (value == 0 || value == 2)) {
        c->opt_splitck = value;
        return SED_OK;
    }
    if (key == SED_OPT_ZEROCOPY && (value == 0 || value == 2)) {
        c->opt_zc = value;
        return SED_OK;
    }
    if (key == SED_OPT_SCALED && (value == 0 || value == 2)) {
        c->opt_scaled = value;
        return SED_OK;
    }
    if (key == SED_OPT_DOT && (value == 0 || value == 2 || value == 3)) {
        c->opt_dot = value;
        return SED_OK;
    }
    if (key == SED_OPT_CHAIN_WAVES && value >= 0) {
        c->opt_chain_waves = value;
        return SED_OK;
    }
    if (key == SED_OPT_DEBUG_CORRUPT && value >= 0) {
        c->opt_debug_corrupt = value;
        return SED_OK;
    }
    if (key == SED_OPT_CHAIN && value >= 0 && value <= 1024) {
        c->opt_chain = value;
        return SED_OK;
    }
    if (key == SED_OPT_ROWS_PER_LANE && (value == 0 || value == 1 || value == 2 || value == 4 || value == 8 ||
                                         value == 16 || value == 32)) {
        c->opt_R = value;
        return SED_OK;
    }
    return c->fail(SED_E_ARG, "bad option %d=%d", key, value);
}

int sed_set_costs(sed_ctx *c, int K, const double *sub, const uint8_t *sub_int, double ins, int ins_is_int,
                  double del, int del_is_int) {
    if (!c) return SED_E_ARG;
    if (c->pair_pending) return c->fail(SED_E_STATE, "a submitted pair has not been waited for");
    if (K < 1 || K > 255 || !sub || !sub_int) return c->fail(SED_E_ARG, "bad cost table (K=%d)", K);
    if (!std::isfinite(ins) || !std::isfinite(del)) return c->fail(SED_E_ARG, "non-finite insert/delete cost");
    for (int e = 0; e < K * K; ++e)
        if (!std::isfinite(sub[e])) return c->fail(SED_E_ARG, "non-finite update cost at %d", e);
    (void)hipSetDevice(c->device);
    c->K = K;
    c->sub.assign(sub, sub + K * K);
    c->sub_int.assign(sub_int, sub_int + K * K);
    c->ins = ins;
    c->del = del;
    c->ins_int = ins_is_int ? 1 : 0;
    c->del_int = del_is_int ? 1 : 0;
    if (K <= SED_MAX_K) {
        std::vector<uint64_t> t(2 * K * K);
        for (int e = 0; e < K * K; ++e) {
            memcpy(&t[2 * e], &sub[e], 8);
            t[2 * e + 1] = sub_int[e] ? 1 : 0;
        }
        if (!c->gtab.reserve(t.size() * 8)) return c->fail(SED_E_OOM, "cost table allocation");
        hipError_t e = hipMemcpy(c->gtab.p, t.data(), t.size() * 8, hipMemcpyHostToDevice);
        if (e != hipSuccess) return c->hipfail(e, "upload cost table");
    }
    c->have_costs = true;
    return SED_OK;
}

sed_batch *sed_batch_create(sed_ctx *c, const uint8_t *codes_a, const int64_t *off_a, const int32_t *len_a,
                            const uint8_t *codes_b, const int64_t *off_b, const int32_t *len_b, int32_t npairs,
                            uint32_t flags) {
    if (!c) return nullptr;
    (void)hipSetDevice(c->device);
    sed_batch *b = new sed_batch();
    b->ctx = c;
    if (fill_batch(b, codes_a, off_a, len_a, codes_b, off_b, len_b, npairs, flags) != SED_OK) {
        delete b;
        return nullptr;
    }
    return b;
}

void sed_batch_destroy(sed_batch *b) {
    if (!b) return;
    (void)hipSetDevice(b->ctx->device);
    delete b;
}

int sed_batch_mode(const sed_batch *b) { return b ? b->mode : SED_E_ARG; }
int sed_batch_rows_per_lane(const sed_batch *b) { return b ? b->R : SED_E_ARG; }
int sed_batch_lane_pairs(const sed_batch *b) { return b ? b->nlane : SED_E_ARG; }
int sed_batch_chains(const sed_batch *b) { return b ? b->nchains : SED_E_ARG; }
int sed_batch_traceback_mode(const sed_batch *b) {
    if (!b || !(b->flags & SED_WANT_SCRIPT)) return 0;
    return b->ck ? 2 : b->split_ck ? 4 : (b->tbpar ? 3 : 1);
}

int sed_dot_factor(const double *sub, double ins, double del, int maxmin, int ladder_maxsum, uint32_t *out) {
    if (!sub || !out || maxmin < 0 || ladder_maxsum < 0) return SED_E_ARG;
    int64_t kap[4][4];
    for (int a = 0; a < 4; ++a)
        for (int bb = 0; bb < 4; ++bb) {
            const double v = ins + del - sub[a * 4 + bb];
            if (v != (double)(int64_t)v) return 0;  // integer tables only (the packed-integer kernels' domain)
            kap[a][bb] = (int64_t)v;
        }
    // ladder: the wide ladder's factorisation where it exists, else the 3-bit one (as batch creation); out[9] = the L unit
    // (the wide ladder's bound is on min(n, m): maxmin, or ladder_maxsum when maxmin is 0)
    const int64_t lmin = maxmin > 0 ? std::min<int64_t>(maxmin, ladder_maxsum) : ladder_maxsum;
    DotKeys dk = ladder_maxsum > 0 ? dot_keys(kap, 0, 16 * lmin + 16, 15) : dot_keys(kap, maxmin);
    uint32_t unit = 16;
    if (ladder_maxsum > 0 && !dk.ok) {
        dk = dot_keys(kap, 0, 8 * (int64_t)ladder_maxsum + 8, 7);
        unit = 8;
    }
    if (!dk.ok) return 0;
    for (int a = 0; a < 4; ++a) {
        out[a] = dk.row[a];
        out[4 + a] = dk.col[a];
    }
    out[8] = dk.S;  // decode shift (dot keys) or sentinel byte (ladder)
    out[9] = ladder_maxsum > 0 ? unit : dk.M;  // decode multiplier (dot keys) or the L unit (ladder)
    return (int)dk.A;
}

int sed_batch_dot_keys(const sed_batch *b) {
    return b ? (b->dot ? 1 : 0) | (b->lad ? 2 : 0) | (b->lad && b->ip.lad == 2 ? 4 : 0) : SED_E_ARG;
}

int sed_batch_chain_stats(sed_batch *b, int32_t *fetched, int32_t *max_per_wave) {
    if (!b) return SED_E_ARG;
    sed_ctx *c = b->ctx;
    (void)hipSetDevice(c->device);
    if (!b->ran) return c->fail(SED_E_STATE, "batch has not been run");
    int rc = sync_batch(b);
    if (rc != SED_OK) return rc;
    int32_t f = 0, mx = 0;
    if (b->nchains > 0 && b->npairs > 0) {
        hipError_t e;
        const int kk = (int)((b->runs + b->nbuf - 1) % b->nbuf);  // the last run's slot
        if (b->chain_dyn && b->chain_launches[kk] > 0) {  // every persistent wave ends with one failed grab: a run takes list + waves
            uint32_t cnt = 0;
            if ((e = hipMemcpy(&cnt, (uint32_t *)b->p_chain + b->chain_npairs + 1 + kk, 4, hipMemcpyDeviceToHost)) !=
                hipSuccess)
                return c->hipfail(e, "download chain counter");
            const uint32_t base =
                (uint32_t)((uint64_t)(b->chain_launches[kk] - 1) * (uint64_t)(b->chain_npairs + b->nchains));
            f = (int32_t)(cnt - base) - b->nchains;
        }
        std::vector<sed_result> h(b->npairs);
        if ((e = hipMemcpy(h.data(), b->p_res[b->cur()], sizeof(sed_result) * b->npairs, hipMemcpyDeviceToHost)) !=
            hipSuccess)
            return c->hipfail(e, "download results");
        for (int p = 0; p < b->npairs; ++p)
            if (!b->pd[p].lane && b->n[p] > 0 && b->m[p] > 0) mx = std::max(mx, (int32_t)h[p].seq + 1);
    }
    if (fetched) *fetched = f;
    if (max_per_wave) *max_per_wave = mx;
    return SED_OK;
}

int sed_batch_bitpar_pairs(const sed_batch *b) {
    return b ? (b->lane_bitpar ? b->nlane : b->nbitpar_f64) : SED_E_ARG;
}

int sed_batch_segment_pairs(const sed_batch *b) { return b ? b->nseg : SED_E_ARG; }

int sed_batch_split_tasks(const sed_batch *b) { return b ? (b->split ? b->ntasks : 0) : SED_E_ARG; }

int sed_batch_scaled_pairs(const sed_batch *b) {
    return b ? (b->scaled ? b->nlane - b->nbitpar_f64 : 0) : SED_E_ARG;
}

int sed_batch_packed_pairs(const sed_batch *b) {
    return b ? (b->nlane_x2 > 0 ? b->nlane : 0) + 2 * b->nwave_x2 : SED_E_ARG;
}

int sed_batch_run(sed_batch *b) {
    if (!b) return SED_E_ARG;
    (void)hipSetDevice(b->ctx->device);
    return run_batch(b);
}

int sed_batch_sync(sed_batch *b) {
    if (!b) return SED_E_ARG;
    return sync_batch(b);
}

int sed_batch_last_times(const sed_batch *b, float *dp_ms, float *tb_ms) {
    if (!b || !b->ran) return SED_E_STATE;
    float a = 0, t = 0;
    const bool script = (b->flags & SED_WANT_SCRIPT) != 0;
    if (b->npairs) {
        const std::array<hipEvent_t, 4> &ev = b->evk[b->cur()];
        if (!ev[0]) return SED_E_STATE;  // the last run was not timed (sed_batch_set_timing)
        if (hipEventElapsedTime(&a, ev[0], ev[1]) != hipSuccess) return SED_E_DEVICE;
        if (script && hipEventElapsedTime(&t, ev[2], ev[3]) != hipSuccess) return SED_E_DEVICE;
        if (b->nparts > 1 && b->last_log >= 0 && (size_t)b->last_log < b->plog.size()) {  // the mean over the parts
            const std::array<hipEvent_t, 12> &pl = b->plog[b->last_log];
            for (int p = 1; p < b->nparts; ++p) {
                float ap = 0, tp = 0;
                if (hipEventElapsedTime(&ap, pl[4 * (p - 1)], pl[4 * (p - 1) + 1]) != hipSuccess ||
                    (script && hipEventElapsedTime(&tp, pl[4 * (p - 1) + 2], pl[4 * (p - 1) + 3]) != hipSuccess))
                    return SED_E_DEVICE;
                a += ap;
                t += tp;
            }
            a /= b->nparts;
            t /= b->nparts;
        }
    }
    if (dp_ms) *dp_ms = a;
    if (tb_ms) *tb_ms = t;
    return SED_OK;
}

int sed_batch_spans(sed_batch *b, float *out, int max_runs) {
    if (!b || (!out && max_runs > 0)) return SED_E_ARG;
    int rc = sync_batch(b);
    if (rc != SED_OK) return rc;
    const int cnt = (int)std::min<size_t>(b->nlog, (size_t)std::max(0, max_runs));
    const bool script = (b->flags & SED_WANT_SCRIPT) != 0;
    const int P = b->nparts;
    for (int i = 0; i < cnt; ++i)
        for (int p = 0; p < P; ++p)
            for (int k = 0; k < 4; ++k) {
                float t = 0;
                if (k < 2 || script) {
                    const hipEvent_t ev = p == 0 ? b->log[i][k] : b->plog[i][4 * (p - 1) + k];
                    if (hipEventElapsedTime(&t, b->log[0][0], ev) != hipSuccess)
                        return b->ctx->fail(SED_E_DEVICE, "event timing");
                }
                out[((size_t)i * P + p) * 4 + k] = t;
            }
    return cnt;
}

int sed_batch_times(sed_batch *b, float *dp_ms, float *tb_ms, int max_runs) {
    if (!b) return SED_E_ARG;
    int rc = sync_batch(b);
    if (rc != SED_OK) return rc;
    const int cnt = (int)std::min<size_t>(b->nlog, (size_t)std::max(0, max_runs));
    const bool script = (b->flags & SED_WANT_SCRIPT) != 0;
    for (int i = 0; i < cnt; ++i) {
        float a = 0, t = 0;
        if (hipEventElapsedTime(&a, b->log[i][0], b->log[i][1]) != hipSuccess ||
            (script && hipEventElapsedTime(&t, b->log[i][2], b->log[i][3]) != hipSuccess))
            return b->ctx->fail(SED_E_DEVICE, "event timing");
        if (b->nparts > 1 && (size_t)i < b->plog.size()) {  // parts: the mean launch of the run's parts
            for (int p = 1; p < b->nparts; ++p) {
                float ap = 0, tp = 0;
                const std::array<hipEvent_t, 12> &pl = b->plog[i];
                if (hipEventElapsedTime(&ap, pl[4 * (p - 1)], pl[4 * (p - 1) + 1]) != hipSuccess ||
                    (script && hipEventElapsedTime(&tp, pl[4 * (p - 1) + 2], pl[4 * (p - 1) + 3]) != hipSuccess))
                    return b->ctx->fail(SED_E_DEVICE, "event timing");
                a += ap;
                t += tp;
            }
            a /= b->nparts;
            t /= b->nparts;
        }
        if (dp_ms) dp_ms[i] = a;
        if (tb_ms) tb_ms[i] = t;
    }
    return cnt;
}

int sed_batch_set_timing(sed_batch *b, int every) {
    if (!b || every < 0) return SED_E_ARG;
    b->time_every = every;
    return SED_OK;
}

int sed_batch_reset_times(sed_batch *b) {
    if (!b) return SED_E_ARG;
    b->nlog = 0;
    return SED_OK;
}

int sed_batch_results(sed_batch *b, double *out_dist, uint8_t *out_is_int, int32_t *out_len, uint32_t *out_ops,
                      const int64_t *ops_off) {
    if (!b) return SED_E_ARG;
    (void)hipSetDevice(b->ctx->device);
    return fetch_results(b, out_dist, out_is_int, out_len, out_ops, ops_off);
}

int sed_batch_dp_launches(const sed_batch *b) { return b ? b->nparts : SED_E_ARG; }

int sed_batch_device_results(const sed_batch *b, uint64_t *d_dist, uint64_t *d_is_int, uint64_t *d_len,
                             uint64_t *d_ops, uint64_t *ops_words) {
    if (!b) return SED_E_ARG;
    const uint64_t base = (uint64_t)(uintptr_t)b->p_res[b->runs ? b->cur() : 0];
    if (d_dist) *d_dist = base + offsetof(sed_result, dist);
    if (d_len) *d_len = base + offsetof(sed_result, len);
    if (d_is_int) *d_is_int = base + offsetof(sed_result, is_int);
    if (d_ops) *d_ops = (uint64_t)(uintptr_t)b->p_ops;
    if (ops_words) *ops_words = b->ops_words;
    return SED_OK;
}

int sed_batch_export(sed_batch *b, uint64_t d_dist, uint64_t d_len, uint64_t d_ops) {
    if (!b) return SED_E_ARG;
    sed_ctx *c = b->ctx;
    (void)hipSetDevice(c->device);
    if (!b->ran) return c->fail(SED_E_STATE, "batch has not been run");
    const int np = b->npairs;
    int rc = sync_batch(b);
    if (rc != SED_OK) return rc;
    const void *resp = b->p_res[b->cur()];
    hipError_t e = hipSuccess;
    if (np && d_dist)
        e = hipMemcpy2DAsync((void *)(uintptr_t)d_dist, sizeof(double), (const char *)resp + offsetof(sed_result, dist),
                             sizeof(sed_result), sizeof(double), np, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess && np && d_len)
        e = hipMemcpy2DAsync((void *)(uintptr_t)d_len, sizeof(int32_t), (const char *)resp + offsetof(sed_result, len),
                             sizeof(sed_result), sizeof(int32_t), np, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess && d_ops && (b->flags & SED_WANT_SCRIPT) && b->ops_words)
        e = hipMemcpyAsync((void *)(uintptr_t)d_ops, b->p_ops, 4 * b->ops_words, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? SED_OK : c->hipfail(e, "export results");
}

int sed_batch_work(const sed_batch *b, double *cells, double *algo_bytes) {
    if (!b) return SED_E_ARG;
    if (cells) *cells = b->cells;
    if (algo_bytes) *algo_bytes = b->algo_bytes;
    return SED_OK;
}

int sed_run_batch(sed_ctx *c, const uint8_t *codes_a, const int64_t *off_a, const int32_t *len_a,
                  const uint8_t *codes_b, const int64_t *off_b, const int32_t *len_b, int32_t npairs, uint32_t flags,
                  double *out_dist, uint8_t *out_is_int, int32_t *out_len, uint32_t *out_ops,
                  const int64_t *ops_off) {
    if (!c) return SED_E_ARG;
    if (c->pair_pending) return c->fail(SED_E_STATE, "a submitted pair has not been waited for");
    (void)hipSetDevice(c->device);
    if (!c->scratch) {
        c->scratch = new sed_batch();
        c->scratch->ctx = c;
        c->scratch->time_every = 0;  // nobody reads a one-shot run's times: no timing events on its kernels
    }
    if (npairs < 0 || (npairs > 0 && (!off_a || !len_a || !off_b || !len_b)))
        return c->fail(SED_E_ARG, "bad batch arguments");
    // Host-buffer batches are cut into chunks whose traceback workspace (2 bits per cell plus the
    // wavefront skew, and the SPLIT route's checkpoints beside its codes: ~0.13 B per cell more) stays under
    // SED_TB_BUDGET_GB (default 48): a list of many long pairs then runs in several launches instead of failing
    // with SED_E_OOM.
    double budget = 48e9;
    if (const char *e = getenv("SED_TB_BUDGET_GB")) budget = std::max(1e6, atof(e) * 1e9);
    int32_t p0 = 0;
    while (p0 < npairs || (npairs == 0 && p0 == 0)) {
        int32_t p1 = p0;
        double bytes = 0;
        if (flags & SED_WANT_SCRIPT) {
            while (p1 < npairs) {
                const double pb = 0.39 * (double)std::max(0, len_a[p1]) * (double)(std::max(0, len_b[p1]) + 127);
                if (p1 > p0 && bytes + pb > budget) break;
                bytes += pb;
                ++p1;
            }
        } else {
            p1 = npairs;
        }
        const int32_t np = p1 - p0;
        int rc = fill_batch(c->scratch, codes_a, off_a + p0, len_a + p0, codes_b, off_b + p0, len_b + p0, np, flags);
        if (rc != SED_OK) return rc;
        if ((rc = run_batch(c->scratch)) != SED_OK) return rc;
        rc = fetch_results(c->scratch, out_dist ? out_dist + p0 : nullptr, out_is_int ? out_is_int + p0 : nullptr,
                           out_len ? out_len + p0 : nullptr, out_ops, ops_off ? ops_off + p0 : nullptr);
        if (rc != SED_OK) return rc;
        if (npairs == 0) break;
        p0 = p1;
    }
    return SED_OK;
}

int sed_run_pair(sed_ctx *c, const uint8_t *codes_a, int32_t n, const uint8_t *codes_b, int32_t m, uint32_t flags,
                 double *out_dist, uint8_t *out_is_int, int32_t *out_len, uint32_t *out_ops) {
    if (!c) return SED_E_ARG;
    if (n < 0 || m < 0 || (n && !codes_a) || (m && !codes_b)) return c->fail(SED_E_ARG, "bad pair arguments");
    static const uint8_t none = 0;
    const int64_t off = 0;
    int32_t len = 0;
    return sed_run_batch(c, n ? codes_a : &none, &off, &n, m ? codes_b : &none, &off, &m, 1, flags, out_dist, out_is_int,
                         out_len ? out_len : &len, (flags & SED_WANT_SCRIPT) ? out_ops : nullptr,
                         (flags & SED_WANT_SCRIPT) && out_ops ? &off : nullptr);
}

int sed_pair_submit(sed_ctx *c, const uint8_t *codes_a, int32_t n, const uint8_t *codes_b, int32_t m, uint32_t flags) {
    if (!c) return SED_E_ARG;
    if (c->pair_pending) return c->fail(SED_E_STATE, "a submitted pair has not been waited for");
    if (n < 0 || m < 0 || (n && !codes_a) || (m && !codes_b)) return c->fail(SED_E_ARG, "bad pair arguments");
    (void)hipSetDevice(c->device);
    if (!c->scratch) {
        c->scratch = new sed_batch();
        c->scratch->ctx = c;
        c->scratch->time_every = 0;
    }
    static const uint8_t none = 0;
    const int64_t off = 0;
    int rc = fill_batch(c->scratch, n ? codes_a : &none, &off, &n, m ? codes_b : &none, &off, &m, 1,
                        flags & ~(uint32_t)SED_PIPELINE);
    if (rc == SED_OK) rc = run_batch(c->scratch);
    c->pair_pending = rc == SED_OK;
    return rc;
}

int sed_pair_wait(sed_ctx *c, double *out_dist, uint8_t *out_is_int, int32_t *out_len, uint32_t *out_ops) {
    if (!c) return SED_E_ARG;
    if (!c->pair_pending) return c->fail(SED_E_STATE, "no pair submitted");
    c->pair_pending = false;
    (void)hipSetDevice(c->device);
    const int64_t off = 0;
    int32_t len = 0;
    const bool script = (c->scratch->flags & SED_WANT_SCRIPT) != 0;
    return fetch_results(c->scratch, out_dist, out_is_int, out_len ? out_len : &len, script ? out_ops : nullptr,
                         script && out_ops ? &off : nullptr);
}

int sed_full_matrix(sed_ctx *c, const uint8_t *codes_a, int32_t n, const uint8_t *codes_b, int32_t m, double *D,
                    uint8_t *M) {
    if (!c) return SED_E_ARG;
    if (c->pair_pending) return c->fail(SED_E_STATE, "a submitted pair has not been waited for");
    if (n < 0 || m < 0 || !D || !M || (n && !codes_a) || (m && !codes_b)) return c->fail(SED_E_ARG, "bad arguments");
    (void)hipSetDevice(c->device);
    if (!c->have_costs) return c->fail(SED_E_STATE, "sed_set_costs() was not called");
    const int save_mode = c->opt_mode, save_R = c->opt_R;
    c->opt_mode = simple_typing(c) ? 2 : 3;
    c->opt_R = 4;
    sed_batch tmp;
    tmp.ctx = c;
    const int64_t zero = 0;
    int rc = fill_batch(&tmp, codes_a, &zero, &n, codes_b, &zero, &m, 1, 0);
    c->opt_mode = save_mode;
    c->opt_R = save_R;
    if (rc != SED_OK) return rc;
    const size_t cells = (size_t)(n + 1) * (size_t)(m + 1);
    DevBuf fD, fM;
    if (!fD.reserve(8 * cells) || !fM.reserve(cells)) {
        fD.release();
        fM.release();
        return c->fail(SED_E_OOM, "full matrix allocation (%zu cells)", cells);
    }
    sed_launch L{};
    L.pd = (const sed_pair_desc *)tmp.p_pd;
    L.npairs = 1;
    L.seqa = tmp.p_seqa;
    L.seqb = tmp.p_seqb;
    L.tb = nullptr;
    L.bnd = (uint32_t *)tmp.d_bnd.p;
    L.res = (sed_result *)tmp.p_res[0];
    L.R = 4;
    L.tasks = tmp.split ? (const int2 *)tmp.p_tasks : nullptr;  // (a pair past 32 symbols: SPLIT)
    L.ntasks = tmp.split ? tmp.ntasks : 0;
    L.stream = c->stream;
    sed_full_out fo{(double *)fD.p, (uint8_t *)fM.p, n, m};
    sed_f64_params fp = tmp.fp;
    hipError_t e = next_split_epoch(&tmp, c->stream, &fp.epoch);
    if (e == hipSuccess) e = sed_launch_f64_full(L, (const double *)c->gtab.p, fp, tmp.mode == SED_MODE_F64_TYPED, fo);
    if (e == hipSuccess) e = hipMemcpyAsync(D, fD.p, 8 * cells, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(M, fM.p, cells, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    fD.release();
    fM.release();
    return e == hipSuccess ? SED_OK : c->hipfail(e, "full matrix");
}

int sed_selftest(sed_ctx *c) {
    if (!c) return SED_E_ARG;
    (void)hipSetDevice(c->device);
    if (!c->selftest.reserve(4)) return c->fail(SED_E_OOM, "selftest buffer");
    hipError_t e;
    uint32_t h = 0;
    if ((e = hipMemsetAsync(c->selftest.p, 0, 4, c->stream)) != hipSuccess) return c->hipfail(e, "memset");
    if ((e = sed_launch_selftest((uint32_t *)c->selftest.p, c->stream)) != hipSuccess) return c->hipfail(e, "launch");
    if ((e = hipMemcpyAsync(&h, c->selftest.p, 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
        return c->hipfail(e, "copy");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hipfail(e, "sync");
    return (int)h;
}

}  // extern "C"

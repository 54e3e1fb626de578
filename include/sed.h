/*
 * sed.h — C-ABI of libsed.so, the MI355X (gfx950) engine for the weighted
 * Wagner–Fischer edit distance and its canonical edit script.
 *
 * It replaces the compute inside the reference's Python module
 * StringEditDistance (plsakr/rna-sequence-diff-patch):
 *   wagnerFisher(str1, str2, userCosts)   StringEditDistance.py:133-224  -> sed_run_batch / sed_batch_*
 *   min_cost / cost (per-cell recurrence) StringEditDistance.py:76-128   -> the DP kernels
 *   create_paths(dp)[0] (canonical path)  StringEditDistance.py:228-271  -> SED_WANT_SCRIPT traceback
 *   generate_es op sequence               StringEditDistance.py:274-334  -> packed op codes
 *   wf_score distance                     IRMethods.py:435-440           -> out_dist
 * The reference has no FFI; its boundary is the Python module itself.  The
 * Python shim (rna-sequence-diff-patch_amd/StringEditDistance.py) keeps that
 * module's names and calls this ABI through ctypes (binding shown in
 * INTEGRATION.md).
 *
 * Conventions
 *   - Sequences are passed as per-call alphabet codes (uint8, 0..K-1); the
 *     caller resolves characters -> codes and the reference's cost() into a
 *     K x K matrix (value + "is a Python int" flag) and raises the
 *     reference's KeyError itself before calling.
 *   - Every host buffer is caller-allocated.  The context owns device memory
 *     and its HIP stream.  No C++ exception crosses this ABI; functions return
 *     SED_OK or a negative SED_E_* code, with text in sed_last_error().
 *   - Threading: one context per thread and device; calls on one context are
 *     serialised by the caller; distinct contexts are independent.
 *   - Op codes of a script, origin -> sink order, 2 bits each, 16 per uint32
 *     (op p at bits 2*(p%16) of word p/16): 0 insert, 1 delete, 2 update.
 */
#ifndef SED_H
#define SED_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    SED_OK = 0,
    SED_E_ARG = -1,       /* bad argument (NULL, negative length, non-finite cost ...) */
    SED_E_DEVICE = -2,    /* HIP error */
    SED_E_OOM = -3,       /* device allocation failed */
    SED_E_RANGE = -4,     /* forced integer mode but the packed key would overflow */
    SED_E_ALPHABET = -5,  /* alphabet larger than the kernel supports (K > 32) */
    SED_E_STATE = -6      /* call order (no costs set, batch not run ...) */
};

/* flags for sed_run_batch / sed_batch_create */
#define SED_WANT_SCRIPT 1u
/* sed_batch only, a hint:
 *  - batches with per-cell traceback codes get three traceback/result buffers and a traceback stream, so the
 *    traceback of run k overlaps the DP kernel of run k+1 (device memory for the traceback triples); dynamic-CHAIN
 *    script batches also put odd runs' DP on a second DP stream (one device counter per buffer);
 *  - distance-only batches of lane pairs alternate their runs over two streams with one result slot each;
 *  - checkpoint batches (sed_batch_traceback_mode 2, the default for script batches of > 256 pairs) ignore it.
 *    Instead, one of >= 2048 wave pairs always runs in parts: part i (a contiguous range of pairs, >= 1024 wave
 *    pairs) runs forward then traceback on its own stream, 2 parts by default (environment SED_CK_HALVES = parts,
 *    1..4: up to 4 streams, the hardware queues a process gets), and nothing joins the streams at a run's end, so
 *    one part's traceback overlaps another part's forward (see sed_batch_dp_launches).
 * sed_batch_sync / _results / _export / _times wait for every stream a batch uses, and a refill waits first. */
#define SED_PIPELINE 2u
/* distance only (no SED_WANT_SCRIPT): out_len is not computed (-1), which lets the integer
 * kernels drop the op-count field of their keys (3 instead of ~4.2 VALU ops per cell). */
#define SED_NO_LEN 4u

/* sed_set_option keys */
#define SED_OPT_MODE 1          /* 0 auto, 1 packed-integer kernel, 2 fp64 kernel, 3 fp64 + int-typing */
#define SED_OPT_ROWS_PER_LANE 2 /* 0 auto, else 4,8,16,32 (integer) / 4,8 (fp64) */
#define SED_OPT_SPLIT 3         /* integer kernel, one wave per stripe: 0 auto (small batches of long
                                   pairs), 1 always, 2 never */
#define SED_OPT_LANE 4          /* one lane per pair for short str2 (m <= 32, n <= 512): 0 auto (on), 2 never */
#define SED_OPT_CHAIN 5         /* integer kernel, single-stripe pairs run back to back in one wave (no
                                   per-pair ramp): 0 auto (large batches), 1 whenever eligible, 2 never,
                                   L >= 3 whenever eligible with chains of L pairs */
#define SED_OPT_TB 7            /* integer script batches at R = 4/8/16 (stripe and CHAIN kernels, not SPLIT): 0 auto
                                   (checkpoints + recompute for > 256 pairs averaging >= 512 cells per path op,
                                   i.e. sum n*m >= 512 * sum (n+m)), 1 per-cell traceback codes, 2 checkpoints
                                   whenever eligible */
#define SED_OPT_PACK 6          /* distance-only integer batches (SED_NO_LEN): two pairs per lane (equal n) or per
                                   wave (equal n and m) in packed 16-bit cells: 0 auto (on), 2 never */
#define SED_OPT_CHAIN_WAVES 8   /* dynamic CHAIN mode: persistent waves, 0 auto (every SIMD's resident waves), else a
                                   cap (tests: several counter-fetched pairs per wave) */
#define SED_OPT_DOT 10          /* checkpoint batches of the stripe kernel and CHAIN batches: 0 auto (dot keys when
                                   the cost table's update addends factor over signed bytes and the pairs fit the
                                   bound), 2 never, 3 (tests) CHAIN ladder dot keys on the 3-bit ladder only */
#define SED_OPT_BITPAR 11       /* distance-only batches under unit costs (insert = delete = 1, every mismatch 1): lane
                                   pairs (m <= 32) run one per lane bit-parallel; in fp64 batches (e.g. costs.json with N)
                                   the lane pairs whose symbols all have unit costs among themselves: 0 auto (on),
                                   2 never */
#define SED_OPT_SCALED 12       /* distance-only fp64 batches whose costs are dyadic over <= 8 symbols (costs.json with N:
                                   multiples of 1/4): lane pairs run an exact integer DP of the costs scaled by 2^k
                                   (3 VALU per cell instead of the fp64 cell): 0 auto (on), 2 never */
#define SED_OPT_SEG 13          /* fp64 batches of > 256 wave pairs: pairs whose cost model favours it run in 16-lane
                                   segments, four per wave (stripes of 16 R rows, a 15-step ramp instead of 63: the
                                   timing.py sweep's short pairs): 0 auto, 1 every such pair, 2 never */
#define SED_OPT_SPLITCK 14      /* SPLIT script batches (<= 256 long pairs: config 2, GUI calls): the forward runs distance
                                   or dot keys with checkpoints and every 64 x 64 tile's codes are then recomputed at once
                                   for the stripe-parallel traceback (sed_batch_traceback_mode 4): 0 auto (on), 2 never
                                   (per-cell codes from the ladder-key forward) */
#define SED_OPT_ZEROCOPY 15     /* small batches (the per-call path) whose kernels write results and scripts with plain
                                   stores: the kernels write them into the batch's pinned host block, so no download
                                   follows the run: 0 auto (on), 2 never */
#define SED_OPT_DEBUG_CORRUPT 9 /* testing only: p + 1 overwrites one checkpoint word of pair p before its traceback,
                                   which must then fail with SED_E_DEVICE naming the pair; 0 off */

/* modes reported by sed_batch_mode */
#define SED_MODE_I32 1
#define SED_MODE_F64 2
#define SED_MODE_F64_TYPED 3

typedef struct sed_ctx sed_ctx;
typedef struct sed_batch sed_batch;

const char *sed_version(void);

/* Create a context on HIP device `device` (NULL on failure). */
sed_ctx *sed_create(int device);
void sed_destroy(sed_ctx *ctx);
const char *sed_last_error(const sed_ctx *ctx);
int sed_set_option(sed_ctx *ctx, int key, int value);

/* Cost model (replaces default_costs / user_costs lookups, StringEditDistance.py:6-18,76-99).
 * sub[a*K+b] = cost(symbol a -> symbol b) as the reference's cost() returns it
 * (0 for case-insensitive matches), sub_int[a*K+b] = 1 when that value is a Python int. */
int sed_set_costs(sed_ctx *ctx, int K, const double *sub, const uint8_t *sub_int,
                  double ins, int ins_is_int, double del, int del_is_int);

/* One-shot batch: host inputs, host outputs (blocking).
 * Pair p: str1 = codes_a[off_a[p] .. +len_a[p]), str2 = codes_b[off_b[p] .. +len_b[p]).
 * out_dist[p]  = dp[n][m].value as fp64; out_is_int[p] = 1 when it is a Python int.
 * out_len[p]   = number of ops in the canonical script.
 * With SED_WANT_SCRIPT: out_ops + ops_off[p] receives ceil((n+m)/16) words for pair p: the out_len[p] ops, then
 * zeros (the bits past the last op in its word and every spare word after it, on every route, so a pair's words
 * are a function of its script alone; the device buffers of sed_batch_device_results / _export hold the same).
 * Script batches whose traceback workspace (~n*m/4 bytes per pair) exceeds SED_TB_BUDGET_GB
 * (environment, default 48) run as several consecutive launches. */
int sed_run_batch(sed_ctx *ctx,
                  const uint8_t *codes_a, const int64_t *off_a, const int32_t *len_a,
                  const uint8_t *codes_b, const int64_t *off_b, const int32_t *len_b,
                  int32_t npairs, uint32_t flags,
                  double *out_dist, uint8_t *out_is_int, int32_t *out_len,
                  uint32_t *out_ops, const int64_t *ops_off);

/* One pair, blocking: sed_run_batch with npairs = 1 and plain pointers (the drop-in module's per-call path:
 * wagnerFisher of one (str1, str2), StringEditDistance.py:133-224, as IRMethods.wf_score calls it per document,
 * IRMethods.py:435-440,469-470).  out_len may be NULL; with SED_WANT_SCRIPT, out_ops receives ceil((n+m)/16) words.
 * Small batches like this one go to the device as one blob from pinned staging and come back in one download, and
 * one-shot runs carry no timing events. */
int sed_run_pair(sed_ctx *ctx, const uint8_t *codes_a, int32_t n, const uint8_t *codes_b, int32_t m, uint32_t flags,
                 double *out_dist, uint8_t *out_is_int, int32_t *out_len, uint32_t *out_ops);

/* sed_run_pair in two halves (round 6): sed_pair_submit uploads the pair and enqueues its kernels, then returns; the
 * caller may do host work while the device computes (the drop-in module builds the edit-script records of
 * generate_es, StringEditDistance.py:274-334, for the GUI's wagnerFisher -> create_paths -> generate_es call,
 * gui.py:360,385-391); sed_pair_wait then waits and writes the results exactly as sed_run_pair would.  The inputs may
 * be freed once submit returns.  One pair in flight per context: until sed_pair_wait, sed_set_costs, sed_run_batch,
 * sed_run_pair, sed_full_matrix and another submit fail with SED_E_STATE. */
int sed_pair_submit(sed_ctx *ctx, const uint8_t *codes_a, int32_t n, const uint8_t *codes_b, int32_t m, uint32_t flags);
int sed_pair_wait(sed_ctx *ctx, double *out_dist, uint8_t *out_is_int, int32_t *out_len, uint32_t *out_ops);

/* Device-resident batch: upload once, run many times (bench), fetch results. */
sed_batch *sed_batch_create(sed_ctx *ctx,
                            const uint8_t *codes_a, const int64_t *off_a, const int32_t *len_a,
                            const uint8_t *codes_b, const int64_t *off_b, const int32_t *len_b,
                            int32_t npairs, uint32_t flags);
void sed_batch_destroy(sed_batch *b);
int sed_batch_mode(const sed_batch *b);               /* SED_MODE_* chosen for this batch */
int sed_batch_rows_per_lane(const sed_batch *b);
int sed_batch_lane_pairs(const sed_batch *b);         /* pairs on the lane-per-pair kernel (short str2) */
int sed_batch_chains(const sed_batch *b);             /* CHAIN mode: number of chains (0 = not used) */
int sed_batch_packed_pairs(const sed_batch *b);       /* pairs computed two per lane / wave (SED_OPT_PACK) */
int sed_batch_bitpar_pairs(const sed_batch *b);       /* lane pairs computed bit-parallel (SED_OPT_BITPAR) */
int sed_batch_scaled_pairs(const sed_batch *b);       /* fp64 lane pairs on the scaled-integer DP (SED_OPT_SCALED) */
int sed_batch_segment_pairs(const sed_batch *b);      /* fp64 wave pairs run in 16-lane segments (SED_OPT_SEG) */
int sed_batch_split_tasks(const sed_batch *b);        /* SPLIT: workgroups (pair, stripe) per run, 0 = not SPLIT */
/* The byte factorisation behind SED_OPT_DOT, without a device (tests): for the 4 x 4 table sub (a -> b, row-major)
 * and insert/delete costs, the dot keys for pairs with min(n, m) <= maxmin (ladder_maxsum = 0) or the ladder dot
 * keys for n + m <= ladder_maxsum (the wide ladder's, L unit 16, for min(n, m) <= maxmin (or ladder_maxsum when
 * maxmin is 0) where it exists, else the 3-bit ladder's, unit 8).
 * out[0..3] = row vectors, out[4..7] = column vectors (4 signed bytes each), out[8] = decode shift / ladder sentinel
 * byte, out[9] = decode multiplier / ladder L unit.  Returns A (> 0), 0 when the table has no such factorisation,
 * or SED_E_ARG. */
int sed_dot_factor(const double *sub, double ins, double del, int maxmin, int ladder_maxsum, uint32_t *out);
int sed_batch_dot_keys(const sed_batch *b);           /* bit 0: the checkpoint forward kernel runs dot keys, bit 1: the
                                                         CHAIN kernel runs ladder dot keys (SED_OPT_DOT), bit 2: over
                                                         the wide ladder (L unit 16) */
int sed_batch_traceback_mode(const sed_batch *b);     /* 0 no script, 1 per-cell codes, 2 checkpoints (SED_OPT_TB),
                                                         3 per-cell codes walked stripe-parallel (<= 64 pairs, R = 4),
                                                         4 SPLIT checkpoints recomputed into per-cell codes
                                                         (SED_OPT_SPLITCK), walked as 3 or 1 */
/* CHAIN diagnostics of the last run (waits for it): pairs handed out by the dynamic-CHAIN device counter, and
 * the most pairs one wave computed back to back (0 when CHAIN mode is off). */
int sed_batch_chain_stats(sed_batch *b, int32_t *fetched, int32_t *max_per_wave);
int sed_batch_run(sed_batch *b);                      /* enqueue on the batch's streams (SED_PIPELINE), returns at once */
int sed_batch_sync(sed_batch *b);                     /* wait for the last run (every stream the batch uses) */
/* Forward launches per run: a checkpoint batch of >= 2048 wave pairs runs in parts on as many streams
 * (SED_CK_HALVES = parts, default 2, >= 1024 wave pairs each), else 1.  With parts, the run times below are the mean
 * launch over the parts (the launches overlap each other's kernels); part 0's DP window includes the lane kernel
 * of the batch's short pairs, if any. */
int sed_batch_dp_launches(const sed_batch *b);
/* device time of the last run, from HIP events on the launching stream(s) (ms; with parts the mean over them) */
int sed_batch_last_times(const sed_batch *b, float *dp_ms, float *traceback_ms);
/* Device times of every run since the last sed_batch_reset_times (waits for them):
 * dp_ms[i] / traceback_ms[i] for run i; returns the number of runs reported (<= max_runs). */
int sed_batch_times(sed_batch *b, float *dp_ms, float *traceback_ms, int max_runs);
/* The same runs as intervals (waits for them): out[(i * parts + p) * 4 + k] for run i, part p
 * (parts = sed_batch_dp_launches), k = {DP start, DP end, traceback start, traceback end} in ms from the DP start of
 * the first run since sed_batch_reset_times (traceback fields 0 without SED_WANT_SCRIPT).  The union of the DP
 * intervals is the time some forward kernel ran, which overlapping parts do not double-count.  Returns the number
 * of runs reported (<= max_runs). */
int sed_batch_spans(sed_batch *b, float *out, int max_runs);
int sed_batch_reset_times(sed_batch *b);
/* Timing events on the batch's kernels: every = 1 on every run (default), k > 1 on every k-th run, 0 never.  Untimed
 * runs are left out of sed_batch_times / _spans / _last_times (SED_E_STATE when the last run was untimed).  Pipelined
 * batches that order buffer reuse through their events keep them on every run. */
int sed_batch_set_timing(sed_batch *b, int every);
int sed_batch_results(sed_batch *b, double *out_dist, uint8_t *out_is_int, int32_t *out_len,
                      uint32_t *out_ops, const int64_t *ops_off);
/* Device pointers of the result arrays (for an RCCL gather); any may be NULL.  Call sed_batch_sync first: the
 * pointers are not ordered after the batch's streams. */
int sed_batch_device_results(const sed_batch *b, uint64_t *d_dist, uint64_t *d_is_int,
                             uint64_t *d_len, uint64_t *d_ops, uint64_t *ops_words);
/* Copy dist (f64[npairs]), len (i32[npairs]) and the packed scripts (u32[ops_words]) of the last
 * run into caller device memory (e.g. tensors an RCCL gather sends); any pointer may be 0. Blocking. */
int sed_batch_export(sed_batch *b, uint64_t d_dist, uint64_t d_len, uint64_t d_ops);
/* Algorithmic counts of one run: DP cells (sum n*m) and HBM bytes (inputs + traceback + outputs). */
int sed_batch_work(const sed_batch *b, double *cells, double *algo_bytes);

/* Full DP matrix of one pair (the dp object the GUI renders, StringEditDistance.py:143-224):
 * D[i*(m+1)+j] = dp[i][j].value, M[...] = optimal incoming edges (1 insert, 2 delete,
 * 4 update) | (1 << 3 when the value is a Python int).  Always runs the fp64 kernel. */
int sed_full_matrix(sed_ctx *ctx, const uint8_t *codes_a, int32_t n, const uint8_t *codes_b, int32_t m,
                    double *D, uint8_t *M);

/* Kernel self-test on the device (DPP lane shifts, byte permute); 0 = pass, else a failure bitmask. */
int sed_selftest(sed_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* SED_H */

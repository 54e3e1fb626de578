/*
 * sed_oracle.c — TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * A plain-C restatement of the reference's weighted Wagner–Fischer path, used
 * only as the parity checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  The product path (libsed.so, HIP) never links or calls it.
 *
 * What it restates (reference = plsakr/rna-sequence-diff-patch @ /root/reference):
 *   - border cells  D[0][j] = j*insert, D[i][0] = i*delete, D[0][0] = int 0
 *                                   StringEditDistance.py:146-182
 *   - cost(c1,c2): int 0 when the characters match case-insensitively, else the
 *     table entry (the caller passes the K x K matrix already resolved, with a
 *     per-entry "is Python int" flag)           StringEditDistance.py:76-89
 *   - min_cost: candidates [insert, delete, update], each ONE fp64 add, value =
 *     first minimal element (keeps its int/float typing), optimal set = every
 *     candidate equal to it                       StringEditDistance.py:92-128
 *   - wagnerFisher interior loop                  StringEditDistance.py:185-222
 *   - create_paths(dp)[0] (BFS from the sink, FIFO): the shortest co-optimal
 *     path, ties broken insert < delete < update reading from the sink; realised
 *     here as L = min edge count from the origin over optimal edges and
 *     choice = first optimal op whose predecessor has L-1.
 *                                                 StringEditDistance.py:228-271
 *     (pinned against create_paths on the G1 golden vectors)
 *
 * Op codes in the returned script (origin -> sink order): 0 insert, 1 delete, 2 update.
 * Parity: pinned by the JSON fixtures in tests/golden, generated from the reference itself.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef struct {
    int K;                     /* alphabet size of the codes */
    const double *sub;         /* K*K: cost(a,b) value (0 for case-insensitive matches) */
    const uint8_t *sub_int;    /* K*K: 1 if the Python value is an int */
    double ins, del;
    int ins_int, del_int;
} sed_oracle_costs;

/* One pair.  Outputs: *dist, *is_int, *len (ops in the canonical script).
 * ops (capacity n+m) may be NULL.  Dm/Tm/Mm (size (n+1)*(m+1), row-major)
 * may be NULL; when given they receive every cell's value, int flag and
 * optimal-incoming-edge mask (1 insert, 2 delete, 4 update).
 * Returns 0, or -1 on allocation failure. */
int sed_oracle_pair(const uint8_t *a, int n, const uint8_t *b, int m, const sed_oracle_costs *c,
                    double *dist, int *is_int, int *len, uint8_t *ops,
                    double *Dm, uint8_t *Tm, uint8_t *Mm)
{
    const int W = m + 1;
    double *D0 = (double *)malloc(sizeof(double) * W), *D1 = (double *)malloc(sizeof(double) * W);
    int32_t *L0 = (int32_t *)malloc(sizeof(int32_t) * W), *L1 = (int32_t *)malloc(sizeof(int32_t) * W);
    uint8_t *T0 = (uint8_t *)malloc(W), *T1 = (uint8_t *)malloc(W);
    uint8_t *choice = ops ? (uint8_t *)malloc((size_t)(n + 1) * W) : NULL;
    if (!D0 || !D1 || !L0 || !L1 || !T0 || !T1 || (ops && !choice)) {
        free(D0); free(D1); free(L0); free(L1); free(T0); free(T1); free(choice);
        return -1;
    }
    /* row 0 */
    D0[0] = 0.0; L0[0] = 0; T0[0] = 1;
    if (Dm) { Dm[0] = 0.0; Tm[0] = 1; Mm[0] = 0; }
    for (int j = 1; j <= m; ++j) {
        D0[j] = (double)j * c->ins; L0[j] = j; T0[j] = (uint8_t)c->ins_int;
        if (choice) choice[j] = 0;
        if (Dm) { Dm[j] = D0[j]; Tm[j] = T0[j]; Mm[j] = 1; }
    }
    for (int i = 1; i <= n; ++i) {
        const uint8_t ai = a[i - 1];
        const double *srow = c->sub + (size_t)ai * c->K;
        const uint8_t *trow = c->sub_int + (size_t)ai * c->K;
        D1[0] = (double)i * c->del; L1[0] = i; T1[0] = (uint8_t)c->del_int;
        if (choice) choice[(size_t)i * W] = 1;
        if (Dm) { size_t o = (size_t)i * W; Dm[o] = D1[0]; Tm[o] = T1[0]; Mm[o] = 2; }
        for (int j = 1; j <= m; ++j) {
            const uint8_t bj = b[j - 1];
            double cand[3];
            uint8_t ctyp[3];
            int32_t lp[3];
            cand[0] = D1[j - 1] + c->ins;  ctyp[0] = T1[j - 1] & (uint8_t)c->ins_int;  lp[0] = L1[j - 1];
            cand[1] = D0[j] + c->del;      ctyp[1] = T0[j] & (uint8_t)c->del_int;      lp[1] = L0[j];
            cand[2] = D0[j - 1] + srow[bj]; ctyp[2] = T0[j - 1] & trow[bj];             lp[2] = L0[j - 1];
            int first = 0;                         /* Python min(): first minimal element */
            if (cand[1] < cand[first]) first = 1;
            if (cand[2] < cand[first]) first = 2;
            const double v = cand[first];
            int32_t best = INT32_MAX;
            int bk = 0, mask = 0;
            for (int k = 0; k < 3; ++k) {
                if (cand[k] == v) {
                    mask |= 1 << k;
                    if (lp[k] < best) { best = lp[k]; bk = k; }
                }
            }
            D1[j] = v; T1[j] = ctyp[first]; L1[j] = best + 1;
            if (choice) choice[(size_t)i * W + j] = (uint8_t)bk;
            if (Dm) { size_t o = (size_t)i * W + j; Dm[o] = v; Tm[o] = T1[j]; Mm[o] = (uint8_t)mask; }
        }
        double *td = D0; D0 = D1; D1 = td;
        int32_t *tl = L0; L0 = L1; L1 = tl;
        uint8_t *tt = T0; T0 = T1; T1 = tt;
    }
    *dist = D0[m];
    *is_int = T0[m];
    *len = L0[m];
    if (ops) {
        int i = n, j = m, q = L0[m];
        while (i > 0 || j > 0) {
            uint8_t op = choice[(size_t)i * W + j];
            ops[--q] = op;
            if (op != 1) --j;
            if (op != 0) --i;
        }
    }
    free(D0); free(D1); free(L0); free(L1); free(T0); free(T1); free(choice);
    return 0;
}

/* ---- batch driver (pthreads) for the CPU baseline ---- */
typedef struct {
    const uint8_t *codes_a, *codes_b;
    const int64_t *off_a, *off_b, *ops_off;
    const int32_t *len_a, *len_b;
    int npairs, nthreads, tid;
    const sed_oracle_costs *c;
    double *dist; int32_t *is_int, *len; uint8_t *ops;
    int err;
} batch_job;

static void *batch_worker(void *p)
{
    batch_job *jb = (batch_job *)p;
    for (int k = jb->tid; k < jb->npairs; k += jb->nthreads) {
        int ii, ll;
        if (sed_oracle_pair(jb->codes_a + jb->off_a[k], jb->len_a[k], jb->codes_b + jb->off_b[k], jb->len_b[k],
                            jb->c, &jb->dist[k], &ii, &ll, jb->ops ? jb->ops + jb->ops_off[k] : NULL,
                            NULL, NULL, NULL)) { jb->err = -1; return NULL; }
        jb->is_int[k] = ii; jb->len[k] = ll;
    }
    return NULL;
}

int sed_oracle_batch(const uint8_t *codes_a, const int64_t *off_a, const int32_t *len_a,
                     const uint8_t *codes_b, const int64_t *off_b, const int32_t *len_b,
                     int npairs, const sed_oracle_costs *c,
                     double *dist, int32_t *is_int, int32_t *len, uint8_t *ops, const int64_t *ops_off,
                     int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    batch_job *jobs = (batch_job *)calloc(nthreads, sizeof(batch_job));
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        batch_job j = {codes_a, codes_b, off_a, off_b, ops_off, len_a, len_b, npairs, nthreads, t,
                       c, dist, is_int, len, ops, 0};
        jobs[t] = j;
        pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < nthreads; ++t) { pthread_join(th[t], NULL); err |= jobs[t].err; }
    free(jobs); free(th);
    return err;
}

/* ---- the splitmix64 synthetic generator (same definition as synth.py) ---- */
static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void sed_synth_codes(uint64_t base, uint64_t pair, int stream, int length, uint8_t *out)
{
    const uint64_t seed = ((base + pair) << 1) | (uint64_t)stream;
    for (int k = 0; k < length; ++k) {
        uint64_t w = mix64(seed + (uint64_t)(k / 32 + 1) * 0x9E3779B97F4A7C15ULL);
        out[k] = (uint8_t)((w >> (2 * (k % 32))) & 3);
    }
}

"""GPU parity of the production routes large batches take (config 3's dynamic CHAIN mode, the default
checkpoint traceback with lane-kernel pairs in the same batch, pipelined batches) and the traceback's
error path.  Every pair is checked against the C oracle (multithreaded), op by op, and every script region's
padding past the last op is zero (sed.h), so runs of one batch on two routes compare as whole buffers."""
import os

import numpy as np
import pytest

from conftest import padding_errors
import oracle
import sedcost
import sedgpu

pytestmark = pytest.mark.gpu
THREADS = min(16, len(os.sched_getaffinity(0)))


def _ragged(seed, count, nlo, nhi, mlo, mhi, related=0.5):
    rng = np.random.default_rng(seed)
    A, B = [], []
    for _ in range(count):
        n, m = int(rng.integers(nlo, nhi + 1)), int(rng.integers(mlo, mhi + 1))
        a = rng.integers(0, 4, size=n).astype(np.uint8)
        if rng.random() < related:
            src = np.resize(a, m) if n else rng.integers(0, 4, size=m).astype(np.uint8)
            mut = rng.random(m) < 0.12
            b = np.where(mut, rng.integers(0, 4, size=m), src).astype(np.uint8)
        else:
            b = rng.integers(0, 4, size=m).astype(np.uint8)
        A.append(a)
        B.append(b)
    return A, B


def _plan(table):
    return sedcost.build_plan(table, ["ACGU"], ["ACGU"])


def _check_all(plan, packed, dist, is_int, ln, ops, script=True, no_len=False):
    """Every pair vs the oracle: distance bits, typing, length and (script) every op."""
    cs = oracle.Costs.from_plan(plan)
    P = packed.npairs
    od, oi, ol, oops, ooff = oracle.batch(cs, packed.codes_a, packed.off_a, packed.len_a, packed.codes_b,
                                          packed.off_b, packed.len_b, P, want_ops=script, nthreads=THREADS)
    assert np.array_equal(dist, od), np.flatnonzero(dist != od)[:10]
    assert np.array_equal(is_int.astype(bool), oi.astype(bool))
    if no_len:
        assert np.all((ln == -1) | (ln == ol))
    else:
        assert np.array_equal(ln, ol), np.flatnonzero(ln != ol)[:10]
    if script:
        bad = [p for p in range(P)
               if not np.array_equal(sedgpu.unpack_ops(ops, packed.ops_off, p, int(ln[p])),
                                     oops[ooff[p]:ooff[p] + ol[p]])]
        assert not bad, bad[:10]
        bad = padding_errors(ops, packed.ops_off, packed.len_a, packed.len_b, ln)
        assert not bad, ("nonzero script padding", bad[:10])


def _batch_run(ctx, packed, script, no_len=False, pipeline=False, runs=1):
    b = sedgpu.Batch(ctx, packed, script, pipeline=pipeline, no_len=no_len)
    try:
        for _ in range(runs):
            b.run()
        out = b.results()
        return b, out
    except Exception:
        b.close()
        raise


def test_dynamic_chain_pipelined_two_dp_streams(gpu, tables):
    """A pipelined dynamic-CHAIN script batch (config 3's route) runs odd runs' DP on a second stream, so a run's
    persistent waves start in the previous run's tail; each buffer slot has its own device counter.  Seven runs
    (every slot reused, both streams, counters past their first base), every pair of the last run against the
    oracle, and the counter accounting of the last run."""
    A, B = _ragged(4242, 12000, 1, 512, 1, 700)
    plan = _plan(tables[False])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, pipeline=True, runs=7)
    try:
        assert b.rows_per_lane == 8 and b.chains == 5120 and b.traceback_mode == 1
        fetched, per_wave = b.chain_stats()
        assert fetched == packed.npairs - b.lane_pairs and per_wave >= 2, (fetched, per_wave)
    finally:
        b.close()
    _check_all(plan, packed, d, ii, ln, ops, script=True)


@pytest.mark.parametrize("alphabet", ["ACGU", "ACGUN"])
def test_lane_batches_pipelined_on_two_streams(gpu, tables, alphabet):
    """Distance-only batches of lane pairs (config 5: bit-parallel; with N: the fp64 lane kernel) pipelined: odd runs
    on a second stream beside the previous run, three result buffers.  Five runs, every pair of the last one
    against the oracle (ACGUN exercises the fp64 mode, costs.json)."""
    rng = np.random.default_rng(777 + len(alphabet))
    seqs = ["".join(rng.choice(list(alphabet), p=None if alphabet == "ACGU" else [0.2475] * 4 + [0.01],
                               size=int(rng.integers(20, 33)))) for _ in range(120)]
    pairs = [(a, b) for a in seqs for b in seqs]
    plan = sedcost.build_plan(tables[False], [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(b) for _, b in pairs])
    b, (d, ii, ln, ops) = _batch_run(gpu, packed, False, no_len=True, pipeline=True, runs=5)
    try:
        assert b.lane_pairs == len(pairs) and b.bitpar_pairs > 0
        assert b.mode == ("i32" if alphabet == "ACGU" else "f64")
    finally:
        b.close()
    _check_all(plan, packed, d, ii, ln, ops, script=False, no_len=True)


@pytest.mark.parametrize("user", [False, True])
def test_dynamic_chain_config3_route(gpu, tables, user):
    """12 000 ragged single-stripe pairs (n 1..512, m 1..700): more than twice the 5120 resident waves, so
    the automatic route is dynamic CHAIN (persistent waves fetching pairs from the device counter) at R = 8.
    Every pair is checked; the counter handed out every wave pair and waves ran several pairs back to back."""
    A, B = _ragged(3000 + user, 12000, 1, 512, 1, 700)
    plan = _plan(tables[user])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    # scripts on the automatic route (per-cell codes at this size) and forced onto checkpoints (SED_OPT_TB = 2)
    ref = None
    for script, no_len, tb in ((True, False, 0), (True, False, 2), (False, False, 0), (False, True, 0)):
        gpu.set_option(sedgpu.SED_OPT_TB, tb)
        try:
            b, (d, ii, ln, ops) = _batch_run(gpu, packed, script, no_len=no_len)
        finally:
            gpu.set_option(sedgpu.SED_OPT_TB, 0)
        try:
            nwave = packed.npairs - b.lane_pairs
            if not no_len:  # distance-only batches pack pairs two per wave instead (SED_OPT_PACK)
                assert b.rows_per_lane == 8 and b.chains == 5120
                assert b.traceback_mode == (0 if not script else 2 if tb == 2 else 1)
                fetched, per_wave = b.chain_stats()
                assert fetched == nwave and per_wave >= 2, (fetched, nwave, per_wave)
                # costs.json's addends factor over bytes with A > 16 min(n, m): the ladder keys run on v_dot4 over
                # the wide ladder (user_costs' would need A > 16 * 512 with kappa up to 5: no byte factorisation)
                assert b.ladder_dot_keys == (not user and tb != 2) and b.ladder_wide == b.ladder_dot_keys
        finally:
            b.close()
        _check_all(plan, packed, d, ii, ln, ops, script=script, no_len=no_len)
        if script and ref is None:
            ref = (d, ii, ln, ops)
        elif script:
            _same((d, ii, ln, ops), ref, packed.ops_off)  # checkpoints against per-cell codes, whole buffers
    # the wide-ladder dot keys against the perm ladder (SED_OPT_DOT = 2) and the 3-bit ladder's dot keys (3) on the
    # same batch, whole buffers
    if not user:
        for dot, lad in ((2, False), (3, True)):
            gpu.set_option(sedgpu.SED_OPT_DOT, dot)
            try:
                b, (d2, ii2, ln2, ops2) = _batch_run(gpu, packed, True)
                try:
                    assert b.ladder_dot_keys == lad and not b.ladder_wide and b.chains == 5120
                finally:
                    b.close()
            finally:
                gpu.set_option(sedgpu.SED_OPT_DOT, 0)
            _check_all(plan, packed, d2, ii2, ln2, ops2)
            _same((d2, ii2, ln2, ops2), ref, packed.ops_off)


def test_dynamic_chain_capped_waves(gpu, tables):
    """The same route with the persistent waves capped (SED_OPT_CHAIN_WAVES = 300): ~30 fetched pairs per
    wave, so every wave crosses many pair switches; scripts and lengths vs the oracle.  Each batch runs three
    times (the pair counter is not reset between runs: a run's values start at runs * (list + waves))."""
    A, B = _ragged(3100, 9000, 1, 512, 33, 700)
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    gpu.set_option(sedgpu.SED_OPT_CHAIN, 1)
    gpu.set_option(sedgpu.SED_OPT_CHAIN_WAVES, 300)
    try:
        for tb in (0, 2):  # per-cell codes, then checkpoints
            gpu.set_option(sedgpu.SED_OPT_TB, tb)
            b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, pipeline=tb == 0, runs=3)
            try:
                assert b.chains == 300 and b.traceback_mode == (2 if tb else 1)
                fetched, per_wave = b.chain_stats()
                assert fetched == packed.npairs - b.lane_pairs and per_wave >= 25, (fetched, per_wave)
            finally:
                b.close()
            _check_all(plan, packed, d, ii, ln, ops)
    finally:
        gpu.set_option(sedgpu.SED_OPT_CHAIN, 0)
        gpu.set_option(sedgpu.SED_OPT_CHAIN_WAVES, 0)
        gpu.set_option(sedgpu.SED_OPT_TB, 0)


def test_checkpoint_default_route_with_lane_pairs_and_pipeline(gpu, tables):
    """> 256 mixed pairs under automatic options: short str2 (m <= 32) on the lane kernel with per-cell
    codes, long pairs (n up to 2600) on the R = 16 checkpoint route, in one batch.  Every pair vs the
    oracle, then the same batch pipelined (SED_PIPELINE, ignored by checkpoint batches) run 3 times."""
    A1, B1 = _ragged(3200, 200, 1, 512, 1, 32)
    A2, B2 = _ragged(3201, 120, 1200, 2600, 1200, 2600)  # large enough for the automatic checkpoint route
    A, B = A1 + A2, B1 + B2
    order = np.random.default_rng(3202).permutation(len(A))
    A, B = [A[i] for i in order], [B[i] for i in order]
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    b, (d, ii, ln, ops) = _batch_run(gpu, packed, True)
    try:
        assert b.traceback_mode == 2 and b.rows_per_lane == 16 and b.lane_pairs >= 150
    finally:
        b.close()
    _check_all(plan, packed, d, ii, ln, ops)
    b, (d2, ii2, ln2, ops2) = _batch_run(gpu, packed, True, pipeline=True, runs=3)
    b.close()
    _same((d2, ii2, ln2, ops2), (d, ii, ln, ops), packed.ops_off)


@pytest.mark.parametrize("user", [False, True])
def test_checkpoint_dot_keys_route(gpu, tables, user):
    """Dot keys (SED_OPT_DOT): the checkpoint forward kernel's cell is one v_dot4_i32_i8 (row vector of str1's
    symbol . column vector of str2's symbol, added to the diagonal) and one v_max3 when the table's update addends
    A*kappa + 1 factor over signed bytes (both shipped tables do).  300 ragged pairs (1..2600, related and
    unrelated) at R = 16, 8 and 4: every pair vs the oracle, op by op, and identical to the perm-based distance
    keys (SED_OPT_DOT = 2)."""
    A, B = _ragged(3400 + user, 300, 1, 2600, 1, 2600)
    plan = _plan(tables[user])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    gpu.set_option(sedgpu.SED_OPT_TB, 2)
    gpu.set_option(sedgpu.SED_OPT_CHAIN, 2)
    try:
        for R in (16, 8, 4):
            gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, R)
            b, (d, ii, ln, ops) = _batch_run(gpu, packed, True)
            try:
                assert b.dot_keys and b.traceback_mode == 2 and b.rows_per_lane == R and b.chains == 0
            finally:
                b.close()
            _check_all(plan, packed, d, ii, ln, ops)
            gpu.set_option(sedgpu.SED_OPT_DOT, 2)
            try:
                b, (d2, ii2, ln2, ops2) = _batch_run(gpu, packed, True)
                try:
                    assert not b.dot_keys and b.traceback_mode == 2
                finally:
                    b.close()
            finally:
                gpu.set_option(sedgpu.SED_OPT_DOT, 0)
            _same((d2, ii2, ln2, ops2), (d, ii, ln, ops), packed.ops_off)
    finally:
        gpu.set_option(sedgpu.SED_OPT_TB, 0)
        gpu.set_option(sedgpu.SED_OPT_CHAIN, 0)
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)


def test_dot_keys_fall_back_past_their_bound(gpu, tables):
    """user_costs' byte factorisation has A = 2880.  Dot keys order the candidates of a cell correctly while
    A > min(n, m) (kmax - kmin) / kmin (kappa = insert + delete - cost in 3..5), i.e. min(n, m) < 4320: a batch
    holding a 4400 x 4400 pair keeps the perm-based distance keys, the same batch without it takes dot keys, and
    both match the oracle."""
    A, B = _ragged(3500, 259, 100, 1500, 100, 1500)
    a, b = _ragged(3501, 1, 4400, 4400, 4400, 4400, related=1.0)
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    gpu.set_option(sedgpu.SED_OPT_TB, 2)
    try:
        for extra, want in (([], True), (list(zip(a, b)), False)):
            packed = sedgpu.PackedPairs(A + [x for x, _ in extra], B + [y for _, y in extra])
            bt, (d, ii, ln, ops) = _batch_run(gpu, packed, True)
            try:
                assert bt.dot_keys == want and bt.traceback_mode == 2
            finally:
                bt.close()
            _check_all(plan, packed, d, ii, ln, ops)
    finally:
        gpu.set_option(sedgpu.SED_OPT_TB, 0)


def test_checkpoint_traceback_reports_a_corrupt_checkpoint(gpu, tables):
    """SED_OPT_DEBUG_CORRUPT overwrites one column-checkpoint word (the sink row's, in the chunk before the
    sink's tile) of one pair with the smallest key between the DP and the traceback: the recomputed tile then contradicts the path
    length, and the run fails with SedError naming that pair instead of returning a wrong script."""
    A, B = _ragged(3300, 300, 200, 1500, 100, 1500)
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    victim = 123
    gpu.set_option(sedgpu.SED_OPT_TB, 2)
    gpu.set_option(sedgpu.SED_OPT_DEBUG_CORRUPT, victim + 1)
    try:
        with pytest.raises(sedgpu.SedError, match="pair %d: traceback failed" % victim):
            gpu.run(packed, True)
    finally:
        gpu.set_option(sedgpu.SED_OPT_DEBUG_CORRUPT, 0)
    try:
        d, ii, ln, ops = gpu.run(packed, True)  # the same context recovers
    finally:
        gpu.set_option(sedgpu.SED_OPT_TB, 0)
    _check_all(plan, packed, d, ii, ln, ops)


def test_checkpoint_parts_on_streams(gpu, tables):
    """A checkpoint batch of >= 2048 wave pairs runs in parts on as many streams (SED_CK_HALVES, default 2 parts of
    >= 1024 wave pairs: one part's traceback beside another part's forward, no join between runs).  3100 ragged wave
    pairs plus 101 lane-kernel pairs, shuffled (an odd count): three runs back to back, every pair vs the oracle;
    then a corrupted checkpoint of a last-part pair fails the run naming that pair, and the next run is right
    again."""
    A1, B1 = _ragged(3600, 3100, 200, 700, 200, 700)
    A2, B2 = _ragged(3601, 101, 1, 300, 1, 32)
    A, B = A1 + A2, B1 + B2
    order = np.random.default_rng(3602).permutation(len(A))
    A, B = [A[i] for i in order], [B[i] for i in order]
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    gpu.set_option(sedgpu.SED_OPT_TB, 2)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 4)
    try:
        b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, runs=3)
        try:
            assert b.traceback_mode == 2 and b.dp_launches == 2 and b.lane_pairs == 101
        finally:
            b.close()
        _check_all(plan, packed, d, ii, ln, ops)
        victim = max(p for p in range(len(A)) if len(B[p]) > 32)  # a wave pair of the last part
        gpu.set_option(sedgpu.SED_OPT_DEBUG_CORRUPT, victim + 1)
        try:
            with pytest.raises(sedgpu.SedError, match="pair %d: traceback failed" % victim):
                gpu.run(packed, True)
        finally:
            gpu.set_option(sedgpu.SED_OPT_DEBUG_CORRUPT, 0)
        d2, ii2, ln2, ops2 = gpu.run(packed, True)
        _same((d2, ii2, ln2, ops2), (d, ii, ln, ops), packed.ops_off)
    finally:
        gpu.set_option(sedgpu.SED_OPT_TB, 0)
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)


def test_headline_config4_route(gpu, tables):
    """The exact route of the bench's headline (config 4's shard) under automatic options: R = 16, checkpoints +
    recompute, dot keys, 2 parts on 2 streams (>= 2048 wave pairs), user_costs.  The batch mixes
      - 2100 ragged wave pairs of 64..1100 (related and unrelated),
      - 48 pairs of 4096 x 4096 (the headline's shape; 48 rather than fewer so that the automatic rule
        sum n*m >= 512 * sum (n + m) still picks checkpoints with the short pairs in the batch),
      - 6 pairs with min(n, m) in 4097..4319, which must still take dot keys (user_costs' A = 2880 orders a cell's
        candidates while min(n, m) < 4320),
    shuffled, run 3 times back to back, every pair vs the oracle op by op (StringEditDistance.py:133-271).  The same
    batch plus 2 pairs with min(n, m) >= 4320 must fall back to the perm-based distance keys, still in 2 parts, with
    the same results for the common pairs and the oracle's for the 2 new ones."""
    rng = np.random.default_rng(4400)
    A1, B1 = _ragged(4401, 2100, 64, 1100, 64, 1100)
    A2, B2 = _ragged(4402, 48, 4096, 4096, 4096, 4096)
    A3, B3 = [], []
    for k in range(6):
        n, m = int(rng.integers(4097, 4320)), int(rng.integers(4097, 4320))
        a, b = _ragged(4403 + k, 1, n, n, m, m, related=float(k % 2))
        A3 += a
        B3 += b
    A, B = A1 + A2 + A3, B1 + B2 + B3
    order = rng.permutation(len(A))
    A, B = [A[i] for i in order], [B[i] for i in order]
    la = np.array([len(x) for x in A], np.float64)
    lb = np.array([len(x) for x in B], np.float64)
    assert (la * lb).sum() >= 512 * (la + lb).sum()  # the automatic checkpoint rule (sed_runtime.cpp: b->ck)
    assert np.minimum(la, lb).max() < 4320 and (np.minimum(la, lb) > 4096).sum() == 6
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, runs=3)
    try:
        assert b.mode == "i32" and b.rows_per_lane == 16 and b.traceback_mode == 2
        assert b.dp_launches == 2 and b.dot_keys and b.chains == 0 and b.lane_pairs == 0
    finally:
        b.close()
    _check_all(plan, packed, d, ii, ln, ops)
    # + 2 pairs past the dot-key bound: the whole batch keeps the distance keys
    a4, b4 = _ragged(4410, 1, 4320, 4320, 4350, 4350, related=1.0)
    a5, b5 = _ragged(4411, 1, 4400, 4400, 4330, 4330, related=0.0)
    A6, B6 = A + a4 + a5, B + b4 + b5
    packed6 = sedgpu.PackedPairs(A6, B6)
    b, (d6, ii6, ln6, ops6) = _batch_run(gpu, packed6, True, runs=3)
    try:
        assert b.rows_per_lane == 16 and b.traceback_mode == 2 and b.dp_launches == 2 and not b.dot_keys
    finally:
        b.close()
    P = len(A)
    assert np.array_equal(d6[:P], d) and np.array_equal(ii6[:P], ii) and np.array_equal(ln6[:P], ln)
    W = int(packed.ops_off[P])  # the common pairs' script words sit at the same offsets in both buffers
    assert np.array_equal(ops6[:W], ops[:W]), np.flatnonzero(ops6[:W] != ops[:W])[:8]
    tail = sedgpu.PackedPairs(a4 + a5, b4 + b5)
    o = tail.ops_off
    _check_all(plan, tail, d6[P:], ii6[P:], ln6[P:],
               np.concatenate([ops6[packed6.ops_off[P + q]:packed6.ops_off[P + q + 1]] for q in range(2)]))
    assert o[2] == packed6.ops_off[P + 2] - packed6.ops_off[P]


def test_repeated_runs_reuse_the_context(gpu, tables):
    """sed_run_batch refills one scratch batch per call (event log reused, not grown): many small calls in
    a row stay correct."""
    A, B = _ragged(3400, 40, 1, 300, 1, 300)
    plan = _plan(tables[False])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    first = gpu.run(packed, True)
    for _ in range(300):
        d, ii, ln, ops = gpu.run(packed, True)
    _same((d, ii, ln, ops), first, packed.ops_off)


@pytest.mark.parametrize("R,split", [(4, 0), (4, 2), (8, 2), (16, 2)])
def test_stripe_parallel_traceback(gpu, tables, R, split):
    """Few pairs (<= 64) with per-cell codes at R = 4 (config 2's SPLIT route): the traceback maps every stripe's
    exits (one lane per stripe and column, codes staged in LDS), composes them from the sink and walks the stripe
    segments in parallel (sed_tb_stripe*_kernel); other R keep the one-chain window walk.
    Ragged pairs of 1..12 stripes with empty strings, lane-kernel pairs, exits through the column-0 border
    (n >> m) and segment boundaries inside script words; every op vs the oracle and vs the one-chain walk."""
    rows = 64 * R
    A, B = _ragged(5200 + R + split, 9, 1, 12 * rows if R == 4 else 4 * rows, 1, 2600)
    rng = np.random.default_rng(5300 + R)
    # (3 rows, 3000) and (4 rows, 4000): insert-heavy paths that leave the map kernel's staged columns
    for n, m in ((0, 40), (60, 0), (700, 20), (3 * rows, 3), (3 * rows + 1, 2 * rows), (2 * rows, 500), (5 * rows - 1, 17),
                 (3 * rows, 3000), (4 * rows, 4000)):
        A.append(rng.integers(0, 4, size=n).astype(np.uint8))
        B.append(rng.integers(0, 4, size=m).astype(np.uint8))
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, R)
    gpu.set_option(sedgpu.SED_OPT_SPLIT, split)
    try:
        b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, runs=2)
        try:
            # stripe walk at R = 4; SPLIT batches there take the checkpoint forward + tile-parallel code recompute
            assert b.traceback_mode == ((4 if split != 2 else 3) if R == 4 else 1) and b.rows_per_lane == R
        finally:
            b.close()
        _check_all(plan, packed, d, ii, ln, ops, script=True)
    finally:
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
        gpu.set_option(sedgpu.SED_OPT_SPLIT, 0)


def test_stripe_walk_only_with_three_stripes(gpu, tables):
    """A few-pair script batch at R = 4 whose pairs all have fewer than 3 stripes (<= 512 rows) has no stripe map
    to build: it takes the window walk (traceback_mode 1, zero-copy results); one pair of 3 stripes brings the
    stripe-parallel walk (mode 3) back.  Both against the oracle."""
    rng = np.random.default_rng(5400)
    shapes = [(100, 100), (250, 240), (512, 700), (1, 3000), (300, 0)]
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 4)
    gpu.set_option(sedgpu.SED_OPT_SPLIT, 2)
    try:
        for extra, want in (([], 1), ([(513, 600)], 3)):
            A = [rng.integers(0, 4, size=n).astype(np.uint8) for n, _ in shapes + extra]
            B = [rng.integers(0, 4, size=m).astype(np.uint8) for _, m in shapes + extra]
            packed = sedgpu.PackedPairs(A, B)
            b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, runs=2)
            try:
                assert b.traceback_mode == want
            finally:
                b.close()
            _check_all(plan, packed, d, ii, ln, ops, script=True)
    finally:
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
        gpu.set_option(sedgpu.SED_OPT_SPLIT, 0)


def _same(out, ref, ops_off):
    """Identical results, the packed script buffers word for word (padding included: zero on every route)."""
    for name, x, y in zip(("dist", "is_int", "len", "ops"), out, ref):
        assert np.array_equal(x, y), (name, np.flatnonzero(x != y)[:8])


@pytest.mark.parametrize("R,pipeline", [(4, False), (4, True), (16, False)])
def test_split_handoff_repeated_runs(gpu, tables, R, pipeline):
    """SPLIT's stripes hand their bottom rows over as 64-bit {epoch tag, value} words (sed_kernels.hip): words of
    an earlier run carry another epoch and must never be taken for this run's.  One batch run 40 times (results
    after each run), and the one-shot path (its scratch batch refilled per call, epoch restarting at 1), must
    match the oracle every time; the 4096^2 pair is config 2's shape."""
    A, B = _ragged(5400 + R, 3, 700, 3000, 1, 2600)
    rng = np.random.default_rng(5410)
    A.append(rng.integers(0, 4, size=4096).astype(np.uint8))
    B.append(rng.integers(0, 4, size=4096).astype(np.uint8))
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, R)
    gpu.set_option(sedgpu.SED_OPT_SPLIT, 1)
    try:
        b = sedgpu.Batch(gpu, packed, True, pipeline=pipeline)
        try:
            first = None
            for _ in range(40):
                b.run()
                out = b.results()
                if first is None:
                    first = out
                    _check_all(plan, packed, *out, script=True)
                else:
                    _same(out, first, packed.ops_off)
        finally:
            b.close()
        for _ in range(3):
            out = gpu.run(packed, True)
            _check_all(plan, packed, *out, script=True)
            _same(out, first, packed.ops_off)
    finally:
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
        gpu.set_option(sedgpu.SED_OPT_SPLIT, 0)


def _factorable_tables(seed, want_ck, want_lad, maxmin, maxsum):
    """Seeded random integer ACGU tables (insert / delete 1..3, substitutions 1..2, as a GUI edit could write them)
    that sed_dot_factor accepts: want_ck for dot keys at min(n, m) <= maxmin, want_lad for ladder dot keys at
    n + m <= maxsum."""
    rng = np.random.default_rng(seed)
    ck, lad = [], []
    K = "ACGU"
    while len(ck) < want_ck or len(lad) < want_lad:
        ins, de = int(rng.integers(1, 4)), int(rng.integers(1, 4))
        sub = rng.integers(1, min(2, ins + de) + 1, size=(4, 4)).astype(float)
        np.fill_diagonal(sub, 0)
        table = {"insert": float(ins), "delete": float(de),
                 "update": {a: {b: float(sub[i, j]) for j, b in enumerate(K) if b != a} for i, a in enumerate(K)}}
        if len(ck) < want_ck and sedgpu.dot_factor(sub, ins, de, maxmin, 0) is not None:
            ck.append(table)
        if len(lad) < want_lad and sedgpu.dot_factor(sub, ins, de, 0, maxsum) is not None:
            lad.append(table)
    return ck, lad


def test_dot_keys_on_random_factorable_tables(gpu):
    """Dot keys and ladder dot keys are picked automatically for any integer table that factors over signed bytes,
    not only the two shipped ones (a GUI-edited user_costs.json can hold others).  Seeded random tables the
    factorisation accepts: the checkpoint route (R = 16) must take dot keys, the dynamic-CHAIN route with per-cell
    codes (R = 8) ladder dot keys; every pair vs the oracle and identical to SED_OPT_DOT = 2."""
    ck_tables, lad_tables = _factorable_tables(3600, 3, 2, 1500, 1024)
    A, B = _ragged(3601, 300, 1, 1500, 1, 1500)
    a2, b2 = _ragged(3602, 2200, 1, 512, 1, 512)
    cases = [(t, A, B, {sedgpu.SED_OPT_TB: 2, sedgpu.SED_OPT_CHAIN: 2, sedgpu.SED_OPT_ROWS_PER_LANE: 16}, "dot")
             for t in ck_tables]
    cases += [(t, a2, b2, {sedgpu.SED_OPT_TB: 1, sedgpu.SED_OPT_CHAIN: 1, sedgpu.SED_OPT_ROWS_PER_LANE: 8,
                           sedgpu.SED_OPT_LANE: 2}, "lad") for t in lad_tables]
    for table, AA, BB, opts, kind in cases:
        plan = _plan(table)
        gpu.set_costs(plan)
        packed = sedgpu.PackedPairs(AA, BB)
        for k, v in opts.items():
            gpu.set_option(k, v)
        try:
            b, (d, ii, ln, ops) = _batch_run(gpu, packed, True)
            try:
                assert (b.dot_keys if kind == "dot" else b.ladder_dot_keys), (kind, table)
                if kind == "lad":
                    assert b.chains > 0
            finally:
                b.close()
            _check_all(plan, packed, d, ii, ln, ops)
            gpu.set_option(sedgpu.SED_OPT_DOT, 2)
            b, (d2, ii2, ln2, ops2) = _batch_run(gpu, packed, True)
            try:
                assert not b.dot_keys and not b.ladder_dot_keys
            finally:
                b.close()
            _same((d2, ii2, ln2, ops2), (d, ii, ln, ops), packed.ops_off)
        finally:
            for k in list(opts) + [sedgpu.SED_OPT_DOT]:
                gpu.set_option(k, 0)


@pytest.mark.parametrize("user,dot", [(True, True), (False, True), (True, False)])
def test_split_checkpoint_codes_route(gpu, tables, user, dot):
    """SPLIT script batches (config 2, GUI pairs; SED_OPT_SPLITCK): the SPLIT forward on dot keys (or distance keys
    with SED_OPT_DOT = 2) stores checkpoints, sed_ck_codes_kernel recomputes every 64 x 64 tile's codes into the
    per-cell code layout, and the stripe-parallel walk reads them.  Ragged pairs of 1..12 stripes (lengths not
    multiples of 64 or 256, single-stripe pairs, n >> m, m >> n, empty sides), two runs back to back; every op vs the
    oracle and identical to the ladder-key forward (SED_OPT_SPLITCK = 2)."""
    A, B = _ragged(5400 + user + 2 * dot, 10, 1, 12 * 256, 1, 3000)
    rng = np.random.default_rng(5500 + user)
    for n, m in ((0, 40), (60, 0), (257, 5), (300, 1), (256, 64), (255, 63), (3 * 256 + 1, 2 * 256 + 3), (40, 2900),
                 (4096, 4096)):
        A.append(rng.integers(0, 4, size=n).astype(np.uint8))
        B.append(rng.integers(0, 4, size=m).astype(np.uint8))
    plan = _plan(tables[user])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    outs = []
    try:
        if not dot:
            gpu.set_option(sedgpu.SED_OPT_DOT, 2)
        for opt in (0, 2):
            gpu.set_option(sedgpu.SED_OPT_SPLITCK, opt)
            b, out = _batch_run(gpu, packed, True, runs=2)
            try:
                assert b.rows_per_lane == 4
                assert b.traceback_mode == (4 if opt == 0 else 3)
                if opt == 0:
                    assert b.dot_keys == dot
            finally:
                b.close()
            outs.append(out)
    finally:
        gpu.set_option(sedgpu.SED_OPT_SPLITCK, 0)
        gpu.set_option(sedgpu.SED_OPT_DOT, 0)
    d, ii, ln, ops = outs[0]
    _check_all(plan, packed, d, ii, ln, ops, script=True)
    for x, y in zip(outs[0], outs[1]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("user", [False, True])
def test_split_band_map_unknown_entries(gpu, tables, user):
    """Stripe-parallel walks whose band maps leave entries unknown (sed_tb_bandmap_kernel: a walk past 64 + 64 ceil(m/n)
    steps, a run of more than 96 inserts, or past the staged columns), so the banded emit kernel walks them itself:
    pairs with a block of 300-700 symbols inserted or deleted in the middle, m = 3n and n = 3m, against the oracle,
    with padding checked (the ops buffer compared whole)."""
    rng = np.random.default_rng(5600 + user)
    A, B = [], []
    for n, ins, at in ((2048, 400, 1000), (1500, 700, 200), (3000, 300, 2600)):
        a = rng.integers(0, 4, size=n).astype(np.uint8)
        mid = rng.integers(0, 4, size=ins).astype(np.uint8)
        b = np.concatenate([a[:at], mid, a[at:]])
        mut = rng.random(len(b)) < 0.05  # point mutations around the block
        b[mut] = rng.integers(0, 4, size=int(mut.sum())).astype(np.uint8)
        A += [a, b]
        B += [b, a]  # the insert block as inserts, then as deletes
    for n, m in ((700, 2100), (2100, 700), (1024, 4000)):
        A.append(rng.integers(0, 4, size=n).astype(np.uint8))
        B.append(rng.integers(0, 4, size=m).astype(np.uint8))
    plan = _plan(tables[user])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, runs=2)
    try:
        assert b.rows_per_lane == 4 and b.traceback_mode == 4  # the SPLIT checkpoint route with the stripe-parallel walk
    finally:
        b.close()
    _check_all(plan, packed, d, ii, ln, ops, script=True)


@pytest.mark.parametrize("user", [False, True])
def test_split_checkpoint_window_walk(gpu, tables, user):
    """SPLIT script batches of 65..256 pairs: the SPLIT checkpoint forward and the tile-parallel code recompute, then
    the window walk (sed_traceback_window_kernel) over the plain op codes (tb_ladder off), since the stripe-parallel
    walk takes <= 64 pairs only.  100 ragged pairs of 257..1500 (some with an empty side), every op vs the oracle and
    identical to the ladder-key forward (SED_OPT_SPLITCK = 2)."""
    A, B = _ragged(5600 + user, 96, 257, 1500, 1, 1500)
    rng = np.random.default_rng(5610 + user)
    for n, m in ((300, 0), (0, 700), (1024, 1), (257, 1500)):
        A.append(rng.integers(0, 4, size=n).astype(np.uint8))
        B.append(rng.integers(0, 4, size=m).astype(np.uint8))
    plan = _plan(tables[user])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    outs = []
    try:
        for opt in (0, 2):
            gpu.set_option(sedgpu.SED_OPT_SPLITCK, opt)
            b, out = _batch_run(gpu, packed, True, runs=2)
            try:
                assert b.rows_per_lane == 4 and b.traceback_mode == (4 if opt == 0 else 1)
            finally:
                b.close()
            outs.append(out)
    finally:
        gpu.set_option(sedgpu.SED_OPT_SPLITCK, 0)
    _check_all(plan, packed, *outs[0], script=True)
    _same(outs[1], outs[0], packed.ops_off)


def test_split_script_batch_with_only_empty_sides(gpu, tables):
    """A SPLIT script batch (n > 256) whose every pair has an empty side has no tile to recompute: it must run on
    per-cell codes (the border walk), not fail the code-recompute launch.  wagnerFisher(s1, "") with len(s1) > 256
    followed by the script is the GUI's way there (sed_run_pair), and a small batch of such pairs (all-delete and
    all-insert scripts) the batch way; both vs the oracle."""
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    rng = np.random.default_rng(5700)
    a = rng.integers(0, 4, size=300).astype(np.uint8)
    d, ii, ln, ops = gpu.run_pair(a.tobytes(), b"", True)
    packed1 = sedgpu.PackedPairs([a], [np.zeros(0, np.uint8)])
    _check_all(plan, packed1, np.array([d]), np.array([ii]), np.array([ln], np.int32), ops)
    A = [rng.integers(0, 4, size=n).astype(np.uint8) for n in (300, 0, 4096, 257)]
    B = [rng.integers(0, 4, size=m).astype(np.uint8) for m in (0, 900, 0, 0)]
    packed = sedgpu.PackedPairs(A, B)
    b, out = _batch_run(gpu, packed, True, runs=2)
    try:
        assert b.traceback_mode in (1, 3)
    finally:
        b.close()
    _check_all(plan, packed, *out, script=True)


def test_checkpoint_two_residency_rounds_every_pair(gpu, tables):
    """More checkpoint wave pairs than the forward kernel holds resident at once (5 waves per SIMD x 1024 SIMDs =
    5120): 5600 ragged pairs of 1000..1500 (related and unrelated) under automatic options take R = 16, checkpoints +
    recompute, dot keys and 2 parts on 2 streams, and the second residency round of each part runs.  Two runs back
    to back; EVERY pair vs the multithreaded oracle op by op (StringEditDistance.py:133-334), not a sample."""
    A, B = _ragged(5800, 5600, 1000, 1500, 1000, 1500)
    la = np.array([len(x) for x in A], np.float64)
    lb = np.array([len(x) for x in B], np.float64)
    assert (la * lb).sum() >= 512 * (la + lb).sum()  # the automatic checkpoint rule (sed_runtime.cpp: b->ck)
    plan = _plan(tables[True])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs(A, B)
    b, (d, ii, ln, ops) = _batch_run(gpu, packed, True, runs=2)
    try:
        assert b.mode == "i32" and b.rows_per_lane == 16 and b.traceback_mode == 2
        assert b.dp_launches == 2 and b.dot_keys and b.chains == 0 and b.lane_pairs == 0
    finally:
        b.close()
    _check_all(plan, packed, d, ii, ln, ops)

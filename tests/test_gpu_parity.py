"""GPU parity: libsed.so (HIP, gfx950) against the golden fixtures generated
from the reference and against the C oracle on seeded inputs.

Bar: bit-exact — fp64 distance bits, Python int/float typing, script length
and every op of the canonical edit script.
"""
import hashlib
import json

import numpy as np
import pytest

from conftest import load_golden
import oracle
import sedcost
import sedgpu
import synth

pytestmark = pytest.mark.gpu
OPCH = "idu"
IUPAC = "AGCUYRWSKMDVHBN"


def gpu_run(ctx, table, pairs, mode=0, R=0, script=True, split=0, lane=0, no_len=False, chain=0, pack=0, tb=0,
            bitpar=0, scaled=0):
    """Run (s1, s2) pairs through the engine; returns [(dist, is_int, len, opstr)]."""
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    ctx.set_mode(mode)
    ctx.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, R)
    ctx.set_option(sedgpu.SED_OPT_SPLIT, split)
    ctx.set_option(sedgpu.SED_OPT_LANE, lane)
    ctx.set_option(sedgpu.SED_OPT_CHAIN, chain)
    ctx.set_option(sedgpu.SED_OPT_PACK, pack)
    ctx.set_option(sedgpu.SED_OPT_TB, tb)
    ctx.set_option(sedgpu.SED_OPT_BITPAR, bitpar)
    ctx.set_option(sedgpu.SED_OPT_SCALED, scaled)
    ctx.set_costs(plan)
    packed = sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(b) for _, b in pairs])
    dist, is_int, ln, ops = ctx.run(packed, script, no_len=no_len)
    out = []
    for p in range(len(pairs)):
        s = None
        if script:
            s = "".join(OPCH[c] for c in sedgpu.unpack_ops(ops, packed.ops_off, p, int(ln[p])))
        out.append((float(dist[p]), bool(is_int[p]), int(ln[p]), s))
    ctx.set_mode(0)
    ctx.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
    ctx.set_option(sedgpu.SED_OPT_SPLIT, 0)
    ctx.set_option(sedgpu.SED_OPT_LANE, 0)
    ctx.set_option(sedgpu.SED_OPT_CHAIN, 0)
    ctx.set_option(sedgpu.SED_OPT_PACK, 0)
    ctx.set_option(sedgpu.SED_OPT_TB, 0)
    ctx.set_option(sedgpu.SED_OPT_BITPAR, 0)
    ctx.set_option(sedgpu.SED_OPT_SCALED, 0)
    return out


def test_selftest(gpu):
    assert gpu.selftest() == 0


@pytest.mark.parametrize("mode", [0, 2, 3])
def test_g1_small_all_modes(gpu, tables, mode):
    g1 = load_golden("g1_small.json")
    for user in (False, True):
        for alpha in ("acgu", "iupac"):
            recs = [r for r in g1 if r["user"] == user and
                    (set(r["s1"] + r["s2"]) <= set("ACGU")) == (alpha == "acgu")]
            got = gpu_run(gpu, tables[user], [(r["s1"], r["s2"]) for r in recs], mode=mode)
            for r, (d, ii, ln, s) in zip(recs, got):
                assert (float.fromhex(r["dist"][0]), r["dist"][1]) == (d, ii), (r["s1"], r["s2"], user)
                assert s == r["canon"], (r["s1"], r["s2"], user, s, r["canon"])
                assert ln == len(r["canon"])


def test_g2_medium(gpu, tables):
    for r in load_golden("g2_medium.json"):
        for mode in (0, 2):
            (d, ii, ln, s), = gpu_run(gpu, tables[r["user"]], [(r["s1"], r["s2"])], mode=mode)
            assert (d, ii) == (float.fromhex(r["dist"][0]), r["dist"][1])
            assert ln == r["len"] and s == r["canon"], (r["kind"], len(r["s1"]), mode)


def test_g3_config2_pair(gpu, tables):
    g3 = load_golden("g3_config2.json")
    s1, s2 = synth.pair_strings(g3["pair_id"], g3["n"], g3["m"], g3["base_seed"])
    assert hashlib.sha256(s1.encode()).hexdigest() == g3["s1_sha256"]
    for R, split in ((0, 0), (4, 2), (8, 2), (16, 2), (32, 2), (4, 1), (8, 1), (16, 1)):
        (d, ii, ln, s), = gpu_run(gpu, tables[True], [(s1, s2)], R=R, split=split)
        assert d == float.fromhex(g3["dist"][0]) and not ii
        assert ln == g3["len"] and s == g3["canon"], (R, split)


@pytest.mark.parametrize("R", [4, 8, 16])
def test_split_mode_vs_oracle(gpu, tables, R):
    """One wave per stripe with inter-workgroup hand-offs (forced on), ragged pairs."""
    pairs = _random_pairs(100 + R, 24, "ACGU", 0, 1500, related=True)
    _oracle_check(tables[True], pairs, gpu_run(gpu, tables[True], pairs, R=R, split=1))


def _random_pairs(seed, count, alphabet, lo, hi, related=False):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(count):
        n, m = rng.integers(lo, hi + 1, size=2)
        a = "".join(rng.choice(list(alphabet), size=n))
        if related:
            b = "".join(c if rng.random() > 0.1 else rng.choice(list(alphabet)) for c in a)
        else:
            b = "".join(rng.choice(list(alphabet), size=m))
        out.append((a, b))
    return out


def _oracle_check(table, pairs, got, no_len=False):
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    cs = oracle.Costs.from_plan(plan)
    for (a, b), (d, ii, ln, s) in zip(pairs, got):
        o = oracle.pair(cs, plan.encode(a), plan.encode(b))
        assert (d, ii) == (o["dist"], bool(o["is_int"])), (len(a), len(b))
        if no_len:  # lane kernels skip the length; the wave kernels may still report it
            assert ln in (-1, o["len"]), (len(a), len(b))
        else:
            assert ln == o["len"], (len(a), len(b))
        if s is not None:
            assert s == oracle.ops_to_str(o["ops"]), (len(a), len(b))


@pytest.mark.parametrize("user", [False, True])
@pytest.mark.parametrize("related", [False, True])
def test_random_ragged_acgu_vs_oracle(gpu, tables, user, related):
    pairs = _random_pairs(7 + user + 2 * related, 96, "ACGU", 0, 700, related)
    for R in (0, 4, 16):
        _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, R=R))


@pytest.mark.parametrize("user", [False, True])
def test_random_iupac_fp64_vs_oracle(gpu, tables, user):
    pairs = _random_pairs(11 + user, 64, IUPAC, 1, 520, related=True)
    for mode in (0, 3):
        _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, mode=mode))


def test_edge_lengths(gpu, tables):
    pairs = [("", ""), ("", "A"), ("A", ""), ("ACGU", ""), ("", "GGGG"), ("A", "A"), ("A", "C")]
    pairs += [("A" * n, "C" * m) for n in (1, 63, 64, 65, 255, 256, 257) for m in (1, 2, 61, 62, 63, 64, 65, 127)]
    for user in (False, True):
        for mode in (0, 2):
            _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, mode=mode))


def test_zero_copy_results_match_download(gpu, tables):
    """Small batches (the per-call path) have their kernels write results and scripts straight into pinned host
    memory (SED_OPT_ZEROCOPY); every small-batch route gives the same answer as with the download: integer lane and
    wave pairs, fp64 SPLIT, the window traceback (65..256 pairs), distance-only and scripts, empty sides.  The
    stripe-parallel walk (<= 64 pairs, atomicOr on the script words) keeps the download."""
    rng = np.random.default_rng(9500)
    acgu = [("".join(rng.choice(list("ACGU"), size=int(rng.integers(1, 40)))),
             "".join(rng.choice(list("ACGU"), size=int(rng.integers(1, 40))))) for _ in range(80)]
    acgu += [("ACGU" * 80, "AGU" * 90), ("", "ACG"), ("GGA", ""), ("", "")]
    iupac = _random_pairs(9600, 70, IUPAC, 1, 300, related=True) + [("", "ACG"), ("GUA" * 50, "")]
    for table, pairs in ((tables[True], acgu), (tables[False], acgu[:5]), (tables[False], iupac), (tables[False], iupac[:3])):
        for flags in (dict(script=True), dict(script=False), dict(script=False, no_len=True)):
            got = gpu_run(gpu, table, pairs, **flags)
            gpu.set_option(sedgpu.SED_OPT_ZEROCOPY, 2)
            try:
                assert gpu_run(gpu, table, pairs, **flags) == got, (len(pairs), flags)
            finally:
                gpu.set_option(sedgpu.SED_OPT_ZEROCOPY, 0)
            _oracle_check(table, pairs, got, no_len=flags.get("no_len", False))
    # one pair per call through sed_run_pair, repeated (the batch's pinned block is reused)
    plan = sedcost.build_plan(tables[False], [a for a, _ in iupac], [b for _, b in iupac])
    gpu.set_costs(plan)
    cs = oracle.Costs.from_plan(plan)
    for a, y in iupac[:20]:
        d, ii, ln, ops = gpu.run_pair(plan.encode_bytes(a), plan.encode_bytes(y), True)
        o = oracle.pair(cs, plan.encode(a), plan.encode(y))
        assert (d, bool(ii), ln) == (o["dist"], bool(o["is_int"]), o["len"])
        assert "".join(OPCH[c] for c in sedgpu.unpack_ops(ops, np.zeros(1, np.int64), 0, ln)) == oracle.ops_to_str(o["ops"])


def test_full_matrix_g1(gpu, tables):
    for r in load_golden("g1_small.json")[::3]:
        plan = sedcost.build_plan(tables[r["user"]], [r["s1"]], [r["s2"]])
        gpu.set_costs(plan)
        D, M = gpu.full_matrix(plan.encode(r["s1"]), plan.encode(r["s2"]))
        want = [[float.fromhex(h), bool(ii), mk] for h, ii, mk in r["cells"]]
        have = [[float(d), bool(mm >> 3), int(mm & 7)] for d, mm in zip(D.ravel(), M.ravel())]
        assert want == have, (r["s1"], r["s2"])


@pytest.mark.parametrize("user", [False, True])
def test_lane_kernel_short_str2_vs_oracle(gpu, tables, user):
    """Lane-per-pair kernel (m <= 32, n <= 512) mixed in one batch with wave-kernel pairs
    (m > 32 or n > 512): scripts, distance + length, distance only (SED_NO_LEN)."""
    rng = np.random.default_rng(31 + user)
    pairs = []
    for _ in range(300):
        n = int(rng.choice([rng.integers(1, 40), rng.integers(1, 513), rng.integers(500, 700)]))
        m = int(rng.choice([rng.integers(1, 33), 32, 33, rng.integers(20, 80)]))
        a = "".join(rng.choice(list("ACGU"), size=n))
        b = "".join(rng.choice(list("ACGU"), size=m)) if rng.random() < 0.5 else \
            "".join(c if rng.random() > 0.1 else rng.choice(list("ACGU")) for c in a[:m])
        pairs.append((a, b or "A"))
    pairs += [("A", "C"), ("ACGU" * 128, "ACGU" * 8), ("G" * 512, "G" * 32), ("G" * 513, "G" * 32)]
    _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs))
    _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, script=False))
    _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, script=False, no_len=True), no_len=True)
    # the same batch with the lane kernel disabled (every pair on the wave kernel)
    _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, lane=2))
    _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, script=False, no_len=True, lane=2),
                  no_len=True)


def test_lane_kernel_all_vs_all_shape(gpu, tables):
    """Config-5 shape: every pair on the lane kernel (piRNA-like lengths 24..32)."""
    rng = np.random.default_rng(5)
    seqs = ["".join(rng.choice(list("ACGU"), size=int(rng.integers(24, 33)))) for _ in range(40)]
    pairs = [(a, b) for a in seqs for b in seqs]
    _oracle_check(tables[False], pairs, gpu_run(gpu, tables[False], pairs, script=False, no_len=True), no_len=True)
    _oracle_check(tables[False], pairs[::7], gpu_run(gpu, tables[False], pairs[::7]))


@pytest.mark.parametrize("alphabet", ["ACGUN", "AGCUYRWSKMDVHBN"])
def test_lane_f64_distance_vs_oracle(gpu, tables, alphabet):
    """fp64 lane-per-pair kernel (distance only, SED_NO_LEN) on short IUPAC / N pairs, mixed
    with wave-kernel pairs; the same batch with the lane route disabled."""
    rng = np.random.default_rng(77 + len(alphabet))
    pairs = []
    for _ in range(400):
        n = int(rng.choice([rng.integers(1, 40), rng.integers(1, 513), rng.integers(500, 600)]))
        m = int(rng.choice([rng.integers(1, 33), 32, 33, rng.integers(20, 70)]))
        pairs.append(("".join(rng.choice(list(alphabet), size=n)), "".join(rng.choice(list(alphabet), size=m))))
    pairs += [("N", "N"), ("A", "N"), ("N" * 30, "A" * 32), ("ACGU" * 128, "N" * 32)]
    for user in (False, True):
        got = gpu_run(gpu, tables[user], pairs, script=False, no_len=True)
        _oracle_check(tables[user], pairs, got, no_len=True)
        assert sum(1 for g in got if g[2] == -1) > 100  # the lane route ran
        _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, script=False, no_len=True, lane=2),
                      no_len=True)


@pytest.mark.parametrize("R", [4, 8])
def test_chain_mode_vs_oracle(gpu, tables, R):
    """CHAIN mode (forced): single-stripe pairs back to back in one wave, lanes switching pairs
    one step apart; ragged m (1..700, including 63/64/65 and multiples of 64), n up to 64R,
    scripts / lengths / distance only, both tables; lane route off so short m chains too."""
    rng = np.random.default_rng(500 + R)
    rows = 64 * R
    pairs = []
    for _ in range(120):
        n = int(rng.choice([rng.integers(1, rows + 1), rows, 1]))
        m = int(rng.choice([rng.integers(1, 701), 63, 64, 65, 128, 1, 2, 33]))
        a = "".join(rng.choice(list("ACGU"), size=n))
        if rng.random() < 0.5:
            b = "".join(c if rng.random() > 0.1 else rng.choice(list("ACGU")) for c in (a * 3)[:m])
        else:
            b = "".join(rng.choice(list("ACGU"), size=m))
        pairs.append((a, b))
    for user in (False, True):
        _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, R=R, chain=1, lane=2))
        _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, R=R, chain=1, lane=2, script=False))
        _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, R=R, chain=1, lane=2, script=False,
                                                   no_len=True), no_len=True)
    # long chains (7 ragged pairs each: many switch windows per wave)
    _oracle_check(tables[True], pairs, gpu_run(gpu, tables[True], pairs, R=R, chain=7, lane=2))
    _oracle_check(tables[False], pairs, gpu_run(gpu, tables[False], pairs, R=R, chain=7, lane=2, script=False))
    # mixed with lane-kernel pairs, default routing otherwise
    _oracle_check(tables[True], pairs, gpu_run(gpu, tables[True], pairs, R=R, chain=1))


def test_chain_mode_is_used(gpu, tables):
    plan = sedcost.build_plan(tables[False], ["ACGU"], ["ACGU"])
    gpu.set_costs(plan)
    A = synth.pair_codes(np.arange(64, dtype=np.uint64), 512, 0)
    B = synth.pair_codes(np.arange(64, dtype=np.uint64), 512, 1)
    gpu.set_option(sedgpu.SED_OPT_CHAIN, 1)
    try:
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs.from_arrays(A, B), True)
        assert b.chains == 64 and b.rows_per_lane == 8  # dynamic: one persistent wave per pair here
        b.run()
        d, ii, ln, ops = b.results()
        b.close()
    finally:
        gpu.set_option(sedgpu.SED_OPT_CHAIN, 0)
    cs = oracle.Costs.from_plan(plan)
    packed = sedgpu.PackedPairs.from_arrays(A, B)
    for p in range(0, 64, 7):
        o = oracle.pair(cs, A[p], B[p])
        assert (d[p], ln[p]) == (o["dist"], o["len"])
        assert np.array_equal(sedgpu.unpack_ops(ops, packed.ops_off, p, int(ln[p])), o["ops"])


def test_script_batches_are_chunked_by_traceback_budget(gpu, tables, monkeypatch):
    """sed_run_batch cuts a script batch into several launches when its traceback workspace
    exceeds SED_TB_BUDGET_GB; results are unchanged (here ~45 chunks of ~1 MB)."""
    pairs = _random_pairs(909, 90, "ACGU", 0, 900, related=True)
    monkeypatch.setenv("SED_TB_BUDGET_GB", "0.001")
    got = gpu_run(gpu, tables[True], pairs)
    monkeypatch.delenv("SED_TB_BUDGET_GB")
    _oracle_check(tables[True], pairs, got)


def test_large_pairs_across_the_integer_key_limits(gpu, tables):
    """Near the packed-key limits (L < 2^14, D < 2^16 - 256 for the padded problem): a 12000 x 4000
    pair still runs the integer kernel, a 9000 x 9000 pair falls back to fp64; both bit-exact."""
    rng = np.random.default_rng(1234)
    a1 = "".join(rng.choice(list("ACGU"), size=12000))
    b1 = "".join(c if rng.random() > 0.15 else rng.choice(list("ACGU")) for c in a1[:4000])
    a2 = "".join(rng.choice(list("ACGU"), size=9000))
    b2 = "".join(c if rng.random() > 0.15 else rng.choice(list("ACGU")) for c in a2)
    for pairs in ([(a1, b1)], [(a2, b2)]):
        plan = sedcost.build_plan(tables[True], [p[0] for p in pairs], [p[1] for p in pairs])
        gpu.set_costs(plan)
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(x) for x, _ in pairs],
                                                 [plan.encode(y) for _, y in pairs]), True)
        assert b.mode == ("i32" if len(pairs[0][0]) == 12000 else "f64")
        b.close()
        _oracle_check(tables[True], pairs, gpu_run(gpu, tables[True], pairs))


@pytest.mark.parametrize("user", [False, True])
def test_lane_x2_packed_distance_vs_oracle(gpu, tables, user):
    """Distance-only lane pairs run two per lane in 16-bit halves (pairs of equal n; a pair without
    a partner shares its lane with itself).  Same results as one pair per lane and as the oracle."""
    rng = np.random.default_rng(404 + user)
    pairs = []
    for _ in range(500):
        n = int(rng.choice([rng.integers(1, 8), rng.integers(20, 33), rng.integers(1, 513)]))
        m = int(rng.integers(1, 33))
        pairs.append(("".join(rng.choice(list("ACGU"), size=n)), "".join(rng.choice(list("ACGU"), size=m))))
    pairs += [("A", "A"), ("G" * 512, "C" * 32), ("ACGU" * 128, "U"), ("C" * 511, "A" * 32)]
    plan = sedcost.build_plan(tables[user], [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    gpu.set_option(sedgpu.SED_OPT_BITPAR, 2)  # (costs.json's unit costs would take the bit-parallel kernel)
    try:
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                                 [plan.encode(y) for _, y in pairs]), False, no_len=True)
        assert b.lane_pairs == len(pairs) and b.packed_pairs == len(pairs) and b.bitpar_pairs == 0
        b.close()
    finally:
        gpu.set_option(sedgpu.SED_OPT_BITPAR, 0)
    got = gpu_run(gpu, tables[user], pairs, script=False, no_len=True, bitpar=2)
    _oracle_check(tables[user], pairs, got, no_len=True)
    assert got == gpu_run(gpu, tables[user], pairs, script=False, no_len=True, pack=2, bitpar=2)


def _unit_table():
    """costs.json's ACGU block as its own table: insert = delete = 1, every mismatch 1 (unit costs)."""
    sub = {a: {b: 1.0 for b in "ACGU"} for a in "ACGU"}
    return {"insert": 1.0, "delete": 1.0, "update": sub}


@pytest.mark.parametrize("seed", [0, 1])
def test_lane_bitpar_unit_costs_vs_oracle(gpu, tables, seed):
    """Unit costs (costs.json on ACGU), distance only: lane pairs (m <= 32, n <= 512) run one per lane
    bit-parallel, mixed with wave-kernel pairs (m > 32 or n > 512).  Every ragged shape against the oracle,
    and against the 16-bit packed lane kernel and the one-pair-per-lane DP kernel (SED_OPT_BITPAR = 2)."""
    rng = np.random.default_rng(8080 + seed)
    pairs = []
    for _ in range(1500):
        n = int(rng.choice([rng.integers(1, 17), rng.integers(15, 34), rng.integers(1, 513), rng.integers(500, 560)]))
        m = int(rng.choice([rng.integers(1, 33), 32, 31, 1, 16, 17, 33, rng.integers(20, 60)]))
        a = "".join(rng.choice(list("ACGU"), size=n))
        if rng.random() < 0.4:  # related: long diagonals and ties
            b = "".join(c if rng.random() > 0.1 else rng.choice(list("ACGU")) for c in (a * 40)[:m])
        else:
            b = "".join(rng.choice(list("ACGU"), size=m))
        pairs.append((a, b))
    pairs += [("A", "A"), ("A", "C"), ("G" * 512, "G" * 32), ("G" * 512, "C" * 32), ("ACGU" * 128, "U"),
              ("U", "ACGU" * 8), ("C" * 511, "A" * 32), ("ACGU" * 8, "ACGU" * 8), ("A" * 513, "A" * 32)]
    for table in (tables[False], _unit_table()):
        plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
        gpu.set_costs(plan)
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                                 [plan.encode(y) for _, y in pairs]), False, no_len=True)
        lanes = b.lane_pairs
        assert lanes > 800 and b.bitpar_pairs == lanes and b.packed_pairs < len(pairs) - lanes  # (wave pairs pack)
        b.close()
        got = gpu_run(gpu, table, pairs, script=False, no_len=True)
        _oracle_check(table, pairs, got, no_len=True)
        assert got == gpu_run(gpu, table, pairs, script=False, no_len=True, bitpar=2)
        assert got == gpu_run(gpu, table, pairs, script=False, no_len=True, bitpar=2, pack=2)


@pytest.mark.parametrize("alphabet,pn", [("ACGUN", 0.01), ("ACGUN", 0.2), ("AGCUYRWSKMDVHBN", 0.0)])
def test_lane_f64_unit_subset_bitpar_vs_oracle(gpu, tables, alphabet, pn):
    """fp64 distance-only batches (costs.json with N or IUPAC codes; config 5 with N): lane pairs whose symbols all
    lie in a unit-cost subset of the table run bit-parallel inside the fp64 lane kernel, the others the fp64 DP.
    Against the oracle and against SED_OPT_BITPAR = 2; the counts show both routes ran."""
    rng = np.random.default_rng(6060 + int(100 * pn) + len(alphabet))
    base = list(alphabet[:4]) if alphabet == "ACGUN" else list(alphabet)

    def seq(k):
        return "".join("N" if rng.random() < pn else rng.choice(base) for _ in range(k))
    seqs = [seq(int(rng.integers(1, 33))) for _ in range(70)]
    pairs = [(a, b) for a in seqs for b in seqs[:40]]
    pairs += [(seq(int(rng.integers(1, 513))), seq(int(rng.integers(1, 33)))) for _ in range(200)]
    pairs += [(seq(40), seq(40)) for _ in range(20)]  # wave-kernel pairs (m > 32)
    table = tables[False]
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                             [plan.encode(y) for _, y in pairs]), False, no_len=True)
    assert b.mode == "f64"
    nbp, lanes = b.bitpar_pairs, b.lane_pairs
    b.close()
    if alphabet == "ACGUN":
        assert 0 < nbp < lanes or (pn == 0.2 and nbp > 0)
    got = gpu_run(gpu, table, pairs, script=False, no_len=True)
    _oracle_check(table, pairs, got, no_len=True)
    assert got == gpu_run(gpu, table, pairs, script=False, no_len=True, bitpar=2)


def _dyadic_tables(tables):
    """(name, table, alphabet, scaled expected) for the scaled-integer lane route."""
    out = [("costs.json ACGUN", tables[False], "ACGUN", True), ("user_costs ACGUN", tables[True], "ACGUN", True)]
    # 8 symbols, eighths, insert != delete
    al = "ACGUNRYS"
    t = {"insert": 0.625, "delete": 1.25, "update": {}}
    rng = np.random.default_rng(77)
    for a in al:
        t["update"][a] = {b: (0.0 if a == b else float(rng.integers(1, 15)) / 8.0) for b in al}
    out.append(("eighths 8 symbols", t, al, True))
    # N at 0.66 (costs.json's IUPAC values are not dyadic): the fp64 lane kernel
    t2 = json.loads(json.dumps(tables[False]))
    for a in "ACGU":
        t2["update"][a]["N"] = 0.66
    out.append(("N at 0.66", t2, "ACGUN", False))
    # a substitution dearer than insert + delete: the offset keys' update byte cannot hold it
    t3 = json.loads(json.dumps(tables[False]))
    t3["update"]["A"]["N"] = 2.5
    out.append(("A->N 2.5", t3, "ACGUN", False))
    # 9 symbols of the same kind: beyond the 8-byte column table
    al9 = al + "K"
    t4 = {"insert": 0.625, "delete": 1.25, "update": {}}
    for a in al9:
        t4["update"][a] = {b: (0.0 if a == b else float(rng.integers(1, 15)) / 8.0) for b in al9}
    out.append(("9 symbols", t4, al9, False))
    return out


@pytest.mark.parametrize("pn", [0.01, 0.2])
def test_lane_scaled_dyadic_vs_oracle(gpu, tables, pn):
    """fp64 distance-only lane pairs under dyadic costs over <= 8 symbols (config 5 with N: costs.json's ACGUN block is
    1.0 but 0.75 for N) run an exact integer DP of the costs scaled by 2^k (sed_lane_scaled_kernel).  Against the
    oracle, against the fp64 lane kernel (SED_OPT_SCALED = 2) and without the bit-parallel pairs (SED_OPT_BITPAR = 2);
    non-dyadic tables, a cost above insert + delete and 9 symbols keep the fp64 lane kernel."""
    for name, table, al, want in _dyadic_tables(tables):
        rng = np.random.default_rng(7070 + int(100 * pn) + len(name))
        base = list(al[:4]) if al.startswith("ACGUN") and len(al) == 5 else list(al)

        def seq(k):
            return "".join("N" if rng.random() < pn else rng.choice(base) for _ in range(k))
        seqs = [seq(int(rng.integers(1, 33))) for _ in range(60)]
        pairs = [(a, b) for a in seqs for b in seqs[:30]]
        pairs += [(seq(int(rng.integers(1, 513))), seq(int(rng.integers(1, 33)))) for _ in range(150)]
        pairs += [(seq(40), seq(40)) for _ in range(10)]  # wave-kernel pairs (m > 32)
        plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
        gpu.set_costs(plan)
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                                 [plan.encode(y) for _, y in pairs]), False, no_len=True)
        try:
            assert b.mode == "f64", name
            assert (b.scaled_pairs > 0) == want, (name, b.scaled_pairs)
            if want:
                assert b.scaled_pairs + b.bitpar_pairs == b.lane_pairs, name
        finally:
            b.close()
        got = gpu_run(gpu, table, pairs, script=False, no_len=True)
        _oracle_check(table, pairs, got, no_len=True)
        assert got == gpu_run(gpu, table, pairs, script=False, no_len=True, scaled=2), name
        assert got == gpu_run(gpu, table, pairs, script=False, no_len=True, bitpar=2), name


def test_lane_bitpar_needs_unit_costs(gpu, tables):
    """user_costs (insert 2, delete 3), a unit table with one mismatch of cost 2, and script / length batches keep
    the DP lane kernels."""
    pairs = _random_pairs(99, 64, "ACGU", 1, 32)
    off = _unit_table()
    off["update"]["A"]["C"] = 2.0
    for table, flags in ((tables[True], dict(script=False, no_len=True)), (off, dict(script=False, no_len=True)),
                         (tables[False], dict(script=False)), (tables[False], dict(script=True))):
        plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
        gpu.set_costs(plan)
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                                 [plan.encode(y) for _, y in pairs]), flags["script"],
                         no_len=flags.get("no_len", False))
        assert b.lane_pairs == len(pairs) and b.bitpar_pairs == 0
        b.close()
        _oracle_check(table, pairs, gpu_run(gpu, table, pairs, **flags), no_len=flags.get("no_len", False))


@pytest.mark.parametrize("R", [0, 4, 8, 16])
def test_wave_x2_packed_distance_vs_oracle(gpu, tables, R):
    """Distance-only wave pairs of equal n run two per wave in 16-bit halves (m within 4x; the wave
    runs the larger m); pairs without a partner, lane pairs and empty pairs in the same batch take
    their usual kernels."""
    rng = np.random.default_rng(808 + R)
    shapes = [(40, 100), (300, 257), (700, 64), (1100, 90), (1, 40), (64, 33), (300, 70), (300, 1000),
              (700, 300), (1100, 400), (1100, 95)]
    pairs = []
    for n, m in shapes:
        for _ in range(int(rng.integers(2, 6))):
            a = "".join(rng.choice(list("ACGU"), size=n))
            b = "".join(rng.choice(list("ACGU"), size=m)) if rng.random() < 0.5 else \
                "".join(c if rng.random() > 0.1 else rng.choice(list("ACGU")) for c in (a * 2)[:m])
            pairs.append((a, b))
    pairs += [("ACGU" * 10, "A" * 20), ("A" * 77, "C" * 91), ("", "ACG"), ("GG", "")]  # lane, single, empties
    order = rng.permutation(len(pairs))
    pairs = [pairs[i] for i in order]
    user = bool(R & 8)
    plan = sedcost.build_plan(tables[user], [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, R)
    gpu.set_option(sedgpu.SED_OPT_SPLIT, 2)  # a batch this small would otherwise run SPLIT (never packed)
    b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                             [plan.encode(y) for _, y in pairs]), False, no_len=True)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
    gpu.set_option(sedgpu.SED_OPT_SPLIT, 0)
    assert b.packed_pairs >= 12
    b.close()
    got = gpu_run(gpu, tables[user], pairs, R=R, split=2, script=False, no_len=True)
    _oracle_check(tables[user], pairs, got, no_len=True)
    assert got == gpu_run(gpu, tables[user], pairs, R=R, split=2, script=False, no_len=True, pack=2)


def _int_table(ins, dele, sub):
    """An integer cost table over ACGU in the reference's format (sub(a, b) for a != b)."""
    return {"insert": float(ins), "delete": float(dele),
            "update": {a: {b: (0.0 if a == b else float(sub(a, b))) for b in "ACGU"} for a in "ACGU"}}


@pytest.mark.parametrize("case", ["sum", "over", "wide", "tight"])
def test_offset_key_eligibility_edges(gpu, case):
    """The offset-key kernels need cost <= insert + delete <= 255 (sed_runtime.cpp: i32_eligible) and the
    16-bit packed distance keys cost < insert + delete.  At the edges: substitutions costing exactly
    insert + delete stay on the integer kernel (packing off), costlier ones or insert + delete > 255 fall
    back to fp64; every route bit-exact against the oracle (script, length, distance-only packed/unpacked)."""
    rng = np.random.default_rng(77)
    tabs = {
        "sum": (_int_table(1, 2, lambda a, b: 3), "i32"),
        "over": (_int_table(1, 1, lambda a, b: 3 if (a, b) == ("A", "C") else 1), "f64"),
        "wide": (_int_table(200, 100, lambda a, b: 7), "f64"),
        "tight": (_int_table(2, 5, lambda a, b: int(rng.integers(1, 8))), "i32"),
    }
    table, mode = tabs[case]
    pairs = _random_pairs(500 + len(case), 64, "ACGU", 0, 300, related=True)
    pairs += _random_pairs(600 + len(case), 64, "ACGU", 1, 40)
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(x) for x, _ in pairs],
                                             [plan.encode(y) for _, y in pairs]), True)
    assert b.mode == mode
    b.close()
    _oracle_check(table, pairs, gpu_run(gpu, table, pairs))
    _oracle_check(table, pairs, gpu_run(gpu, table, pairs, script=False))
    for pack in (0, 2):
        _oracle_check(table, pairs, gpu_run(gpu, table, pairs, script=False, no_len=True, pack=pack), no_len=True)


def test_ladder_rows_and_long_paths(gpu, tables):
    """Ladder keys (sed_kernels.hip): every rung of the 16-row ladder at the sink (n = 1..48), stripes of
    R = 4/8/16, and script lengths past 8192 (L read modulo 8192 inside [max(n,m), n+m])."""
    rng = np.random.default_rng(4242)
    pairs = [("".join(rng.choice(list("ACGU"), size=n)), "".join(rng.choice(list("ACGU"), size=int(m))))
             for n in range(1, 49) for m in rng.integers(33, 90, size=2)]
    for R in (4, 8, 16):
        for user in (False, True):
            _oracle_check(tables[user], pairs, gpu_run(gpu, tables[user], pairs, R=R))
    a = "".join(rng.choice(list("ACGU"), size=9000))
    b = "".join(rng.choice(list("ACGU"), size=300))  # L >= max(n, m) = 9000 > 8192
    got = gpu_run(gpu, tables[True], [(a, b)])
    assert got[0][2] > 8192
    _oracle_check(tables[True], [(a, b)], got)


@pytest.mark.parametrize("user", [False, True])
def test_checkpoint_traceback_vs_oracle(gpu, tables, user):
    """CK traceback (SED_OPT_TB = 2): the R = 16 kernel stores column / row checkpoints instead of per-cell
    codes and the traceback recomputes 64-row tiles.  Ragged multi-stripe batches (lengths 1..2600, related
    and unrelated, border lengths around tiles, chunks and stripes) give the oracle's scripts, and the same
    as the per-cell codes (SED_OPT_TB = 1)."""
    pairs = _random_pairs(900 + user, 24, "ACGU", 1, 2600, related=True)
    pairs += _random_pairs(910 + user, 16, "ACGU", 1, 1500)
    rng = np.random.default_rng(920 + user)
    for n, m in ((64, 64), (65, 63), (1024, 64), (1025, 129), (2048, 1), (1, 2048), (1088, 1090), (63, 4000)):
        a = "".join(rng.choice(list("ACGU"), size=n))
        pairs.append((a, "".join(c if rng.random() > 0.2 else rng.choice(list("ACGU")) for c in a)[:m].ljust(m, "G")))
    plan = sedcost.build_plan(tables[user], [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs([plan.encode(x) for x, _ in pairs], [plan.encode(y) for _, y in pairs])
    for tb, want in ((2, 2), (1, 1), (0, 1)):  # auto: codes below 257 pairs
        gpu.set_option(sedgpu.SED_OPT_TB, tb)
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 16)
        gpu.set_option(sedgpu.SED_OPT_SPLIT, 2)
        b = sedgpu.Batch(gpu, packed, True)
        assert b.traceback_mode == want
        b.close()
    gpu.set_option(sedgpu.SED_OPT_TB, 0)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
    gpu.set_option(sedgpu.SED_OPT_SPLIT, 0)
    got = gpu_run(gpu, tables[user], pairs, R=16, split=2, lane=2, tb=2)
    _oracle_check(tables[user], pairs, got)
    assert got == gpu_run(gpu, tables[user], pairs, R=16, split=2, lane=2, tb=1)


def test_checkpoint_traceback_config2_pair(gpu, tables):
    """The G3 pair (4096 x 4096, user_costs) through the CK traceback."""
    g3 = load_golden("g3_config2.json")
    s1, s2 = synth.pair_strings(g3["pair_id"], g3["n"], g3["m"], g3["base_seed"])
    (d, ii, ln, s), = gpu_run(gpu, tables[True], [(s1, s2)], R=16, split=2, tb=2)
    assert (d, ii) == (float.fromhex(g3["dist"][0]), g3["dist"][1])
    assert ln == len(g3["canon"]) and s == g3["canon"]


@pytest.mark.parametrize("mode", [0, 2, 3])
def test_g8_gui_cost_tables_small(gpu, mode):
    """G8 (reference-generated): cost tables the GUI can write, in every kernel mode; the auto mode
    routes the integer table to the packed kernel and the rest to fp64 / fp64-typed."""
    g8 = load_golden("g8_cost_tables.json")
    for name, table in g8["tables"].items():
        recs = [r for r in g8["small"] if r["table"] == name]
        if mode == 0 and name == "gui_int":
            acgu = [(r["s1"], r["s2"]) for r in recs if set(r["s1"] + r["s2"]) <= set("ACGU")]
            plan = sedcost.build_plan(table, [a for a, _ in acgu], [b for _, b in acgu])
            gpu.set_costs(plan)
            b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in acgu],
                                                     [plan.encode(y) for _, y in acgu]), True)
            assert b.mode == "i32"
            b.close()
        got = gpu_run(gpu, table, [(r["s1"], r["s2"]) for r in recs], mode=mode)
        for r, (d, ii, ln, s) in zip(recs, got):
            assert (d, ii) == (float.fromhex(r["dist"][0]), r["dist"][1]), (name, r["s1"], r["s2"], mode)
            assert s == r["canon"] and ln == len(r["canon"]), (name, r["s1"], r["s2"], mode)


def test_g8_gui_cost_tables_full_matrix(gpu):
    g8 = load_golden("g8_cost_tables.json")
    for r in g8["small"][::2]:
        table = g8["tables"][r["table"]]
        plan = sedcost.build_plan(table, [r["s1"]], [r["s2"]])
        gpu.set_costs(plan)
        D, M = gpu.full_matrix(plan.encode(r["s1"]), plan.encode(r["s2"]))
        want = [[float.fromhex(h), bool(ii), mk] for h, ii, mk in r["cells"]]
        have = [[float(d), bool(mm >> 3), int(mm & 7)] for d, mm in zip(D.ravel(), M.ravel())]
        assert want == have, (r["table"], r["s1"], r["s2"])


def test_g8_gui_cost_tables_medium(gpu):
    """G8 medium pairs (256..1024): distance bits, typing, length and canonical script in auto mode, forced
    fp64-typed mode, and (integer table) at every R with per-cell codes and with checkpoints."""
    g8 = load_golden("g8_cost_tables.json")
    for r in g8["medium"]:
        table = g8["tables"][r["table"]]
        runs = [dict(mode=0), dict(mode=3)]
        if r["table"] == "gui_int" and set(r["s1"] + r["s2"]) <= set("ACGU"):
            runs += [dict(R=4, split=2), dict(R=8, split=2), dict(R=16, split=2, tb=1), dict(R=16, split=2, tb=2),
                     dict(split=1)]
        for kw in runs:
            (d, ii, ln, s), = gpu_run(gpu, table, [(r["s1"], r["s2"])], **kw)
            assert (d, ii) == (float.fromhex(r["dist"][0]), r["dist"][1]), (r["table"], r["kind"], kw)
            assert ln == r["len"] and s == r["canon"], (r["table"], r["kind"], kw)
        # distance only: the fp64 lane kernel / packed integer kernels where the table allows them
        (d, ii, ln, s), = gpu_run(gpu, table, [(r["s1"], r["s2"])], script=False, no_len=True)
        assert (d, ii) == (float.fromhex(r["dist"][0]), r["dist"][1]), (r["table"], r["kind"], "distance")


@pytest.mark.parametrize("name", ["frac_indel", "zero_sub", "sub_over", "int_literals", "gui_int",
                                  "zero_insert", "negative_sub"])
def test_g8_tables_random_batches_vs_oracle(gpu, name):
    """The G8 tables on ragged random batches (lane and wave pairs, ACGU and IUPAC) vs the oracle, which
    test_oracle_golden.py pins to the same tables; scripts, lengths and distance-only routes."""
    table = load_golden("g8_cost_tables.json")["tables"][name]
    pairs = _random_pairs(1300 + len(name), 80, "ACGU", 0, 600, related=True)
    pairs += _random_pairs(1400 + len(name), 80, IUPAC, 1, 300, related=True)
    pairs += _random_pairs(1500 + len(name), 120, "ACGUN", 1, 40)
    _oracle_check(table, pairs, gpu_run(gpu, table, pairs))
    _oracle_check(table, pairs, gpu_run(gpu, table, pairs, script=False))
    _oracle_check(table, pairs, gpu_run(gpu, table, pairs, script=False, no_len=True), no_len=True)
    _oracle_check(table, pairs, gpu_run(gpu, table, pairs, mode=3))


@pytest.mark.parametrize("R", [4, 8, 16])
@pytest.mark.parametrize("chain", [1, 2])
def test_checkpoint_route_every_R_stripe_and_chain(gpu, tables, R, chain):
    """Checkpoints (SED_OPT_TB = 2) at R = 4/8/16 rows per lane: tiles of 64/R bands of R rows.  Stripe kernel
    (chain off) on ragged multi-stripe pairs, CHAIN kernel (forced, static chains of 5 and dynamic; CHAIN runs
    at R = 4/8 only, R = 16 stays on the stripe kernel) on ragged single-stripe pairs, lane route off so short
    str2 chain too; scripts equal the oracle's and the per-cell codes'."""
    rng = np.random.default_rng(1700 + R + chain)
    rows = 64 * R
    pairs = []
    for _ in range(90):
        n = int(rng.choice([rng.integers(1, rows + 1), rows, 1]) if chain == 1 else rng.integers(1, 3 * rows + 70))
        m = int(rng.choice([rng.integers(1, 700), 63, 64, 65, 128, 1, 2, 33]))
        a = "".join(rng.choice(list("ACGU"), size=n))
        if rng.random() < 0.5:
            b = "".join(c if rng.random() > 0.12 else rng.choice(list("ACGU")) for c in (a * 3)[:m])
        else:
            b = "".join(rng.choice(list("ACGU"), size=m))
        pairs.append((a, b))
    for user in (False, True):
        for ch in ([1, 5] if chain == 1 else [2]):
            got = gpu_run(gpu, tables[user], pairs, R=R, split=2, lane=2, chain=ch, tb=2)
            _oracle_check(tables[user], pairs, got)
            assert got == gpu_run(gpu, tables[user], pairs, R=R, split=2, lane=2, chain=ch, tb=1)
    plan = sedcost.build_plan(tables[True], [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    gpu.set_option(sedgpu.SED_OPT_TB, 2)
    gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, R)
    gpu.set_option(sedgpu.SED_OPT_CHAIN, chain)
    gpu.set_option(sedgpu.SED_OPT_LANE, 2)
    gpu.set_option(sedgpu.SED_OPT_SPLIT, 2)  # a batch this small would otherwise run SPLIT (codes)
    try:
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(x) for x, _ in pairs], [plan.encode(y) for _, y in pairs]),
                         True)
        assert b.traceback_mode == 2 and b.rows_per_lane == R and (b.chains > 0) == (chain == 1 and R < 16)
        b.close()
    finally:
        for k in (sedgpu.SED_OPT_TB, sedgpu.SED_OPT_ROWS_PER_LANE, sedgpu.SED_OPT_CHAIN, sedgpu.SED_OPT_LANE,
                  sedgpu.SED_OPT_SPLIT):
            gpu.set_option(k, 0)


@pytest.mark.parametrize("table_name", ["costs.json", "int_literals", "frac_indel"])
def test_fp64_split_vs_oracle(gpu, tables, table_name):
    """fp64 SPLIT (sed_wf_f64_split_kernel): batches of <= 256 pairs run one 128-thread workgroup per stripe of 128
    rows (R = 2; 256 rows at SED_OPT_ROWS_PER_LANE = 4), the stripes handing their bottom rows down through tagged
    {D low, D high, L key | typing} words (timing.py's one-call loop at 300-500 nt, GUI calls over IUPAC symbols;
    timing.py:45-57, StringEditDistance.py:92-128).  Ragged IUPAC pairs of 257..1400 rows, one-stripe and empty sides, m past and
    below a chunk, scripts and distances, every pair against the oracle and identical to SED_OPT_SPLIT = 2 (lone
    waves); the forced route (SED_OPT_SPLIT = 1) on the same batch."""
    table = tables[False] if table_name == "costs.json" else load_golden("g8_cost_tables.json")["tables"][table_name]
    pairs = _random_pairs(9100 + len(table_name), 14, IUPAC, 257, 1400, related=True)
    pairs += _random_pairs(9200 + len(table_name), 6, IUPAC, 1, 700)
    rng = np.random.default_rng(9300)
    for n, m in ((257, 1), (1000, 5), (300, 64), (513, 65), (768, 700), (200, 900), (1, 1200)):
        pairs.append(("".join(rng.choice(list(IUPAC), size=n)), "".join(rng.choice(list(IUPAC), size=m))))
    pairs += [("", "ACG" * 100), ("GUA" * 100, ""), ("", "")]
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    for script in (True, False):
        for R in (2, 4):  # the default (R = 2: stripes of 128 rows) and SED_OPT_ROWS_PER_LANE = 4
            gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0 if R == 2 else R)
            b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                                     [plan.encode(y) for _, y in pairs]), script)
            try:
                assert b.mode in ("f64", "f64-typed") and b.rows_per_lane == R
                assert b.split_tasks == sum(-(-len(a) // (64 * R)) if a and y else 1 for a, y in pairs), b.split_tasks
            finally:
                b.close()
                gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
        got = gpu_run(gpu, table, pairs, script=script)
        _oracle_check(table, pairs, got)
        assert gpu_run(gpu, table, pairs, script=script, R=4) == got, (table_name, script)
        assert gpu_run(gpu, table, pairs, script=script, split=2) == got, (table_name, script)
        assert gpu_run(gpu, table, pairs, script=script, split=1) == got, (table_name, script)
    # the run repeated on one batch: the hand-off words of run k + 1 carry another epoch than run k's
    b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(y) for _, y in pairs]),
                     True)
    try:
        for _ in range(3):
            b.run()
            b.sync()
    finally:
        b.close()


def test_fp64_split_full_matrix(gpu, tables):
    """The dp proxy's full matrix (sed_full_matrix, fp64 at R = 4) of pairs past 256 rows runs SPLIT: every cell's
    value, typing and edge mask identical to the lone-wave kernel's (SED_OPT_SPLIT = 2), the sink to the oracle's."""
    rng = np.random.default_rng(9400)
    shapes = ((600, 450), (257, 300), (1000, 40), (300, 1))
    for user in (False, True):
        table = tables[user]
        for n, m in shapes:
            a = "".join(rng.choice(list(IUPAC), size=n))
            b = "".join(rng.choice(list(IUPAC), size=m))
            plan = sedcost.build_plan(table, [a], [b])
            gpu.set_costs(plan)
            D, M = gpu.full_matrix(plan.encode(a), plan.encode(b))
            gpu.set_option(sedgpu.SED_OPT_SPLIT, 2)
            try:
                D2, M2 = gpu.full_matrix(plan.encode(a), plan.encode(b))
            finally:
                gpu.set_option(sedgpu.SED_OPT_SPLIT, 0)
            assert np.array_equal(D.view(np.uint64), D2.view(np.uint64)) and np.array_equal(M, M2), (user, n, m)
            o = oracle.pair(oracle.Costs.from_plan(plan), plan.encode(a), plan.encode(b))
            assert (float(D[n, m]), bool(M[n, m] >> 3)) == (o["dist"], bool(o["is_int"])), (user, n, m)


def test_fp64_split_forced_over_segments_and_r2_fallback(gpu, tables):
    """An fp64 batch of > 256 wave pairs takes the 16-lane segments on the automatic route; SED_OPT_SPLIT = 1 forces
    the fp64 SPLIT route over them (no segment pairs), and rows per lane 2 outside SPLIT (SED_OPT_SPLIT = 2) falls back
    to the automatic R instead of failing.  Results identical on every route, the oracle's on a sample."""
    pairs = _random_pairs(9500, 290, IUPAC, 1, 300)
    pairs += _random_pairs(9501, 6, IUPAC, 257, 600, related=True)
    table = tables[False]
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    packed = sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(y) for _, y in pairs])
    try:
        b = sedgpu.Batch(gpu, packed, True)
        assert b.segment_pairs > 0 and b.split_tasks == 0
        b.close()
        gpu.set_option(sedgpu.SED_OPT_SPLIT, 1)
        b = sedgpu.Batch(gpu, packed, True)
        assert b.segment_pairs == 0 and b.split_tasks > 0 and b.rows_per_lane == 2
        b.close()
        gpu.set_option(sedgpu.SED_OPT_SPLIT, 2)
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 2)
        b = sedgpu.Batch(gpu, packed, True)
        assert b.split_tasks == 0 and b.rows_per_lane in (4, 8)
        b.close()
    finally:
        gpu.set_option(sedgpu.SED_OPT_SPLIT, 0)
        gpu.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 0)
    got = gpu_run(gpu, table, pairs)
    assert gpu_run(gpu, table, pairs, split=1) == got
    assert gpu_run(gpu, table, pairs, split=2, R=2) == got
    _oracle_check(table, pairs[::7] + pairs[-6:], got[::7] + got[-6:])


@pytest.mark.parametrize("script", [True, False])
def test_fp64_split_gate(gpu, tables, script):
    """The automatic fp64 SPLIT route of <= 256 pairs is gated on its cost model (sed_runtime.cpp: f64_split_pays):
    128 long narrow pairs (2000 x 100, 16 stripes each, whose chains hold the resident workgroups mostly waiting on the
    stripe lag) run one wave per pair; 16 pairs of 1000^2 run SPLIT.  Identical results on both routes, the oracle's
    on a sample."""
    table = tables[False]
    rng = np.random.default_rng(9600 + script)
    for shape, count, want_split in (((2000, 100), 128, False), ((1000, 1000), 16, True)):
        pairs = [("".join(rng.choice(list(IUPAC), size=shape[0])), "".join(rng.choice(list(IUPAC), size=shape[1])))
                 for _ in range(count)]
        plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
        gpu.set_costs(plan)
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(y) for _, y in pairs]),
                         script)
        try:
            assert (b.split_tasks > 0) == want_split, (shape, b.split_tasks)
        finally:
            b.close()
        got = gpu_run(gpu, table, pairs, script=script)
        assert gpu_run(gpu, table, pairs, script=script, split=1) == got
        assert gpu_run(gpu, table, pairs, script=script, split=2) == got
        _oracle_check(table, pairs[::16], got[::16])



@pytest.mark.parametrize("table_name", ["costs.json", "int_literals", "frac_indel"])
def test_fp64_segments_vs_oracle(gpu, tables, table_name):
    """fp64 batches of > 256 wave pairs run the pairs their cost model favours in 16-lane segments, four per wave
    (sed_wf_f64_kernel SW = 16: row DPP moves, 16-step chunks, a 15-step ramp) with the per-cell-code traceback of
    that layout: the timing.py sweep's short IUPAC pairs (timing.py:45-57).  Ragged pairs of 1..300 (one or more
    16 R-row stripes, columns past a chunk), scripts and distance-only, the typed fp64 kernel (int literals) and
    fractional indels: every pair vs the oracle, and identical to SED_OPT_SEG = 2 (no segments) and = 1 (every wave
    pair in segments)."""
    table = tables[False] if table_name == "costs.json" else load_golden("g8_cost_tables.json")["tables"][table_name]
    pairs = _random_pairs(8800 + len(table_name), 420, IUPAC, 1, 300, related=True)
    pairs += _random_pairs(8900 + len(table_name), 60, IUPAC, 33, 700)
    pairs += [("", "ACG"), ("GUA", ""), ("", ""), ("A", "C")]  # empty sides stay on the one-wave-per-pair kernel
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    for script in (True, False):
        b = sedgpu.Batch(gpu, sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs],
                                                 [plan.encode(y) for _, y in pairs]), script)
        try:
            assert b.mode in ("f64", "f64-typed") and b.lane_pairs == 0
            nseg = b.segment_pairs
            assert 0 < nseg <= len(pairs) - 3, nseg
        finally:
            b.close()
        got = gpu_run(gpu, table, pairs, script=script)
        _oracle_check(table, pairs, got)
        for opt in (2, 1):
            gpu.set_option(sedgpu.SED_OPT_SEG, opt)
            try:
                assert gpu_run(gpu, table, pairs, script=script) == got, (table_name, script, opt)
            finally:
                gpu.set_option(sedgpu.SED_OPT_SEG, 0)

"""CPU: the host half of the drop-in module — cost-table resolution and the
reference's KeyError, the dp proxy's list protocol and repr, co-optimal path
enumeration order, edit-script formatting, reversal and patching.

No GPU here: where a dp needs device results, the test fills the proxy from
the oracle (test infrastructure) so the host logic can be checked alone.
"""
import importlib
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
import oracle
import sedcost

OPS = {"i": "insert", "d": "delete", "u": "update"}


@pytest.fixture(scope="module")
def SED():
    cwd = os.getcwd()
    os.chdir(GOLDEN)
    try:
        sys.modules.pop("StringEditDistance", None)
        mod = importlib.import_module("StringEditDistance")
    finally:
        os.chdir(cwd)
    return mod


def oracle_dp(SED, table, s1, s2):
    """A DPMatrix whose device results come from the oracle (test only)."""
    plan = sedcost.build_plan(table, [s1], [s2])
    dp = SED.DPMatrix(s1, s2, plan)
    o = oracle.pair(oracle.Costs.from_plan(plan), plan.encode(s1), plan.encode(s2), True, True)
    dp._final = int(o["dist"]) if o["is_int"] else o["dist"]
    dp._script = o["ops"]
    dp._full = (o["D"], (o["M"] | (o["T"] << 3)).astype(np.uint8))
    return dp


def es_compact(es):
    return [[e["operation"][0], e["source"]["character"], e["source"]["index"],
             e["destination"]["character"], e["destination"]["index"]] for e in es]


def test_module_globals(SED, tables):
    assert SED.default_costs == tables[False] and SED.user_costs == tables[True]
    for name in ("wagnerFisher", "create_paths", "generate_es", "patching", "generate_rev_es",
                 "generate_sequence_from_es", "reload_user_costs", "cost", "min_cost", "Node", "Edge"):
        assert hasattr(SED, name)


def test_key_errors_like_reference(SED, tables):
    for r in load_golden("g6_errors.json"):
        table = tables[r["user"]]
        if "error" in r:
            with pytest.raises(KeyError) as ei:
                sedcost.check_pair(table, r["s1"], r["s2"])
            assert [str(a) for a in ei.value.args] == r["error"][1], (r["s1"], r["s2"])
        else:
            sedcost.check_pair(table, r["s1"], r["s2"])


def test_missing_table_keys():
    with pytest.raises(KeyError) as ei:
        sedcost.check_pair({"delete": 1.0, "update": {}}, "A", "C")
    assert ei.value.args == ("insert",)
    with pytest.raises(KeyError) as ei:
        sedcost.check_pair({"insert": 1.0, "update": {}}, "A", "C")
    assert ei.value.args == ("delete",)
    with pytest.raises(KeyError) as ei:
        sedcost.check_pair({"insert": 1.0, "delete": 1.0}, "A", "C")
    assert ei.value.args == ("update",)
    sedcost.check_pair({"insert": 1.0, "delete": 1.0}, "A", "a")  # matches never read the table
    sedcost.check_pair({}, "", "")


def test_cost_and_min_cost(SED, tables):
    assert SED.cost("A", "a") == 0 and isinstance(SED.cost("A", "a"), int)
    assert SED.cost("A", "C", True) == tables[True]["update"]["A"]["C"]
    with pytest.raises(KeyError):
        SED.cost("x", "A")
    dp = oracle_dp(SED, tables[True], "AGRGA", "AGGGAA")
    val, ops = SED.min_cost(dp, 3, 3, "AGRGA", "AGGGAA", True)
    assert val == dp[3][3].value and ops[2] == (2, 2, "update")


def test_dp_proxy_protocol_and_repr(SED, tables):
    for r in load_golden("g6_errors.json"):
        if "error" in r or r.get("matrix_repr") is None:
            continue
        dp = oracle_dp(SED, tables[r["user"]], r["s1"], r["s2"])
        assert repr(dp) == r["matrix_repr"], (r["s1"], r["s2"])
        assert len(dp) == len(r["s1"]) + 1 and len(dp[0]) == len(r["s2"]) + 1
        assert repr(dp[-1][-1]) == r["repr"]
        assert dp[len(dp) - 1][len(dp[0]) - 1] is dp[-1][-1]
    with pytest.raises(IndexError):
        oracle_dp(SED, tables[False], "AC", "G")[3]


def test_g1_all_paths_in_reference_order(SED, tables):
    g1 = load_golden("g1_small.json")
    for r in g1:
        dp = oracle_dp(SED, tables[r["user"]], r["s1"], r["s2"])
        want = [[float.fromhex(h), bool(ii)] for h, ii, _ in r["cells"]]
        have = [[float(c.value), isinstance(c.value, int)] for row in dp for c in row]
        assert want == have
        paths = SED.create_paths(dp)
        ops = ["".join("idu"[o] for o in p.ops) for p in paths]
        if r["paths"] == "deadlock":
            assert ops[0] == r["canon"] and len(set(ops)) == len(ops)
            continue
        assert ops == r["paths"][:len(ops)] and len(ops) == r["npaths"], (r["s1"], r["s2"], r["user"])
        for p, es in zip(paths, r["es"]):
            if isinstance(es, dict):
                with pytest.raises(IndexError):
                    SED.generate_es(p, r["s1"], r["s2"])
            else:
                assert es_compact(SED.generate_es(p, r["s1"], r["s2"])) == es
                # the generic (edge-walking) formatter agrees with the fast one
                assert es_compact(SED.generate_es(list(p), r["s1"], r["s2"])) == es


def test_nodes_edges_like_reference(SED, tables):
    dp = oracle_dp(SED, tables[True], "AGRGA", "AGGGAA")
    sink = dp[5][6]
    assert [e.operation for e in sink.incoming_edges] == ["insert", "update"]
    for e in sink.incoming_edges:
        assert e.destination is sink and e in e.source.edges
    assert dp[1][0].edges[0].operation == "delete"  # column 0 is linked before the interior (reference :167-182)
    assert [e.operation for e in dp[0][1].edges][0] == "insert"
    assert dp[0][0].value == 0 and isinstance(dp[0][0].value, int)
    assert (dp[2][3].i, dp[2][3].j) == (1, 2)


def test_g5_reverse_sequence_patching(SED):
    for r in load_golden("g5_patching.json"):
        es = [{"operation": OPS[o], "source": {"character": sc, "index": si},
               "destination": {"character": dc, "index": di}} for o, sc, si, dc, di in r["es"]]
        rev = SED.generate_rev_es(es)
        assert es_compact(rev) == r["rev"]
        assert SED.generate_sequence_from_es(es) == r["seq_from_es"]
        assert SED.generate_sequence_from_es(rev) == r["seq_from_rev"]
        for probe, code, out in r["patch_es"]:
            assert list(SED.patching(es, probe)) == [code, out], (r["s1"], r["s2"], probe)
        for probe, code, out in r["patch_rev"]:
            assert list(SED.patching(rev, probe)) == [code, out], (r["s1"], r["s2"], probe)


def test_g5_canonical_scripts(SED, tables):
    for r in load_golden("g5_patching.json"):
        dp = oracle_dp(SED, tables[r["user"]], r["s1"], r["s2"])
        es = SED.generate_es(SED.create_paths(dp)[0], r["s1"], r["s2"])
        assert es_compact(es) == r["es"]
        assert SED.patching(es, r["s1"]) == (0, r["s2"])
        assert SED.patching(SED.generate_rev_es(es), r["s2"]) == (0, r["s1"])


def test_generate_es_errors(SED, tables):
    dp = oracle_dp(SED, tables[False], "", "")
    with pytest.raises(IndexError):
        SED.generate_es(SED.create_paths(dp)[0], "", "")
    dp = oracle_dp(SED, tables[False], "AC", "AG")
    with pytest.raises(IndexError):  # not an edge of the graph
        SED.generate_es([dp[0][0], dp[2][2]], "AC", "AG")


def test_plan_encoding_roundtrip(tables):
    plan = sedcost.build_plan(tables[False], ["ACGUN", "aY"], ["RRA", "Ww"])
    for s in ("ACGUN", "aY", "RRA", "Ww"):
        codes = plan.encode(s)
        assert "".join(plan.alphabet[c] for c in codes) == s
    k = plan.code
    assert plan.sub[k["a"], k["A"]] == 0 and plan.sub_int[k["a"], k["A"]] == 1
    assert plan.sub[k["Y"], k["W"]] == tables[False]["update"]["Y"]["W"]


def _first_error(fn):
    try:
        fn()
    except KeyError as ex:
        return ("KeyError", ex.args)
    return None


def test_check_batch_like_sequential_checks(tables):
    """sedcost.check_batch (distance_batch, wfsearch) raises exactly what check_pair over the pairs in order raises:
    its fast path (every combination over the union alphabets resolves) must never hide an error, and the slow
    path finds the first offending pair.  Random batches over valid symbols, lowercase (free on a case-insensitive
    match, an error on a mismatch), unknown symbols and empty strings; both tables and tables missing keys."""
    rng = np.random.default_rng(77)
    pools = ["ACGU", "ACGUYRN", "ACGUa", "ACGUT", "ACGUacgu", "AGRGA"]
    extra = [{"insert": 1.0, "delete": 1.0, "update": {"A": {"C": 1.0}, "C": {"A": 2.0}}},
             {"delete": 1.0, "update": {}}, {"insert": 1.0, "update": {}}]
    for trial in range(400):
        table = (tables[False], tables[True], *extra)[trial % 5]
        pool = pools[trial % len(pools)] if trial % 5 < 2 else "ACac"
        P = int(rng.integers(1, 12))
        s1 = ["".join(rng.choice(list(pool), size=int(rng.integers(0, 6)))) for _ in range(P)]
        s2 = ["".join(rng.choice(list(pool), size=int(rng.integers(0, 6)))) for _ in range(P)]
        if trial % 3 == 0:  # the one-vs-many shape of wfsearch
            s1 = [s1[0]] * P

        def seq():
            for a, b in zip(s1, s2):
                sedcost.check_pair(table, a, b)
        want = _first_error(seq)
        got = _first_error(lambda: sedcost.check_batch(table, s1, s2))
        assert got == want, (trial, s1, s2, got, want)


def test_batch_plan_and_packing_match_per_string(tables):
    """build_plan over the joined strings, encode_many and PackedPairs.from_concat equal the per-string versions."""
    import sedgpu
    rng = np.random.default_rng(5)
    s1 = ["".join(rng.choice(list("ACGUNY"), size=int(rng.integers(0, 40)))) for _ in range(50)]
    s2 = ["".join(rng.choice(list("ACGUR"), size=int(rng.integers(0, 40)))) for _ in range(50)]
    plan = sedcost.build_plan(tables[False], s1, s2)
    seen = {}
    for s in s1 + s2:
        for c in s:
            seen.setdefault(c, 0)
    assert set(plan.alphabet) == set(seen)
    assert plan.alphabet[:len(dict.fromkeys("".join(s1)))] == list(dict.fromkeys("".join(s1)))
    ca, la = plan.encode_many(s1)
    cb, lb = plan.encode_many(s2)
    p1 = sedgpu.PackedPairs.from_concat(ca, la, cb, lb)
    p0 = sedgpu.PackedPairs([plan.encode(a) for a in s1], [plan.encode(b) for b in s2])
    for f in ("codes_a", "codes_b", "len_a", "len_b", "off_a", "off_b", "ops_off"):
        assert np.array_equal(getattr(p1, f), getattr(p0, f)), f
    assert p1.npairs == p0.npairs == 50


def test_distinct_first_occurrence_order():
    """sedcost.distinct (the delete-pass scan with the remembered alphabet, a histogram past 16 new symbols) equals
    dict.fromkeys on random strings over small, IUPAC-sized and large byte alphabets, non-latin text and empty
    strings, in any order of calls (the remembered symbols change between them)."""
    import random
    rnd = random.Random(11)
    pools = ["ACGU", "ACGUN", "ACGUYRWSKMDVHBNX", "".join(chr(i) for i in range(1, 256)), "aé€Ω", "\x00A"]
    for _ in range(4000):
        pool = rnd.choice(pools)
        s = "".join(rnd.choice(pool) for _ in range(rnd.randint(0, 80)))
        assert sedcost.distinct(s) == list(dict.fromkeys(s)), s
        assert sedcost.distinct_many([s, s[::-1], ""]) == list(dict.fromkeys(s + s[::-1])), s
    assert sedcost.distinct(list("ACCA")) == ["A", "C"]


def test_encode_many_repeated_query(tables):
    """The one-query-many-documents fast path of encode_many (codes tiled once) equals per-string encoding."""
    plan = sedcost.build_plan(tables[False], ["ACGUN"], ["ACGU"])
    for strs in (["ACGUNNA"] * 7, ["A"] * 2, ["ACG", "ACG", "AC"], [""] * 3):
        codes, lens = plan.encode_many(strs)
        want = np.concatenate([plan.encode(s) for s in strs]) if strs else np.zeros(0, np.uint8)
        assert np.array_equal(codes, want) and lens.tolist() == [len(s) for s in strs], strs


def test_pair_plan_shared_by_symbol_sets_and_fresh_after_edits(tables):
    """pair_plan caches one plan per (str1 symbols, str2 symbols, resolved costs): pairs over the same symbols in any
    order share it; editing the table in place (the GUI's cost editors), including an int/float change of one
    value, gives a new plan with the new value; a missing entry raises the reference's KeyError."""
    import copy
    t = copy.deepcopy(tables[True])
    p1 = sedcost.pair_plan(t, "ACGU", "UGCA")
    p2 = sedcost.pair_plan(t, "UUGCAA", "CAGU")
    assert p1 is p2
    for s1, s2 in (("ACGU", "UGCA"), ("UUGCAA", "CAGU")):
        want = sedcost.build_plan(t, [s1], [s2])
        for a in set(s1):
            for b in set(s2):
                assert p2.sub[p2.code[a], p2.code[b]] == want.sub[want.code[a], want.code[b]]
    old = t["update"]["A"]["C"]
    t["update"]["A"]["C"] = float(old) + 0.5
    p3 = sedcost.pair_plan(t, "CAGU", "GUCA")
    assert p3 is not p1 and p3.sub[p3.code["A"], p3.code["C"]] == float(old) + 0.5
    t["update"]["A"]["C"] = int(old) if float(old).is_integer() else old
    t["update"]["A"]["C"] = float(t["update"]["A"]["C"])
    t["update"]["A"]["G"] = int(t["update"]["A"]["G"])
    p4 = sedcost.pair_plan(t, "ACGU", "UGCA")
    assert p4.sub_int[p4.code["A"], p4.code["G"]] == 1
    del t["update"]["G"]["U"]
    with pytest.raises(KeyError):
        sedcost.pair_plan(t, "GA", "AU")

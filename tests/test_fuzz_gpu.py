"""Time-bounded randomized route fuzz (GPU): random batches through the C-ABI against the C oracle, bit for bit.

Every iteration draws a cost table (costs.json, user_costs.json or one of the G8 GUI tables), an alphabet (ACGU or
the table's whole alphabet), a batch size around the routing thresholds (1, 16, 17, 64, 65, 256, 257 ... pairs),
ragged lengths (empty sides included, now and then a pair past 1000 rows), a flag set (script, distance with length,
distance only) and a routing override (SPLIT on / off, lane kernels off, rows per lane, fp64 forced, zero-copy off,
16-lane segments on / off, per-cell codes or checkpoints, SPLIT's ladder-key forward, CHAIN mode on the wide, 3-bit
or perm ladder), then compares every pair's distance, typing, length and script with the oracle, and checks that the script
region's bits past the last op are zero (sed.h)
(oracle/sed_oracle.c: StringEditDistance.py:92-334).  SED_FUZZ_SECONDS sets the budget (default 20 s) and
SED_FUZZ_SEED the first seed (default 2026), so the default run is reproducible; a failure names its seed.
"""
import os
import time

import numpy as np
import pytest

from conftest import load_golden, padding_errors
import oracle
import sedcost
import sedgpu

pytestmark = pytest.mark.gpu

SIZES = [1, 1, 2, 3, 5, 16, 17, 40, 64, 65, 100, 256, 257, 300]
OPTIONS = [
    (None, 0),
    (sedgpu.SED_OPT_SPLIT, 1), (sedgpu.SED_OPT_SPLIT, 2),
    (sedgpu.SED_OPT_LANE, 2),
    (sedgpu.SED_OPT_ROWS_PER_LANE, 4), (sedgpu.SED_OPT_ROWS_PER_LANE, 8),
    (sedgpu.SED_OPT_ZEROCOPY, 2),
    (sedgpu.SED_OPT_SEG, 1), (sedgpu.SED_OPT_SEG, 2),
    (sedgpu.SED_OPT_TB, 1), (sedgpu.SED_OPT_TB, 2),
    (sedgpu.SED_OPT_SPLITCK, 2),
    ("mode", 2), ("mode", 3),  # the fp64 kernels forced (simple / full typing)
    # CHAIN mode forced at R = 8 / 4 (dynamic, or static chains of 3), on the wide-ladder dot keys where the table
    # factors, the 3-bit ladder's (SED_OPT_DOT = 3) or the perm ladder (2)
    ((sedgpu.SED_OPT_CHAIN, 1), (sedgpu.SED_OPT_ROWS_PER_LANE, 8)),
    ((sedgpu.SED_OPT_CHAIN, 1), (sedgpu.SED_OPT_ROWS_PER_LANE, 4)),
    ((sedgpu.SED_OPT_CHAIN, 3), (sedgpu.SED_OPT_ROWS_PER_LANE, 8)),
    ((sedgpu.SED_OPT_CHAIN, 1), (sedgpu.SED_OPT_ROWS_PER_LANE, 8), (sedgpu.SED_OPT_DOT, 3)),
    ((sedgpu.SED_OPT_CHAIN, 1), (sedgpu.SED_OPT_ROWS_PER_LANE, 8), (sedgpu.SED_OPT_DOT, 2)),
]
CELL_CAP = 2.5e7  # oracle work per iteration


def _tables():
    out = [("costs.json", load_golden("costs.json")), ("user_costs.json", load_golden("user_costs.json"))]
    out += sorted(load_golden("g8_cost_tables.json")["tables"].items())
    return out


def _batch(rng, alphabet):
    npairs = int(rng.choice(SIZES))
    related = rng.random() < 0.5
    pairs, cells = [], 0.0
    for _ in range(npairs):
        r = rng.random()
        hi = 40 if r < 0.4 else (600 if r < 0.93 else 1500)
        n = int(rng.integers(0, hi + 1))
        m = int(rng.integers(0, hi + 1)) if not related else max(0, n + int(rng.integers(-n // 8 - 1, n // 8 + 2)))
        if cells + n * m > CELL_CAP:
            n, m = min(n, 40), min(m, 40)
        cells += n * m
        a = "".join(rng.choice(alphabet, size=n))
        if related:
            b = "".join(c if rng.random() > 0.15 else rng.choice(alphabet) for c in a)[:m]
            b += "".join(rng.choice(alphabet, size=max(0, m - len(b))))
        else:
            b = "".join(rng.choice(alphabet, size=m))
        pairs.append((a, b))
    return pairs


def _check(gpu, table, pairs, script, no_len, opt, seed):
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    gpu.set_costs(plan)
    settings = list(opt) if isinstance(opt[0], tuple) else [opt]
    for key, val in settings:
        if key == "mode":
            gpu.set_mode(val)
        elif key is not None:
            gpu.set_option(key, val)
    try:
        packed = sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(b) for _, b in pairs])
        dist, is_int, ln, ops = gpu.run(packed, script, no_len=no_len)
    finally:
        for key, val in settings:
            if key == "mode":
                gpu.set_mode(0)
            elif key is not None:
                gpu.set_option(key, 0)
    cs = oracle.Costs.from_plan(plan)
    for p, (a, b) in enumerate(pairs):
        o = oracle.pair(cs, plan.encode(a), plan.encode(b), want_ops=script)
        where = "seed %d, pair %d of %d (%d x %d), script %s, no_len %s, option %s" % (
            seed, p, len(pairs), len(a), len(b), script, no_len, opt)
        assert (float(dist[p]), bool(is_int[p])) == (o["dist"], bool(o["is_int"])), where
        if not no_len or script:
            assert int(ln[p]) == o["len"], where
        if script:
            got = sedgpu.unpack_ops(ops, packed.ops_off, p, int(ln[p]))
            assert np.array_equal(got, o["ops"]), where
            assert not padding_errors(ops, packed.ops_off, packed.len_a, packed.len_b, ln, [p]), \
                "nonzero script padding: " + where


def test_route_fuzz_vs_oracle(gpu):
    budget = float(os.environ.get("SED_FUZZ_SECONDS", "20"))
    seed = int(os.environ.get("SED_FUZZ_SEED", "2026"))
    tabs = _tables()
    t_end = time.monotonic() + budget
    t_note = time.monotonic() + 20.0
    runs = 0
    while time.monotonic() < t_end or runs < 8:
        if time.monotonic() > t_note:  # (progress for long budgets)
            print("route fuzz: %d batches, seed %d" % (runs, seed), flush=True)
            t_note += 20.0
        rng = np.random.default_rng(seed)
        name, table = tabs[int(rng.integers(0, len(tabs)))]
        full = [s for s in table["update"] if all(s in table["update"][t] for t in table["update"])]
        acgu = [s for s in "ACGU" if s in full]
        alphabet = list(acgu if (rng.random() < 0.5 and len(acgu) == 4) else full)
        pairs = _batch(rng, alphabet)
        mode = int(rng.integers(0, 3))
        script, no_len = (True, False) if mode == 0 else ((False, False) if mode == 1 else (False, True))
        opt = OPTIONS[int(rng.integers(0, len(OPTIONS)))]
        _check(gpu, table, pairs, script, no_len, opt, seed)
        seed += 1
        runs += 1
    print("route fuzz: %d batches" % runs)


def test_module_fuzz_vs_pyref():
    """The drop-in module's calls as the reference's callers make them, on random short pairs, against the
    pure-Python node graph (oracle/pyref.py, pinned to the reference's fixtures by tests/test_pyref.py):
    wagnerFisher's sink value and int/float typing, create_paths(dp)[0] and generate_es, then generate_rev_es and
    patching back to str1 (StringEditDistance.py:133-457).  SED_FUZZ_MODULE_SECONDS sets the budget (default 8 s)."""
    import importlib
    import sys
    from conftest import GOLDEN
    import pyref
    cwd = os.getcwd()
    os.chdir(GOLDEN)
    try:
        sys.modules.pop("StringEditDistance", None)
        SED = importlib.import_module("StringEditDistance")
    finally:
        os.chdir(cwd)
    tables = {False: load_golden("costs.json"), True: load_golden("user_costs.json")}
    iupac = list("AGCUYRWSKMDVHBN")
    rng = np.random.default_rng(int(os.environ.get("SED_FUZZ_SEED", "2026")) + 7)
    t_end = time.monotonic() + float(os.environ.get("SED_FUZZ_MODULE_SECONDS", "8"))
    t_note = time.monotonic() + 20.0
    runs = 0
    kept = []  # long scripts the 'caller' holds (some with their reversal): never reused, never changed
    while time.monotonic() < t_end or runs < 20:
        if time.monotonic() > t_note:  # (progress for long budgets)
            print("module fuzz: %d pairs" % runs, flush=True)
            t_note += 20.0
        user = bool(rng.random() < 0.5)
        al = list("ACGU") if rng.random() < 0.5 else iupac
        if rng.random() < 0.05:  # a long pair: the script-list build / reuse path (n + m >= 512), vs the C oracle
            _long_module_case(SED, rng, al, tables[user], user, kept)
            runs += 1
            continue
        n, m = int(rng.integers(0, 48)), int(rng.integers(0, 48))
        s1 = "".join(rng.choice(al, size=n))
        s2 = "".join(c if rng.random() > 0.2 else rng.choice(al) for c in s1)[:m] if rng.random() < 0.5 else \
            "".join(rng.choice(al, size=m))
        v, ops, es = pyref.run_pair(s1, s2, tables[user])
        dp = SED.wagnerFisher(s1, s2, user)
        got = dp[len(dp) - 1][len(dp[0]) - 1].value
        assert (got, type(got)) == (v, type(v)), (s1, s2, user)
        if s1 and s2:
            path = SED.create_paths(dp)[0]
            steps = [(b.i - a.i, b.j - a.j) for a, b in zip(path, path[1:])]
            assert "".join("u" if st == (1, 1) else ("d" if st[0] else "i") for st in steps) == ops, (s1, s2, user)
            got_es = SED.generate_es(path, s1, s2)
            assert got_es == es, (s1, s2, user)
            # (patching returns (error code, string), StringEditDistance.py:457)
            assert SED.patching(SED.generate_rev_es(got_es), s2) == (0, s1), (s1, s2, user)
            assert SED.patching(got_es, s1) == (0, s2), (s1, s2, user)
        runs += 1
    for es, copy, _ in kept:
        assert es == copy
    print("module fuzz: %d pairs" % runs)


def _long_module_case(SED, rng, al, table, user, kept):
    """One GUI-style call on a pair of 260..900 symbols a side (the records are built during the device run and a
    released previous list may be reused, StringEditDistance._skeleton): the records must equal es_from_ops of the C
    oracle's script; the result is sometimes kept (with a deep copy, sometimes with its reversal) and kept ones are
    sometimes released, so the reuse sees held, shared and released lists."""
    import _sedhost
    import oracle
    import sedcost
    n, m = (int(x) for x in rng.integers(260, 900, size=2))
    s1 = "".join(rng.choice(al, size=n))
    s2 = "".join(c if rng.random() > 0.15 else rng.choice(al) for c in s1)[:m] if rng.random() < 0.5 else \
        "".join(rng.choice(al, size=m))
    plan = sedcost.pair_plan(table, s1, s2)
    want = oracle.pair(oracle.Costs.from_plan(plan), np.frombuffer(plan.encode_bytes(s1), np.uint8),
                       np.frombuffer(plan.encode_bytes(s2), np.uint8))
    SED._script_hint = True
    dp = SED.wagnerFisher(s1, s2, user)
    got = dp[len(dp) - 1][len(dp[0]) - 1].value
    assert got == want["dist"], (n, m, user)
    es = SED.generate_es(SED.create_paths(dp)[0], s1, s2)
    assert es == _sedhost.es_from_ops(want["ops"].tobytes(), s1, s2), (n, m, user)
    if rng.random() < 0.3:
        copy = [dict(r, source=dict(r["source"]), destination=dict(r["destination"])) for r in es]
        kept.append((es, copy, SED.generate_rev_es(es) if rng.random() < 0.5 else None))
    if kept and rng.random() < 0.3:
        es0, copy0, _ = kept.pop(int(rng.integers(0, len(kept))))
        assert es0 == copy0

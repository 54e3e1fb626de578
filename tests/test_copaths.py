"""CPU: co-optimal path enumeration in the reference's create_paths order (copaths.py) on the
G1 golden masks (generated from the reference's own dp graphs and create_paths)."""
import itertools
import math

import numpy as np
import pytest

from conftest import load_golden
import copaths


def _mask(rec):
    n, m = len(rec["s1"]), len(rec["s2"])
    return np.array([c[2] for c in rec["cells"]], np.uint8).reshape(n + 1, m + 1)


def test_g1_paths_in_reference_order():
    for r in load_golden("g1_small.json"):
        M = _mask(r)
        got = ["".join("idu"[o] for o in p) for p in copaths.iter_paths(M)]
        assert got[0] == r["canon"], (r["s1"], r["s2"])
        if r["paths"] == "deadlock":
            # the reference blocks forever here (bounded queue); the count stands in for it
            assert len(got) == copaths.count_paths(M) > (len(r["s1"]) + 1) * (len(r["s2"]) + 1)
            continue
        assert got == r["paths"], (r["s1"], r["s2"], r["user"])
        assert copaths.count_paths(M) == r["npaths"] == len(got)


def test_lazy_prefix_and_big_count():
    # every edge optimal: the count is the Delannoy number D(n, m) (a 100-bit integer here)
    n = m = 40
    M = np.full((n + 1, m + 1), 7, np.uint8)
    M[0, :] = 1
    M[:, 0] = 2
    M[0, 0] = 0
    dela = sum(math.comb(n, k) * math.comb(m, k) * 2 ** k for k in range(min(n, m) + 1))
    assert copaths.count_paths(M) == dela
    first = list(itertools.islice(copaths.iter_paths(M), 5))
    assert [len(p) for p in first] == [40, 41, 41, 41, 41]  # the all-update path, then one i+d pair
    assert "".join("idu"[o] for o in first[0]) == "u" * 40
    assert "".join("idu"[o] for o in first[1]) == "u" * 39 + "di"  # from the sink: i first
    # shortest paths have exactly n updates; the next lengths come only after all of them
    lengths = [len(p) for p in itertools.islice(copaths.iter_paths(M), 200)]
    assert lengths == sorted(lengths)


def test_lex_order_from_sink():
    M = np.full((4, 4), 7, np.uint8)
    M[0, :] = 1
    M[:, 0] = 2
    M[0, 0] = 0
    paths = ["".join("idu"[o] for o in p) for p in copaths.iter_paths(M)]
    assert len(paths) == copaths.count_paths(M) == 63  # Delannoy D(3,3)
    key = [(len(p), p[::-1].translate(str.maketrans("idu", "012"))) for p in paths]
    assert key == sorted(key)


def test_g8_path_order_on_gui_cost_tables():
    """Ordered enumeration and counts on the G8 tables (zero/negative costs give many co-optimal paths)."""
    g8 = load_golden("g8_cost_tables.json")
    n = 0
    for r in g8["small"]:
        if r["paths"] == "deadlock":
            continue
        M = np.array([mk for _, _, mk in r["cells"]], np.uint8).reshape(len(r["s1"]) + 1, len(r["s2"]) + 1)
        got = []
        for p in copaths.iter_paths(M):
            got.append("".join("idu"[c] for c in p))
            if len(got) == len(r["paths"]):
                break
        assert got == r["paths"], (r["table"], r["s1"], r["s2"])
        assert copaths.count_paths(M) == r["npaths"]
        n += 1
    assert n > 300


def test_c_windows_and_count_match_the_python_restatement():
    """_sedhost.length_windows / count_paths (C) against the Python bitsets and big-int count on random
    masks of real DPs (oracle full matrices), including windows narrower than the path-length spread."""
    import oracle
    import sedcost
    rng = np.random.default_rng(11)
    table = load_golden("g8_cost_tables.json")["tables"]["zero_insert"]  # many co-optimal paths
    for _ in range(30):
        a = "".join(rng.choice(list("ACGU"), size=int(rng.integers(0, 25))))
        b = "".join(rng.choice(list("ACGU"), size=int(rng.integers(0, 25))))
        plan = sedcost.build_plan(table, [a], [b])
        M = oracle.pair(oracle.Costs.from_plan(plan), plan.encode(a), plan.encode(b), full=True)["M"]
        sets = copaths.length_sets(M)
        for words in (1, 2):
            w = copaths.LengthWindows(M, words)
            for i in range(M.shape[0]):
                for j in range(M.shape[1]):
                    s = sets[i][j]
                    assert w.lo[i * w.cols + j] == ((s & -s).bit_length() - 1 if s else -1)
                    assert w.hi[i * w.cols + j] == (s.bit_length() - 1 if s else -1)
                    for ell in range(w.lo[i * w.cols + j], w.lo[i * w.cols + j] + 64 * words):
                        assert w.has(i, j, ell) == (s >> ell) & 1
        assert copaths.count_paths(M) == copaths._count_paths_py(np.asarray(M))
        got = list(itertools.islice(copaths.iter_paths(M), 300))
        saved, copaths._sedhost = copaths._sedhost, None
        try:
            ref = list(itertools.islice(copaths.iter_paths(M), 300))
        finally:
            copaths._sedhost = saved
        assert [p.tolist() for p in got] == [p.tolist() for p in ref]


def test_window_bounds_and_large_counts():
    """Every monotone path is co-optimal (all edges set): length classes come out in order, the sink's
    window reports its exact range, and the C count equals the Python big-int count (Delannoy D(40, 40))."""
    n = m = 40
    M = np.zeros((n + 1, m + 1), np.uint8)
    M[0, 1:] = 1
    M[1:, 0] = 2
    M[1:, 1:] = 7
    lengths = []
    for p in copaths.iter_paths(M):
        if not lengths or len(p) != lengths[-1]:
            lengths.append(len(p))
        if len(lengths) > 3:
            break
    assert lengths == [40, 41, 42, 43]
    w = copaths.LengthWindows(M)
    assert w.lengths_at_sink() == (40, 80) and w.exact_up_to() == 103
    total = copaths.count_paths(M)
    assert total == copaths._count_paths_py(M) and total.bit_length() > 64  # Delannoy D(40, 40)


def test_window_widening_is_capped(monkeypatch):
    """Widening the length windows past MAX_WORDS words or SED_COPATHS_MAX_GB raises a SedError that names the
    limit instead of allocating without bound."""
    import sedgpu
    assert copaths._wider(1, 40, 40, 140, 40) == 2
    monkeypatch.setenv("SED_COPATHS_MAX_GB", "0.00001")  # 10 kB
    with pytest.raises(sedgpu.SedError, match="SED_COPATHS_MAX_GB"):
        copaths._wider(1, 40, 40, 140, 40)
    monkeypatch.delenv("SED_COPATHS_MAX_GB")
    with pytest.raises(sedgpu.SedError, match="1024 words"):
        copaths._wider(1024, 4, 4, 70000, 8)

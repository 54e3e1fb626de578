"""GPU: the drop-in StringEditDistance module end to end (wagnerFisher on the
device, the dp proxy, create_paths, generate_es ...) against the golden
fixtures generated from the reference, including the callers' idioms
(IRMethods.wf_score, the GUI's table / script loops)."""
import hashlib
import importlib
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

pytestmark = pytest.mark.gpu


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


def es_compact(es):
    return [[e["operation"][0], e["source"]["character"], e["source"]["index"],
             e["destination"]["character"], e["destination"]["index"]] for e in es]


def wf_score(SED, seq1, seq2, user_cost=False):
    """IRMethods.wf_score's body (IRMethods.py:435-440), verbatim in behaviour."""
    dp = SED.wagnerFisher(seq1, seq2, user_cost)
    cost = dp[len(dp) - 1][len(dp[0]) - 1].value
    return 1 / (1 + cost)


def test_g1_through_the_module(SED):
    for r in load_golden("g1_small.json"):
        dp = SED.wagnerFisher(r["s1"], r["s2"], r["user"])
        v = dp[len(dp) - 1][len(dp[0]) - 1].value
        assert (float(v), isinstance(v, int)) == (float.fromhex(r["dist"][0]), r["dist"][1])
        paths = SED.create_paths(dp)
        first = "".join("idu"[o] for o in paths[0].ops)
        assert first == r["canon"]
        # the GUI loop: every cell value, then every path's script
        cells = [[float(c.value), isinstance(c.value, int)] for row in dp for c in row]
        assert cells == [[float.fromhex(h), bool(ii)] for h, ii, _ in r["cells"]]
        if r["paths"] != "deadlock":
            ops = ["".join("idu"[o] for o in p.ops) for p in paths]
            assert ops == r["paths"][:len(ops)] and len(ops) == r["npaths"]
            for p, es in zip(paths, r["es"]):
                if isinstance(es, dict):
                    with pytest.raises(IndexError):
                        SED.generate_es(p, r["s1"], r["s2"])
                else:
                    assert es_compact(SED.generate_es(p, r["s1"], r["s2"])) == es


def test_g6_errors_typing_repr(SED):
    for r in load_golden("g6_errors.json"):
        if "error" in r:
            with pytest.raises(KeyError) as ei:
                SED.wagnerFisher(r["s1"], r["s2"], r["user"])
            assert [str(a) for a in ei.value.args] == r["error"][1]
            continue
        dp = SED.wagnerFisher(r["s1"], r["s2"], r["user"])
        v = dp[-1][-1].value
        assert (float(v), isinstance(v, int)) == (float.fromhex(r["dist"][0]), r["dist"][1])
        assert repr(dp[-1][-1]) == r["repr"]
        if r.get("matrix_repr") is not None:
            assert repr(dp) == r["matrix_repr"]
        if "es0" in r:
            assert es_compact(SED.generate_es(SED.create_paths(dp)[0], r["s1"], r["s2"])) == r["es0"]
        if "es_error" in r:
            with pytest.raises(IndexError):
                SED.generate_es(SED.create_paths(dp)[0], r["s1"], r["s2"])


def test_g2_canonical_scripts(SED):
    for r in load_golden("g2_medium.json"):
        dp = SED.wagnerFisher(r["s1"], r["s2"], r["user"])
        assert dp[-1][-1].value == float.fromhex(r["dist"][0])
        es = SED.generate_es(SED.create_paths(dp)[0], r["s1"], r["s2"])
        assert hashlib.sha256(json.dumps(es_compact(es)).encode()).hexdigest() == r["es_sha256"]
        assert SED.patching(es, r["s1"]) == (0, r["s2"])
        assert SED.patching(SED.generate_rev_es(es), r["s2"]) == (0, r["s1"])


def test_g4_wf_score_all_vs_all(SED):
    g4 = load_golden("g4_wf_score.json")
    seqs = g4["seqs"]
    for user, key in ((False, "wf_score"), (True, "wf_score_user")):
        want = [[float.fromhex(x) for x in row] for row in g4[key]]
        got = [[wf_score(SED, a, b, user) for b in seqs] for a in seqs]
        assert got == want
        # one launch for the whole matrix
        vals = SED.distance_batch([a for a in seqs for _ in seqs], [b for _ in seqs for b in seqs], user)
        assert [[1 / (1 + vals[i * len(seqs) + j]) for j in range(len(seqs))] for i in range(len(seqs))] == want


def test_all_vs_all_single_rank(SED):
    import sedshard
    g4 = load_golden("g4_wf_score.json")
    M = sedshard.all_vs_all(g4["seqs"], False)
    want = np.array([[1 / float.fromhex(x) - 1 for x in row] for row in g4["wf_score"]])
    assert np.allclose(M, want, rtol=0, atol=1e-9)


def test_edit_script_batch_matches_single_calls(SED):
    g5 = load_golden("g5_patching.json")
    for user in (False, True):
        recs = [r for r in g5 if r["user"] == user]
        out = SED.edit_script_batch([r["s1"] for r in recs], [r["s2"] for r in recs], user)
        for r, (v, es) in zip(recs, out):
            assert es_compact(es) == r["es"]


def test_reload_user_costs(SED, tmp_path, monkeypatch):
    table = json.load(open(os.path.join(GOLDEN, "user_costs.json")))
    table["insert"] = 5.0
    (tmp_path / "user_costs.json").write_text(json.dumps(table))
    monkeypatch.chdir(tmp_path)
    old = SED.user_costs
    try:
        SED.reload_user_costs()
        assert SED.wagnerFisher("", "AC", True)[-1][-1].value == 10.0
        SED.user_costs["insert"] = 1.0  # the GUI edits the dict in place
        assert SED.wagnerFisher("", "AC", True)[-1][-1].value == 2.0
    finally:
        SED.user_costs = old


def test_count_paths_and_enumeration(SED):
    import itertools
    import copaths
    for r in load_golden("g1_small.json")[::5]:
        dp = SED.wagnerFisher(r["s1"], r["s2"], r["user"])
        if r["paths"] != "deadlock":
            assert SED.count_paths(dp) == r["npaths"]
    # medium pairs: the device's canonical script is the first path of the ordered enumeration,
    # and the next paths come quickly (the reference's BFS frontier would be exponential here)
    for r in load_golden("g2_medium.json")[:6]:
        dp = SED.wagnerFisher(r["s1"], r["s2"], r["user"])
        paths = SED.create_paths(dp)
        first = next(copaths.iter_paths(dp._materialise()[1]))
        assert np.array_equal(first, paths[0].ops)
        more = [p.ops for p in itertools.islice(iter(paths), 20)]
        keys = [(len(o), tuple(o[::-1])) for o in more]
        assert keys == sorted(keys) and len(set(keys)) == len(keys)
        assert SED.count_paths(dp) >= len(more)


def test_search_collection_matches_reference(SED):
    import seqio
    import wfsearch
    g7 = load_golden("g7_ingest_search.json")
    coll = seqio.ListCollection.from_sequences(list(g7["test_input"].values()))
    wfsearch.clear_cache()
    for s in g7["searches"]:
        want = [[seq, float.fromhex(h)] for seq, h in s["scores"]]
        got = wfsearch.search_collection(s["query"], None, coll, wfsearch.wf_score)
        assert [[a, b] for a, b in got] == want
        rd = {}
        wfsearch.search_collection(s["query"], "tf", coll, wfsearch.wf_score, return_dict=rd)  # cached
        assert [[a, b] for a, b in rd["wf_score"]] == want
        seen = []
        wfsearch.search_collection(s["query"], None, coll, wfsearch.wf_score, callback=seen.append)
        assert [[a, b] for a, b in seen[0]] == want
        assert wfsearch.wf_score(s["query"], want[3][0]) == want[3][1]


def test_script_hint_runs_agree(SED):
    """wagnerFisher runs distance-only, or DP + traceback when the previous matrix was asked for its
    script (the GUI pattern).  Both runs must give the same value, type, canonical path and script."""
    for r in load_golden("g1_small.json")[:120]:
        seen = []
        for hint in (False, True):
            SED._script_hint = hint
            dp = SED.wagnerFisher(r["s1"], r["s2"], r["user"])
            assert (dp._script is not None) == hint
            v = dp[len(dp) - 1][len(dp[0]) - 1].value
            assert (float(v), isinstance(v, int)) == (float.fromhex(r["dist"][0]), r["dist"][1])
            assert "".join("idu"[o] for o in SED.create_paths(dp)[0].ops) == r["canon"]
            assert SED._script_hint  # create_paths asked for the script: the next call predicts it
            seen.append((v, type(v), list(dp.script())))
        assert seen[0] == seen[1]
    SED._script_hint = True
    assert SED.wagnerFisher("ACGU", "AGU")._script is not None
    assert SED.wagnerFisher("ACGU", "AGU")._script is None  # nobody asked for the last script: distance-only again


def test_gui_call_builds_es_records_during_the_run(SED):
    """The GUI's call (wagnerFisher -> create_paths -> generate_es, gui.py:360,385-391) on pairs of >= 512 symbols
    submits the pair (sed_pair_submit), builds generate_es' records while the device runs and fills them after
    (sed_pair_wait, _sedhost.es_fill): the records equal es_from_ops', a second generate_es returns new ones, and the
    context refuses another call while a pair is in flight (SED_E_STATE)."""
    import _sedhost
    import sedcost
    import sedgpu
    import synth
    for n, m, user in ((700, 650, True), (200, 200, False), (4096, 4096, True)):
        s1, s2 = synth.pair_strings(n + m, n, m)
        SED._script_hint = True
        dp = SED.wagnerFisher(s1, s2, user)
        assert (dp._skel is not None) == (n + m >= SED._SKEL_MIN)
        p0 = SED.create_paths(dp)[0]
        es = SED.generate_es(p0, s1, s2)
        assert dp._skel is None
        want = _sedhost.es_from_ops(np.asarray(p0.ops, np.uint8).tobytes(), s1, s2)
        assert es == want and len(es) == len(p0.ops)
        es2 = SED.generate_es(p0, s1, s2)
        assert es2 == es and es2 is not es and es2[0] is not es[0]
        assert SED.patching(es, s1) == (0, s2)
    ctx = sedgpu.context()
    plan = sedcost.pair_plan(SED._table(False), "ACGUACGU", "ACGGU")
    ctx.set_costs(plan)
    a, b = plan.encode_bytes("ACGUACGU"), plan.encode_bytes("ACGGU")
    ctx.submit_pair(a, b, True)
    try:
        assert ctx._lib.sed_pair_submit(ctx.ptr, a, len(a), b, len(b), 1) == -6  # SED_E_STATE: one pair in flight
        with pytest.raises(sedgpu.SedError, match="waited for"):
            ctx.run_pair(a, b, False)
    finally:
        got = ctx.wait_pair()
    assert got[:3] == ctx.run_pair(a, b, True)[:3]


def test_gui_calls_recycle_released_scripts(SED):
    """Repeated GUI calls (gui.py:385-391 drops the previous call's scripts, edit_scripts.clear()) reuse a released
    generate_es list as the next call's records (StringEditDistance._skeleton, _sedhost.es_recycle: its records still
    carry the old values until generate_es fills them): every call's records equal es_from_ops', and a list the caller
    still holds (one with its reversal too) is never reused nor changed."""
    import _sedhost
    import synth

    def want(p0, s1, s2):
        return _sedhost.es_from_ops(np.asarray(p0.ops, np.uint8).tobytes(), s1, s2)

    held, reused = [], []
    shapes = [(700, 650), (640, 700), (600, 610), (700, 700), (650, 600), (4096, 4096), (4000, 4090), (700, 690),
              (690, 700), (700, 700)]
    for k, (n, m) in enumerate(shapes):
        s1, s2 = synth.pair_strings(3000 + k, n, m)
        SED._script_hint = True
        dp = SED.wagnerFisher(s1, s2, True)
        reused.append(dp._skel is not None and dp._skel[0][0]["operation"] is not None)  # (new records hold None)
        p0 = SED.create_paths(dp)[0]
        es = SED.generate_es(p0, s1, s2)
        assert es == want(p0, s1, s2)
        if k in (1, 4):  # kept by the caller, with a deep copy of its values (and for k = 4 its reversal)
            copy = [dict(r, source=dict(r["source"]), destination=dict(r["destination"])) for r in es]
            held.append((es, copy, SED.generate_rev_es(es) if k == 4 else None))
        del es, p0, dp
    assert sum(reused) >= 5, reused
    for es, copy, _ in held:
        assert es == copy


def _ref_search_collection(query, vector_type, collection, method, return_dict=None, callback=None):
    """IRMethods.search_collection (IRMethods.py:443-477) for method == wf_score: one wagnerFisher per
    document through the drop-in module, exactly as the unchanged caller does."""
    scores = []
    for doc in collection.find({}):
        scores.append((doc['sequence'], method(query, doc['sequence'])))
    if callback is not None:
        callback(scores)
    elif return_dict is not None:
        return_dict[method.__name__] = scores
    else:
        return scores


def test_create_search_threads_process_model(SED):
    """gui.py:360 runs wagnerFisher in the GUI process (HIP initialised there), then
    IRMethods.create_search_threads forks a Process per method and another for wf_score, delivering through
    Manager dicts (IRMethods.py:480-515).  The forked children are served by a thread of this process over a socket
    pair made at fork time (sedgpu._before_fork); results match G7."""
    import multiprocessing as mp
    import seqio
    import sedgpu
    import wfsearch
    g7 = load_golden("g7_ingest_search.json")
    coll = seqio.ListCollection.from_sequences(list(g7["test_input"].values()))
    SED.wagnerFisher("AGRGA", "AGGGAA", True)  # the parent's GPU call (gui.py:360)
    assert isinstance(sedgpu.context(), sedgpu.Context)
    fork = mp.get_context("fork")
    manager = fork.Manager()
    for s in g7["searches"][:2]:
        want = [[seq, float.fromhex(h)] for seq, h in s["scores"]]
        return_dict, wagner_dict = manager.dict(), manager.dict()
        jobs = [fork.Process(target=_ref_search_collection, args=(s["query"], "tf", coll, wfsearch.wf_score,
                                                                  return_dict))]
        for p in jobs:
            p.start()
        for p in jobs:
            p.join(timeout=120)
            assert p.exitcode == 0
        p = fork.Process(target=_ref_search_collection, args=(s["query"], "tf", coll, wfsearch.wf_score, wagner_dict))
        p.start()
        p.join(timeout=120)
        assert p.exitcode == 0
        assert [[a, b] for a, b in return_dict["wf_score"]] == want
        assert [[a, b] for a, b in wagner_dict["wf_score"]] == want
    manager.shutdown()
    dp = SED.wagnerFisher("ACGU", "AGU")  # the parent's own context still works
    assert dp[len(dp) - 1][len(dp[0]) - 1].value == 1


def _child_searches(query, coll, return_dict, key):
    """A forked child: the reference's per-document search, then the batched one (wfsearch), both delivered."""
    import wfsearch
    per_doc = _ref_search_collection(query, "tf", coll, wfsearch.wf_score)
    wfsearch.clear_cache()
    batched = wfsearch.search_collection(query, "tf", coll, wfsearch.wf_score)
    return_dict[key] = (per_doc, batched)


def test_concurrent_forked_children_served_by_the_parent(SED):
    """Four children forked at once from a HIP process (a multiprocessing pool's shape), each running the
    per-document and the batched search, while the parent keeps calling wagnerFisher on its own context: the
    parent serves them on as many threads and pooled contexts at the same time.  Every child's results match G7,
    and so do the parent's."""
    import multiprocessing as mp
    import seqio
    import sedgpu
    g7 = load_golden("g7_ingest_search.json")
    coll = seqio.ListCollection.from_sequences(list(g7["test_input"].values()))
    SED.wagnerFisher("AGRGA", "AGGGAA", True)
    assert isinstance(sedgpu.context(), sedgpu.Context)
    fork = mp.get_context("fork")
    manager = fork.Manager()
    out = manager.dict()
    searches = g7["searches"][:4]
    jobs = [fork.Process(target=_child_searches, args=(s["query"], coll, out, k)) for k, s in enumerate(searches)]
    for p in jobs:
        p.start()
    for _ in range(50):  # the parent's own calls while the children are served
        dp = SED.wagnerFisher("ACGU", "AGU")
        assert dp[len(dp) - 1][len(dp[0]) - 1].value == 1
    for p in jobs:
        p.join(timeout=180)
        assert p.exitcode == 0
    for k, s in enumerate(searches):
        want = [[seq, float.fromhex(h)] for seq, h in s["scores"]]
        per_doc, batched = out[k]
        assert [[a, b] for a, b in per_doc] == want, k
        assert [[a, b] for a, b in batched] == want, k
    manager.shutdown()


def test_import_time_demo_globals(SED):
    """StringEditDistance.py:459-466 leaves str1, str2, dp, all_paths, path (the last path) and es (its edit
    script) as module globals; the drop-in computes them on first access (G1 holds the same case)."""
    rec = next(r for r in load_golden("g1_small.json") if (r["s1"], r["s2"], r["user"]) == ("AGRGA", "AGGGAA", True))
    assert (SED.str1, SED.str2) == ("AGRGA", "AGGGAA")
    v = SED.dp[len(SED.dp) - 1][len(SED.dp[0]) - 1].value
    assert (float(v), isinstance(v, int)) == (float.fromhex(rec["dist"][0]), rec["dist"][1])
    assert len(SED.all_paths) == rec["npaths"]
    ops = "".join("u" if (b.i - a.i, b.j - a.j) == (1, 1) else ("d" if b.i > a.i else "i")
                  for a, b in zip(SED.path, SED.path[1:]))
    assert ops == rec["paths"][-1]
    assert SED.es == SED.generate_es(SED.path, "AGRGA", "AGGGAA")

"""Wall time of the two unchanged-caller paths that the per-call numbers of call_latency.py do not cover.

1. IRMethods.create_search_threads (IRMethods.py:480-515): the GUI process has already called wagnerFisher
   (gui.py:360, so HIP lives in the parent), then forks one multiprocessing.Process for the search
   (search_collection over every document, one wf_score = one wagnerFisher per document, IRMethods.py:435-440,
   469-470) and, after joining it, a second Process for the same search again (:511-514).  Results travel
   back through Manager dicts.  Recorded per round: the parent's start -> join wall time, the child's time to
   its first result (engine start-up inside the child), the mean of its remaining per-document calls, and the
   same search in-process, per document and batched (wfsearch.search_collection, one launch).
2. timing.py:45-57: one wagnerFisher per random 15-symbol IUPAC pair of equal lengths 10, 20, .., 500
   (costs.json, so the fp64 kernels), timed per call like the reference does.

    python tools/caller_paths.py [out.json]
"""
import json
import multiprocessing as mp
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else None
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd")]
os.chdir(os.path.join(REPO, "tests", "golden"))  # the module loads costs.json / user_costs.json from the CWD
import numpy as np  # noqa: E402

import StringEditDistance as SED  # noqa: E402
import sedgpu  # noqa: E402
import seqio  # noqa: E402
import synth  # noqa: E402
import wfsearch  # noqa: E402

NDOCS = 500


def wf_score(seq1, seq2, user_cost=False):
    """IRMethods.wf_score (IRMethods.py:435-440), as the unchanged caller has it."""
    dp = SED.wagnerFisher(seq1, seq2, user_cost)
    cost = dp[len(dp) - 1][len(dp[0]) - 1].value
    return 1 / (1 + cost)


def search_collection(query, vector_type, collection, method, return_dict=None, stamps=None, t_fork=None):
    """IRMethods.search_collection for wf_score (IRMethods.py:443-477): one call per document.  `stamps` (a
    Manager dict) receives the child's own timings: its start after the parent's Process() (t_fork, same
    monotonic clock), first result and the loop end."""
    t0 = time.perf_counter()
    if stamps is not None and t_fork is not None:
        stamps["start_ms"] = (t0 - t_fork) * 1e3
    scores, first = [], None
    for doc in collection.find({}):
        scores.append((doc['sequence'], method(query, doc['sequence'])))
        if first is None:
            first = time.perf_counter() - t0
    t1 = time.perf_counter() - t0
    if stamps is not None:
        stamps["first_ms"] = first * 1e3
        stamps["loop_ms"] = t1 * 1e3
        stamps["rest_per_call_ms"] = (t1 - first) * 1e3 / max(1, len(scores) - 1)
        c = sedgpu.context()
        stamps["engine"] = getattr(c, "served_by", None) or type(c).__name__
    if return_dict is not None:
        return_dict[method.__name__] = scores
    return scores


def batched_search(query, vector_type, collection, method, return_dict=None, stamps=None, t_fork=None):
    """The same search through wfsearch.search_collection (the drop-in for IRMethods.search_collection): one
    request to the parent's engine for all documents."""
    t0 = time.perf_counter()
    wfsearch.clear_cache()
    scores = wfsearch.search_collection(query, vector_type, collection, wfsearch.wf_score)
    t1 = time.perf_counter() - t0
    if stamps is not None:
        stamps["start_ms"] = (t0 - t_fork) * 1e3
        stamps["first_ms"] = stamps["loop_ms"] = t1 * 1e3
        stamps["rest_per_call_ms"] = 0.0
        t2 = time.perf_counter()  # the same search again in this child: the first request's set-up excluded
        wfsearch.clear_cache()
        wfsearch.search_collection(query, vector_type, collection, wfsearch.wf_score)
        stamps["second_ms"] = (time.perf_counter() - t2) * 1e3
        stamps["phases"] = search_phases(query, collection)
        prof = os.environ.get("CALLER_PATHS_PROFILE")  # a file: cProfile of one more search in this child
        if prof:
            import cProfile
            import io
            import pstats
            pr = cProfile.Profile()
            wfsearch.clear_cache()
            pr.enable()
            wfsearch.search_collection(query, vector_type, collection, wfsearch.wf_score)
            pr.disable()
            out = io.StringIO()
            pstats.Stats(pr, stream=out).sort_stats("cumulative").print_stats(25)
            with open(prof, "a") as f:
                f.write(out.getvalue())
        c = sedgpu.context()
        stamps["engine"] = (getattr(c, "served_by", None) or type(c).__name__) + ", batched"
    if return_dict is not None:
        return_dict["wf_score"] = scores
    return scores


def search_phases(query, collection, reps=5):
    """The batched search's phases, warm, in ms: the batch's cost plan, the packed codes, and the engine call (in a
    forked child: one request to the parent's serving thread)."""
    seqs = [doc['sequence'] for doc in collection.find({})]
    queries = [query] * len(seqs)
    acc = [0.0, 0.0, 0.0]
    for _ in range(reps):
        t0 = time.perf_counter()
        plan = SED.batch_plan(queries, seqs, False)
        t1 = time.perf_counter()
        packed = SED._packed(plan, queries, seqs)
        t2 = time.perf_counter()
        ctx = sedgpu.context()
        ctx.set_costs(plan)
        ctx.run(packed, False, no_len=True)
        t3 = time.perf_counter()
        acc[0] += t1 - t0
        acc[1] += t2 - t1
        acc[2] += t3 - t2
    return {k: v * 1e3 / reps for k, v in zip(("plan_ms", "pack_ms", "run_ms"), acc)}


def collection():
    ids = np.arange(NDOCS, dtype=np.uint64)
    ln = synth.lengths(ids, 24, 32)
    seqs = ["".join(synth.ALPHABET[c] for c in synth.pair_codes([i], int(n), 0)[0]) for i, n in zip(ids, ln)]
    return seqs[0], seqs, seqio.ListCollection.from_sequences(seqs)


def process_model(out):
    query, seqs, coll = collection()
    fork = mp.get_context("fork")
    manager = fork.Manager()
    SED.wagnerFisher("AGRGA", "AGGGAA", True)  # the GUI process's own call (gui.py:360): HIP in the parent
    want = search_collection(query, "tf", coll, wf_score)
    rounds = []
    # create_search_threads' two Process rounds and one more search after them (per-document wagnerFisher, the
    # unchanged caller), then three with the child on wfsearch.search_collection (one batched request)
    for rnd in range(6):
        return_dict, stamps = manager.dict(), manager.dict()
        t0 = time.perf_counter()
        target = search_collection if rnd < 3 else batched_search
        p = fork.Process(target=target, args=(query, "tf", coll, wf_score, return_dict, stamps, t0))
        p.start()
        p.join()
        wall = (time.perf_counter() - t0) * 1e3
        assert p.exitcode == 0 and list(return_dict["wf_score"]) == want
        rounds.append(dict(stamps, wall_ms=wall))
    manager.shutdown()
    # in-process references: the same per-document loop, and one batched launch (cache cleared each time)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        search_collection(query, "tf", coll, wf_score)
    loop_ms = (time.perf_counter() - t0) * 1e3 / reps
    got = None
    t0 = time.perf_counter()
    for _ in range(reps):
        wfsearch.clear_cache()
        got = wfsearch.search_collection(query, "tf", coll, wfsearch.wf_score)
    batch_ms = (time.perf_counter() - t0) * 1e3 / reps
    assert got == want
    phases = search_phases(query, coll)
    out["process_model"] = {
        "docs": NDOCS, "doc_lengths": "U[24,32] synthetic ACGU", "costs": "costs.json",
        "rounds": rounds, "inproc_per_doc_loop_ms": loop_ms, "inproc_wfsearch_batched_ms": batch_ms,
        "inproc_phases": phases,
        "fork_engine": os.environ.get("SED_FORK_ENGINE", "parent"),
    }
    for k, r in enumerate(rounds):
        print("forked search round %d (%s): wall %.1f ms, child started at %.2f ms, first result %.2f ms, loop "
              "%.2f ms, then %.4f ms per document" % (k, r["engine"], r["wall_ms"], r["start_ms"], r["first_ms"],
                                                     r["loop_ms"], r["rest_per_call_ms"])
              + ("; again in the child %.2f ms" % r["second_ms"] if "second_ms" in r else "")
              + ("; phases %s" % {k: round(v, 3) for k, v in r["phases"].items()} if "phases" in r else ""))
    print("in-process: per-document loop %.2f ms, wfsearch batched %.3f ms; phases %s"
          % (loop_ms, batch_ms, {k: round(v, 3) for k, v in phases.items()}))


def timing_loop(out):
    random.seed(20261015)
    nuc = ['A', 'G', 'C', 'U', 'Y', 'R', 'W', 'S', 'K', 'M', 'D', 'V', 'H', 'B', 'N']
    rows = []
    for rep in range(3):
        for i in range(10, 510, 10):
            s1 = "".join(random.choices(nuc, k=i))
            s2 = "".join(random.choices(nuc, k=i))
            t0 = time.perf_counter()
            dp = SED.wagnerFisher(s1, s2)
            v = dp[len(dp) - 1][len(dp[0]) - 1].value
            rows.append((rep, i, (time.perf_counter() - t0) * 1e3, v))
    last = [r for r in rows if r[0] == 2]
    per_len = {i: ms for _, i, ms, _ in last}
    total = sum(per_len.values())
    out["timing_py_loop"] = {"lengths": "10..500 step 10, one wagnerFisher per pair (timing.py:45-57)",
                             "per_call_ms_rep3": per_len, "sweep_ms_rep3": total,
                             "sweep_ms_rep1": sum(ms for r, _, ms, _ in rows if r == 0),
                             "cells_per_s_rep3": sum(i * i for i in per_len) / (total * 1e-3)}
    print("timing.py loop: sweep of 50 calls %.2f ms (first sweep %.2f ms); 10 nt %.3f ms, 250 nt %.3f ms, "
          "500 nt %.3f ms per call" % (total, out["timing_py_loop"]["sweep_ms_rep1"], per_len[10], per_len[250],
                                       per_len[500]))


if __name__ == "__main__":
    res = {}
    process_model(res)
    timing_loop(res)
    if OUT:
        with open(OUT, "w") as f:
            json.dump(res, f, indent=1)

#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE.

This script runs only in the build container (it needs /root/reference); the
fixtures it writes are small JSON files that travel with the repo.  Nothing on
the GPU box reads /root/reference.

    python -B tests/golden/make_golden.py            # G1, G2, G4, G5, G6
    python -B tests/golden/make_golden.py --g3       # the 4096^2 config-2 pair (~2 min, ~12 GB RAM)

Fixture sets:
  G1  small pairs, every co-optimal path in reference order (create_paths),
      the full DP matrix (value, int-typing, optimal-edge mask) and the ES list.
  G2  medium pairs: distance, canonical ES and a digest of the full matrix.  The
      canonical path is walked on the reference's OWN dp graph with the
      (L, insert<delete<update) rule, which G1 verifies equals create_paths(dp)[0].
  G3  config-2 pair (4096x4096 synthetic ACGU, user_costs): distance + canonical ES.
  G4  25x25 wf_score matrix over test_input.xml (IRMethods.wf_score).
  G5  generate_rev_es / generate_sequence_from_es / patching cases.
  G6  error and typing cases (KeyError, IndexError, int-zero typing).
  G7  ingest + search: import_xml on test_input.xml and on seqxml_cases.xml (T/X
      normalisation, duplicate ids), and IRMethods.search_collection(query, ..., wf_score)
      over a list-backed collection of the test_input.xml sequences.

    python -B tests/golden/make_golden.py --g7       # G7 only
    python -B tests/golden/make_golden.py --g8       # G8 only
    python -B tests/golden/make_golden.py --g9       # G9 only

  G9  FASTA ingest: the reference's fa_import.py itself (its import-time loop,
      fa_import.py:39-62) run on synthetic ./data/ocu.fa files in a scratch
      directory, with pymongo's MongoClient replaced by a list-backed collection
      (the inserted documents are recorded); data, get_all_keys() and the
      inserted sequences per file.

  G8  cost tables the GUI (gui.py:193-252) and hand-edited JSON can produce, each
      installed as the reference's user_costs global (what reload_user_costs does):
      fractional insert/delete (border products j*ins, i*del), zero and negative
      substitutions (int/float typing), substitutions dearer than insert + delete,
      int literals, a zero insert, and an integer table the packed kernel takes.
      Per table: G1-style small pairs (every path, full matrix) and G2-style
      medium pairs (canonical ES, length, matrix digest).
"""
import copy
import hashlib
import io
import json
import os
import random
import signal
import sys
import contextlib

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "rna-sequence-diff-patch_amd"))
import synth  # noqa: E402

OPS = {"insert": "i", "delete": "d", "update": "u"}
MASK = {"insert": 1, "delete": 2, "update": 4}
IUPAC = "AGCUYRWSKMDVHBN"


def load_reference():
    os.chdir(REF)
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        import StringEditDistance as S  # prints its smoke block on import
        import IRMethods as IR
        import import_xml as IX
    return S, IR, IX


def vrec(v):
    return [float(v).hex(), isinstance(v, int) and not isinstance(v, bool)]


def cell_mask(node):
    m = 0
    for e in node.incoming_edges:
        m |= MASK[e.operation]
    return m


def path_ops(path):
    out = []
    for a, b in zip(path, path[1:]):
        di, dj = b.i - a.i, b.j - a.j
        out.append("u" if (di, dj) == (1, 1) else ("d" if di == 1 else "i"))
    return "".join(out)


def es_compact(es):
    return [[OPS[e["operation"]], e["source"]["character"], e["source"]["index"],
             e["destination"]["character"], e["destination"]["index"]] for e in es]


def canonical_from_graph(dp):
    """Shortest co-optimal path, ties insert<delete<update read from the sink.

    Computed on the reference's own Node graph: L = min edge count from the
    origin over optimal (incoming) edges; at each cell take the first incoming
    edge (they are stored insert, delete, update) whose source has L = L-1.
    Returns the node path origin->sink.
    """
    rows, cols = len(dp), len(dp[0])
    L = [[0] * cols for _ in range(rows)]
    for i in range(rows):
        for j in range(cols):
            if i == 0 and j == 0:
                continue
            n = dp[i][j]
            L[i][j] = 1 + min(L[e.source.i + 1][e.source.j + 1] for e in n.incoming_edges)
    i, j = rows - 1, cols - 1
    path = [dp[i][j]]
    while (i, j) != (0, 0):
        n = dp[i][j]
        for e in n.incoming_edges:
            si, sj = e.source.i + 1, e.source.j + 1
            if L[si][sj] == L[i][j] - 1:
                i, j = si, sj
                break
        path.append(dp[i][j])
    return path[::-1], L[rows - 1][cols - 1]


def matrix_digest(dp):
    h = hashlib.sha256()
    for row in dp:
        for n in row:
            h.update(("%s|%d|%d;" % (float(n.value).hex(), int(isinstance(n.value, int)), cell_mask(n))).encode())
    return h.hexdigest()


class _Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise _Timeout()


def create_paths_or_deadlock(S, dp, seconds=0.5):
    signal.signal(signal.SIGALRM, _alarm)
    signal.setitimer(signal.ITIMER_REAL, seconds)
    try:
        return S.create_paths(dp)
    except _Timeout:
        return None
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0)


def rand_str(rng, alphabet, lo, hi):
    return "".join(rng.choice(alphabet) for _ in range(rng.randint(lo, hi)))


def gen_g1(S):
    rng = random.Random(1015)
    cases = []
    for user in (False, True):
        for alpha in ("ACGU", IUPAC):
            for _ in range(110):
                s1, s2 = rand_str(rng, alpha, 0, 7), rand_str(rng, alpha, 0, 7)
                cases.append((s1, s2, user))
    # a few hand-picked ones: the survey's deadlock example and the smoke block
    cases += [("ACGCGCG", "UUU", False), ("AGRGA", "AGGGAA", True), ("A", "CA", False),
              ("", "", False), ("", "ACG", True), ("GU", "", False), ("AAAA", "AAAA", False)]
    out = []
    for s1, s2, user in cases:
        dp = S.wagnerFisher(s1, s2, user)
        rec = {"s1": s1, "s2": s2, "user": user, "dist": vrec(dp[-1][-1].value),
               "cells": [[*vrec(n.value), cell_mask(n)] for row in dp for n in row]}
        cpath, clen = canonical_from_graph(dp)
        rec["canon"] = path_ops(cpath)
        paths = create_paths_or_deadlock(S, dp)
        if paths is None:
            rec["paths"] = "deadlock"
        else:
            ops = [path_ops(p) for p in paths]
            assert ops[0] == rec["canon"], (s1, s2, user)
            rec["npaths"] = len(ops)
            rec["paths"] = ops[:400]
            es_list = []
            for p in paths[:6]:
                try:
                    es_list.append(es_compact(S.generate_es(p, s1, s2)))
                except Exception as ex:  # IndexError on empty strings
                    es_list.append({"error": type(ex).__name__})
            rec["es"] = es_list
        out.append(rec)
    return out


def gen_g2(S):
    specs = []
    for n, m in ((64, 64), (96, 64), (256, 256), (200, 300)):
        for user in (False, True):
            specs.append(("rand", "ACGU", n, m, user))
            specs.append(("related", "ACGU", n, n, user))
            specs.append(("rand", IUPAC, n, m, user))
    specs += [("rand", "ACGU", 1024, 1024, True), ("related", "ACGU", 1024, 1024, False),
              ("rand", IUPAC, 1024, 1024, False)]
    rng = random.Random(2026)
    out = []
    for kind, alpha, n, m, user in specs:
        s1 = "".join(rng.choice(alpha) for _ in range(n))
        if kind == "related":
            s2 = "".join(c if rng.random() >= 0.1 else rng.choice(alpha) for c in s1)
        else:
            s2 = "".join(rng.choice(alpha) for _ in range(m))
        dp = S.wagnerFisher(s1, s2, user)
        cpath, clen = canonical_from_graph(dp)
        es = S.generate_es(cpath, s1, s2)
        out.append({"s1": s1, "s2": s2, "user": user, "kind": kind,
                    "dist": vrec(dp[-1][-1].value), "canon": path_ops(cpath), "len": clen,
                    "es_sha256": hashlib.sha256(json.dumps(es_compact(es)).encode()).hexdigest(),
                    "digest": matrix_digest(dp)})
        print("G2", kind, len(alpha), n, m, user, out[-1]["dist"], file=sys.stderr)
    return out


def gen_g3(S):
    s1, s2 = synth.pair_strings(0, 4096, 4096)
    dp = S.wagnerFisher(s1, s2, True)
    cpath, clen = canonical_from_graph(dp)
    ops = path_ops(cpath)
    es = es_compact(S.generate_es(cpath, s1, s2))
    return {"pair_id": 0, "base_seed": synth.BASE_SEED, "n": 4096, "m": 4096, "user": True,
            "s1_sha256": hashlib.sha256(s1.encode()).hexdigest(),
            "s2_sha256": hashlib.sha256(s2.encode()).hexdigest(),
            "dist": vrec(dp[-1][-1].value), "len": clen, "canon": ops,
            "es_sha256": hashlib.sha256(json.dumps(es).encode()).hexdigest()}


def gen_g4(IR, IX):
    seqs = IX.import_xml(os.path.join(REF, "test_input.xml"))
    ids = list(seqs)
    rec = {"ids": ids, "seqs": [seqs[k] for k in ids]}
    for user in (False, True):
        rec["wf_score_user" if user else "wf_score"] = [
            [float(IR.wf_score(seqs[a], seqs[b], user)).hex() for b in ids] for a in ids]
    return rec


def gen_g5(S):
    rng = random.Random(55)
    out = []
    pairs = [("ACG", "AG"), ("AGRGA", "AGGGAA"), ("A", "CA"), ("GAUUACA", "GCAUGCU"), ("AAAA", "AAAA")]
    for _ in range(60):
        alpha = rng.choice(("ACGU", IUPAC))
        pairs.append((rand_str(rng, alpha, 1, 12), rand_str(rng, alpha, 1, 12)))
    for s1, s2 in pairs:
        for user in (False, True):
            dp = S.wagnerFisher(s1, s2, user)
            cpath, _ = canonical_from_graph(dp)
            es = S.generate_es(cpath, s1, s2)
            rev = S.generate_rev_es(es)
            probes = [s1, s2, s1 + "A", s1[:-1], "UUUU", "", s1[::-1]]
            rec = {"s1": s1, "s2": s2, "user": user, "es": es_compact(es), "rev": es_compact(rev),
                   "seq_from_es": S.generate_sequence_from_es(es),
                   "seq_from_rev": S.generate_sequence_from_es(rev),
                   "patch_es": [[p, *S.patching(es, p)] for p in probes],
                   "patch_rev": [[p, *S.patching(rev, p)] for p in probes]}
            out.append(rec)
    return out


def gen_g6(S):
    cases = [("a", "G", False), ("A", "T", False), ("A", "T", True), ("T", "T", False),
             ("a", "A", False), ("A", "A", False), ("AT", "GA", False), ("GA", "AT", False),
             ("ACGx", "ACGU", False), ("ACGU", "xyz", False), ("aC", "Ac", False), ("", "", False),
             ("", "ACG", False), ("ACG", "", True), ("N", "N", True), ("NNA", "ANN", True),
             ("AC", "ACGT", False), ("UUx", "UU", True), ("Tx", "AG", False)]
    out = []
    for s1, s2, user in cases:
        rec = {"s1": s1, "s2": s2, "user": user}
        try:
            dp = S.wagnerFisher(s1, s2, user)
            rec["dist"] = vrec(dp[-1][-1].value)
            rec["repr"] = repr(dp[-1][-1])
            rec["matrix_repr"] = repr(dp) if len(s1) * len(s2) <= 64 else None
            try:
                paths = S.create_paths(dp)
                rec["es0"] = es_compact(S.generate_es(paths[0], s1, s2))
            except Exception as ex:
                rec["es_error"] = [type(ex).__name__, [str(a) for a in ex.args]]
        except Exception as ex:
            rec["error"] = [type(ex).__name__, [str(a) for a in ex.args]]
        out.append(rec)
    return out


SEQXML_CASES = """<?xml version="1.0"?>
<seqXML source="synthetic" seqXMLversion="0.4">
    <entry id="t-and-x"><RNAseq>ACGTTXGA</RNAseq></entry>
    <entry id="plain"><RNAseq>GGGAAAUUUCCC</RNAseq></entry>
    <entry id="dup"><RNAseq>AAAA</RNAseq></entry>
    <entry id="lower"><RNAseq>acgtx</RNAseq></entry>
    <entry id="dup"><RNAseq>TTTT</RNAseq></entry>
    <entry id="iupac"><RNAseq>RYKMSWBDHVNX</RNAseq></entry>
</seqXML>
"""


class _ListCollection:
    """pymongo-collection stand-in: find({}) over a list of {'sequence': ...} docs."""

    def __init__(self, seqs):
        self.docs = [{"sequence": s} for s in seqs]

    def find(self, flt):
        assert flt == {}
        return iter(self.docs)


def gen_g7(IR, IX):
    cases_path = os.path.join(HERE, "seqxml_cases.xml")
    with open(cases_path, "w") as f:
        f.write(SEQXML_CASES)
    seqs = IX.import_xml(os.path.join(REF, "test_input.xml"))
    docs = list(seqs.values())
    coll = _ListCollection(docs)
    searches = []
    for q in (docs[0], docs[7], docs[-1], "ACGUACGUNN"):
        scores = IR.search_collection(q, None, coll, IR.wf_score)
        searches.append({"query": q, "scores": [[s, float(v).hex()] for s, v in scores]})
    return {"test_input": seqs, "cases": IX.import_xml(cases_path), "searches": searches}


def g8_tables():
    """Cost tables reachable through the GUI's editors (float(val) writes, gui.py:193-252) or a
    hand-edited user_costs.json, derived from the shipped tables."""
    with open(os.path.join(REF, "user_costs.json")) as f:
        user = json.load(f)
    with open(os.path.join(REF, "costs.json")) as f:
        dflt = json.load(f)
    T = {}
    t = copy.deepcopy(user)
    t["insert"], t["delete"] = 0.66, 0.83
    T["frac_indel"] = t
    t = copy.deepcopy(user)
    t["update"]["A"]["C"] = 0.0
    t["update"]["G"]["U"] = 0.0
    t["update"]["Y"]["N"] = 0.0
    T["zero_sub"] = t
    t = copy.deepcopy(dflt)
    t["insert"], t["delete"] = 1.0, 2.0
    t["update"]["A"]["G"] = 7.0
    t["update"]["C"]["U"] = 3.5
    t["update"]["R"]["A"] = 4.0
    T["sub_over"] = t

    def ints(x):
        if isinstance(x, dict):
            return {k: ints(v) for k, v in x.items()}
        return int(x) if float(x).is_integer() else x
    T["int_literals"] = ints(copy.deepcopy(user))
    t = copy.deepcopy(user)
    t["insert"], t["delete"] = 3.0, 1.0
    for a, row in zip("ACGU", ((0, 2, 1, 4), (3, 0, 4, 1), (1, 4, 0, 2), (4, 1, 3, 0))):
        for b, v in zip("ACGU", row):
            t["update"][a][b] = float(v)
    T["gui_int"] = t
    t = copy.deepcopy(dflt)
    t["insert"] = 0.0
    T["zero_insert"] = t
    t = copy.deepcopy(user)
    t["update"]["A"]["G"] = -1.0
    t["update"]["U"]["C"] = -0.5
    T["negative_sub"] = t
    return T


def gen_g8(S):
    tables = g8_tables()
    rng = random.Random(8008)
    saved = S.user_costs
    out = {"tables": tables, "small": [], "medium": []}
    try:
        for name, table in tables.items():
            S.user_costs = table  # what reload_user_costs() does after the GUI rewrote user_costs.json
            for alpha in ("ACGU", IUPAC):
                for _ in range(24):
                    s1, s2 = rand_str(rng, alpha, 0, 6), rand_str(rng, alpha, 0, 6)
                    dp = S.wagnerFisher(s1, s2, True)
                    rec = {"table": name, "s1": s1, "s2": s2, "dist": vrec(dp[-1][-1].value),
                           "cells": [[*vrec(n.value), cell_mask(n)] for row in dp for n in row]}
                    cpath, clen = canonical_from_graph(dp)
                    rec["canon"] = path_ops(cpath)
                    paths = create_paths_or_deadlock(S, dp)
                    if paths is None:
                        rec["paths"] = "deadlock"
                    else:
                        ops = [path_ops(p) for p in paths]
                        assert ops[0] == rec["canon"], (name, s1, s2)
                        rec["npaths"] = len(ops)
                        rec["paths"] = ops[:200]
                    out["small"].append(rec)
            for kind, alpha, n, m in (("rand", "ACGU", 256, 256), ("related", "ACGU", 512, 512),
                                      ("rand", IUPAC, 300, 280), ("related", "ACGU", 1024, 1000)):
                s1 = "".join(rng.choice(alpha) for _ in range(n))
                if kind == "related":
                    s2 = "".join(c if rng.random() >= 0.1 else rng.choice(alpha) for c in s1)[:m]
                else:
                    s2 = "".join(rng.choice(alpha) for _ in range(m))
                dp = S.wagnerFisher(s1, s2, True)
                cpath, clen = canonical_from_graph(dp)
                es = S.generate_es(cpath, s1, s2)
                out["medium"].append({"table": name, "s1": s1, "s2": s2, "kind": kind,
                                      "dist": vrec(dp[-1][-1].value), "canon": path_ops(cpath), "len": clen,
                                      "es_sha256": hashlib.sha256(json.dumps(es_compact(es)).encode()).hexdigest(),
                                      "digest": matrix_digest(dp)})
                print("G8", name, kind, len(alpha), n, m, out["medium"][-1]["dist"], file=sys.stderr)
    finally:
        S.user_costs = saved
    return out


FASTA_CASES = {
    # multi-line records, T->U / X->N on the accumulated sequence, IUPAC codes, an empty record, duplicate
    # titles; the last record is never stored.  (Symbols outside the 15-letter alphabet -- lowercase, a
    # '\r' kept by line[:-1] -- make the reference's tf vector, IRMethods.convert_to_tf_vector, raise
    # ValueError inside fa_import, so they are not fixture material.)
    "quirks": ">piR-1 first\nACGT\nTTXA\n>piR-2\nGGGG\n>empty\n>piR-3\nAXT\nRYKM\n>piR-1 first\nUUUU\n"
              ">piR-4\nCCCC\nNN\n>last\nAAAA\n",
    "no_trailing_newline": ">a\nACGT\n>b\nTTTT\n>c\nGGXX",
}


def _fasta_cap_case():
    rng = random.Random(99)
    lines = []
    for k in range(520):  # more than the 500-record cap (fa_import.py:22)
        lines.append(">piR-ocu-%d some description\n" % k)
        seq = "".join(rng.choice("ACGTX") for _ in range(rng.randint(24, 32)))
        for a in range(0, len(seq), 10):
            lines.append(seq[a:a + 10] + "\n")
    return "".join(lines)


class _MongoStandIn:
    """pymongo.MongoClient stand-in for fa_import.py's import-time code (fa_import.py:14-16,49): no
    server; insert_one appends to a list."""

    inserted = []

    class _Coll:
        def insert_one(self, doc):
            _MongoStandIn.inserted.append(doc["sequence"])

        def find(self, flt):
            return iter([])

    class _Db:
        def __init__(self):
            self.sequences = _MongoStandIn._Coll()

    def __init__(self, *a, **k):
        self.rna_db = _MongoStandIn._Db()


def gen_g9():
    import tempfile
    import types
    cases = dict(FASTA_CASES)
    cases["cap_520_records"] = _fasta_cap_case()
    fake = types.ModuleType("pymongo")
    fake.MongoClient = _MongoStandIn
    real = sys.modules.get("pymongo")
    sys.modules["pymongo"] = fake
    out = {}
    cwd = os.getcwd()
    try:
        for name, text in cases.items():
            with tempfile.TemporaryDirectory() as tmp:
                os.mkdir(os.path.join(tmp, "data"))
                with open(os.path.join(tmp, "data", "ocu.fa"), "w", newline="") as f:
                    f.write(text)
                os.chdir(tmp)
                _MongoStandIn.inserted = []
                sys.modules.pop("fa_import", None)
                with contextlib.redirect_stdout(io.StringIO()):
                    import fa_import  # runs the reference's import loop on ./data/ocu.fa
                out[name] = {"fasta": text, "data": list(fa_import.data.items()),
                             "keys": fa_import.get_all_keys(), "inserted": list(_MongoStandIn.inserted)}
                os.chdir(cwd)
    finally:
        os.chdir(cwd)
        sys.modules.pop("fa_import", None)
        if real is not None:
            sys.modules["pymongo"] = real
        else:
            sys.modules.pop("pymongo", None)
    return out


def dump(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes", file=sys.stderr)


def main():
    S, IR, IX = load_reference()
    if "--g3" in sys.argv:
        dump("g3_config2.json", gen_g3(S))
        return
    if "--g7" in sys.argv:
        dump("g7_ingest_search.json", gen_g7(IR, IX))
        return
    if "--g8" in sys.argv:
        dump("g8_cost_tables.json", gen_g8(S))
        return
    if "--g9" in sys.argv:
        dump("g9_fasta.json", gen_g9())
        return
    dump("g1_small.json", gen_g1(S))
    dump("g6_errors.json", gen_g6(S))
    dump("g5_patching.json", gen_g5(S))
    dump("g4_wf_score.json", gen_g4(IR, IX))
    dump("g2_medium.json", gen_g2(S))
    dump("g7_ingest_search.json", gen_g7(IR, IX))
    dump("g8_cost_tables.json", gen_g8(S))
    dump("g9_fasta.json", gen_g9())


if __name__ == "__main__":
    main()

"""CPU: the pure-Python node-graph restatement (oracle/pyref.py, bench.py's reference-regime CPU baseline)
reproduces the reference's own outputs: every G1 distance (value and int typing), canonical path and the
first edit script, the G2 medium scripts, and the G8 GUI cost tables."""
from conftest import load_golden
import pyref

OPS = {"insert": "i", "delete": "d", "update": "u"}


def _es_compact(es):
    return [[OPS[e["operation"]], e["source"]["character"], e["source"]["index"],
             e["destination"]["character"], e["destination"]["index"]] for e in es]


def test_g1(tables):
    for r in load_golden("g1_small.json"):
        v, ops, es = pyref.run_pair(r["s1"], r["s2"], tables[r["user"]])
        assert (float(v), isinstance(v, int)) == (float.fromhex(r["dist"][0]), r["dist"][1]), (r["s1"], r["s2"])
        assert ops == r["canon"], (r["s1"], r["s2"])
        if r["paths"] != "deadlock" and isinstance(r["es"][0], list):
            assert _es_compact(es) == r["es"][0], (r["s1"], r["s2"])


def test_g2_medium(tables):
    for r in load_golden("g2_medium.json"):
        if len(r["s1"]) > 256:
            continue
        v, ops, _ = pyref.run_pair(r["s1"], r["s2"], tables[r["user"]])
        assert float(v) == float.fromhex(r["dist"][0]) and ops == r["canon"]


def test_g8_tables():
    g8 = load_golden("g8_cost_tables.json")
    for r in g8["small"]:
        v, ops, _ = pyref.run_pair(r["s1"], r["s2"], g8["tables"][r["table"]])
        assert (float(v), isinstance(v, int)) == (float.fromhex(r["dist"][0]), r["dist"][1]), r["table"]
        assert ops == r["canon"], (r["table"], r["s1"], r["s2"])

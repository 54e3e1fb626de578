"""CPU: the host C edit-script helpers (_sedhost, csrc/sedhost.c) against the
module's Python restatement of the reference (StringEditDistance.py:274-457, gui.py:629-657):
the G5 golden cases through both paths, and a fuzz of well-formed and malformed scripts
(negative / out-of-range indices, multi-character and non-ASCII characters, unknown
operations, missing keys) where results and exception types must agree."""
import importlib
import json
import os
import random
import sys

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
import _sedhost

OPS = {"i": "insert", "d": "delete", "u": "update"}


class _NoFast:
    """Stand-in for _sedhost that declines every call (forces the Python restatement)."""

    def __getattr__(self, name):
        return lambda *a, **k: NotImplemented


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


def both(SED, fn, *args):
    """(result-or-exception-type) of SED.fn through the C path and through the Python path."""
    out = []
    for fast in (True, False):
        saved = SED._sedhost
        if not fast:
            SED._sedhost = _NoFast()
        try:
            out.append(("ok", getattr(SED, fn)(*args)))
        except Exception as ex:  # noqa: BLE001 - comparing exception types is the point
            out.append(("err", type(ex).__name__))
        finally:
            SED._sedhost = saved
    return out


def test_g5_through_both_paths(SED):
    for r in load_golden("g5_patching.json"):
        es = [{"operation": OPS[o], "source": {"character": sc, "index": si},
               "destination": {"character": dc, "index": di}} for o, sc, si, dc, di in r["es"]]
        a, b = both(SED, "generate_rev_es", es)
        assert a == b and a[0] == "ok"
        rev = a[1]
        assert both(SED, "generate_sequence_from_es", es) == [("ok", r["seq_from_es"])] * 2
        assert both(SED, "generate_sequence_from_es", rev) == [("ok", r["seq_from_rev"])] * 2
        for probe, code, out in r["patch_es"]:
            assert both(SED, "patching", es, probe) == [("ok", (code, out))] * 2
        for probe, code, out in r["patch_rev"]:
            assert both(SED, "patching", rev, probe) == [("ok", (code, out))] * 2
        assert SED.es_to_json(es) == json.dumps({"edit_script": es}, indent=4)
        assert SED.es_to_json(rev, 2) == json.dumps({"edit_script": rev}, indent=2)


def test_rev_es_shares_dicts_like_reference(SED):
    es = _sedhost.es_from_ops(bytes([2, 0, 1, 2]), "ACG", "UAC")
    rev = SED.generate_rev_es(es)
    for e, r in zip(es, rev):
        if e["operation"] in ("insert", "update"):
            assert r["source"] is e["destination"] and r["destination"] is e["source"]
        else:
            assert r["destination"] is e["source"] and list(r["source"]) == ["index", "character"]


def test_es_from_ops_matches_records(SED):
    rng = random.Random(3)
    for _ in range(300):
        s1 = "".join(rng.choice("ACGUN") for _ in range(rng.randint(1, 12)))
        s2 = "".join(rng.choice("ACGUN") for _ in range(rng.randint(1, 12)))
        ops = [2] * min(len(s1), len(s2)) + [0] * max(0, len(s2) - len(s1)) + [1] * max(0, len(s1) - len(s2))
        rng.shuffle(ops)
        got = _sedhost.es_from_ops(bytes(ops), s1, s2)
        want, r, c = [], 0, 0
        for op in ops:
            c += op != 1
            r += op != 0
            want.append(SED._op_record(SED._OPNAME[op], s1, s2, r - 1, c - 1))
        assert got == want
    with pytest.raises(IndexError):
        _sedhost.es_from_ops(bytes([0]), "", "A")  # str1[-1] of an empty string, as the reference


def test_es_skeleton_fill_equals_es_from_ops():
    """The drop-in module builds generate_es' records during the device run (es_skeleton) and fills their values after
    it (es_fill): equal to es_from_ops whatever the skeleton's size (fewer, as many or more records than ops), with
    independent dicts per record, also on non-ASCII strings (the slow character path)."""
    rng = random.Random(4)
    for trial in range(300):
        al = "ACGUN" if trial % 10 else "ACGéU"
        s1 = "".join(rng.choice(al) for _ in range(rng.randint(1, 40)))
        s2 = "".join(rng.choice(al) for _ in range(rng.randint(1, 40)))
        ops = [2] * min(len(s1), len(s2)) + [0] * max(0, len(s2) - len(s1)) + [1] * max(0, len(s1) - len(s2))
        rng.shuffle(ops)
        want = _sedhost.es_from_ops(bytes(ops), s1, s2)
        recs, sides = _sedhost.es_skeleton(rng.choice([0, 1, max(len(s1), len(s2)), len(ops), len(ops) + 5]))
        got = _sedhost.es_fill(recs, sides, bytes(ops), s1, s2)
        assert got == want and got is recs
        assert len({id(r["source"]) for r in got} | {id(r["destination"]) for r in got}) == 2 * len(got)
    with pytest.raises(IndexError):
        recs, sides = _sedhost.es_skeleton(1)
        _sedhost.es_fill(recs, sides, bytes([0]), "", "A")


def test_es_recycle_reuses_only_unshared_records():
    """es_recycle takes a previous generate_es list as the next skeleton only when every record and side dict is held by
    the list alone, unmodified in shape: filled again, it equals es_from_ops of the new script (also with fewer or more
    records than ops); a record or side held elsewhere (rev_es shares side dicts), an added key or a reordered record is
    refused (None)."""
    rng = random.Random(5)

    def script(k):
        s1 = "".join(rng.choice("ACGU") for _ in range(rng.randint(1, 30)))
        s2 = "".join(rng.choice("ACGU") for _ in range(rng.randint(1, 30)))
        ops = [2] * min(len(s1), len(s2)) + [0] * max(0, len(s2) - len(s1)) + [1] * max(0, len(s1) - len(s2))
        rng.shuffle(ops)
        return bytes(ops), s1, s2

    for trial in range(200):
        ops, s1, s2 = script(trial)
        old = _sedhost.es_from_ops(*script(trial))
        count = rng.choice([0, 1, len(ops), len(ops) + 7])
        got = _sedhost.es_recycle(old, count)
        assert got is not None and got[0] is old and len(old) >= count
        assert _sedhost.es_fill(got[0], got[1], ops, s1, s2) == _sedhost.es_from_ops(ops, s1, s2)
    ops, s1, s2 = script(0)
    base = _sedhost.es_from_ops(ops, s1, s2)
    held = base[len(base) // 2]
    assert _sedhost.es_recycle(base, 0) is None  # a record held outside the list
    del held
    assert _sedhost.es_recycle(base, 0) is not None
    rev = _sedhost.rev_es(base)
    assert _sedhost.es_recycle(base, 0) is None  # side dicts shared with the reversed script
    del rev
    base[0]["extra"] = 1
    assert _sedhost.es_recycle(base, 0) is None
    del base[0]["extra"]
    base[0]["source"] = base[0].pop("source")  # same keys, another order
    assert _sedhost.es_recycle(base, 0) is None


def _rand_side(rng):
    d = {}
    keys = ["character", "index"]
    if rng.random() < 0.1:
        keys.reverse()
    for k in keys:
        if rng.random() < 0.03:
            continue  # missing key -> KeyError in both paths
        if k == "character":
            d[k] = rng.choice(["A", "C", "G", "U", "", "AC", "é", '"', "\\", "\n"] if rng.random() < 0.2 else "ACGU")
        else:
            d[k] = rng.randint(-12, 14) if rng.random() < 0.97 else rng.choice([2.0, "3", 10 ** 30])
    return d


def test_fuzz_c_and_python_agree(SED):
    rng = random.Random(11)
    for _ in range(3000):
        es = []
        for _ in range(rng.randint(0, 9)):
            op = rng.choice(["insert", "delete", "update"] * 10 + ["noop"])
            es.append({"operation": op, "source": _rand_side(rng), "destination": _rand_side(rng)})
        probe = "".join(rng.choice("ACGU") for _ in range(rng.randint(0, 10)))
        for fn, args in (("patching", (es, probe)), ("generate_rev_es", (es,)),
                         ("generate_sequence_from_es", (es,))):
            a, b = both(SED, fn, *args)
            assert a == b, (fn, es, probe)
        try:
            want = json.dumps({"edit_script": es}, indent=4)
        except TypeError:
            continue
        assert SED.es_to_json(es) == want


def test_save_and_load_es(SED, tmp_path):
    es = _sedhost.es_from_ops(bytes([2, 0, 1, 2, 2]), "ACGU", "GACU")
    p = tmp_path / "es.json"
    SED.save_es(str(p), es)
    assert p.read_text() == json.dumps({"edit_script": es}, indent=4)
    assert SED.load_es(str(p)) == es

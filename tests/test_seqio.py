"""CPU: sequence ingest (seqio.py) against the reference's own outputs: import_xml (G7) and
fa_import.py's import loop (G9: the reference module run on synthetic ./data/ocu.fa files with a
list-backed stand-in for its MongoDB collection, tests/golden/make_golden.py --g9)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
import seqio


def test_import_xml_matches_reference():
    g7 = load_golden("g7_ingest_search.json")
    assert seqio.import_xml(os.path.join(GOLDEN, "test_input.xml")) == g7["test_input"]
    got = seqio.import_xml(os.path.join(GOLDEN, "seqxml_cases.xml"))
    assert got == g7["cases"]
    assert list(got) == list(g7["cases"])  # dict order: first occurrence of each id


FASTA = [">piR-1 first\n", "ACGT\n", "TTXA\n", ">piR-2\n", "GGGG\n", ">empty\n", ">piR-3\n", "AXT\n",
         ">piR-4\n", "CCCC\n"]


def test_fasta_reference_quirks():
    recs = seqio.read_fasta(FASTA)
    # multi-line records joined, T->U and X->N; the empty record is not stored and its title
    # is replaced by the next one; the last record (piR-4) is never stored (fa_import.py:41-62)
    assert recs == [("piR-1 first", "ACGUUUNA"), ("piR-2", "GGGG"), ("piR-3", "ANU")]
    assert seqio.fasta_dict(FASTA) == dict(recs)
    # the 500-record cap (fa_import.py:22,49-53): the loop stops at the '>' after the cap
    assert seqio.read_fasta(FASTA, limit=2) == recs[:2]
    # line[:-1] drops the last character of an unterminated line, as the reference does
    assert seqio.read_fasta([">a\n", "ACG", ">b\n", "A\n"]) == [("a", "AC")]


def test_fasta_clean_mode(tmp_path):
    p = tmp_path / "x.fa"
    p.write_text(">a\r\nACGT\r\n>b\nGG")
    assert seqio.read_fasta(str(p), reference_quirks=False) == [("a", "ACGU"), ("b", "GG")]
    assert seqio.read_fasta(str(p)) == [("a", "ACGU")]  # text mode folds \r\n; last record dropped


def test_list_collection():
    c = seqio.ListCollection.from_fasta(FASTA)
    assert [d["sequence"] for d in c.find({})] == ["ACGUUUNA", "GGGG", "ANU"]
    assert c.count_documents({}) == 3 and len(c) == 3
    c.insert_one({"sequence": "AAA", "tf": b"x"})
    assert c.sequences()[-1] == "AAA"
    with pytest.raises(NotImplementedError):
        c.find({"sequence": "AAA"})


def test_encode_many():
    code = {ch: i for i, ch in enumerate("AGCU")}
    codes, offs, lens = seqio.encode_many(["ACG", "", "UUA"], code)
    assert codes.tolist() == [0, 2, 1, 3, 3, 0] and offs.tolist() == [0, 3, 3] and lens.tolist() == [3, 0, 3]
    with pytest.raises(KeyError) as ei:
        seqio.encode_many(["ACX"], code)
    assert ei.value.args == ("X",)
    assert seqio.encode_many([], code)[0].size == 0


@pytest.mark.parametrize("case", ["quirks", "no_trailing_newline", "cap_520_records"])
def test_fasta_matches_reference_fa_import(case):
    """G9: fa_import.data (title -> sequence, dict order), get_all_keys() and the documents it inserted
    (order, T->U / X->N, 500-record cap, the dropped last record) from the same file."""
    g9 = load_golden("g9_fasta.json")[case]
    lines = g9["fasta"].splitlines(keepends=True)
    recs = seqio.read_fasta(lines)
    assert [s for _, s in recs] == g9["inserted"]
    d = seqio.fasta_dict(lines)
    assert list(d.items()) == [tuple(x) for x in g9["data"]]
    assert list(d) == g9["keys"]
    assert seqio.ListCollection.from_fasta(lines).sequences() == g9["inserted"]

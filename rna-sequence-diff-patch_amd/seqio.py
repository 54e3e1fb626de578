"""Sequence ingest for the engine: FASTA and SeqXML readers with the
reference's normalisation, a list-backed stand-in for the MongoDB `sequences` collection,
and packing of many sequences into the engine's code arrays.

Reference behaviour mirrored here:
  * `fa_import.py:39-62`: '>' lines start a record (title = line[1:-1]); sequence lines are
    appended as line[:-1] and the *accumulated* sequence gets T->U then X->N after every
    line; a record is stored when the next '>' arrives and only if its sequence is
    non-empty; the import stops after 500 stored records (`imported = 500`, `:22`), and the
    file's last record is never stored (nothing follows it).  `reference_quirks=False`
    keeps the last record and strips line ends properly instead.
  * `import_xml.py:4-17`: every <entry id=...><RNAseq>...</RNAseq> of a SeqXML file, T->U
    then X->N, into a dict id -> sequence (later duplicates overwrite earlier ones).
  * the collection documents `{'sequence': ...}` that `IRMethods.search_collection`
    iterates with `collection.find({})` (`IRMethods.py:443-477`).
"""
import xml.etree.ElementTree as ET

import numpy as np

FASTA_LIMIT = 500  # fa_import.py:22


def _normalise(seq):
    return seq.replace('T', 'U').replace('X', 'N')


def read_fasta(source, limit=FASTA_LIMIT, reference_quirks=True):
    """[(title, sequence)] in file order (the order fa_import.py inserts documents).

    source: a path or an iterable of lines (with their '\\n').  Duplicate titles are kept
    as separate records here; `fasta_dict` gives the reference's title -> sequence dict."""
    if isinstance(source, str):
        with open(source) as f:
            return read_fasta(f.readlines(), limit, reference_quirks)
    out = []
    title, seq = '', ''
    remaining = limit
    for line in source:
        body = line[:-1] if reference_quirks else line.rstrip('\r\n')
        if line[:1] == '>':
            if seq != '':
                out.append((title, seq))
                remaining -= 1
                seq = ''
            if remaining <= 0:
                break
            title = body[1:]
        else:
            seq = _normalise(seq + body) if reference_quirks else seq + _normalise(body)
    if not reference_quirks and seq != '' and remaining > 0:
        out.append((title, seq))
    return out


def fasta_dict(source, limit=FASTA_LIMIT, reference_quirks=True):
    """fa_import.data: title -> sequence (a repeated title keeps the later sequence)."""
    return {t: s for t, s in read_fasta(source, limit, reference_quirks)}


def import_xml(file_name):
    """import_xml.import_xml: SeqXML entry id -> RNA sequence (T->U, X->N)."""
    root = ET.parse(file_name).getroot()
    out = {}
    for entry in root.findall('entry'):
        out[entry.get('id')] = _normalise(entry.find('RNAseq').text)
    return out


class ListCollection:
    """In-memory stand-in for the pymongo collection `rna_db.sequences` (fa_import.py:14-16):
    documents are dicts with at least 'sequence'; `find({})` yields them in insertion order."""

    def __init__(self, docs=()):
        self._docs = [dict(d) for d in docs]

    @classmethod
    def from_sequences(cls, seqs):
        return cls({'sequence': s} for s in seqs)

    @classmethod
    def from_fasta(cls, source, limit=FASTA_LIMIT, reference_quirks=True):
        return cls.from_sequences(s for _, s in read_fasta(source, limit, reference_quirks))

    def insert_one(self, doc):
        self._docs.append(dict(doc))

    def find(self, flt=None):
        if flt:
            raise NotImplementedError("ListCollection.find supports the empty filter only")
        return iter(list(self._docs))

    def count_documents(self, flt=None):
        if flt:
            raise NotImplementedError("ListCollection.count_documents supports the empty filter only")
        return len(self._docs)

    def sequences(self):
        return [d['sequence'] for d in self._docs]

    def __len__(self):
        return len(self._docs)


def encode_many(seqs, code_of):
    """Codes of many sequences with one lookup table: (codes u8[], offsets i64[], lengths i32[]).
    code_of: dict char -> code (CostPlan.code).  Unknown characters raise KeyError(char)."""
    lut = np.full(256, 255, np.uint8)
    for ch, c in code_of.items():
        if len(ch) == 1 and ord(ch) < 256:
            lut[ord(ch)] = c
    lens = np.array([len(s) for s in seqs], np.int32)
    offs = np.zeros(len(seqs), np.int64)
    if len(seqs):
        offs[1:] = np.cumsum(lens[:-1])
    raw = np.frombuffer(''.join(seqs).encode('latin-1'), np.uint8)
    codes = lut[raw]
    bad = np.nonzero(codes == 255)[0]
    if bad.size:
        raise KeyError(chr(raw[bad[0]]))
    return codes, offs, lens

"""Cost tables -> per-call alphabet codes and a K x K cost matrix.

Host-side half of the reference's cost model (StringEditDistance.py:6-27,
76-99).  The reference looks costs up per DP cell in a dict of dicts; the
engine instead resolves, once per call, every (str1 symbol, str2 symbol)
combination into

    sub[a][b]      the value cost(a, b) returns (int 0 when a.lower() == b.lower())
    sub_int[a][b]  1 when that value is a Python int (typing of dp values)

and raises the same KeyError the reference would raise at the first offending
cell in row-major order (insert / delete keys first, as the border loops read
them before any update lookup, StringEditDistance.py:156,174).
"""
import operator

import numpy as np

UPDATE, INSERT, DELETE = "update", "insert", "delete"


def _is_py_int(v):
    return isinstance(v, int)


class CostPlan:
    """Alphabet + resolved cost matrix for a set of (str1, str2) pairs."""

    __slots__ = ("alphabet", "code", "sub", "sub_int", "ins", "ins_int", "dele", "del_int", "_key", "_lut", "_trans")

    def __init__(self, alphabet, sub, sub_int, ins, ins_int, dele, del_int):
        self.alphabet = alphabet
        self.code = {c: k for k, c in enumerate(alphabet)}
        self.sub = sub
        self.sub_int = sub_int
        self.ins, self.ins_int, self.dele, self.del_int = ins, ins_int, dele, del_int
        self._key = (tuple(alphabet), sub.tobytes(), sub_int.tobytes(), ins, ins_int, dele, del_int)
        lut = np.full(256, 255, dtype=np.uint8)
        for c, k in self.code.items():
            if len(c) == 1 and ord(c) < 256:
                lut[ord(c)] = k
        self._lut = lut
        self._trans = lut.tobytes()  # str.encode('latin-1').translate: characters -> codes (255 = not in the alphabet)

    @property
    def K(self):
        return len(self.alphabet)

    def key(self):
        return self._key

    def encode(self, s):
        """uint8 codes of a sequence whose symbols are all in the alphabet."""
        if isinstance(s, str):
            try:
                raw = np.frombuffer(s.encode("latin-1"), dtype=np.uint8)
                out = self._lut[raw]
                if not (out == 255).any():
                    return out
            except UnicodeEncodeError:
                pass
        return np.fromiter((self.code[c] for c in s), dtype=np.uint8, count=len(s))

    def encode_many(self, strs):
        """(concatenated uint8 codes, int32 lengths) of a list of sequences: one byte translate over the joined string
        when they are latin-1 strs (the query of a one-vs-many search is encoded once), else per sequence."""
        if _all_str(strs) and self.K < 255:
            try:
                if len(strs) > 1 and strs.count(strs[0]) == len(strs):  # one query against many documents
                    one = strs[0].encode("latin-1").translate(self._trans)
                    if b"\xff" not in one:
                        return (np.frombuffer(one * len(strs), dtype=np.uint8),
                                np.full(len(strs), len(strs[0]), dtype=np.int32))
                lens = np.fromiter(map(len, strs), dtype=np.int32, count=len(strs))
                out = "".join(strs).encode("latin-1").translate(self._trans)
                if b"\xff" not in out:
                    return np.frombuffer(out, dtype=np.uint8), lens
            except UnicodeEncodeError:
                pass
        lens = np.fromiter(map(len, strs), dtype=np.int32, count=len(strs))
        parts = [self.encode(x) for x in strs]
        return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), lens

    def encode_bytes(self, s):
        """The codes of encode(s) as bytes (one translate for latin-1 strings)."""
        if isinstance(s, str) and self.K < 255:
            try:
                out = s.encode("latin-1").translate(self._trans)
                if b"\xff" not in out:
                    return out
            except UnicodeEncodeError:
                pass
        return self.encode(s).tobytes()


def _scalar(table, key):
    v = table[key]  # KeyError(key) exactly like the reference
    return float(v), 1 if _is_py_int(v) else 0


def _all_str(xs):
    return not xs or set(map(type, xs)) == {str}


_SEEN = [b""]  # symbols distinct() has met (latin-1 bytes, at most 64): one delete pass finds any others


def distinct(s):
    """The distinct symbols of a sequence in first-occurrence order (dict.fromkeys(s)).  For latin-1 strings: one
    bytes.translate pass deletes the symbols met before; the rest is found by deleting one new symbol at a time
    (the first byte left is the next new one), and the order is by first occurrence (bytes.find).  ~15 us for a
    14 000-symbol string of 4 symbols, against ~70 us for dict.fromkeys."""
    if isinstance(s, str):
        try:
            b = s.encode("latin-1")
        except UnicodeEncodeError:
            return list(dict.fromkeys(s))
        seen = _SEEN[0]
        rest = b.translate(None, seen) if seen else b
        new = b""
        while rest and len(new) < 16:
            c = rest[:1]
            new += c
            rest = rest.translate(None, c)
        if rest:  # a large alphabet: a histogram
            return sorted((chr(c) for c in np.flatnonzero(np.bincount(np.frombuffer(b, dtype=np.uint8),
                                                                          minlength=256))), key=s.find)
        if new:
            _SEEN[0] = seen + new if len(seen) + len(new) <= 64 else new
        pos = [(b.find(c), c) for c in seen if c in b] if seen else []
        pos += [(b.find(c), c) for c in new]
        pos.sort()
        return [chr(c) for _, c in pos]
    return list(dict.fromkeys(s))


def distinct_many(strs):
    """distinct over the concatenation of strs (first occurrence in order), from the distinct strings only: a
    repeated string adds no new symbol (wfsearch repeats the query once per document)."""
    return distinct("".join(dict.fromkeys(strs)))


def check_pair(table, s1, s2):
    """Raise the reference's exception for wagnerFisher(s1, s2), if any.

    Order (StringEditDistance.py:146-222): row 0 reads table['insert'] when
    len(s2) >= 1, column 0 reads table['delete'] when len(s1) >= 1, then the
    interior cells in row-major order call cost(s1[i-1], s2[j-1]).
    """
    n, m = len(s1), len(s2)
    if m >= 1:
        table[INSERT]
    if n >= 1:
        table[DELETE]
    if n == 0 or m == 0:
        return
    first_j = {c: s2.find(c) for c in distinct(s2)} if isinstance(s2, str) else {}
    if not isinstance(s2, str):
        for j, c in enumerate(s2):
            first_j.setdefault(c, j)
    bad = {}  # str1 symbol -> (first offending j, exception)
    for a in distinct(s1):
        best = None
        for b, j in first_j.items():
            if a.lower() == b.lower():
                continue
            try:
                table[UPDATE][a][b]
            except KeyError as ex:
                if best is None or j < best[0]:
                    best = (j, ex)
        if best is not None:
            bad[a] = best
    if not bad:
        return
    for a in s1:
        if a in bad:
            raise bad[a][1]


def check_batch(table, strs1, strs2, u=None):
    """check_pair over the pairs in order (the first offending pair raises), with a fast path for batches of strs
    (wfsearch, distance_batch: ~500 documents cost ~21 us each as check_pair loops): when every (str1 symbol, str2
    symbol) combination over the union alphabets of the pairs that have cells resolves, and insert / delete exist
    where the borders read them, no pair can raise and nothing else is looked up."""
    strs1, strs2 = list(strs1), list(strs2)
    if _batch_resolves(table, strs1, strs2, u):
        return
    for a, b in zip(strs1, strs2):
        check_pair(table, a, b)


def _batch_resolves(table, strs1, strs2, u=None):
    """u: (distinct_many(strs1), distinct_many(strs2)) when the caller has them (batch_plan)."""
    if not _all_str(strs1) or not _all_str(strs2):
        return False
    try:
        if any(strs2):
            table[INSERT]
        if any(strs1):
            table[DELETE]
        if all(strs1) and all(strs2):  # (every pair has cells)
            u1, u2 = u if u is not None else (distinct_many(strs1), distinct_many(strs2))
        else:
            inner = [(a, b) for a, b in zip(strs1, strs2) if a and b]
            if not inner:
                return True
            u1, u2 = distinct_many([a for a, _ in inner]), distinct_many([b for _, b in inner])
        upd = table[UPDATE]
        for a in u1:
            la = a.lower()
            row = None
            for b in u2:
                if la != b.lower():
                    if row is None:
                        row = upd[a]
                    row[b]
    except (KeyError, TypeError, IndexError, AttributeError):
        return False
    return True


_PLANS = {}  # pair_plan's cache: resolved costs -> CostPlan
_GETTERS = {}  # (sorted str1 symbols, sorted str2 symbols) -> [(str1 symbol, itemgetter of the str2 symbols it is
#               compared with, their count)] for the rows with at least one such symbol


def _row_getters(u1, u2):
    g = _GETTERS.get((u1, u2))
    if g is None:
        g = []
        for a in u1:
            la = a.lower()
            keys = [b for b in u2 if la != b.lower()]
            if keys:
                g.append((a, operator.itemgetter(*keys), len(keys)))
        if len(_GETTERS) > 4096:
            _GETTERS.clear()
        _GETTERS[(u1, u2)] = g
    return g


def pair_plan(table, s1, s2):
    """check_pair(table, s1, s2) then build_plan(table, [s1], [s2]) for one pair of non-empty strs, with the plan
    cached by the costs the pair resolves to.  The table is read on every call (the GUI edits user_costs in place,
    gui.py:193-252), and any lookup that fails goes through check_pair, which raises the reference's exception.
    The key takes the symbol sets in sorted order: two pairs over the same symbols share one plan whatever order
    the symbols first occur in (timing.py's random IUPAC pairs, wf_score's documents), so set_costs is skipped and
    no plan is rebuilt.  A plan's alphabet order is that of the first pair it was built for; codes go through
    plan.code, so any order encodes any pair over the same sets."""
    u1 = tuple(sorted(set(s1) if len(s1) <= 256 else distinct(s1)))
    u2 = tuple(sorted(set(s2) if len(s2) <= 256 else distinct(s2)))
    try:
        ins, dele = table[INSERT], table[DELETE]
        vals = []
        rows = _row_getters(u1, u2)
        if rows:
            upd = table[UPDATE]
            for a, g, cnt in rows:
                v = g(upd[a])
                vals.append(v if cnt > 1 else (v,))
    except (KeyError, TypeError, IndexError, AttributeError):
        check_pair(table, s1, s2)  # the reference's exception, if any
        return build_plan(table, [s1], [s2])
    vals = tuple(vals)
    key = (u1, u2, vals, tuple(tuple(map(type, v)) for v in vals), ins, type(ins), dele, type(dele))
    try:
        plan = _PLANS.get(key)
    except TypeError:  # unhashable cost values
        return build_plan(table, [s1], [s2])
    if plan is None:
        plan = build_plan(table, [s1], [s2])
        if len(_PLANS) > 512:
            _PLANS.clear()
        _PLANS[key] = plan
    return plan


def build_plan(table, strs1, strs2, u=None):
    """CostPlan over the union alphabet of the given sequences (already checked).  u: (distinct_many(strs1),
    distinct_many(strs2)) when the caller has them."""
    seen, seen2 = {}, {}
    if u is not None:
        seen, seen2 = dict.fromkeys(u[0], 0), dict.fromkeys(u[1], 0)
    elif _all_str(strs1) and _all_str(strs2):
        # (first occurrence over the concatenation = over the strings in order)
        seen = dict.fromkeys(distinct_many(strs1), 0)
        seen2 = dict.fromkeys(distinct_many(strs2), 0)
    else:
        for s in strs1:
            for c in distinct(s):
                seen.setdefault(c, 0)
        for s in strs2:
            for c in distinct(s):
                seen2.setdefault(c, 0)
    syms1 = list(seen)
    alphabet = syms1 + [c for c in seen2 if c not in seen]
    set1, set2 = set(syms1), set(seen2)
    K = len(alphabet)
    sub = np.zeros((K, K), dtype=np.float64)
    sub_int = np.ones((K, K), dtype=np.uint8)  # unreachable combinations: int 0
    upd = None
    for a_i, a in enumerate(alphabet):
        if a not in set1:
            continue
        for b_i, b in enumerate(alphabet):
            if b not in set2 or a.lower() == b.lower():
                continue
            if upd is None:
                upd = table[UPDATE]
            row = upd.get(a) if hasattr(upd, "get") else None
            if row is None or b not in row:
                continue  # never met as a (str1, str2) cell of a checked pair
            v = row[b]
            sub[a_i, b_i] = float(v)
            sub_int[a_i, b_i] = 1 if _is_py_int(v) else 0
    ins, ins_int = _scalar(table, INSERT) if INSERT in table else (1.0, 0)
    dele, del_int = _scalar(table, DELETE) if DELETE in table else (1.0, 0)
    if not K:
        alphabet = ["A"]
        sub = np.zeros((1, 1))
        sub_int = np.ones((1, 1), dtype=np.uint8)
    return CostPlan(alphabet, sub, sub_int, ins, ins_int, dele, del_int)

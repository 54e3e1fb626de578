"""Co-optimal paths of a DP matrix, in the reference's create_paths order, without its
exponential BFS queue.

The reference (`StringEditDistance.py:228-271`) runs a FIFO BFS from the sink over each
cell's incoming edges (stored insert, delete, update) and records a path when it reaches
the origin.  BFS pops partial paths level by level, so its output order is

    path length ascending, then the op sequence read from the sink, insert < delete < update

(verified on every G1 and G8 golden case).  Enumerating that order directly needs, per
cell, which lengths an origin->cell co-optimal path can have; with them a depth-first search
that tries insert, delete, update in turn never enters a dead end, so each path costs
O(length) and the first k paths cost O(k * length) instead of the BFS's exponential
frontier.

The lengths are kept as windows above each cell's shortest length (_sedhost.length_windows,
C): 64 * words bits per cell, exact for every path up to lmin(sink) + 64 * words - 1 ops, and
widened (recomputed with twice the words) only when the enumeration gets there.  A 4097 x
4097 matrix then needs 268 MB instead of Python bitsets of up to n + m bits per cell.  The
path count is a multi-limb row-by-row sum in C (_sedhost.count_paths).  Both fall back to
the Python restatements below when the host extension is not built.

Input everywhere is the edge mask M[(n+1) x (m+1)] of the full matrix (sed_full_matrix:
bit 1 insert from the left, 2 delete from above, 4 update from the diagonal, 8 int typing).
"""
import numpy as np

try:
    import _sedhost
except ImportError:  # host C extension not built: the Python restatements below
    _sedhost = None

_PRED = ((0, -1), (-1, 0), (-1, -1))  # insert, delete, update


def length_sets(M):
    """L[i][j] = Python-int bitset of the lengths of co-optimal origin->(i,j) paths (Python
    restatement; small matrices and the tests)."""
    M = np.asarray(M)
    n, m = M.shape[0] - 1, M.shape[1] - 1
    mk = (M & 7).tolist()
    L = [[0] * (m + 1) for _ in range(n + 1)]
    L[0][0] = 1
    for i in range(n + 1):
        Li, Lu = L[i], L[i - 1] if i else None
        row = mk[i]
        for j in range(m + 1):
            if i == 0 and j == 0:
                continue
            b = row[j]
            acc = 0
            if b & 1:
                acc |= Li[j - 1]
            if b & 2:
                acc |= Lu[j]
            if b & 4:
                acc |= Lu[j - 1]
            Li[j] = acc << 1
    return L


class LengthWindows:
    """has(i, j, length): is there a co-optimal origin->(i, j) path of that many ops."""

    def __init__(self, M, words=1):
        M = np.ascontiguousarray(np.asarray(M, dtype=np.uint8) & 7)
        self.n, self.m = M.shape[0] - 1, M.shape[1] - 1
        self.cols = self.m + 1
        self.words = words
        if _sedhost is not None:
            lo, hi, win = _sedhost.length_windows(M.tobytes(), self.n, self.m, words)
            self.lo = memoryview(lo).cast("i")
            self.hi = memoryview(hi).cast("i")
            self.win = memoryview(win).cast("Q")
            self._sets = None
        else:
            self._sets = length_sets(M)
            lo = [[(s & -s).bit_length() - 1 if s else -1 for s in row] for row in self._sets]
            hi = [[s.bit_length() - 1 if s else -1 for s in row] for row in self._sets]
            self.lo = [x for row in lo for x in row]
            self.hi = [x for row in hi for x in row]

    def exact_up_to(self):
        """Longest total path length this window answers exactly (None: unlimited)."""
        if self._sets is not None:
            return None
        return self.lo[self.n * self.cols + self.m] + 64 * self.words - 1

    def has(self, i, j, length):
        if self._sets is not None:
            return (self._sets[i][j] >> length) & 1
        c = i * self.cols + j
        d = length - self.lo[c]
        if d < 0 or d >= 64 * self.words:
            return 0
        return (self.win[c * self.words + (d >> 6)] >> (d & 63)) & 1

    def lengths_at_sink(self):
        c = self.n * self.cols + self.m
        return self.lo[c], self.hi[c]


# Windows cost 8 * words bytes per cell and every widening recomputes them in O(cells * words).  A window must cover
# [lmin(c), lmin(c) + delta] at every cell c for paths delta ops longer than the shortest (a prefix may be shortest
# while its suffix is long), so it cannot slide; the widening stops at MAX_WORDS (the C limit) or at
# SED_COPATHS_MAX_GB of windows (default 8), with a SedError that says so.
MAX_WORDS = 1024


def _wider(words, n, m, ell, lmin):
    import os
    budget = float(os.environ.get("SED_COPATHS_MAX_GB", "8")) * 1e9
    new = words * 2
    need = 8.0 * new * (n + 1) * (m + 1)
    if new > MAX_WORDS or need > budget:
        from sedgpu import SedError
        raise SedError("create_paths: paths of %d ops are %d longer than the shortest (%d); enumerating them needs "
                       "length windows of %d x 64 bits per cell (%.1f GB for %d x %d cells), past the limit of %d "
                       "words / SED_COPATHS_MAX_GB=%.3g" % (ell, ell - lmin, lmin, new, need / 1e9, n + 1, m + 1,
                                                           MAX_WORDS, budget / 1e9))
    return new


def iter_paths(M, L=None):
    """Yield every co-optimal path as uint8 op codes (0 insert, 1 delete, 2 update,
    origin -> sink) in the reference's create_paths order.

    Memory: the length windows take 8 * words bytes per cell (words = 1 covers paths up to 63 ops longer than the
    shortest; each further doubling is recomputed on demand, see _wider)."""
    M = np.asarray(M)
    n, m = M.shape[0] - 1, M.shape[1] - 1
    mk = memoryview(np.ascontiguousarray(M & 7, dtype=np.uint8).tobytes())
    cols = m + 1
    win = L if isinstance(L, LengthWindows) else LengthWindows(M)
    lo, hi = win.lengths_at_sink()
    if lo < 0:
        return
    for ell in range(lo, hi + 1):
        lim = win.exact_up_to()
        while lim is not None and ell > lim:  # beyond the window: twice as wide
            win = LengthWindows(M, _wider(win.words, n, m, ell, lo))
            lim = win.exact_up_to()
        if not win.has(n, m, ell):
            continue
        ops = []
        stack = [[n, m, ell, 0]]  # cell, remaining length, next op to try
        has = win.has
        while stack:
            top = stack[-1]
            i, j, r, k = top
            if r == 0:  # at the origin (the only cell with a length-0 path)
                yield np.array(ops[::-1], np.uint8)
                stack.pop()
                if ops:
                    ops.pop()
                continue
            b = mk[i * cols + j]
            for op in range(k, 3):
                if b & (1 << op):
                    di, dj = _PRED[op]
                    if has(i + di, j + dj, r - 1):
                        top[3] = op + 1
                        stack.append([i + di, j + dj, r - 1, 0])
                        ops.append(op)
                        break
            else:
                stack.pop()
                if ops:
                    ops.pop()


def count_paths(M):
    """Number of co-optimal paths (exact Python int)."""
    M = np.asarray(M)
    n, m = M.shape[0] - 1, M.shape[1] - 1
    if _sedhost is not None:
        return _sedhost.count_paths(np.ascontiguousarray(M & 7, dtype=np.uint8).tobytes(), n, m)
    return _count_paths_py(M)


def _count_paths_py(M):
    """Python restatement: anti-diagonal by anti-diagonal with object arrays (two diagonals live)."""
    n, m = M.shape[0] - 1, M.shape[1] - 1
    zero = np.zeros(n + 2, dtype=object)
    d2 = zero.copy()  # diagonal d-2, indexed by row i (+1 offset so i-1 = -1 reads 0)
    d1 = zero.copy()
    d1[1] = 1  # origin, diagonal 0
    if n == 0 and m == 0:
        return 1
    for d in range(1, n + m + 1):
        lo, hi = max(0, d - m), min(n, d)
        i = np.arange(lo, hi + 1)
        b = M[i, d - i].astype(np.int64)
        cur = zero.copy()
        left = np.where(b & 1, d1[i + 1], 0)          # (i, j-1) on diagonal d-1
        up = np.where(b & 2, d1[i], 0)                # (i-1, j) on diagonal d-1
        dg = np.where(b & 4, d2[i], 0)                # (i-1, j-1) on diagonal d-2
        cur[i + 1] = left + up + dg
        d2, d1 = d1, cur
    return int(d1[n + 1])

"""TEST INFRASTRUCTURE — the reference's own cost regime, restated in pure Python.

bench.py's second CPU-baseline leg and tests/test_pyref.py use this module; the
product path never imports it.  It reproduces how StringEditDistance.py computes, not just what: one
Python object per DP cell with Python lists of incoming/outgoing edge objects (a-4, a-5), the candidate
list with Python's min() and the == tie list per cell (a-2, a-3), then the canonical path over the
object graph (a-6, the L rule that equals create_paths(dp)[0]) and the edit-script dicts (a-7).  So its
cells/s is the reference regime (~1.5e5 cells/s per core), timed on the GPU box where the
reference itself cannot travel.

Cited semantics (plsakr/rna-sequence-diff-patch, StringEditDistance.py):
  cost           :76-89    int 0 on a case-insensitive match, else table['update'][c1][c2]
  min_cost       :92-128   candidates [insert, delete, update], each one float add; min(); == ties
  wagnerFisher   :133-224  border products j*insert / i*delete, one node per cell, an edge per tie
  create_paths[0]:228-271  shortest co-optimal path, insert < delete < update read from the sink
  generate_es    :274-334  one dict per edge, index -1 / str[-1] on the borders
"""

INSERT, DELETE, UPDATE = "insert", "delete", "update"


class Link:
    """An optimal predecessor edge (StringEditDistance.py:31-40)."""
    __slots__ = ("src", "dst", "op")

    def __init__(self, src, dst, op):
        self.src, self.dst, self.op = src, dst, op


class Cell:
    """One DP cell (StringEditDistance.py:43-71): string indices (row-1, col-1), value, edges."""
    __slots__ = ("i", "j", "value", "out", "inc")

    def __init__(self, i, j, value):
        self.i, self.j, self.value = i, j, value
        self.out, self.inc = [], []

    def link(self, nxt, op):
        e = Link(self, nxt, op)
        self.out.append(e)
        nxt.inc.append(e)


def sub_cost(table, a, b):
    if a.lower() == b.lower():
        return 0
    return table["update"][a][b]


def build(s1, s2, table):
    """The node graph of wagnerFisher(s1, s2) under `table`."""
    n, m = len(s1), len(s2)
    ins, dele = table["insert"], table["delete"]
    grid = [[None] * (m + 1) for _ in range(n + 1)]
    grid[0][0] = Cell(-1, -1, 0)
    for j in range(1, m + 1):
        c = Cell(-1, j - 1, j * ins)
        grid[0][j - 1].link(c, INSERT)
        grid[0][j] = c
    for i in range(1, n + 1):
        c = Cell(i - 1, -1, i * dele)
        grid[i - 1][0].link(c, DELETE)
        grid[i][0] = c
    for i in range(1, n + 1):
        above, row = grid[i - 1], grid[i]
        a = s1[i - 1]
        for j in range(1, m + 1):
            preds = (row[j - 1], above[j], above[j - 1])
            cand = [preds[0].value + ins, preds[1].value + dele, preds[2].value + sub_cost(table, a, s2[j - 1])]
            best = min(cand)
            c = Cell(i - 1, j - 1, best)
            for k in [k for k, v in enumerate(cand) if v == best]:
                preds[k].link(c, (INSERT, DELETE, UPDATE)[k])
            row[j] = c
    return grid


def canonical_path(grid):
    """create_paths(dp)[0]: per cell L = fewest edges from the origin over optimal edges; from the sink take
    the first incoming edge (insert, delete, update order) whose source has L - 1.  Origin -> sink."""
    rows, cols = len(grid), len(grid[0])
    L = {}
    for r in range(rows):
        for c in range(cols):
            cell = grid[r][c]
            L[id(cell)] = 0 if (r, c) == (0, 0) else 1 + min(L[id(e.src)] for e in cell.inc)
    cell = grid[rows - 1][cols - 1]
    path = [cell]
    while cell.inc:
        want = L[id(cell)] - 1
        cell = next(e.src for e in cell.inc if L[id(e.src)] == want)
        path.append(cell)
    return path[::-1]


def edit_script(path, s1, s2):
    """generate_es: one dict per edge of the path (matches are updates), -1 indices on the borders."""
    es = []
    for cur, nxt in zip(path, path[1:]):
        op = next(e.op for e in cur.out if e.dst is nxt)
        es.append({"operation": op, "source": {"character": s1[nxt.i], "index": nxt.i},
                   "destination": {"character": s2[nxt.j], "index": nxt.j}})
    return es


def run_pair(s1, s2, table, script=True):
    """(distance value, canonical op string, edit script or None) the reference regime's way."""
    grid = build(s1, s2, table)
    value = grid[-1][-1].value
    if not script:
        return value, None, None
    path = canonical_path(grid)
    ops = "".join("u" if (b.i - a.i, b.j - a.j) == (1, 1) else ("d" if b.i > a.i else "i")
                  for a, b in zip(path, path[1:]))
    es = edit_script(path, s1, s2) if s1 and s2 else None
    return value, ops, es

"""Per-tile dumps of the checkpoint traceback for one failing pair, from a -DSED_TB_DEBUG build (SED_LIBRARY):
pair 0 = the 208 x 106 costs.json pair that the select-free hold (SED_CK_VHOLD) fails, then 40 dummy pairs whose
script words hold the dumps (136 words per tile visit: entry keys, initial keys, i, j, c, Q, k, sig_end, re, q).
Prints one JSON line {lib, err, visits, tiles: [...]}."""
import json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import sedcost, sedgpu
from test_gpu_parity import _random_pairs

table = json.load(open(os.path.join(REPO, "tests", "golden", "costs.json")))
pairs = _random_pairs(900, 24, "ACGU", 1, 2600, related=True) + _random_pairs(910, 16, "ACGU", 1, 1500)
a0, b0 = pairs[31]
assert (len(a0), len(b0)) == (208, 106), (len(a0), len(b0))
rng = np.random.default_rng(5)
dummy = ["".join(rng.choice(list("ACGU"), size=2000)) for _ in range(400)]
A = [a0] + dummy[:200]
B = [b0] + dummy[200:]
plan = sedcost.build_plan(table, A, B)
ctx = sedgpu.Context(0)
ctx.set_costs(plan)
for k, v in ((sedgpu.SED_OPT_TB, 2), (sedgpu.SED_OPT_ROWS_PER_LANE, 16), (sedgpu.SED_OPT_SPLIT, 2), (sedgpu.SED_OPT_LANE, 2)):
    ctx.set_option(k, v)
packed = sedgpu.PackedPairs([plan.encode(x) for x in A], [plan.encode(y) for y in B])
dist, is_int, ln, ops = ctx.run(packed, True)
w = np.asarray(ops, dtype=np.uint32)
base = (208 + 106 + 15) // 16 + 64
info = int(w[base - 1])
tiles = []
for v in range(min(32, info >> 8)):
    d = w[base + 136 * v: base + 136 * (v + 1)]
    tiles.append({"ent": [int(x) for x in d[:64]], "vinit": [int(x) for x in d[64:128]], "coord": [int(x) for x in d[128:136]]})
steps = w[base + 136 * 32: base + 136 * 32 + 3 * 64 * 127].reshape(127, 3, 64)
print(json.dumps({"lib": os.path.basename(sedgpu.LIB_PATH), "err": info & 255, "visits": info >> 8, "tiles": tiles,
                  "steps": [[[int(x) for x in r] for r in st] for st in steps]}), flush=True)

"""Debug probe for the dot-key checkpoint forward kernel: distances and lengths of the forward kernel alone
(SED_DEBUG_NOTB=1 skips the traceback) against the C oracle, with and without dot keys."""
import os, sys
os.environ["SED_DEBUG_NOTB"] = "1"
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "rna-sequence-diff-patch_amd")]
import numpy as np
from conftest import load_golden
import oracle, sedcost, sedgpu

ctx = sedgpu.Context(0)
rng = np.random.default_rng(5)
CHAIN = len(sys.argv) > 1 and sys.argv[1] == "chain"
cases = ([(100, 100), (64, 64), (1, 1), (5, 70), (256, 200), (250, 700), (3, 3), (200, 64)] if CHAIN else
         [(100, 100), (64, 64), (1, 1), (5, 70), (300, 200), (1024, 1024), (1030, 700), (2000, 2600)])
pairs = []
for n, m in cases:
    a = "".join(rng.choice(list("ACGU"), size=n))
    b = "".join(c if rng.random() > 0.2 else rng.choice(list("ACGU")) for c in a)[:m].ljust(m, "G")
    pairs.append((a, b))
for user in (False, True):
    table = load_golden("user_costs.json" if user else "costs.json")
    plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
    cs = oracle.Costs.from_plan(plan)
    ctx.set_costs(plan)
    packed = sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(b) for _, b in pairs])
    for dot in (0, 2):
        ctx.set_option(sedgpu.SED_OPT_TB, 1 if CHAIN else 2)
        ctx.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, 4 if CHAIN else 16)
        ctx.set_option(sedgpu.SED_OPT_CHAIN, 1 if CHAIN else 0)
        ctx.set_option(sedgpu.SED_OPT_SPLIT, 2)
        ctx.set_option(sedgpu.SED_OPT_LANE, 2)
        ctx.set_option(sedgpu.SED_OPT_DOT, dot)
        b = sedgpu.Batch(ctx, packed, True)
        b.run()
        dist, is_int, ln, ops = b.results()
        print("user", user, "dot_keys", b.dot_keys, "ladder", b.ladder_dot_keys, "chains", b.chains)
        b.close()
        for p, (x, y) in enumerate(pairs):
            o = oracle.pair(cs, plan.encode(x), plan.encode(y))
            print("  %5d x %5d  gpu %8.1f %6d  oracle %8.1f %6d  %s" % (len(x), len(y), dist[p], ln[p], o["dist"], o["len"],
                  "ok" if (dist[p], ln[p]) == (o["dist"], o["len"]) else "MISMATCH"))

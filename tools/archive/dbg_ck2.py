"""ck2 traceback debug: small pairs through the checkpoint route, GPU vs oracle, tile visits printed (debug lib)."""
import os, sys, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("rna-sequence-diff-patch_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, p))
import sedgpu, sedcost, oracle
table = json.load(open(os.path.join(REPO, "tests", "golden", "user_costs.json")))
ctx = sedgpu.Context(0)
plan = sedcost.build_plan(table, ["ACGU"], ["ACGU"])
ctx.set_costs(plan)
cs = oracle.Costs.from_plan(plan)
rng = np.random.default_rng(11)
for R in (16, 4):
    ctx.set_option(sedgpu.SED_OPT_TB, 2)
    ctx.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, R)
    ctx.set_option(sedgpu.SED_OPT_DOT, 2)
    for npairs, n, m in ((1, 40, 50), (1, 100, 90), (2, 100, 90), (1, 700, 650)):
        A = [rng.integers(0, 4, n).astype(np.uint8) for _ in range(npairs)]
        B = [rng.integers(0, 4, m).astype(np.uint8) for _ in range(npairs)]
        pk = sedgpu.PackedPairs(A, B)
        print("=== R", R, "npairs", npairs, n, m, flush=True)
        try:
            d, ii, ln, ops = ctx.run(pk, True)
            bad = []
            for p in range(npairs):
                o = oracle.pair(cs, A[p], B[p])
                g = sedgpu.unpack_ops(ops, pk.ops_off, p, int(ln[p]))
                if not (d[p] == o["dist"] and ln[p] == o["len"] and np.array_equal(g, o["ops"])):
                    bad.append(p)
            print("result ok" if not bad else "MISMATCH %s" % bad, flush=True)
        except sedgpu.SedError as ex:
            print("ERROR", ex, flush=True)
        for p in range(npairs):
            o = oracle.pair(cs, A[p], B[p])
            print("oracle pair", p, "dist", o["dist"], "len", o["len"], flush=True)

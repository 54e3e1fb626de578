"""GPU diagnostic: fp64 kernel (unmasked ramp) vs the oracle on tall/narrow shapes."""
import os, sys, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("rna-sequence-diff-patch_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import sedgpu, sedcost, oracle
table = json.load(open(os.path.join(REPO, "tests", "golden", "costs.json")))
ctx = sedgpu.Context(0)
rng = np.random.default_rng(5)
for alpha, mode in (("ACGU", 2), ("AGCUYRWSKMDVHBN", 0)):
    plan = sedcost.build_plan(table, [alpha], [alpha])
    ctx.set_costs(plan)
    ctx.set_mode(mode)
    cs = oracle.Costs.from_plan(plan)
    for n in (1, 63, 64, 65, 600, 1000, 5000, 70000):
        for m in (1, 2, 5, 40, 100, 700):
            if n * m > 2e7:
                continue
            a = rng.integers(0, len(alpha), n).astype(np.uint8)
            b = rng.integers(0, len(alpha), m).astype(np.uint8)
            pk = sedgpu.PackedPairs([a], [b])
            for script in (False, True):
                d, ii, ln, ops = ctx.run(pk, script)
                o = oracle.pair(cs, a, b)
                ok = d[0] == o["dist"] and ln[0] == o["len"]
                if not ok:
                    print("MISMATCH", alpha[:5], mode, n, m, script, d[0], o["dist"], ln[0], o["len"], flush=True)
    print("done", alpha, flush=True)

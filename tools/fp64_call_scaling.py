"""Engine time of one fp64 wagnerFisher call (costs.json, random IUPAC pairs of equal length) by length: the
per-call cost of timing.py's loop (timing.py:45-57) split by pair size, on the automatic route, with SPLIT forced
(SED_OPT_SPLIT = 1: one workgroup per 256-row stripe) and without it (= 2: one wave per pair).

    python tools/fp64_call_scaling.py [out.txt]
"""
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else None
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd")]
os.chdir(os.path.join(REPO, "tests", "golden"))  # the module loads costs.json from the CWD
import StringEditDistance as SED  # noqa: E402
import sedcost  # noqa: E402
import sedgpu  # noqa: E402

NUC = ['A', 'G', 'C', 'U', 'Y', 'R', 'W', 'S', 'K', 'M', 'D', 'V', 'H', 'B', 'N']


def timed(ctx, table, pairs, script):
    ts = []
    for a, b in pairs:
        plan = sedcost.pair_plan(table, a, b)
        ctx.set_costs(plan)
        ea, eb = plan.encode_bytes(a), plan.encode_bytes(b)
        t0 = time.perf_counter()
        ctx.run_pair(ea, eb, script, no_len=not script)
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[2:])
    return "%s %.1f us (min %.1f)" % ("script" if script else "distance", ts[len(ts) // 2] * 1e6, ts[0] * 1e6)


def main():
    lines = []
    table = SED._table(False)
    ctx = sedgpu.context()
    SED.wagnerFisher("AGRGA", "AGGGAA")  # start-up
    random.seed(11)
    for n in (10, 30, 60, 100, 200, 300, 400, 500, 1000, 2000):
        pairs = [("".join(random.choices(NUC, k=n)), "".join(random.choices(NUC, k=n))) for _ in range(12)]
        for split in (0, 1, 2):
            ctx.set_option(sedgpu.SED_OPT_SPLIT, split)
            row = [timed(ctx, table, pairs, script) for script in (False, True)]
            lines.append("n = m = %4d, split %d: " % (n, split) + ", ".join(row))
            print(lines[-1], flush=True)
    ctx.set_option(sedgpu.SED_OPT_SPLIT, 0)
    if OUT:
        with open(OUT, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()

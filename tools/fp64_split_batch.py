"""fp64 batches of many long pairs: the automatic route (SPLIT for <= 256 pairs with wave pairs, sed_runtime.cpp
fill_batch) against SPLIT forced (SED_OPT_SPLIT = 1) and one wave per pair (= 2).  Random IUPAC pairs of equal length
under costs.json, P pairs per batch, scripts and distances with length (many-pair fp64 batches, e.g.
wf_scores with user costs against a few hundred long documents).  Prints one line per (P, length, flags) with the
median engine time of 5 calls and SPLIT's task count.

    python tools/fp64_split_batch.py [out.txt]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else None
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd")]
import json  # noqa: E402
import sedcost  # noqa: E402
import sedgpu  # noqa: E402

NUC = list("AGCUYRWSKMDVHBN")


def main():
    with open(os.path.join(REPO, "tests", "golden", "costs.json")) as f:
        table = json.load(f)
    ctx = sedgpu.Context(0)
    rng = np.random.default_rng(5)
    lines = []
    # P x n [x m] (m = n when omitted)
    sizes = [tuple(int(v) for v in x.split("x")) for x in os.environ.get(
        "SED_SPLIT_SIZES", "16x1000,64x500,64x1000,64x2000,128x1000,128x2000,256x500,256x1000,256x2000").split(",")]
    for size in sizes:
        P, L, M = size[0], size[1], size[2] if len(size) > 2 else size[1]
        pairs = [("".join(rng.choice(NUC, size=L)), "".join(rng.choice(NUC, size=M))) for _ in range(P)]
        plan = sedcost.build_plan(table, [a for a, _ in pairs], [b for _, b in pairs])
        ctx.set_costs(plan)
        packed = sedgpu.PackedPairs([plan.encode(a) for a, _ in pairs], [plan.encode(b) for _, b in pairs])
        for script in (True, False):
            row, ref = [], None
            for split in (0, 1, 2):
                ctx.set_option(sedgpu.SED_OPT_SPLIT, split)
                b = sedgpu.Batch(ctx, packed, script)
                tasks = b.split_tasks
                b.close()
                ts = []
                for _ in range(6):
                    t0 = time.perf_counter()
                    out = ctx.run(packed, script)
                    ts.append(time.perf_counter() - t0)
                if ref is None:
                    ref = out
                else:  # same results on every route
                    assert all(np.array_equal(x, y) for x, y in zip(out, ref) if x is not None), (P, L, split)
                ts = sorted(ts[1:])
                row.append("split %d %7.2f ms (tasks %d)" % (split, ts[len(ts) // 2] * 1e3, tasks))
            ctx.set_option(sedgpu.SED_OPT_SPLIT, 0)
            lines.append("P %3d  %4d x %4d  %-8s " % (P, L, M, "script" if script else "distance") + "  ".join(row))
            print(lines[-1], flush=True)
    ctx.close()
    if OUT:
        with open(OUT, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()

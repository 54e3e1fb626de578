"""Model of the checkpoint traceback's tile visits (sed_kernels.hip: ck_traceback_pair) on config 4's pairs: the oracle's
canonical path of synthetic 4096 x 4096 pairs (user_costs.json, bench.py's generator) is walked through the kernel's
visit geometry (stripes of 64 R rows, row groups of 64 rows, chunks of 64 forward steps; R = 16) and each visit is
priced at 6 VALU per sweep step (the step: DPP add, perm, add, min3, and, alignbit) plus a fixed per-visit setup.

    python3 tools/tb_window_model.py [pairs]

Windows: one chunk per visit (the round-5 kernel), or two chunks (ce - 1, ce) when the entry step x inside its chunk
is below the entry row re (SED_CKTB_NW = 12), or always two.  Test and design infrastructure: uses oracle/."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rna-sequence-diff-patch_amd"), os.path.join(REPO, "oracle")]
import oracle  # noqa: E402
import sedcost  # noqa: E402
import synth  # noqa: E402

R, G, ROWS = 16, 4, 1024


def paths(npairs):
    table = json.load(open(os.path.join(REPO, "tests", "golden", "user_costs.json")))
    cs = oracle.Costs.from_plan(sedcost.build_plan(table, [synth.ALPHABET], [synth.ALPHABET]))
    out = []
    for pid in range(npairs):
        a = synth.pair_codes(np.array([pid], np.uint64), 4096, 0)[0]
        b = synth.pair_codes(np.array([pid], np.uint64), 4096, 1)[0]
        out.append(oracle.pair(cs, a, b)["ops"])
    return out


def simulate(ops_list, extra, setup=175):
    """extra(re, x, ce) -> chunks added left of the entry chunk; returns visits, sweep steps, ops, VALU per op."""
    visits = steps = nops = 0
    for ops in ops_list:
        q = len(ops)
        i = j = 4096
        while i > 0 and j > 0:
            t = ((i - 1) % ROWS) // R
            ce = (j - 1 + t) >> 6
            rowbase = (i - 1) // ROWS * ROWS + 64 * (t // G)
            re, x = i - rowbase - 1, (j - 1 + t) & 63
            e = extra(re, x, ce)
            visits += 1
            steps += x + 64 * e + re - (G - 2)
            while i > 0 and j > 0:  # the walk inside the window: rows of the group, chunks ce - e .. ce
                tt = ((i - 1) % ROWS) // R
                if not (rowbase <= i - 1 < rowbase + 64 and ce - e <= (j - 1 + tt) >> 6 <= ce):
                    break
                op = ops[q - 1]
                q -= 1
                j -= op != 1
                i -= op != 0
        nops += len(ops)
    return visits, steps, nops, (6 * steps + setup * visits) / nops


def main():
    ps = paths(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
    rules = [("one chunk", lambda re, x, ce: 0),
             ("two chunks when x < re", lambda re, x, ce: int(ce >= 1 and x < re)),
             ("always two chunks", lambda re, x, ce: int(ce >= 1)),
             ("always three chunks", lambda re, x, ce: min(ce, 2))]
    for name, rule in rules:
        v, s, o, vpo = simulate(ps, rule)
        print("%-24s visits/pair %6.1f  sweep steps/visit %6.1f  ops/visit %5.1f  VALU/op %5.2f" % (
            name, v / len(ps), s / v, o / v, vpo))


if __name__ == "__main__":
    main()

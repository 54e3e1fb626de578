"""Lengths of the band-map walks (sed_tb_bandmap_kernel: one lane per 64-row band and entry column, walking the
canonical codes up to the band's top row) on config 2's 4096 x 4096 pair (user_costs.json), from the oracle's edge
mask (update preferred over delete over insert where several are optimal: an approximation of the canonical codes
that keeps the path structure).  Prints the walk length percentiles and those of the longest walk per 64 lanes (a
wave's time).  Test and design infrastructure: uses oracle/.

    python3 tools/tbmap_walks.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd"), os.path.join(REPO, "oracle")]
import oracle  # noqa: E402
import sedcost  # noqa: E402
import synth  # noqa: E402


def main():
    table = json.load(open(os.path.join(REPO, "tests", "golden", "user_costs.json")))
    s1, s2 = synth.pair_strings(0, 4096, 4096)
    plan = sedcost.pair_plan(table, s1, s2)
    a = np.frombuffer(plan.encode_bytes(s1), np.uint8)
    b = np.frombuffer(plan.encode_bytes(s2), np.uint8)
    M = oracle.pair(oracle.Costs.from_plan(plan), a, b, full=True)["M"]
    n, m = len(a), len(b)
    op = np.where(M & 4, 2, np.where(M & 2, 1, 0)).astype(np.int8)
    lens = []
    for g in range(1, (n + 63) // 64):
        top = 64 * g
        i = np.full(m + 1, min(64 * (g + 1), n), np.int64)
        j = np.arange(m + 1, dtype=np.int64)
        cnt = np.zeros(m + 1, np.int64)
        run = np.zeros(m + 1, np.int64)
        live = j > 0
        while live.any():
            idx = np.flatnonzero(live)
            o = op[i[idx], j[idx]]
            cnt[idx] += 1
            run[idx] = np.where(o == 0, run[idx] + 1, 0)
            i[idx] -= o != 0
            j[idx] -= o != 1
            live[idx] = (i[idx] > top) & (j[idx] > 0) & (run[idx] <= 96)
        lens.append(cnt)
    L = np.concatenate(lens)
    W = np.concatenate([np.maximum.reduceat(c[:len(c) // 64 * 64], np.arange(0, len(c) // 64 * 64, 64)) for c in lens])
    print("walk length percentiles 50/90/99/99.9/100:", np.percentile(L, [50, 90, 99, 99.9, 100]))
    print("longest walk per 64 lanes, percentiles 50/90/99/100:", np.percentile(W, [50, 90, 99, 100]), "mean %.1f" % W.mean())


if __name__ == "__main__":
    main()

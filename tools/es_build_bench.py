"""Host cost of generate_es' records for config 2's 4096^2 script (4233 records), CPU only: es_from_ops (build with
values), es_skeleton (the records with None values, what the drop-in module can build while the device computes)
then es_fill (the values), and freeing the list.  Median of 40 of each, after a warm-up.

    python tools/es_build_bench.py
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd"), os.path.join(REPO, "oracle")]
import json  # noqa: E402
import _sedhost  # noqa: E402
import oracle  # noqa: E402
import sedcost  # noqa: E402
import synth  # noqa: E402


def med(f, k=40):
    ts = []
    for _ in range(k + 2):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[2:])
    return ts[len(ts) // 2] * 1e3


def main():
    s1, s2 = synth.pair_strings(0, 4096, 4096)
    with open(os.path.join(REPO, "tests", "golden", "user_costs.json")) as f:
        table = json.load(f)
    plan = sedcost.pair_plan(table, s1, s2)
    o = oracle.pair(oracle.Costs.from_plan(plan), plan.encode(s1), plan.encode(s2))
    ops = np.asarray(o["ops"], np.uint8).tobytes()
    n = len(ops)
    ref = _sedhost.es_from_ops(ops, s1, s2)
    sk = _sedhost.es_skeleton(4096)
    assert _sedhost.es_fill(sk[0], sk[1], ops, s1, s2) == ref
    keep = []
    print("records %d" % n)
    print("es_from_ops          %.3f ms" % med(lambda: keep.append(_sedhost.es_from_ops(ops, s1, s2))))
    lists = list(keep)
    keep.clear()
    print("free (del list)      %.3f ms" % med(lambda: lists.pop().__len__()))  # the pop drops the last reference
    sks = []
    print("es_skeleton(4096)    %.3f ms" % med(lambda: sks.append(_sedhost.es_skeleton(4096))))
    print("es_fill              %.3f ms" % med(lambda: keep.append(_sedhost.es_fill(*sks.pop(), ops, s1, s2))))


if __name__ == "__main__":
    main()

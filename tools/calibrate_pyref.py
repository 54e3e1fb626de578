#!/usr/bin/env python3
"""Calibrate oracle/pyref.py (the bench's reference-regime CPU leg) against the reference's own
StringEditDistance.wagnerFisher, timed on the same core in this container (the reference never travels to the
GPU box, so the bench can only time the restatement there).

Both run distance-only (wagnerFisher builds the whole node graph either way; the reference's create_paths is
exponential and cannot produce a script at these sizes) on the same synthetic ACGU pairs, one process each, pinned
to one core, best of 3.  The ratio reference / pyref (cells/s) goes to profiles/r03/pyref_calibration.json, which
bench.py prints in its python_node_graph object.

    python tools/calibrate_pyref.py [--core 2]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

CHILD = r'''
import io, json, os, sys, time, contextlib
which, n, table_name = sys.argv[1], int(sys.argv[2]), sys.argv[3]
sys.path.insert(0, os.path.join(%(repo)r, "rna-sequence-diff-patch_amd"))
import synth
a = "".join("ACGU"[c] for c in synth.pair_codes([7], n, 0)[0])
b = "".join("ACGU"[c] for c in synth.pair_codes([7], n, 1)[0])
user = table_name == "user_costs.json"
if which == "reference":
    os.chdir(%(ref)r)
    sys.path.insert(0, %(ref)r)
    with contextlib.redirect_stdout(io.StringIO()):  # the module prints its demo on import
        import StringEditDistance as SED
    run = lambda: SED.wagnerFisher(a, b, user)
    val = lambda dp: dp[n][n].value
else:
    sys.path.insert(0, os.path.join(%(repo)r, "oracle"))
    import pyref
    with open(os.path.join(%(repo)r, "tests", "golden", table_name)) as f:
        table = json.load(f)
    run = lambda: pyref.build(a, b, table)
    val = lambda g: g[n][n].value
best = 1e9
for _ in range(3):
    t0 = time.perf_counter()
    out = run()
    best = min(best, time.perf_counter() - t0)
    v = val(out)
    del out
print(json.dumps({"which": which, "n": n, "seconds": best, "cells_per_s": n * n / best, "dist": v}))
''' % {"repo": REPO, "ref": REF}


def run(which, n, table, core):
    cmd = ["taskset", "-c", str(core), sys.executable, "-B", "-c", CHILD, which, str(n), table]
    return json.loads(subprocess.check_output(cmd, text=True).strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--core", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "pyref_calibration.json"))
    args = ap.parse_args()
    rows = []
    for table in ("costs.json", "user_costs.json"):
        for n in (256, 512):
            r = run("reference", n, table, args.core)
            p = run("pyref", n, table, args.core)
            assert r["dist"] == p["dist"], (r, p)
            rows.append({"table": table, "n": n, "reference_cells_per_s": r["cells_per_s"],
                         "pyref_cells_per_s": p["cells_per_s"], "ratio": r["cells_per_s"] / p["cells_per_s"]})
            print(json.dumps(rows[-1]), flush=True)
    ratio = sum(x["ratio"] for x in rows) / len(rows)
    out = {"what": "reference StringEditDistance.wagnerFisher cells/s divided by oracle/pyref.py build() cells/s, "
                   "same core, same synthetic ACGU pairs, distance only, best of 3",
           "cpu_model": open("/proc/cpuinfo").read().split("model name")[1].split(":")[1].split("\n")[0].strip(),
           "core": args.core, "rows": rows, "ratio_mean": ratio}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("ratio (reference / pyref) = %.3f" % ratio)


if __name__ == "__main__":
    main()

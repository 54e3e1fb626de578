"""Timeline of the config-4 shard's parts (sed_batch_spans): per step, how long some forward kernel runs, how long
only tracebacks run, and how long both parts' forwards overlap.  Usage: python tools/c4_timeline.py [steps]
(environment switches such as SED_CK_HALVES / SED_CK_SCHED apply)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd"), REPO]
import bench  # noqa: E402
import sedcost  # noqa: E402
import sedgpu  # noqa: E402
import synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
with open(os.path.join(REPO, "tests", "golden", "user_costs.json")) as f:
    table = json.load(f)
plan = sedcost.build_plan(table, [synth.ALPHABET], [synth.ALPHABET])
A, B = bench.gen_codes(np.arange(8192, dtype=np.uint64), 4096, 4096)
ctx = sedgpu.Context(0)
ctx.set_costs(plan)
b = sedgpu.Batch(ctx, sedgpu.PackedPairs.from_arrays(A, B), True)
for _ in range(3):
    b.run()
b.sync()
b.reset_times()
import time
t0 = time.perf_counter()
for _ in range(steps):
    b.run()
b.sync()
wall = (time.perf_counter() - t0) * 1e3 / steps
sp = b.spans()  # [runs, parts, 4]
fw = [(s[0], s[1]) for run in sp for s in run]
tb = [(s[2], s[3]) for run in sp for s in run]
T0, T1 = min(a for a, _ in fw), max(max(e for _, e in fw), max(e for _, e in tb))
grid = np.linspace(T0, T1, 200001)
def cover(iv):
    c = np.zeros_like(grid, dtype=np.int32)
    for a, e in iv:
        c[(grid >= a) & (grid < e)] += 1
    return c
cf, ct = cover(fw), cover(tb)
dt = (T1 - T0) / (len(grid) - 1)
print("parts %d, steps %d: wall %.3f ms/step, events span %.3f ms/step" % (sp.shape[1], steps, wall, (T1 - T0) / steps))
print("  forward busy (union)      %.3f ms/step" % ((cf > 0).sum() * dt / steps))
print("  two forwards at once      %.3f ms/step" % ((cf > 1).sum() * dt / steps))
print("  tracebacks only           %.3f ms/step" % (((cf == 0) & (ct > 0)).sum() * dt / steps))
print("  nothing                   %.3f ms/step" % (((cf == 0) & (ct == 0)).sum() * dt / steps))
print("  mean forward launch %.3f ms, traceback %.3f ms" % (np.mean([e - a for a, e in fw]), np.mean([e - a for a, e in tb])))
for r in range(min(4, len(sp))):
    print("  run %d: " % r + "  ".join("part%d fwd %.2f-%.2f tb %.2f-%.2f" % (p, *sp[r, p]) for p in range(sp.shape[1])))

"""A few 4096^2 script calls through the engine's submit / wait pair API (the GUI call's engine part), for a
rocprofv3 --kernel-trace --hip-runtime-trace timeline of where the call's time goes before its first kernel."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd")]
import json
import sedcost, sedgpu, synth  # noqa: E402

table = json.load(open(os.path.join(REPO, "tests", "golden", "user_costs.json")))
s1, s2 = synth.pair_strings(0, 4096, 4096)
plan = sedcost.pair_plan(table, s1, s2)
ctx = sedgpu.context()
ctx.set_costs(plan)
a, b = plan.encode_bytes(s1), plan.encode_bytes(s2)
for k in range(8):
    t0 = time.perf_counter()
    ctx.submit_pair(a, b, True)
    t1 = time.perf_counter()
    got = ctx.wait_pair()
    t2 = time.perf_counter()
    print("call %d: submit %.1f us, wait %.1f us" % (k, (t1 - t0) * 1e6, (t2 - t1) * 1e6))

"""Host-side cost of one sed_batch_run (enqueue) vs the GPU time of a step, for the
small-kernel workloads (config 5) where launch overhead matters."""
import json, os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd"), REPO]
import bench, sedcost, sedgpu, synth  # noqa: E402

qa, qb = bench.gen_all_vs_all(500)
table = json.load(open(os.path.join(REPO, "tests", "golden", "costs.json")))
plan = sedcost.build_plan(table, [synth.ALPHABET], [synth.ALPHABET])
ctx = sedgpu.Context(0)
ctx.set_costs(plan)
for pipeline, every in ((False, 1), (True, 1), (False, 0), (True, 0)):  # pipeline: odd runs on a second stream
    b = sedgpu.Batch(ctx, sedgpu.PackedPairs(qa, qb), False, no_len=True, pipeline=pipeline)
    for _ in range(5):
        b.run()
    b.sync()
    b.set_timing(every)  # 0: no timing events on the kernels
    for n in (10, 100, 400):
        b.reset_times()
        t0 = time.perf_counter()
        for _ in range(n):
            b.run()
        t1 = time.perf_counter()
        b.sync()
        t2 = time.perf_counter()
        dp, _ = b.times()
        print("pipeline %d events %d runs %4d  enqueue %.1f us/run  total %.1f us/run  kernel %.1f us" %
              (pipeline, every, n, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6,
               float(np.mean(dp)) * 1e3 if len(dp) else float("nan")), flush=True)
    b.close()

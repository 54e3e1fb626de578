#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/<tag>/:
kernel-trace stats, per-launch HBM traffic from the FETCH_SIZE / WRITE_SIZE
passes (gfx950 corrections from MI355X_MICROARCH.md §HBM: counters are KiB,
FETCH_SIZE reads half the bytes of a wide coalesced stream -> x2) and the SQ
counters, plus the bench lines."""
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", tag)
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)


def pmc(path):
    out = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        out.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return out


stats = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
for w in ("c3", "c5", "c5n"):  # secondary workloads (kernel trace only)
    f = os.path.join(src, "kt_" + w, "kt_kernel_stats.csv")
    if os.path.exists(f):
        shutil.copy(f, os.path.join(dst, "kernel_stats_%s.csv" % w))
        shutil.copy(os.path.join(src, "kt_bench_%s.json" % w), os.path.join(dst, "bench_under_kernel_trace_%s.json" % w))
fetch = pmc(os.path.join(src, "fetch", "pmc_counter_collection.csv"))
write = pmc(os.path.join(src, "write", "pmc_counter_collection.csv"))
sq = pmc(os.path.join(src, "sq", "pmc_counter_collection.csv"))
bench = json.load(open(os.path.join(src, "bench.json")))
kt_bench = json.load(open(os.path.join(src, "kt_bench.json")))
summary = {"tag": tag, "bench": bench, "bench_under_kernel_trace": {k: kt_bench[k] for k in ("value", "ms_per_step")},
           "kernels": {}}
for row in stats:
    name = row["Name"]
    ent = {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) / 1e6,
           "min_ms": float(row["MinNs"]) / 1e6, "max_ms": float(row["MaxNs"]) / 1e6}
    if name in fetch and name in write:
        f = sum(fetch[name]["FETCH_SIZE"]) / len(fetch[name]["FETCH_SIZE"])
        w = sum(write[name]["WRITE_SIZE"]) / len(write[name]["WRITE_SIZE"])
        ent["FETCH_SIZE_KiB"] = f
        ent["WRITE_SIZE_KiB"] = w
        ent["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
    if name in sq:
        ent["sq"] = {k: sum(v) / len(v) for k, v in sq[name].items()}
        g = ent["sq"].get("GRBM_GUI_ACTIVE")
        if g:
            ent["effective_clock_ghz"] = g / 8 / (ent["avg_ms"] * 1e-3) / 1e9
    summary["kernels"][name] = ent
json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
dp = summary["kernels"].get("sed_wf_i32_kernel")
if dp and "hbm_bytes_per_launch" in dp:
    json.dump({"kernel": "sed_wf_i32_kernel", "workload": bench["config"]["workload"],
               "hbm_bytes_per_launch": dp["hbm_bytes_per_launch"],
               "FETCH_SIZE_KiB": dp["FETCH_SIZE_KiB"], "WRITE_SIZE_KiB": dp["WRITE_SIZE_KiB"],
               "correction": "MI355X_MICROARCH.md HBM section: counters in KiB, FETCH_SIZE x2 on gfx950",
               "source": "profiles/%s/summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes); fallback only"
                         % tag},
              open(os.path.join("profiles", "pmc_dp_i32_c4.json"), "w"), indent=1)
print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "sq"} for k, v in summary["kernels"].items()}, indent=1))

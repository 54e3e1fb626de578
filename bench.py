#!/usr/bin/env python3
"""Throughput bench: DP cells/s + edit-script bit-exact rate on MI355X.

Default workload (BASELINE.json config 4, per-GPU shard; weak scaling):
  8192 synthetic ACGU pairs of 4096 x 4096 per GPU, user_costs.json,
  one step = the integer DP kernel + the device traceback over the whole
  batch (distance AND canonical edit script for every pair), inputs resident
  in HBM.  At --gpus 8 that is exactly config 4 (64k pairs).

    python bench.py [--gpus N --steps K --warmup W] [--workload c4|c3|c2]

For N > 1 run under torch.distributed.run (one rank per GPU); each rank
generates its own pair-index shard (no input scatter), the steps run with no
data-path collective, and the per-pair results are gathered to rank 0 over
RCCL once, after the timed region (timed separately as gather_ms).
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "rna-sequence-diff-patch_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import sedcost  # noqa: E402
import sedgpu  # noqa: E402
import synth  # noqa: E402

METRIC = "DP cells/sec (whole node) + edit-script bit-exact rate, 4k×4k RNA pairs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec peak
SIMDS, CLOCK = 1024, 2.4e9
# VALU ceiling of the integer kernels: every op of the dependent DP cell issues at ~4 cycles per wave64
# instruction on gfx950 whatever the op mix (tools/ubench/valu_mix.hip, valu_row.hip: 4.0-4.2 cycles/op,
# the nominal 2-cycle ops do not pair when interleaved with the 4-cycle v_perm/v_min3/v_alignbit).
# Ops per cell in offset-key space (sed_kernels.hip): perm + add + min3 (+ and_or clearing the op for the
# op-count field, + the ladder's delete add on 3 of 16 rows) (+ alignbit for the traceback); packed distance
# keys: perm + pk_add + 2 pk_min per 2 cells.  Checkpoint script batches (traceback mode 2) run the distance
# keys (D << 16 - U carries the path length; the traceback recomputes the op tie-break): "nolen".
VALU_CYCLES_PER_OP = 4.0
# the dot-key cell (v_dot4_i32_i8 + v_max3_u32) measures 4.50-4.75 cycles per op in its dependent row
# (profiles/r02_dot/ubench_valu_dot.txt: 72-75 cycles for 8 dot + 8 max): the model takes 4.5
VALU_CYCLES_DOT = 4.5
CELL_OPS = {"script": 5 + 3 / 16, "len": 4 + 3 / 16, "nolen": 3, "nolen_x2": 2, "dot": 2}
# the bit-parallel unit-cost lane kernel: ~15 VALU per str1 symbol for a whole row of str2 (m <= 32), from its ISA
BITPAR_OPS_PER_ROW = 15


def lad_ops(R):
    """Ladder dot keys with per-cell codes (CHAIN kernel): 4 VALU on the ladder's d = -1 rows, 6 on its jump rows
    (3 of 16 rows at R = 16, 2 of 8 at R = 8, 1 of 4 at R = 4; sed_kernels.hip Ladder<R>)."""
    jumps = {16: 3, 8: 2, 4: 1}.get(R, 3)
    period = min(R, 16) if R in (4, 8, 16) else 16
    return 4.0 + 2.0 * jumps / period

WORKLOADS = {
    # name: (pairs per GPU, n, m, cost table, description)
    "c4": (8192, 4096, 4096, "user_costs.json",
           "config 4 shard: 8192 pairs/GPU of 4096x4096 synthetic ACGU, user_costs.json, distance + edit script"),
    "c3": (65536, 512, 512, "costs.json",
           "config 3: 65536 pairs of 512x512 synthetic ACGU, costs.json, distance + edit script"),
    "c2": (1, 4096, 4096, "user_costs.json",
           "config 2: 1 pair 4096x4096 synthetic ACGU, user_costs.json, distance + edit script"),
    "iupac": (8192, 1024, 1024, "costs.json",
              "fp64 path: 8192 pairs of 1024x1024 synthetic 15-symbol IUPAC, costs.json, distance + edit script"),
    "timing": (51200, 0, 0, "costs.json",
               "timing.py methodology, batched: pair p is two random 15-symbol IUPAC sequences of length 10 + 10 (p mod "
               "50) (timing.py:12-15,45-57: lengths 10..500 step 10), costs.json (fp64 path), distance + edit script"),
    "c5": (500, 0, 0, "costs.json",
           "config 5 (synthetic): all-vs-all wf_score over 500 ACGU sequences of length U[24,32], costs.json, "
           "250000 ordered pairs, distance only"),
    "c5n": (500, 0, 0, "costs.json",
            "config 5 with N (synthetic): all-vs-all wf_score over 500 sequences of length U[24,32], ~1% N "
            "(fp64 path), costs.json, 250000 ordered pairs, distance only"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_codes(pair_ids, n, m, iupac=False):
    gen = synth.iupac_codes if iupac else synth.pair_codes
    A = np.empty((len(pair_ids), n), np.uint8)
    B = np.empty((len(pair_ids), m), np.uint8)
    for s in range(0, len(pair_ids), 512):
        ids = pair_ids[s:s + 512]
        A[s:s + len(ids)] = gen(ids, n, 0)
        B[s:s + len(ids)] = gen(ids, m, 1)
    return A, B


def gen_all_vs_all(nseq, lo=24, hi=32, n_rate=0.0):
    """Config 5 stand-in: nseq synthetic ACGU sequences, every ordered pair (query = str1).
    n_rate > 0: that fraction of positions becomes N (code 4), which forces the fp64 path."""
    ids = np.arange(nseq, dtype=np.uint64)
    ln = synth.lengths(ids, lo, hi)
    seqs = [synth.pair_codes([i], int(l), 0)[0] for i, l in zip(ids, ln)]
    if n_rate > 0:
        rng = np.random.default_rng(20261015)
        seqs = [np.where(rng.random(len(q)) < n_rate, 4, q).astype(np.uint8) for q in seqs]
    return [seqs[a] for a in range(nseq) for _ in range(nseq)], [seqs[b] for _ in range(nseq) for b in range(nseq)]


def script_costs(plan, A, B, ln, ops, ops_off):
    """Vectorised property check over ALL pairs: the script is a monotone
    alignment consuming exactly n rows and m columns and its summed cost equals
    the distance.  Returns (valid mask, cost)."""
    P, n = A.shape
    m = B.shape[1]
    Lmax = n + m
    W = (Lmax + 15) // 16
    words = ops[(ops_off[:P, None] + np.arange(W)[None, :])]
    codes = ((words[:, :, None] >> (2 * np.arange(16, dtype=np.uint32))[None, None, :]) & 3).reshape(P, -1)[:, :Lmax]
    live = np.arange(Lmax)[None, :] < ln[:, None]
    ins = (codes == 0) & live
    dele = (codes == 1) & live
    upd = (codes == 2) & live
    rows = np.cumsum(dele | upd, axis=1)  # rows consumed after each op
    cols = np.cumsum(ins | upd, axis=1)
    ok = (rows[:, -1] == n) & (cols[:, -1] == m) & (((codes == 3) & live).sum(1) == 0)
    ri = np.clip(rows - 1, 0, n - 1)
    cj = np.clip(cols - 1, 0, m - 1)
    a_sym = np.take_along_axis(A, ri, axis=1)
    b_sym = np.take_along_axis(B, cj, axis=1)
    sub = plan.sub[a_sym, b_sym]
    cost = ins.sum(1) * plan.ins + dele.sum(1) * plan.dele + (sub * upd).sum(1)
    return ok, cost


def cpu_share():
    """Host cores this process may use: the affinity mask, capped by the cgroup CPU quota and by the
    per-job thread budget the box exports (OMP_NUM_THREADS), whichever is smallest."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _pyref_task(args):
    """One reference-regime job (oracle/pyref.py, the node graph of StringEditDistance.py:133-334)."""
    import pyref
    s1, s2, table, script = args
    t0 = time.perf_counter()
    pyref.run_pair(s1, s2, table, script)
    return len(s1) * len(s2), time.perf_counter() - t0


def cpu_baseline_python(table, alphabet, A, B, qa, qb, want_script, cores, seconds):
    """Reference-regime leg: the pure-Python node-graph restatement on `cores` processes over a bounded
    sample of the workload.  Long pairs are sampled as leading B x B blocks (one node graph of ~0.6 M
    cells, ~0.4 GB, per process at a time); short pairs run whole.  Returns the bench object."""
    import multiprocessing as mp
    if A is not None:
        P, n = A.shape
        m = B.shape[1]
        blk = min(n, m, 768)
        jobs = []
        for k in range(4 * cores):  # leading blocks of successive pairs (of the one pair's diagonal for c2)
            p = k % P
            o = 0 if P > 1 else (k * blk) % max(1, min(n, m) - blk + 1)
            jobs.append(("".join(alphabet[c] for c in A[p, o:o + blk]), "".join(alphabet[c] for c in B[p, o:o + blk]),
                         table, want_script))
        what = "leading %dx%d blocks of the first %d pairs" % (blk, blk, min(P, len(jobs))) if P > 1 else \
            "%d diagonal %dx%d blocks of the pair" % (len(jobs), blk, blk)
    else:
        budget = 1.5e5 * cores * seconds  # ~cells the sample may hold at the reference's rate
        jobs, cells = [], 0
        for a, b in zip(qa, qb):
            jobs.append(("".join(alphabet[c] for c in a), "".join(alphabet[c] for c in b), table, want_script))
            cells += len(a) * len(b)
            if cells >= budget:
                break
        what = "the first %d of the pairs" % len(jobs)
    ctx = mp.get_context("spawn")
    with ctx.Pool(cores) as pool:
        t0 = time.perf_counter()
        res = pool.map(_pyref_task, jobs, chunksize=max(1, len(jobs) // (4 * cores)))
        dt = time.perf_counter() - t0
    cells = float(sum(c for c, _ in res))
    cal = None
    cal_path = os.path.join(REPO, "profiles", "r03", "pyref_calibration.json")
    if os.path.exists(cal_path):  # tools/calibrate_pyref.py: the reference itself, timed against pyref on one core
        with open(cal_path) as f:
            c = json.load(f)
        cal = {"reference_over_pyref": c["ratio_mean"], "source": os.path.relpath(cal_path, REPO),
               "reference_estimate": cells / dt * c["ratio_mean"]}
    return {"value": cells / dt, "unit": "cells/s", "cores": cores, "kind": "port", "calibration": cal,
            "sample": "%s, pure-Python node graph (oracle/pyref.py: the reference's Node/Edge regime, %s), "
                      "%.1f s" % (what, "distance + canonical edit script" if want_script else "distance", dt)}


def strided_sample(P, count):
    """About `count` pair indices spread over all P pairs: every ceil(P / count)-th pair from pair 0, plus the last
    pair, so the sample spans every part (SED_CK_HALVES), every residency round of the waves and every rank's shard
    end to end (not a prefix).  Returns (indices, stride)."""
    count = int(max(1, min(P, count)))
    stride = -(-P // count)
    idx = np.arange(0, P, stride, dtype=np.int64)
    if idx[-1] != P - 1:
        idx = np.append(idx, P - 1)
    return idx, int(stride)


def oracle_subset(cs, packed, idx, want_ops, threads):
    """The C oracle over the pairs `idx` of `packed` (descriptor arrays gathered, sequence buffers shared)."""
    import oracle
    sel = lambda a: np.ascontiguousarray(np.asarray(a)[idx])  # noqa: E731
    return oracle.batch(cs, packed.codes_a, sel(packed.off_a), sel(packed.len_a), packed.codes_b, sel(packed.off_b),
                        sel(packed.len_b), len(idx), want_ops=want_ops, nthreads=threads)


def cpu_baseline(plan, packed, seconds, threads, want_ops):
    """Oracle (C restatement, test infrastructure) on a bounded, strided sample of the same pairs: about `seconds`
    of work on `threads` threads, spread over the whole batch (strided_sample)."""
    import oracle
    cs = oracle.Costs.from_plan(plan)
    P = packed.npairs
    la, lb = packed.len_a[:P], packed.len_b[:P]
    cells_p = la.astype(np.float64) * lb
    cum = np.cumsum(cells_p)
    probe = int(min(P, np.searchsorted(cum, 2e6) + 1))  # ~2M cells, single thread (rate probe only)
    t0 = time.perf_counter()
    oracle.batch(cs, packed.codes_a, packed.off_a, la, packed.codes_b, packed.off_b, lb, probe, want_ops=want_ops)
    per_cell = (time.perf_counter() - t0) / max(1.0, float(cum[probe - 1]))
    budget = seconds * threads / max(per_cell, 1e-12)  # cells the sample may hold
    count = int(min(P, max(threads, budget / max(1.0, float(cells_p.mean())))))
    idx, stride = strided_sample(P, count)
    t0 = time.perf_counter()
    dist, is_int, ln, ops, ops_off = oracle_subset(cs, packed, idx, want_ops, threads)
    dt = time.perf_counter() - t0
    return {"value": float(cells_p[idx].sum()) / dt, "seconds": dt, "count": len(idx), "idx": idx, "stride": stride,
            "dist": dist, "len": ln, "ops": ops, "ops_off": ops_off}


def sample_exact(idx, o_dist, o_len, o_ops, o_off, dist, ln, ops, ops_off, want_script):
    """Per sampled pair: distance, length and (script mode) every op equal to the oracle's."""
    exact = (o_dist == dist[idx]) & ((o_len == ln[idx]) | (ln[idx] == -1))
    if want_script:
        for k, p in enumerate(idx):
            if exact[k]:
                g = sedgpu.unpack_ops(ops, ops_off, int(p), int(ln[p]))
                exact[k] = np.array_equal(g, o_ops[o_off[k]: o_off[k] + o_len[k]])
    return exact


def pmc_pass(counters, kernels, timeout=240):
    """One rocprofv3 --pmc pass over this bench re-run as a child process for one step (no warmup, no CPU legs, no
    nested measurement).  Returns ({kernel: {counter: value per launch}}, None) or (None, reason)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if any(k.startswith("ROCPROF") for k in os.environ):
        return None, "this bench already runs under rocprofv3"  # no nested profilers
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="sedpmc_", dir="/tmp")
    # argparse keeps the last occurrence of each flag
    child = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:] + [
        "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--traffic", "none"]
    cmd = ["timeout", "-s", "KILL", str(timeout), rp, "--pmc"] + list(counters) + [
        "-T", "-d", d, "-o", "pmc", "--output-format", "csv", "--"] + child
    try:
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           env=dict(os.environ, TMPDIR="/tmp"), timeout=timeout + 60)
    except subprocess.TimeoutExpired:
        return None, "%s pass timed out" % "+".join(counters)
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] in counters and row["Kernel_Name"] in kernels:
                    vals.setdefault(row["Kernel_Name"], {}).setdefault(row["Counter_Name"], []).append(
                        float(row["Counter_Value"]))
    shutil.rmtree(d, ignore_errors=True)
    if r.returncode != 0 or not vals:
        return None, "%s pass failed (rc %d)" % ("+".join(counters), r.returncode)
    return {k: {c: sum(v) / len(v) for c, v in cv.items()} for k, cv in vals.items()}, None


def measure_traffic(kernels):
    """HBM bytes per launch of `kernels` (summed), measured now, one pass per counter (FETCH_SIZE and WRITE_SIZE do
    not fit one pass).  Units and the gfx950 correction per MI355X_MICROARCH.md "HBM": both counters in KiB,
    FETCH_SIZE reports half the bytes of wide streaming reads, so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
    Returns (bytes, detail) or (None, reason)."""
    kib = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        got, why = pmc_pass([ctr], kernels)
        if got is None:
            return None, why
        kib[ctr] = sum(v.get(ctr, 0.0) for v in got.values())
    total = 2.0 * kib["FETCH_SIZE"] * 1024.0 + kib["WRITE_SIZE"] * 1024.0
    return total, {"FETCH_SIZE_KiB": kib["FETCH_SIZE"], "WRITE_SIZE_KiB": kib["WRITE_SIZE"],
                   "correction": "KiB; FETCH_SIZE x2 on gfx950 (MI355X_MICROARCH.md HBM)"}


def measure_issue(kernels):
    """VALU / SALU issue per kernel from one SQ pass: SQ_INSTS_VALU and SQ_INSTS_SALU (wave-instructions per launch)
    and GRBM_GUI_ACTIVE (cycles, summed over the 8 XCDs).  A wave64 VALU instruction occupies its SIMD's issue
    port 4 cycles (tools/ubench/valu_mix.hip), so valu_issue = SQ_INSTS_VALU * 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8);
    the scalar unit issues one instruction per CU per cycle, so salu_issue = SQ_INSTS_SALU / 256 CUs / (GRBM / 8)."""
    got, why = pmc_pass(["SQ_INSTS_VALU", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"], kernels)
    if got is None:
        return None, why
    out = {}
    for k, c in got.items():
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc <= 0:
            continue
        out[k] = {"SQ_INSTS_VALU": c.get("SQ_INSTS_VALU"), "SQ_INSTS_SALU": c.get("SQ_INSTS_SALU"),
                  "GRBM_GUI_ACTIVE": c.get("GRBM_GUI_ACTIVE"),
                  "valu_issue": c.get("SQ_INSTS_VALU", 0.0) * 4.0 / SIMDS / cyc,
                  "salu_issue": c.get("SQ_INSTS_SALU", 0.0) / (SIMDS / 4) / cyc}
    return out, None


def s8d_bytes(len_a, len_b, script):
    """SURVEY.md §8(d)'s algorithmic HBM bytes of one launch: 2-bit packed inputs (n+m)/4 + an 8-byte distance per
    pair; script mode adds the 2-bit traceback choice of every cell (0.25 B/cell), the path's (n+m) sparse reads of
    it and the (n+m) 2-bit ops out."""
    n = np.asarray(len_a, np.float64)
    m = np.asarray(len_b, np.float64)
    per_pair = (n + m) / 4.0 + 8.0
    if script:
        per_pair = per_pair + 0.25 * n * m + (n + m) + (n + m) / 4.0
    return float(per_pair.sum())


def interval_union(iv):
    """Total length of the union of intervals [(start, end), ...] (ms)."""
    tot, cur_s, cur_e = 0.0, None, None
    for s, e in sorted((float(a), float(b)) for a, b in iv if b > a):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def launcher_cmd(n, argv, port):
    """The torch.distributed.run command bench.py starts for itself when run as `bench.py --gpus N` (N > 1)
    outside a launcher: one rank per GPU on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def self_launch(n, argv):
    """Run this bench as n ranks (a child launcher; this process never touches HIP) and return its exit code.
    The ranks' rank 0 prints the JSON line on the inherited stdout."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log("bench.py: launching %d ranks: %s" % (n, " ".join(launcher_cmd(n, argv, port))))
    return subprocess.call(launcher_cmd(n, argv, port), env=env)


def refuse_reason(gpus, environ):
    """Why this rank must not run (None if it may): a world size that differs from --gpus, or a debug switch of
    the engine in the environment (SED_DEBUG_*, e.g. one that drops work from the timed region)."""
    world = int(environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        return "--gpus %d but WORLD_SIZE=%d: the line would misreport the GPU count" % (gpus, world)
    dbg = sorted(k for k in environ if k.startswith("SED_DEBUG"))
    if dbg:
        return "debug switch(es) %s set: refusing to time the engine under them" % ", ".join(dbg)
    return None


def gen_timing(pair_ids):
    """timing.py's sweep (timing.py:45-57: random 15-symbol pairs of equal length 10, 20, .., 500), batched: pair id p
    has length 10 + 10 (p mod 50) on both sides."""
    ids = np.asarray(pair_ids, dtype=np.uint64)
    ln = 10 + 10 * (ids % np.uint64(50)).astype(np.int64)
    qa = [None] * len(ids)
    qb = [None] * len(ids)
    for L in np.unique(ln):
        sel = np.flatnonzero(ln == L)
        a = synth.iupac_codes(ids[sel], int(L), 0)
        b = synth.iupac_codes(ids[sel], int(L), 1)
        for k, x in enumerate(sel):
            qa[x] = a[k]
            qb[x] = b[k]
    return qa, qb


def shard_inputs(workload, P, n, m, world, r):
    """Rank r's inputs, regenerated from the seeds: (A, B, None, None) for fixed-shape workloads (pair ids
    [r*P, (r+1)*P)), (None, None, qa, qb) for the all-vs-all rows of config 5 and the ragged timing sweep."""
    if workload == "timing":
        qa, qb = gen_timing(np.arange(r * P, (r + 1) * P, dtype=np.uint64))
        return None, None, qa, qb
    if workload in ("c5", "c5n"):
        import sedshard
        lo, hi = sedshard.shard_range(P, world, r)  # query rows of this rank
        qa, qb = gen_all_vs_all(P, n_rate=0.01 if workload == "c5n" else 0.0)
        return None, None, qa[lo * P:hi * P], qb[lo * P:hi * P]
    ids = np.arange(r * P, (r + 1) * P, dtype=np.uint64)
    A, B = gen_codes(ids, n, m, workload == "iupac")
    return A, B, None, None


def shard_bounds(workload, P, world, r):
    """[first, stop) of rank r's shard as shard_inputs draws it: pair ids, or config 5's query rows."""
    if workload in ("c5", "c5n"):
        import sedshard
        return sedshard.shard_range(P, world, r)
    return r * P, (r + 1) * P


def valid_scripts(plan, A, B, dist, ln, ops, ops_off, exact_int):
    """Pairs (of A, B) whose script passes script_costs and whose cost equals the reported distance."""
    good = 0
    P = A.shape[0]
    for s0 in range(0, P, 256):
        sl = slice(s0, min(P, s0 + 256))
        ok, cost = script_costs(plan, A[sl], B[sl], ln[sl], ops, ops_off[sl])
        same = (cost == dist[sl]) if exact_int else np.isclose(cost, dist[sl], rtol=1e-12)
        good += int((ok & same).sum())
    return good


def valid_scripts_ragged(plan, qa, qb, dist, ln, ops, ops_off, exact_int):
    """valid_scripts over ragged pairs, grouped by shape."""
    la = np.array([len(x) for x in qa])
    lb = np.array([len(x) for x in qb])
    good = 0
    for (n, m) in set(zip(la.tolist(), lb.tolist())):
        sel = np.flatnonzero((la == n) & (lb == m))
        if n == 0 or m == 0:
            continue
        A = np.stack([qa[x] for x in sel])
        B = np.stack([qb[x] for x in sel])
        good += valid_scripts(plan, A, B, dist[sel], ln[sel], ops, ops_off[sel], exact_int)
    return good


def oracle_agree(plan, packed, idx, dist, ln, ops, ops_off, want_script, threads):
    """Pairs among `idx` of `packed` whose distance, length and every op equal the C oracle's."""
    import oracle
    cs = oracle.Costs.from_plan(plan)
    od, _, oln, oops, ooff = oracle_subset(cs, packed, idx, want_script, threads)
    return int(sample_exact(idx, od, oln, oops, ooff, dist, ln, ops, ops_off, want_script).sum())


def verify_gathered(args, plan, P, n, m, world, gdist, glen, gops, want_script, mode, threads, seconds):
    """Rank 0 after the gather: every rank's results, checked on rank 0 (N > 1).  The script property check over
    ALL gathered pairs (inputs regenerated from the seeds), and an oracle comparison of a strided sample of each
    rank's pairs (first to last) within `seconds` of CPU time in total.  Returns the bench line's check fields."""
    exact_int = mode == "i32"
    valid = total = agree = sampled = 0
    base = wbase = 0
    per_rank = []
    for r in range(world):
        A, B, qa, qb = shard_inputs(args.workload, P, n, m, world, r)
        packed = sedgpu.PackedPairs.from_arrays(A, B) if A is not None else sedgpu.PackedPairs(qa, qb)
        Pr = packed.npairs
        d = gdist[base:base + Pr]
        ln = glen[base:base + Pr]
        words = int(packed.ops_off[Pr])  # this rank's script words (its segment of the gathered buffer)
        if want_script:
            ops = gops[wbase:wbase + words]
            valid += (valid_scripts(plan, A, B, d, ln, ops, packed.ops_off, exact_int) if A is not None else
                      valid_scripts_ragged(plan, qa, qb, d, ln, ops, packed.ops_off, exact_int))
        else:
            ops = None
        wbase += words
        total += Pr
        # oracle sample: a strided sample over the whole rank shard, about seconds / world of work
        la, lb = packed.len_a[:Pr].astype(np.float64), packed.len_b[:Pr].astype(np.float64)
        budget = 1.5e8 * threads * seconds / world  # cells; the C oracle runs ~1e8-2e8 cells/s per thread
        idx, stride = strided_sample(Pr, budget / max(1.0, float((la * lb).mean())))
        agree += oracle_agree(plan, packed, idx, d, ln, ops, packed.ops_off, want_script, threads)
        sampled += len(idx)
        per_rank.append({"pairs": len(idx), "stride": stride})
        base += Pr
    out = {"verified_on_rank0": {"pairs": total, "oracle_sample_per_rank": per_rank}}
    if want_script:
        out["script_valid_rate"] = valid / max(1, total)
        out["script_exact_rate"] = agree / max(1, sampled)
    else:
        out["dist_exact_rate"] = agree / max(1, sampled)
    out["exact_sample"] = sampled
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (= ranks).  Outside a launcher, N > 1 starts torch.distributed.run with N ranks")
    ap.add_argument("--steps", type=int, default=20)  # per-cell-code batches pipeline traceback k beside DP k+1 (the last one is not overlapped); checkpoint batches run DP then traceback
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--pairs", type=int, default=0, help="override pairs per GPU")
    ap.add_argument("--shape", default="", help="override the pair shape NxM (experiments; fixed-shape workloads)")
    ap.add_argument("--no-script", action="store_true", help="distance only (no traceback)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="no overlap across steps: script batches run DP and traceback back to back on one stream, "
                         "lane batches every step's kernel on one stream")
    ap.add_argument("--rows-per-lane", type=int, default=0)
    ap.add_argument("--no-lane", action="store_true", help="route short pairs to the wave kernels too (A/B)")
    ap.add_argument("--no-pack", action="store_true",
                    help="distance-only pairs one per lane / wave (no packed 16-bit cells; A/B)")
    ap.add_argument("--no-bitpar", action="store_true",
                    help="unit-cost distance-only lane pairs on the DP lane kernels instead of bit-parallel (A/B)")
    ap.add_argument("--seg", type=int, default=0,
                    help="SED_OPT_SEG: fp64 pairs in 16-lane segments: 0 auto, 1 every eligible pair, 2 never (A/B)")
    ap.add_argument("--no-split-ck", action="store_true",
                    help="SPLIT script batches (config 2) keep the ladder-key forward with per-cell codes (SED_OPT_SPLITCK 2; A/B)")
    ap.add_argument("--no-scaled", action="store_true",
                    help="fp64 lane pairs on the fp64 DP instead of the scaled-integer DP of dyadic costs (A/B)")
    ap.add_argument("--timing-every", type=int, default=-1,
                    help="timing events on every run (1), every k-th run, or none (0) in the timed region; with k != 1 "
                         "the roofline takes the step time as the kernels' busy time and the kernel times come from an "
                         "instrumented pass of the same steps afterwards; -1 (default): 0 for distance-only batches of "
                         "lane pairs only (config 5: the events cost the host ~5 us of a ~5 us step), else 1")
    ap.add_argument("--split", type=int, default=0, help="SED_OPT_SPLIT: 0 auto, 1 force, 2 off (A/B)")
    ap.add_argument("--tb", type=int, default=0,
                    help="SED_OPT_TB: 0 auto, 1 per-cell traceback codes, 2 checkpoints + recompute (A/B)")
    ap.add_argument("--chain", type=int, default=0,
                    help="SED_OPT_CHAIN: 0 auto, 1 force, 2 off, L>=3 force with chains of L pairs (A/B)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-python-baseline", action="store_true",
                    help="skip the reference-regime leg (pure-Python node graph, oracle/pyref.py)")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_dp_i32_c4.json"),
                    help="per-launch HBM traffic of the DP kernel from the rocprofv3 FETCH_SIZE/WRITE_SIZE passes "
                         "(tools/profile_round.sh + tools/summarize_profile.py); used when its workload matches")
    ap.add_argument("--traffic", default="measure", choices=["measure", "file", "none"],
                    help="roofline.traffic and valu.issue: measure = three rocprofv3 --pmc child runs of this "
                         "workload (FETCH_SIZE, WRITE_SIZE, SQ issue; one step each) on rank 0 at N = 1; "
                         "file = --pmc-json; none")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse ranks sharing one GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))  # before anything touches HIP
    why = refuse_reason(args.gpus, os.environ)
    if why:
        log("bench.py: " + why)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    local = local % max(1, torch.cuda.device_count())  # ranks > GPUs only in a gloo rehearsal
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    tdev = torch.device("cuda", local) if args.dist_backend == "nccl" else torch.device("cpu")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    P, n, m, costs_file, desc = WORKLOADS[args.workload]
    if args.pairs:
        P = args.pairs
    if args.shape:
        n, m = (int(x) for x in args.shape.lower().split("x"))
        desc += " [shape overridden: %dx%d]" % (n, m)
    want_script = not args.no_script and args.workload not in ("c5", "c5n")
    iupac = args.workload in ("iupac", "timing")
    with open(os.path.join(REPO, "tests", "golden", costs_file)) as f:
        table = json.load(f)
    alpha = synth.IUPAC if iupac else (synth.ALPHABET + "N" if args.workload == "c5n" else synth.ALPHABET)
    plan = sedcost.build_plan(table, [alpha], [alpha])
    t0 = time.perf_counter()
    A, B, qa, qb = shard_inputs(args.workload, P, n, m, world, rank)
    packed = sedgpu.PackedPairs.from_arrays(A, B) if A is not None else sedgpu.PackedPairs(qa, qb)
    Pw = P  # pairs per GPU as configured (config 5: query rows)
    P = packed.npairs
    log("rank %d: generated %d pairs in %.1fs" % (rank, P, time.perf_counter() - t0))

    ctx = sedgpu.Context(local)
    if args.rows_per_lane:
        ctx.set_option(sedgpu.SED_OPT_ROWS_PER_LANE, args.rows_per_lane)
    if args.no_lane:
        ctx.set_option(sedgpu.SED_OPT_LANE, 2)
    if args.no_pack:
        ctx.set_option(sedgpu.SED_OPT_PACK, 2)
    if args.no_bitpar:
        ctx.set_option(sedgpu.SED_OPT_BITPAR, 2)
    if args.no_scaled:
        ctx.set_option(sedgpu.SED_OPT_SCALED, 2)
    if args.no_split_ck:
        ctx.set_option(sedgpu.SED_OPT_SPLITCK, 2)
    if args.seg:
        ctx.set_option(sedgpu.SED_OPT_SEG, args.seg)
    if args.chain:
        ctx.set_option(sedgpu.SED_OPT_CHAIN, args.chain)
    if args.split:
        ctx.set_option(sedgpu.SED_OPT_SPLIT, args.split)
    if args.tb:
        ctx.set_option(sedgpu.SED_OPT_TB, args.tb)
    ctx.set_costs(plan)
    t0 = time.perf_counter()
    pipeline = not args.no_pipeline  # script batches: traceback(k) beside DP(k+1); lane batches: DP(k+1) beside DP(k)
    batch = sedgpu.Batch(ctx, packed, want_script, pipeline=pipeline, no_len=not want_script)
    log("rank %d: batch resident in %.1fs (mode %s, R=%d)" % (rank, time.perf_counter() - t0, batch.mode,
                                                             batch.rows_per_lane))
    cells, design_bytes = batch.work()
    algo_bytes = s8d_bytes(packed.len_a[:P], packed.len_b[:P], want_script)

    if args.timing_every < 0:
        args.timing_every = 0 if (not want_script and batch.lane_pairs == P) else 1
    for _ in range(args.warmup):
        batch.run()
    batch.sync()
    batch.reset_times()
    if args.timing_every != 1:
        batch.set_timing(args.timing_every)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.run()  # DP then traceback; per-cell-code batches overlap traceback(k) with DP(k+1) (SED_PIPELINE)
    batch.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    time_pass = "the timed region"
    if args.timing_every != 1:  # kernel times from an instrumented pass of the same steps (untimed by the bench)
        batch.set_timing(1)
        batch.reset_times()
        for _ in range(args.steps):
            batch.run()
        batch.sync()
        time_pass = "an instrumented pass of %d steps after the timed region (which had timing events on %s)" % (
            args.steps, "no run" if args.timing_every == 0 else "every %d-th run" % args.timing_every)
    dp_ms, tb_ms = batch.times()
    spans = batch.spans()  # [steps, parts, {dp start, dp end, tb start, tb end}] from HIP events
    cells_all = cells
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tc = torch.tensor([cells], dtype=torch.float64, device=tdev)  # shards may differ (config 5's rows)
        dist.all_reduce(tc, op=dist.ReduceOp.SUM)
        cells_all = float(tc.item())
    ms_per_step = elapsed * 1e3 / args.steps
    value = cells_all * args.steps / elapsed

    # ---- results: gather to rank 0 over RCCL (timed separately) ----
    gather_ms = None
    got = None
    if dist is not None:
        import sedshard
        words = int(packed.ops_off[P])
        t_dist = torch.empty(P, dtype=torch.float64, device="cuda")
        t_len = torch.empty(P, dtype=torch.int32, device="cuda")
        t_ops = torch.empty(max(words, 1), dtype=torch.int32, device="cuda")
        batch.export(t_dist.data_ptr(), t_len.data_ptr(), t_ops.data_ptr() if want_script else 0)
        sends = [t.to(tdev) for t in (t_dist, t_len, t_ops)]
        barrier()
        g0 = time.perf_counter()
        got = sedshard.gather_to_rank0(sends, world, rank)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3
        if rank == 0:
            log("rank 0: gathered %d results + %d script words over %s (%.2f ms)"
                % (got[0].numel(), got[2].numel(), args.dist_backend, gather_ms))

    # ---- verification (untimed) ----
    check = {}
    cpu = None
    threads = cpu_share()
    if dist is not None:
        if rank == 0:
            gd = got[0].cpu().numpy()
            gl = got[1].cpu().numpy()
            go = got[2].cpu().numpy().view(np.uint32)
            tv = time.perf_counter()
            check = verify_gathered(args, plan, Pw, n, m, world, gd, gl, go, want_script, batch.mode, threads,
                                    args.cpu_seconds)
            log("rank 0: verified %d gathered pairs in %.1fs" % (len(gd), time.perf_counter() - tv))
    else:
        d_gpu, ii_gpu, ln_gpu, ops = batch.results()
        if want_script and A is not None:
            check["script_valid_rate"] = valid_scripts(plan, A, B, d_gpu, ln_gpu, ops, packed.ops_off,
                                                       batch.mode == "i32") / P
        elif want_script:
            check["script_valid_rate"] = valid_scripts_ragged(plan, qa, qb, d_gpu, ln_gpu, ops, packed.ops_off,
                                                              batch.mode == "i32") / P
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(plan, packed, args.cpu_seconds, threads, want_script)
            c, idx = cpu["count"], cpu["idx"]
            exact = sample_exact(idx, cpu["dist"], cpu["len"], cpu["ops"], cpu["ops_off"], d_gpu, ln_gpu, ops,
                                 packed.ops_off, want_script)
            check["script_exact_rate" if want_script else "dist_exact_rate"] = float(exact.mean())
            check["exact_sample"] = {"pairs": int(c), "stride": cpu["stride"], "first": int(idx[0]),
                                     "last": int(idx[-1]), "of": int(P)}
            shape = "%dx%d" % (n, m) if n else "ragged"
            cpu_obj = {"value": cpu["value"], "unit": "cells/s", "cores": threads, "kind": "port",
                       "sample": "%d of the %d pairs, every %d-th from pair 0 plus the last (%s, %s, %s), C oracle "
                                 "sed_oracle.c, %.1f s" % (c, P, cpu["stride"], shape, costs_file,
                                                           "distance + script" if want_script else "distance",
                                                           cpu["seconds"]),
                       "cpu_model": cpu_model()}
            if not args.no_python_baseline:
                cpu_obj["python_node_graph"] = cpu_baseline_python(
                    table, alpha, A, B, qa if A is None else None, qb if A is None else None, want_script, threads,
                    args.cpu_seconds)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    dp_avg = float(np.mean(dp_ms))
    # A checkpoint batch of >= 2048 pairs runs in parts on as many streams (SED_CK_HALVES), and pipelined batches
    # put consecutive runs' DP kernels on two streams: launches overlap.  The roofline therefore divides a step's
    # bytes and cells by the DP kernels' busy time per step, the union of every DP launch's event interval over the
    # timed steps / steps (<= ms_per_step).  The mean launch (what a rocprofv3 kernel trace averages) and the
    # per-launch fraction it gives are kept beside it.
    launches = batch.dp_launches
    algo_launch, design_launch, cells_launch = algo_bytes / launches, design_bytes / launches, cells / launches
    dp_busy = interval_union([(s[0], s[1]) for run in spans for s in run]) / max(1, len(spans))
    if args.timing_every != 1:
        # the instrumented pass enqueues slower (timing events cost the host ~5 us per run, tools/host_overhead.py),
        # so its overlap differs from the timed region's: the roofline takes the timed step itself as the kernels'
        # busy time (an upper bound), and the pass's union stays beside it
        dp_busy_pass, dp_busy = dp_busy, ms_per_step
        time_pass = "the timed region's step time (no timing events in it; the union over %s was %.4g ms)" % (
            time_pass, dp_busy_pass)
    achieved = algo_bytes / (dp_busy * 1e-3) / 1e9
    achieved_launch = algo_launch / (dp_avg * 1e-3) / 1e9
    nl, npk, nbp = batch.lane_pairs, batch.packed_pairs, batch.bitpar_pairs
    lane_x2 = batch.mode == "i32" and not want_script and nl > 0 and not args.no_pack and nbp == 0
    wave_x2 = npk - (nl if lane_x2 else 0)  # wave pairs computed two per wave
    ops_cell = None
    R = batch.rows_per_lane
    if batch.mode == "i32":
        # checkpoint batches (SED_OPT_TB 2): the forward kernel runs dot keys (v_dot4 + v_max3, 2 ops/cell) or
        # distance keys (3 ops/cell); the traceback's recompute runs after it on the same SIMDs and is not in
        # this model (kernel_ms is the DP).  Per-cell codes on ladder dot keys (CHAIN, config 3): v_dot4, v_min3,
        # v_and_or, v_alignbit on the d = -1 rows, plus 2 adds on the ladder's jump rows (2 of 8 at R = 8).
        if want_script and batch.traceback_mode in (2, 4):
            ops_cell = CELL_OPS["dot" if batch.dot_keys else "nolen"]
        elif want_script:
            ops_cell = lad_ops(R) if batch.ladder_dot_keys else CELL_OPS["script"]
        elif nbp == P:
            ops_cell = BITPAR_OPS_PER_ROW * float(np.sum(packed.len_a[:P])) / max(cells, 1.0)
        else:
            ops_cell = CELL_OPS["nolen_x2" if npk == P else "nolen"]
    dot_cell = batch.mode == "i32" and want_script and batch.traceback_mode in (2, 4) and batch.dot_keys
    cyc = VALU_CYCLES_DOT if dot_cell else VALU_CYCLES_PER_OP
    valu_peak = SIMDS * CLOCK * 64 / (cyc * ops_cell) if ops_cell else None
    rate = cells / (dp_busy * 1e-3)
    if batch.mode != "i32":
        parts = (["sed_wf_f64_kernel"] if nl < P else []) + \
            ([("sed_lane_scaled_kernel" if batch.scaled_pairs else "sed_lane_f64_kernel")] if nl else [])
    else:
        wave_k = "sed_wf_i32_chain_kernel" if batch.chains else "sed_wf_i32_kernel"
        parts = ((["sed_wf_i32x2_kernel"] if wave_x2 else []) + ([wave_k] if nl + wave_x2 < P else []) +
                 (["sed_ck_codes_kernel"] if want_script and batch.traceback_mode == 4 else []) +
                 ([("sed_lane_bitpar_kernel" if nbp else "sed_lane_i32x2_kernel" if lane_x2 else
                    "sed_lane_i32_kernel")] if nl else []))
    tb_kernels = []
    if want_script and nl < P:
        tb_kernels = {2: ["sed_traceback_ck_kernel"], 3: ["sed_tb_stripemap_kernel", "sed_tb_stripeemit_kernel"],
                      4: ["sed_tb_stripemap_kernel", "sed_tb_stripeemit_kernel", "sed_traceback_kernel",
                          "sed_traceback_window_kernel"],
                      1: ["sed_traceback_kernel", "sed_traceback_window_kernel"]}.get(batch.traceback_mode, [])
    kname = "+".join(parts)
    traffic, traffic_src, issue, issue_src = None, None, None, None
    if args.traffic == "measure" and world == 1:
        traffic, detail = measure_traffic(set(parts))
        traffic_src = {"measured": "rocprofv3 --pmc, this workload, one step per counter", **detail} \
            if traffic is not None else {"measure_failed": detail}
        issue, why = measure_issue(set(parts) | set(tb_kernels))
        issue_src = "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE, this workload, one step" \
            if issue is not None else {"measure_failed": why}
    if traffic is None and args.traffic != "none" and args.pmc_json and os.path.exists(args.pmc_json):
        with open(args.pmc_json) as f:
            pm = json.load(f)
        if pm.get("workload") == desc and batch.mode == "i32" and want_script and P == WORKLOADS[args.workload][0]:
            traffic = pm.get("hbm_bytes_per_launch")
            traffic_src = dict(traffic_src or {}, file=os.path.relpath(args.pmc_json, REPO))
    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith("SED_")}
    line = {
        "metric": METRIC, "value": value, "unit": "cells/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32" if batch.mode == "i32" else "f64", "data": "synthetic",
        "config": {"workload": desc, "pairs_per_gpu": P, "timing_every": args.timing_every, "n": n, "m": m, "costs": costs_file,
                   "script": want_script, "pipeline": pipeline and batch.traceback_mode != 2, "mode": batch.mode,
                   "rows_per_lane": R, "lane_pairs": nl, "packed_pairs": npk, "bitpar_pairs": nbp,
                   "scaled_pairs": batch.scaled_pairs, "segment_pairs": batch.segment_pairs,
                   "chains": batch.chains, "dot_keys": batch.dot_keys, "ladder_dot_keys": batch.ladder_dot_keys,
                   "traceback": {0: None, 1: "per-cell codes", 2: "checkpoints + recompute",
                                 3: "per-cell codes, stripe-parallel walk",
                                 4: "checkpoints, every tile's codes recomputed, stripe-parallel walk"}[batch.traceback_mode],
                   "parallelism": "dp%d" % world, "env": env},
        # the kernels issue VALU on most cycles and move a fraction of the HBM peak: "bound" names the VALU; the
        # HBM figures are the roofline the north star asks for (SURVEY.md 8(d) bytes), "valu" the binding one
        "roofline": {"bound": "valu" if valu_peak is not None else "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "time_basis": ("DP kernels' busy time per step: union of every DP launch's HIP-event interval "
                                    "over the steps of %s / steps" % time_pass) if args.timing_every == 1 else time_pass,
                     "traffic": None if traffic is None else traffic * launches,
                     "traffic_per_launch": traffic,
                     "traffic_frac": None if traffic is None else
                     traffic * launches / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "traffic_source": traffic_src,
                     "kernel": kname, "kernel_ms_per_step": dp_busy, "kernel_ms_mean_launch": dp_avg,
                     "launches_per_step": launches,
                     "algo_bytes_per_step": algo_bytes, "algo_bytes_per_launch": algo_launch,
                     "algo_bytes_def": "SURVEY.md 8(d): per pair (n+m)/4 in + 8 out" +
                                       (" + 0.25 B/cell traceback + (n+m) reads + (n+m)/4 ops out" if want_script
                                        else ""),
                     "frac_per_launch_overlapped": achieved_launch / HBM_PEAK_GBS,
                     "frac_step": algo_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "design_bytes_per_step": design_bytes,
                     "design_frac": design_bytes / (dp_busy * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "valu": None if valu_peak is None else {
            "model": "%.4g VALU ops/cell x %.2f cycles/op per wave64 (tools/ubench/valu_row.hip%s), 1024 SIMDs, "
                     "%.1f GHz" % (ops_cell, cyc, ", ubench_valu_dot.txt" if dot_cell else "", CLOCK / 1e9),
            "achieved": rate, "peak": valu_peak, "unit": "cells/s", "frac": rate / valu_peak,
            "time_basis": "kernel_ms_per_step"},
        "issue": issue, "issue_source": issue_src,
        "traceback_ms": float(np.mean(tb_ms)) if want_script else None,
        "gather_ms": gather_ms,
        # each rank's [first, stop) pair ids (config 5: query rows), regenerated from the seeds on rank 0 to verify
        "shards": [list(shard_bounds(args.workload, Pw, world, r)) for r in range(world)],
        "cpu_baseline": cpu_obj if cpu is not None else None,
    }
    if issue and line["valu"] is not None:
        dom = [k for k in parts if k in issue]
        if dom:
            line["valu"]["issue_util"] = issue[dom[0]]["valu_issue"]
    line.update(check)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

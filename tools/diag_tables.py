"""GPU diagnostic: bisect the failing ladder-dot-key CHAIN case of test_dot_keys_on_random_factorable_tables."""
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("rna-sequence-diff-patch_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import sedgpu
import test_gpu_routes as T

ctx = sedgpu.Context(0)
ck_tables, lad_tables = T._factorable_tables(3600, 3, 2, 1500, 1024)
a2, b2 = T._ragged(3602, 2200, 1, 512, 1, 512)


def run(plan, A, B, opts):
    ctx.set_costs(plan)
    for k, v in opts.items():
        ctx.set_option(k, v)
    packed = sedgpu.PackedPairs(A, B)
    try:
        b, (d, ii, ln, ops) = T._batch_run(ctx, packed, True)
        flags = (b.dot_keys, b.ladder_dot_keys, b.chains, b.rows_per_lane)
        b.close()
        try:
            T._check_all(plan, packed, d, ii, ln, ops)
            return "ok", flags
        except AssertionError as ex:
            return "mismatch " + str(ex)[:200], flags
    except sedgpu.SedError as ex:
        return "error " + str(ex), None
    finally:
        for k in opts:
            ctx.set_option(k, 0)


base = {sedgpu.SED_OPT_TB: 1, sedgpu.SED_OPT_CHAIN: 1, sedgpu.SED_OPT_ROWS_PER_LANE: 8, sedgpu.SED_OPT_LANE: 2}
for ti, table in enumerate(lad_tables):
    plan = T._plan(table)
    print("table", ti, table["insert"], table["delete"], plan.sub.tolist(), flush=True)
    for name, extra in (("lad", {}), ("nodot", {sedgpu.SED_OPT_DOT: 2}),
                        ("nochain", {sedgpu.SED_OPT_CHAIN: 2}), ("static3", {sedgpu.SED_OPT_CHAIN: 3})):
        print(" ", name, run(plan, a2, b2, {**base, **extra}), flush=True)
    # bisect the lad failure to a small subset
    idx = list(range(len(a2)))
    while len(idx) > 1:
        h = idx[:len(idx) // 2]
        r, _ = run(plan, [a2[i] for i in h], [b2[i] for i in h], base)
        if r != "ok":
            idx = h
            continue
        h2 = idx[len(idx) // 2:]
        r2, _ = run(plan, [a2[i] for i in h2], [b2[i] for i in h2], base)
        if r2 != "ok":
            idx = h2
            continue
        break
    print("  minimal failing subset:", [(i, len(a2[i]), len(b2[i])) for i in idx[:10]], len(idx), flush=True)
    if len(idx) <= 4:
        for i in idx:
            print("   pair", i, "a", "".join("ACGU"[c] for c in a2[i]), "b", "".join("ACGU"[c] for c in b2[i]),
                  flush=True)
            print("   alone:", run(plan, [a2[i]], [b2[i]], base), flush=True)
            print("   alone nodot:", run(plan, [a2[i]], [b2[i]], {**base, sedgpu.SED_OPT_DOT: 2}), flush=True)

"""Per-call engine time of sed_run_pair under two settings of one option, interleaved: a 30-nt integer distance call
(IRMethods.wf_score's idiom), a 30-nt script call, 100-nt and 250-nt integer script calls and a 300-nt fp64 distance
call.  Default: SED_OPT_ZEROCOPY 0 (results written into pinned host memory) against 2 (the download).

    python tools/zc_ab.py [OPTION A B]      e.g. python tools/zc_ab.py SED_OPT_LANE 0 2
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd")]
os.chdir(os.path.join(REPO, "tests", "golden"))
import StringEditDistance as SED  # noqa: E402
import sedcost  # noqa: E402
import sedgpu  # noqa: E402

NUC = "AGCUYRWSKMDVHBN"


def main():
    import random
    opt_name, va, vb = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("SED_OPT_ZEROCOPY", 0, 2)
    key = getattr(sedgpu, opt_name)
    random.seed(3)
    ctx = sedgpu.context()
    SED.wagnerFisher("AGRGA", "AGGGAA")
    a, b = "AAAAAAAAAAAGGGAGCGAAGUCAAGGCCC", "AAAAAAAAAAAGUGCUACGACAUUUGGGGGU"
    fa = "".join(random.choice(NUC) for _ in range(300))
    fb = "".join(random.choice(NUC) for _ in range(300))
    ia = "".join(random.choice("ACGU") for _ in range(250))
    ib = "".join(c if random.random() > 0.1 else random.choice("ACGU") for c in ia)
    cases = [("30 nt distance", SED._table(False), a, b, False), ("30 nt script", SED._table(False), a, b, True),
             ("100 nt script", SED._table(True), ia[:100], ib[:100], True),
             ("250 nt script", SED._table(True), ia, ib, True),
             ("300 nt fp64 distance", SED._table(False), fa, fb, False)]
    for name, table, x, y, script in cases:
        plan = sedcost.pair_plan(table, x, y)
        ctx.set_costs(plan)
        ex, ey = plan.encode_bytes(x), plan.encode_bytes(y)
        res = {va: [], vb: []}
        for rnd in range(6):
            for opt in (va, vb):
                ctx.set_option(key, opt)
                for _ in range(20):
                    ctx.run_pair(ex, ey, script, no_len=not script)
                t0 = time.perf_counter()
                for _ in range(200):
                    ctx.run_pair(ex, ey, script, no_len=not script)
                res[opt].append((time.perf_counter() - t0) / 200 * 1e6)
        ctx.set_option(key, 0)
        print("%-22s %s=%d: %s us; %d: %s us" % (name, opt_name, va, " ".join("%.1f" % v for v in res[va]), vb,
                                                 " ".join("%.1f" % v for v in res[vb])), flush=True)


if __name__ == "__main__":
    main()

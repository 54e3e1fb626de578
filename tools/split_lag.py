"""Config 2's SPLIT forward split into its per-step cost and its per-stripe hand-off lag: one user_costs ACGU pair
per call with m = 4096 columns and n = 256 .. 4096 rows (1 .. 16 stripes of 256 rows at R = 4), distance + script
(the checkpoint forward on dot keys).  Run under rocprofv3 --kernel-trace; the forward kernel's time against the
stripe count gives the per-step cost (one stripe: m + 63 steps) and the lag each further stripe adds.

    python tools/split_lag.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rna-sequence-diff-patch_amd")]
os.chdir(os.path.join(REPO, "tests", "golden"))  # the module loads the cost files from the CWD
import StringEditDistance as SED  # noqa: E402
import sedcost  # noqa: E402
import sedgpu  # noqa: E402
import synth  # noqa: E402


def main():
    table = SED._table(True)
    ctx = sedgpu.context()
    s1, s2 = synth.pair_strings(0, 4096, 4096)
    for n in (256, 512, 1024, 2048, 4096):
        a = s1[:n]
        plan = sedcost.pair_plan(table, a, s2)
        ctx.set_costs(plan)
        ea, eb = plan.encode_bytes(a), plan.encode_bytes(s2)
        for _ in range(6):
            ctx.run_pair(ea, eb, True)
        print("n = %d done" % n, flush=True)


if __name__ == "__main__":
    main()

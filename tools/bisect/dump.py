"""Debug builds (-DSED_TB_DEBUG): run the config-3 route batch with checkpoints forced and save pair 0's
first-tile dump (ops[0:648]) to gpurun_out/bisect/dump_<tag>.npy."""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", ".."), os.path.join(HERE, "..", "..", "tests"),
                os.path.join(HERE, "..", "..", "rna-sequence-diff-patch_amd")]
import sedgpu, sedcost, json
from test_gpu_routes import _ragged, _plan
tag = sys.argv[1]
tables = json.load(open(os.path.join(HERE, "..", "..", "tests", "golden", "costs.json")))
A, B = _ragged(3000, 12000, 1, 512, 1, 700)
ctx = sedgpu.Context()
ctx.set_costs(_plan(tables))
ctx.set_option(sedgpu.SED_OPT_TB, 2)
packed = sedgpu.PackedPairs(A, B)
b = sedgpu.Batch(ctx, packed, True)
b.run()
d, ii, ln, ops = b.results()
print(tag, "route chains", b.chains, "R", b.rows_per_lane, "tb", b.traceback_mode, "n,m", len(A[0]), len(B[0]), "len0", ln[0])
os.makedirs("gpurun_out/bisect", exist_ok=True)
np.save("gpurun_out/bisect/dump_%s.npy" % tag, ops[:648].copy())
print(tag, "scalars i j c Q k sig_end re q:", ops[640:648].tolist())

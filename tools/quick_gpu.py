import sys, os
sys.path.insert(0, 'rna-sequence-diff-patch_amd'); sys.path.insert(0, 'oracle')
import json, sedgpu, sedcost, oracle
ctx = sedgpu.Context(0)
print('selftest', ctx.selftest(), flush=True)
uc = json.load(open('tests/golden/user_costs.json'))
pairs = [("AGGA", "AGGGAA"), ("ACGU"*40, "AGU"*50)]
plan = sedcost.build_plan(uc, [a for a,_ in pairs], [b for _,b in pairs])
ctx.set_costs(plan)
pk = sedgpu.PackedPairs([plan.encode(a) for a,_ in pairs],[plan.encode(b) for _,b in pairs])
d, ii, ln, ops = ctx.run(pk, True)
cs = oracle.Costs.from_plan(plan)
for p,(a,b) in enumerate(pairs):
    o = oracle.pair(cs, plan.encode(a), plan.encode(b))
    print(p, d[p], ii[p], ln[p], '| oracle', o['dist'], o['is_int'], o['len'], flush=True)
    print(' gpu ', ''.join('idu'[c] for c in sedgpu.unpack_ops(ops, pk.ops_off, p, int(ln[p]))))
    print(' orc ', oracle.ops_to_str(o['ops']))

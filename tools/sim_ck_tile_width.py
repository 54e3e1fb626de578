"""Model of the checkpoint traceback on real canonical paths (as tools/sim_ck_tiles.py) for tiles 2, 3 or 4 column
checkpoints wide (64 rows x TW columns, the sweep starting at the tile's first checkpoint): visits, sweep steps and the
VALU estimate visits x 190 (set-up) + steps x 6 (sweep) + ops (walk v_readlane).  python tools/sim_ck_tile_width.py"""
import sys, json, numpy as np
sys.path[:0]=['rna-sequence-diff-patch_amd','oracle']
import oracle, sedcost, synth
table=json.load(open('tests/golden/user_costs.json'))
plan=sedcost.build_plan(table,['ACGU'],['ACGU'])
cs=oracle.Costs.from_plan(plan)
n=m=4096; R=16; ROWS=64*R; H=64; GH=4
for pid in range(3):
    a=synth.pair_codes([pid],n,0)[0]; b=synth.pair_codes([pid],m,1)[0]
    ops=oracle.pair(cs,a,b)['ops']
    path=[(n,m)]; i,j=n,m
    for op in ops[::-1]:
        if op==0: j-=1
        elif op==1: i-=1
        else: i-=1;j-=1
        path.append((i,j))
    for TW in (64,128,192,256):
        visits=0; steps=0; idx=0; words=0
        while True:
            i,j=path[idx]
            if i==0 or j==0: break
            k=(i-1)//ROWS; t=((i-1)%ROWS)//R; Q=t//GH
            c=(j-1+t)//TW
            rowbase=k*ROWS+H*Q
            J0=TW*c-GH*Q+1
            re=i-rowbase-1
            sig_end=(j-J0+GH-1)+re
            visits+=1; steps+=sig_end-(GH-1)+1
            while True:
                idx+=1
                i,j=path[idx]
                if i==0 or j==0: break
                if i<rowbase+1: break
                tt=((i-1)%ROWS)//R
                if j<TW*c-tt+1: break
        print(pid,'TW',TW,'visits',visits,'steps',steps,'steps/visit',round(steps/visits,1),'VALU est', visits*190+steps*6+len(ops), flush=True)

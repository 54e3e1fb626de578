"""Model of the checkpoint traceback's tile visits (sed_traceback_ck_kernel) on real canonical paths: for tile
heights H (rows per tile) and column-checkpoint intervals C, the number of tile visits and the total sweep steps
per 4096^2 pair (user_costs).  Run on the CPU: python tools/sim_ck_tiles.py (output: profiles/r03/sim_ck_tiles.txt)."""
import sys, json, numpy as np
sys.path[:0]=['rna-sequence-diff-patch_amd','oracle']
import oracle, sedcost, synth
table=json.load(open('tests/golden/user_costs.json'))
plan=sedcost.build_plan(table,['ACGU'],['ACGU'])
cs=oracle.Costs.from_plan(plan)
n=m=4096; R=16; ROWS=64*R
for pid in range(3):
    a=synth.pair_codes([pid],n,0)[0]; b=synth.pair_codes([pid],m,1)[0]
    ops=oracle.pair(cs,a,b)['ops']
    path=[(n,m)]; i,j=n,m
    for op in ops[::-1]:
        if op==0: j-=1
        elif op==1: i-=1
        else: i-=1;j-=1
        path.append((i,j))
    for H in (64,32,16):
      GH=H//R if H>=R else 1
      for C in (64,32):
        visits=0; steps=0; idx=0
        while True:
            i,j=path[idx]
            if i==0 or j==0: break
            k=(i-1)//ROWS; t=((i-1)%ROWS)//R; Q=t//GH
            c=(j-1+t)//C
            rowbase=k*ROWS+H*Q
            J0=C*c-GH*Q+1
            re=i-rowbase-1
            sig_end=(j-J0+GH-1)+re
            visits+=1; steps+=sig_end-(GH-1)+1
            while True:
                idx+=1
                i,j=path[idx]
                if i==0 or j==0: break
                if i<rowbase+1: break
                tt=((i-1)%ROWS)//R
                if j<C*c-tt+1: break
        print(pid,'H',H,'C',C,visits,steps,round(steps/visits,1),flush=True)

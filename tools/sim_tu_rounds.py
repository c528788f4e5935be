#!/usr/bin/env python3
"""Config-4 closed loop: what a CTU row's TU dataflow costs under two schedules
(DESIGN.md §6a), from the oracle's seeded quadtree of the 4K luma plane (CTB 32,
plane id 0, seed 1234) and the round-5 per-call costs (cycles, A/B stamps):
  * per CTU (the product): each CTU's rounds in turn, each (round, size) one call;
  * cross-CTU: one dataflow over the whole row, a TU ready once the TUs above and
    left of it are done even if they lie in the previous CTU.
Also counts the size combinations of the per-CTU rounds (pairs: 2 x the TUs).

    python tools/sim_tu_rounds.py        # needs oracle/ built (g.build())
"""
import sys, numpy as np
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle'))
import oracle as O
W,H,CTB,PID,SEED=3840,2160,32,0,1234
cost={4:3000,8:4800,16:8500,32:5000}
def tus_of_ctu(cx,cy):
    out=[]
    def rec(x,y,s):
        if s>4 and ((x+s>W) or (y+s>H) or O.tu_split(SEED,PID,x,y,s)):
            h=s//2
            for (dx,dy) in ((0,0),(h,0),(0,h),(h,h)): rec(x+dx,y+dy,h)
        else:
            if x+s<=W and y+s<=H: out.append((x,y,s))
    rec(cx*CTB,cy*CTB,CTB); return out
def row_tus(cy):
    return [tus_of_ctu(cx,cy) for cx in range(W//CTB)]
def schedule(tus_list, cross):
    # unit owner map for the row band
    owner={}
    allt=[t for ct in tus_list for t in ct]
    for i,(x,y,s) in enumerate(allt):
        for ux in range(x//4,(x+s)//4):
            for uy in range(y//4,(y+s)//4): owner[(ux,uy)]=i
    ctu_of=[x//CTB for (x,y,s) in allt]
    done=[False]*len(allt)
    total=0; entries=0; rounds=0
    if not cross:
        for c in range(len(tus_list)):
            idx=[i for i in range(len(allt)) if ctu_of[i]==c]
            pend=set(idx)
            while pend:
                ready=[]
                for i in pend:
                    x,y,s=allt[i]; ok=True
                    for k in range(s//4):
                        up=owner.get((x//4+k, y//4-1)); lf=owner.get((x//4-1, y//4+k))
                        if up is not None and not done[up]: ok=False
                        if lf is not None and not done[lf]: ok=False
                    if ok: ready.append(i)
                for i in ready: done[i]=True; pend.discard(i)
                sizes=set(allt[i][2] for i in ready); rounds+=1; entries+=len(sizes)
                total+=sum(cost[s] for s in sizes)
    else:
        pend=set(range(len(allt)))
        while pend:
            ready=[]
            for i in pend:
                x,y,s=allt[i]; ok=True
                for k in range(s//4):
                    up=owner.get((x//4+k, y//4-1)); lf=owner.get((x//4-1, y//4+k))
                    if up is not None and not done[up]: ok=False
                    if lf is not None and not done[lf]: ok=False
                if ok: ready.append(i)
            for i in ready: done[i]=True; pend.discard(i)
            sizes={}
            for i in ready: sizes[allt[i][2]]=sizes.get(allt[i][2],0)+1
            rounds+=1
            # capacity per batch (pairs: 2 planes): N=4:16/2=8, 8:8/2=4,16:4/2=2,32:1
            cap={4:8,8:4,16:2,32:1}
            for s,n in sizes.items():
                nb=-(-n//cap[s]); entries+=nb; total+=nb*cost[s]
    return total, entries, rounds
for cy in (5,30,60):
    tl=row_tus(cy)
    a=schedule(tl,False); b=schedule(tl,True)
    print(cy, 'per-CTU', a, 'cross', b, 'ratio %.2f'%(b[0]/a[0]))
import collections
def combos(tus_list):
    owner={}
    allt=[t for ct in tus_list for t in ct]
    for i,(x,y,s) in enumerate(allt):
        for ux in range(x//4,(x+s)//4):
            for uy in range(y//4,(y+s)//4): owner[(ux,uy)]=i
    ctu_of=[x//CTB for (x,y,s) in allt]
    done=[False]*len(allt); cnt=collections.Counter()
    for c in range(len(tus_list)):
        pend=set(i for i in range(len(allt)) if ctu_of[i]==c)
        while pend:
            ready=[]
            for i in pend:
                x,y,s=allt[i]; ok=True
                for k in range(s//4):
                    up=owner.get((x//4+k, y//4-1)); lf=owner.get((x//4-1, y//4+k))
                    if up is not None and not done[up]: ok=False
                    if lf is not None and not done[lf]: ok=False
                if ok: ready.append(i)
            for i in ready: done[i]=True; pend.discard(i)
            sz=collections.Counter(allt[i][2] for i in ready)
            cnt[tuple(sorted((s, 2*n) for s,n in sz.items()))]+=1
    return cnt
tot=collections.Counter()
for cy in range(0,68,4): tot+=combos(row_tus(cy))
for k,v in tot.most_common(25): print(v, k)

"""Lockstep probe rounds of the frontier's LDS hash table (CPU model, no GPU).

find_batch (csrc/frontier_body.h) probes a wave's 64 lanes x LB = 4 keys in lockstep: a round
reads PROBE_W buckets of 4 slots for every key still unresolved, so the wave pays for the
LONGEST probe sequence among its 256 keys, not the mean.  This inserts n random keys with the
kernel's linear bucket probing and reports the mean probe length and the expected rounds per
256-key batch for one and two buckets per round.  Output: profiles/r04_probe_rounds.txt.
"""
import numpy as np
rng=np.random.default_rng(1)
def sim(nb,n,trials=200,per_round=1,batch=256):
    res=[];mean=[]
    for t in range(trials):
        fill=np.zeros(nb,int); pl=[]
        hs=rng.integers(0,nb,n)
        for h in hs:
            b=h;k=1
            while fill[b]>=4: b=(b+1)%nb;k+=1
            fill[b]+=1; pl.append(k)
        pl=np.array(pl)
        # rounds for a batch of keys sampled from members
        s=rng.choice(pl,batch)
        r=np.ceil(s/per_round).max()
        res.append(r); mean.append(pl.mean())
    return np.mean(res), np.mean(mean)
for nb,label in [(384,"narrow 1536"),(704,"mid 2816"),(1536,"wide 6144")]:
    for n in [int(nb*4*a) for a in (0.25,0.4,0.5,0.6,0.75)]:
        m1,pm=sim(nb,n,100); m2,_=sim(nb,n,100,per_round=2)
        print(f"{label} n={n} load={n/(nb*4):.2f} mean probe {pm:.3f}  lockstep rounds per 256 keys: 1/round {m1:.2f}  2/round {m2:.2f}")

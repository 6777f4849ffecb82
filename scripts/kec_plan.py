#!/usr/bin/env python3
"""Complement plan of the JIT's Keccak-f[1600] subroutine (jit.cpp kKecInit / kKecPlan).

Lanes may be stored complemented; chi at row position x is one AND / OR plus xor (2-cycle VALU
on MI355X) when its operands b1, b2 are stored in opposite states, otherwise xor + v_bfi (v_bfi
issues at 4 cycles); a free output state that differs from the natural one costs an xnor
(4.7 cycles, profiles/r02af/valu_kinds.json).  Costs in issue cycles per 64-bit lane (two
halves) above the all-2-cycle form: bfi position 2 x 1.9, xnor 2 x 2.1, an initially
complemented lane 2 x 2.6 (two v_not).  A beam search over the 24 rounds (theta and rho-pi move
the states, chi's free outputs choose them) minimises the total; prints the init mask and the
per-round chi output states as 25-bit masks (bit x + 5y).

    python scripts/kec_plan.py
"""
import itertools, random
RHOPI = [(10,1),(7,3),(11,6),(17,10),(18,15),(3,21),(5,28),(16,36),(8,45),(21,55),(24,2),(4,14),(15,27),(23,41),(19,56),(13,8),(12,25),(2,43),(20,62),(14,18),(22,39),(9,61),(6,20),(1,44)]
def theta(P):
    c=[0]*5
    for i in range(25): c[i%5]^=P[i]
    d=[c[(x+4)%5]^c[(x+1)%5] for x in range(5)]
    return tuple(P[i]^d[i%5] for i in range(25))
def rhopi(Q):
    R=list(Q); cur=Q[1]
    for dst,_ in RHOPI:
        t=Q[dst]; R[dst]=cur; cur=t
    return tuple(R)
def info(R):
    bad=[]; nat=[]
    for y in range(0,25,5):
        for x in range(5):
            r1=R[y+(x+1)%5]; r2=R[y+(x+2)%5]; i=y+x
            if r1==r2: bad.append(i); nat.append(R[i])
            else: nat.append(R[i] if r1==1 else R[i]^1)
    return bad, nat
CB, CX, CN = 1.9, 2.1, 5.2   # bad position, xnor, initial NOT lane (both halves: x2 for CB/CX)
def step_options(R, maxflip):
    bad, nat = info(R); free=[i for i in range(25) if i not in bad]
    out=[]
    for k in range(maxflip+1):
        for fl in itertools.combinations(free, k):
            P=list(nat)
            for i in fl: P[i]^=1
            out.append((2*CB*len(bad)+2*CX*k, tuple(P)))
    return out
random.seed(0)
# initial patterns: sparse
inits=set([tuple([0]*25)])
for _ in range(3000):
    p=[0]*25
    for i in random.sample(range(25), random.randint(1,6)): p[i]=1
    inits.add(tuple(p))
beam=[(CN*2/2*sum(p), p) for p in inits]  # cost of init NOTs (2 per lane at 2.6)
beam=[(c, rhopi(theta(p)), (p,)) for c,p in beam]
beam.sort(key=lambda t:t[0]+2*CB*len(info(t[1])[0])); beam=beam[:200]
for rnd in range(24):
    cand={}
    for c,R,hist in beam:
        for dc,P in step_options(R, 3 if rnd<23 else 2):
            extra = 0
            if rnd==23:
                extra = 2*2.6*sum(P[:4])  # un-complement digest lanes
                Rn=None; key=P
            else:
                Rn=rhopi(theta(P)); key=Rn
            tot=c+dc+extra
            if key not in cand or cand[key][0]>tot: cand[key]=(tot,Rn,hist+(P,))
    beam=sorted(cand.values(), key=lambda t:t[0] + (2*CB*len(info(t[1])[0]) if t[1] else 0))[:200]
best=beam[0]
base = 24*2*CB*25  # all-bfi baseline
print("baseline extra cycles", base, "best", round(best[0],1), "saving per keccak", round(base-best[0],1))
print("init", best[2][0])
hist = best[2]
mask = lambda P: sum(b << i for i, b in enumerate(P))
print("INIT 0x%07x" % mask(hist[0]))
print("PLAN", ", ".join("0x%07x" % mask(P) for P in hist[1:]))
# re-simulate: bad counts and xnor counts per round
R = rhopi(theta(hist[0])); nb = nx = 0
for P in hist[1:]:
    bad, nat = info(R); nb += len(bad); nx += sum(1 for i in range(25) if i not in bad and P[i] != nat[i])
    R = rhopi(theta(P))
print("bad positions", nb, "xnor positions", nx, "digest lanes complemented", sum(hist[-1][:4]))

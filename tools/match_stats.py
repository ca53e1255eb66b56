#!/usr/bin/env python3
"""LZ77 match statistics of the synthetic BAM (the resolver): lengths and distances of the first
30 BGZF blocks' matches, split at the resolver's near/far distance (2808 B), with the 16-byte copy iterations each
needs.  Restates RFC 1951 decoding in Python (tools/regions_model.py).  Output: profiles/r05/match_stats.log."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "spark-bam_amd")]
import synth, collections
from regions_model import Bits, header, dec, LIT, LEN, DIST, SPEC
raw=synth.SynthBam(tile_mb=8).bytes().tobytes()
pos=0; nb=0
far=collections.Counter(); near=collections.Counter(); L_far=[]; L_near=[]
while pos+18<=len(raw) and nb<30:
    end=pos+(raw[pos+16]|(raw[pos+17]<<8))+1
    pay=raw[pos+18:end-8]; pos=end
    if len(pay)<1000: continue
    nb+=1
    bs=Bits(pay); p=0
    while True:
        fin=bs.get(p,1)
        lt,dt,p=header(bs,p)
        st=0; L=0
        while True:
            k,v,p=dec(bs,lt,dt,p,st)
            if k==SPEC: break
            if k==LEN: L=v-253; st=1
            elif k==DIST:
                d=v-0x7fff+1; st=0
                (L_far if d>2808 else L_near).append((L,d))
            else: st=0
        if fin: break
import statistics
def it(L): return (L+15)//16
print('blocks',nb,'far',len(L_far),'near',len(L_near))
print('far L mean',statistics.mean(l for l,d in L_far),'iters>2 total',sum(max(0,it(l)-2) for l,d in L_far), 'share L>32', sum(1 for l,d in L_far if l>32)/len(L_far))
print('near L mean',statistics.mean(l for l,d in L_near),'overlap(d<L)',sum(1 for l,d in L_near if d<l)/len(L_near), 'iters total', sum(it(l) for l,d in L_near))
print('far iters total', sum(it(l) for l,d in L_far))
h=collections.Counter(min(it(l),10) for l,d in L_far); print('far iter hist', sorted(h.items()))
h=collections.Counter(min(it(l),10) for l,d in L_near); print('near iter hist', sorted(h.items()))

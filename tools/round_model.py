#!/usr/bin/env python3
"""Round model of k_inflate_wave on the synthetic BAM (round 5): per BGZF block its DEFLATE blocks
(bit extents, symbols), the decoder's rounds (64 lanes x 544-bit segments, a 96-symbol warm-up per lane and round)
and the lane-steps they cost, with and without the last (BFINAL) block's rounds sized to the payload's end; and how
zlib splits a BGZF payload (non-final blocks of ~16K zlib symbols = the first ~93 % of the bits).
Output: profiles/r05/round_model.log."""
import math
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "spark-bam_amd")]
import numpy as np  # noqa: E402
import synth  # noqa: E402
from pair_stats import huff  # noqa: E402
from sbam.dist import _CL_ORDER, _LEN_EXTRA, _DIST_EXTRA  # noqa: E402

def dblocks(payload):
    """(final, header_start_bit, data_start_bit, end_bit, nsym) per deflate block"""
    n=len(payload); st={'pos':0,'bb':0,'bc':0,'bit':0}; out=[]
    def need(k):
        while st['bc']<k:
            st['bb'] |= (payload[st['pos']] if st['pos']<n else 0) << st['bc']; st['pos']+=1; st['bc']+=8
    def bits(k):
        need(k); v=st['bb']&((1<<k)-1); st['bb']>>=k; st['bc']-=k; st['bit']+=k; return v
    def sym(t):
        need(15); e=t[st['bb']&32767]; l=e&15; st['bb']>>=l; st['bc']-=l; st['bit']+=l; return e>>4
    while True:
        h0=st['bit']
        fin, typ = bits(1), bits(2)
        hlit, hdist, hclen = bits(5)+257, bits(5)+1, bits(4)+4
        cl=[0]*19
        for i in range(hclen): cl[_CL_ORDER[i]]=bits(3)
        ct=huff(cl); lens=[]
        while len(lens)<hlit+hdist:
            s=sym(ct)
            if s<16: lens.append(s)
            elif s==16: lens += [lens[-1]]*(3+bits(2))
            else: lens += [0]*((3+bits(3)) if s==17 else (11+bits(7)))
        lt, dt = huff(lens[:hlit]), huff(lens[hlit:])
        d0=st['bit']; ns=0
        while True:
            s=sym(lt); ns+=1
            if s<256: continue
            if s==256: break
            k=s-257; bits(_LEN_EXTRA[k]); d=sym(dt); bits(_DIST_EXTRA[d]); ns+=1
        out.append((fin, h0, d0, st['bit'], ns))
        if fin: break
    return out

s = synth.SynthBam(tile_mb=8.0)
raw = s.bytes().tobytes()
pos=0; bl=[]
while pos+18<=len(raw):
    bsize=raw[pos+16]|(raw[pos+17]<<8); end=pos+bsize+1
    isz=int.from_bytes(raw[end-4:end],'little')
    if isz: bl.append(raw[pos+18:end-8])
    pos=end
K=544; W=96; R=64*K
cur=ex=fin_exact=0; nb=0; ndb=0; ns_tot=0; rounds_cur=0; rounds_ex=0
bpsym=[]
for b in bl[10:110]:
    nb+=1
    for (fin,h0,d0,e,ns) in dblocks(b):
        ndb+=1; ns_tot+=ns
        bits=e-d0; r=bits/ns; bpsym.append(r)
        # current: rounds of 64*K bits until the data ends; per-lane steps per round = warm + K/r
        nr=math.ceil(bits/R); rounds_cur+=nr
        cur += nr*(W + K/r)
        # final block sized exactly (the data runs to the payload end); others as now
        if fin:
            k=math.ceil(bits/nr/64); ex += nr*(W + k/r); rounds_ex+=nr
        else:
            ex += nr*(W + K/r); rounds_ex+=nr
print("bgzf blocks", nb, "deflate blocks", ndb, "per bgzf %.2f"%(ndb/nb), "sym/dblock %.0f"%(ns_tot/ndb), "bits/sym %.2f"%np.mean(bpsym))
print("rounds/bgzf %.2f" % (rounds_cur/nb), "lane-steps/bgzf: current %.0f  final-exact %.0f (%.1f%%)" % (cur/nb, ex/nb, 100*(1-ex/cur)))
print("useful symbols per bgzf %.0f per lane %.0f" % (ns_tot/nb, ns_tot/nb/64))
from collections import Counter
c=Counter(); cf=Counter(); fr=[]
for b in bl[10:110]:
    ds=dblocks(b)
    tot=ds[-1][3]-ds[0][1]
    for (fin,h0,d0,e,ns) in ds:
        (cf if fin else c)[ns]+=1
        if not fin: fr.append((e-ds[0][1])/tot)
print("non-final nsym", c.most_common(5))
print("final nsym range", min(cf), max(cf))
print("first-block end fraction of payload: mean %.3f min %.3f max %.3f" % (np.mean(fr), min(fr), max(fr)))

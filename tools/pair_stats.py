#!/usr/bin/env python3
"""Symbol statistics of the synthetic BAM's DEFLATE streams behind the decoder's multi-symbol experiment (round 5):
per symbol its kind and code length, and how many decoder steps two-symbol root entries would save — two literals
whose codes fit a 9-, 10- or 11-bit root, or a length (with its extra bits) and a distance code within 9 bits.
Python zlib-free restatement of RFC 1951 decoding (blocks 20-60 of an 8 MB tile).  Output: profiles/r05/pair_stats.log."""
import os
import sys
import zlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "spark-bam_amd")]
import numpy as np
import synth
from sbam.dist import _CL_ORDER, _LEN_EXTRA, _DIST_EXTRA

def huff(lengths):
    tab = [0] * 32768
    code, nxt, cnt = 0, [0]*16, [0]*16
    for l in lengths: cnt[l] += 1
    cnt[0] = 0
    for l in range(1, 16):
        code = (code + cnt[l-1]) << 1; nxt[l] = code
    for sym, l in enumerate(lengths):
        if l:
            c = nxt[l]; nxt[l] += 1
            r = int(format(c, f"0{l}b")[::-1], 2)
            for j in range(r, 32768, 1 << l): tab[j] = (sym << 4) | l
    return tab

def decode(payload):
    """list of (kind, codelen, extra) per symbol; kind 0 lit,1 len,2 dist,3 eob"""
    n=len(payload); st={'pos':0,'bb':0,'bc':0}; out=[]
    def need(k):
        while st['bc']<k:
            st['bb'] |= (payload[st['pos']] if st['pos']<n else 0) << st['bc']; st['pos']+=1; st['bc']+=8
    def bits(k):
        need(k); v=st['bb']&((1<<k)-1); st['bb']>>=k; st['bc']-=k; return v
    def sym(t):
        need(15); e=t[st['bb']&32767]; st['bb']>>=e&15; st['bc']-=e&15; return e>>4, e&15
    while True:
        fin, typ = bits(1), bits(2)
        assert typ == 2
        hlit, hdist, hclen = bits(5)+257, bits(5)+1, bits(4)+4
        cl=[0]*19
        for i in range(hclen): cl[_CL_ORDER[i]]=bits(3)
        ct=huff(cl); lens=[]
        while len(lens)<hlit+hdist:
            s,_=sym(ct)
            if s<16: lens.append(s)
            elif s==16: lens += [lens[-1]]*(3+bits(2))
            else: lens += [0]*((3+bits(3)) if s==17 else (11+bits(7)))
        lt, dt = huff(lens[:hlit]), huff(lens[hlit:])
        blk=[]
        while True:
            s,l = sym(lt)
            if s<256: blk.append((0,l,0))
            elif s==256: blk.append((3,l,0)); break
            else:
                k=s-257; x=_LEN_EXTRA[k]; bits(x); blk.append((1,l,x))
                d,dl = sym(dt); dx=_DIST_EXTRA[d]; bits(dx); blk.append((2,dl,dx))
        out.append(blk)
        if fin: break
    return out

def main():
    s = synth.SynthBam(tile_mb=8.0)
    raw = s.bytes().tobytes()
    pos = 0; blocks=[]
    while pos + 18 <= len(raw):
        bsize = raw[pos+16] | (raw[pos+17]<<8); end = pos+bsize+1
        isz = int.from_bytes(raw[end-4:end],'little')
        if isz: blocks.append(raw[pos+18:end-8])
        pos = end
    print("blocks", len(blocks))
    tot = {'sym':0,'lit':0,'bits':0,'steps9':0,'steps10':0,'steps11':0,'steps9x':0, 'dblocks':0}
    for b in blocks[20:60]:
        for blk in decode(b):
            tot['dblocks']+=1
            syms=[x for x in blk]
            tot['sym']+=len(syms); tot['lit']+=sum(1 for k,_,_ in syms if k==0)
            tot['bits']+=sum(l+x for _,l,x in syms)
            for R,key in ((9,'steps9'),(10,'steps10'),(11,'steps11')):
                i=0; st=0
                while i<len(syms):
                    k,l,x=syms[i]
                    if k==0 and i+1<len(syms) and syms[i+1][0]==0 and l+syms[i+1][1]<=R: i+=2
                    else: i+=1
                    st+=1
                tot[key]+=st
            # 9-bit root: also lit+len(with no extra bits), len(no extra)+... and len+dist if total<=9
            i=0; st=0
            while i<len(syms):
                k,l,x=syms[i]
                if i+1<len(syms):
                    k2,l2,x2=syms[i+1]
                    if k==0 and k2 in (0,) and l+l2<=9: i+=2; st+=1; continue
                    if k==1 and k2==2 and l+x+l2<=9: i+=2; st+=1; continue
                i+=1; st+=1
            tot['steps9x']+=st
    print(tot)
    print("bits/sym %.2f lit frac %.3f" % (tot['bits']/tot['sym'], tot['lit']/tot['sym']))
    for k in ('steps9','steps10','steps11','steps9x'): print(k, "%.3f"%(tot[k]/tot['sym']))


if __name__ == "__main__":
    main()

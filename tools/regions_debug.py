#!/usr/bin/env python3
"""Check k_inflate_regions' hand-over records against a Python restatement of RFC 1951 (regions
pass): for every BGZF block of a synthetic BAM, its first DEFLATE block's end bit, token count (symbols less the
end-of-block code) and output bytes; reports the pieced blocks whose record differs and the blocks that went from
a successful regions pass to the exact decoder (with their DEFLATE block structure).  Needs the regions build of
branch `exp/regions` (it exports sbam_debug_inflate_resume; the main library does not).
    regions_debug.py [--size-mb 20] [--tile-mb 8]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
from pair_stats import huff  # noqa: E402
from sbam.dist import _CL_ORDER, _LEN_EXTRA, _DIST_EXTRA  # noqa: E402

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]


def dblocks(payload):
    """per DEFLATE block: (final, data_start_bit, end_bit, tokens, out_bytes)"""
    n = len(payload)
    st = {"pos": 0, "bb": 0, "bc": 0, "bit": 0}

    def need(k):
        while st["bc"] < k:
            st["bb"] |= (payload[st["pos"]] if st["pos"] < n else 0) << st["bc"]
            st["pos"] += 1
            st["bc"] += 8

    def bits(k):
        need(k)
        v = st["bb"] & ((1 << k) - 1)
        st["bb"] >>= k
        st["bc"] -= k
        st["bit"] += k
        return v

    def sym(t):
        need(15)
        e = t[st["bb"] & 32767]
        ln = e & 15
        st["bb"] >>= ln
        st["bc"] -= ln
        st["bit"] += ln
        return e >> 4

    out = []
    while True:
        fin, typ = bits(1), bits(2)
        if typ != 2:
            out.append((fin, -1, -1, -1, -1))
            break
        hlit, hdist, hclen = bits(5) + 257, bits(5) + 1, bits(4) + 4
        cl = [0] * 19
        for i in range(hclen):
            cl[_CL_ORDER[i]] = bits(3)
        ct = huff(cl)
        lens = []
        while len(lens) < hlit + hdist:
            s = sym(ct)
            if s < 16:
                lens.append(s)
            elif s == 16:
                lens += [lens[-1]] * (3 + bits(2))
            else:
                lens += [0] * ((3 + bits(3)) if s == 17 else (11 + bits(7)))
        lt, dt = huff(lens[:hlit]), huff(lens[hlit:])
        d0 = st["bit"]
        tok = ob = 0
        while True:
            s = sym(lt)
            if s < 256:
                tok += 1
                ob += 1
                continue
            if s == 256:
                break
            k = s - 257
            ob += LBASE[k] + bits(_LEN_EXTRA[k])
            d = sym(dt)
            bits(_DIST_EXTRA[d])
            tok += 2
        out.append((fin, d0, st["bit"], tok, ob))
        if fin:
            break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mb", type=float, default=20)
    ap.add_argument("--tile-mb", type=float, default=8)
    ap.add_argument("--tiles", type=int, default=1)
    ap.add_argument("--check", type=int, default=400, help="pieced blocks whose records are checked (Python decode)")
    a = ap.parse_args()
    import sbam
    import synth
    s = synth.SynthBam.for_size(int(a.size_mb * 1e6), tile_mb=a.tile_mb, threads=16, distinct=a.tiles > 1,
                                cycle=max(a.tiles, 1))
    data = s.bytes()
    f = sbam.BamFile(data, path="synth.bam")
    nb = f.blocks()[0].size
    rs = np.zeros(4 * nb, np.int32)
    npc = np.zeros(nb, np.int32)
    fn = f.L.sbam_debug_inflate_resume
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    assert fn(f.ctx, rs.ctypes.data, npc.ctypes.data) == 0
    rs = rs.reshape(nb, 4)
    st, cs, us, uo = f.blocks()
    raw = np.frombuffer(bytes(data), np.uint8)
    rep = {"blocks": int(nb), "pieced": int((npc > 0).sum()), "regions_ok": int((rs[:, 0] >= 0).sum()),
           "fallbacks": int(f.inflate_fallbacks()), "record_mismatch": [], "lost_after_regions": []}
    checked = 0
    for b in range(nb):
        if rs[b, 0] < 0 or checked >= a.check:
            continue
        checked += 1
        p0 = int(st[b])
        xlen = int(raw[p0 + 10]) | (int(raw[p0 + 11]) << 8)
        a0 = p0 + 12 + xlen
        pay = raw[a0:p0 + int(cs[b]) - 8].tobytes()
        skip = (a0 - ((a0 >> 4) << 4)) * 8
        ds = dblocks(pay)
        fin, d0, e, tok, ob = ds[0]
        exp = (skip + e, tok, ob, int(fin))
        got = (int(rs[b, 0]), int(rs[b, 1]), int(rs[b, 2]), int(rs[b, 3]) >> 16)
        if exp != got:
            rep["record_mismatch"].append({"block": b, "expected": exp, "got": got, "npm": int(rs[b, 3]) & 0xffff})
        if npc[b] == 0:
            rep["lost_after_regions"].append({"block": b, "record": got, "npm": int(rs[b, 3]) & 0xffff,
                                              "dblocks": [(int(x[0]), int(x[3]), int(x[4])) for x in ds],
                                              "usize": int(us[b])})
    why = {}
    for b in range(nb):
        if rs[b, 0] < 0:
            k = ["not eligible", "header", "short", "no end of block", "rejoin", "stop kind", "bytes", "unknown stops",
                 "slot overflow"][int(rs[b, 1])]
            why[k] = why.get(k, 0) + 1
    rep["not_pieced"] = why
    rep["checked"] = checked
    rep["lost"] = int(((rs[:, 0] >= 0) & (npc == 0)).sum())  # passes whose block then went to the exact decoder
    rep["record_mismatch"] = rep["record_mismatch"][:10]
    rep["lost_after_regions"] = rep["lost_after_regions"][:10]
    print(json.dumps(rep), flush=True)
    f.close()


if __name__ == "__main__":
    main()

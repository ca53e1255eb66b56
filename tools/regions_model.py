#!/usr/bin/env python3
"""Python model of k_inflate_regions' pass (regions pass) over the first DEFLATE block of real
BGZF payloads: 64 lane regions of Rb bits, a kRW-bit warm-up per lane, sub-rounds of Sb bits, stops recorded (the
first two) and decoding on, sub-round-0 checkpoints every 8 steps, then the entry/exit check and the rejoin
re-decode.  Reports how many passes succeed, why the others fail, and checks a successful pass's end-of-block
position, token and byte counts against a straight decode.   regions_model.py [--blocks 40] [--tile-mb 8]"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]
from pair_stats import huff  # noqa: E402
from regions_debug import dblocks, LBASE  # noqa: E402
from sbam.dist import _CL_ORDER, _LEN_EXTRA, _DIST_EXTRA  # noqa: E402

KRS, KRW, KH, KCP, KCPS = 480, 480, 48, 12, 8
LIT, LEN, DIST, SPEC = 0, 1, 2, 3
ST_NONE, ST_EOB, ST_ERR, ST_OUT = 0, 1, 2, 3


class Bits:
    def __init__(self, payload):
        self.v = int.from_bytes(payload + b"\0" * 16, "little")
        self.n = 8 * len(payload)

    def get(self, pos, k):
        return (self.v >> pos) & ((1 << k) - 1)


def header(bs, pos):
    """(lit table, dist table, data start) of the dynamic block at pos"""
    def bits(k):
        nonlocal pos
        v = bs.get(pos, k)
        pos += k
        return v

    def sym(t):
        nonlocal pos
        e = t[bs.get(pos, 15)]
        pos += e & 15
        return e >> 4
    fin, typ = bits(1), bits(2)
    assert typ == 2
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
    return huff(lens[:hlit]), huff(lens[hlit:]), pos


def dec(bs, lt, dt, pos, st):
    """one symbol in state st (0 literal/length, 1 distance): (kind, token, new pos)"""
    t = dt if st else lt
    e = t[bs.get(pos, 15)]
    s, ln = e >> 4, e & 15
    if ln == 0:
        return SPEC, 1, pos + 1
    pos += ln
    if st:
        if s >= 30:
            return SPEC, 1, pos
        x = _DIST_EXTRA[s]
        base = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
                4097, 6145, 8193, 12289, 16385, 24577][s]
        return DIST, 0x7fff + base + bs.get(pos, x), pos + x
    if s < 256:
        return LIT, s, pos
    if s == 256:
        return SPEC, 0, pos
    if s > 285:
        return SPEC, 1, pos
    k = s - 257
    x = _LEN_EXTRA[k]
    return LEN, 253 + LBASE[k] + bs.get(pos, x), pos + x


def run_pass(payload):
    bs = Bits(payload)
    lt, dt, P0 = header(bs, 0)
    pend = bs.n
    Rb = ((pend - P0 + 63) // 64 + 31) & ~31
    NS = (Rb + KRS - 1) // KRS
    Sb = (((Rb + NS - 1) // NS) + 31) & ~31
    lanes = []
    for k in range(64):
        rs, re = P0 + k * Rb, P0 + (k + 1) * Rb
        st, pl, go = 0, 0, rs < pend
        rp = P0 if k == 0 else max(P0, rs - KRW)
        if k > 0 and go:
            while rp < rs:
                kind, v, rp = dec(bs, lt, dt, rp, st)
                pl = v - 253 if kind == LEN else pl
                st = 1 if kind == LEN else 0
        if not go:
            rp = pend
        entry = (rp, st, pl)
        stops, tok, byt, cps = [], 0, 0, {}
        toks = []
        if not go:
            stops.append((rs, rs, ST_OUT, 0, 0))
        for j in range(NS):
            sub_end = min(rs + (j + 1) * Sb, re)
            nsub = 0
            while go and rp < sub_end:
                if j == 0 and nsub % KCPS == 0 and nsub // KCPS < KCP and st == 0:
                    cps[rp] = (tok, byt)
                p0 = rp
                kind, v, rq = dec(bs, lt, dt, rp, st)
                outp = rq > pend
                if kind == SPEC or outp:
                    stops.append((p0, rq, ST_OUT if outp else ST_EOB if v == 0 else ST_ERR, tok, byt))
                    if outp:
                        go = False
                rp = rq
                toks.append(v)
                cnt = not (kind == SPEC or outp)
                if cnt and kind == LEN:
                    byt += v - 253
                    pl = v - 253
                elif cnt and kind == LIT:
                    byt += 1
                tok += 1
                st = 1 if (cnt and kind == LEN) else 0
                nsub += 1
            # checkpoints at group starts the lane reaches after its last step in sub-round 0 are not live
        lanes.append(dict(entry=entry, exit=(rp, st, pl), stops=stops, tok=tok, byt=byt, cps=cps, toks=toks))
    # verification
    res = []
    for k in range(64):
        L = lanes[k]
        pex = L["entry"] if k == 0 else lanes[k - 1]["exit"]
        frm, fixn, fixb, ccb, fstop, bad = 0, 0, 0, 0, None, None
        if pex != L["entry"]:
            r, s4 = pex[0], pex[1]
            cands = sorted(p for p in L["cps"])
            tk = by = 0
            lim = ((min(r, pend) >> 5) + 16) * 32
            while True:
                nxt = [p for p in cands if p >= r]
                if s4 == 0 and nxt and nxt[0] == r:
                    frm, ccb = L["cps"][r]
                    fixn, fixb = tk, by
                    if frm - tk < -KH:
                        bad = "prefix>headroom"
                    break
                if not nxt or r >= lim:
                    bad = "no rejoin"
                    break
                kind, v, r = dec(bs, lt, dt, r, s4)
                if kind == SPEC or r > pend:
                    fstop = (ST_OUT if r > pend else ST_EOB if v == 0 else ST_ERR, r)
                    fixn, fixb = tk, by
                    break
                tk += 1
                by += 1 if kind == LIT else (v - 253 if kind == LEN else 0)
                s4 = 1 if kind == LEN else 0
        if fstop:
            res.append(dict(stop=fstop, n=fixn, b=fixb, bad=bad))
            continue
        later = [s for s in L["stops"] if s[3] >= frm]
        unk = not later and len(L["stops"]) > 2 and False  # (the kernel keeps two stops: see below)
        kept = L["stops"][:2]
        later = [s for s in kept if s[3] >= frm]
        if not later and len(L["stops"]) > 2:
            bad = bad or "stops unknown"
        if later:
            s = later[0]
            res.append(dict(stop=(s[2], s[1]), n=fixn + s[3] - frm, b=fixb + s[4] - ccb, bad=bad))
        else:
            res.append(dict(stop=None, n=fixn + L["tok"] - frm, b=fixb + L["byt"] - ccb, bad=bad))
    for k, r in enumerate(res):
        if r["bad"]:
            return {"ok": False, "why": r["bad"], "lane": k}
        if r["stop"]:
            if r["stop"][0] != ST_EOB:
                return {"ok": False, "why": "stop %d" % r["stop"][0], "lane": k}
            return {"ok": True, "f": k, "pos": r["stop"][1], "tok": sum(x["n"] for x in res[:k + 1]),
                    "byt": sum(x["b"] for x in res[:k + 1])}
    return {"ok": False, "why": "no stop"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=40)
    ap.add_argument("--tile-mb", type=float, default=8)
    a = ap.parse_args()
    import synth
    raw = synth.SynthBam(tile_mb=a.tile_mb).bytes().tobytes()
    pos, pays = 0, []
    while pos + 18 <= len(raw):
        end = pos + (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
        if int.from_bytes(raw[end - 4:end], "little"):
            pays.append(raw[pos + 18:end - 8])
        pos = end
    why = collections.Counter()
    wrong = 0
    for p in pays[5:5 + a.blocks]:
        r = run_pass(p)
        if r["ok"]:
            fin, d0, e, tok, ob = dblocks(p)[0]
            if (r["pos"], r["tok"], r["byt"]) != (e, tok, ob):
                wrong += 1
            why["ok"] += 1
        else:
            why[r["why"]] += 1
    print(json.dumps({"passes": sum(why.values()), "outcomes": dict(why), "wrong_results": wrong}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Python model of k_inflate_resolve's step structure (sbam_inflate.hip) over the synthetic BAM's token streams:
128 tokens per step (two per lane), the step cut kSpan bytes past its base, matches in dependency rounds, copies in
steps of <= 16 bytes with the overlapping-copy distance doubling.  Reports rounds and copy iterations per step (the
wave pays the slowest ready lane of a round) under the kernel's readiness rule and under the exact rule (a match is
ready when its source meets no pending output), so a change to either is priced before it is built.
Restates RFC 1951 decoding in Python (tools/regions_model.py).   resolve_model.py [--blocks 30] [--tile-mb 8]"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "spark-bam_amd")]
import synth  # noqa: E402
from regions_model import Bits, header, dec, LEN, DIST, SPEC  # noqa: E402

NEAR = 4096 - 1024 - 264  # RingGeom<12>::kNear


def block_tokens(pay):
    """the block's tokens as (kind, value): 'l' byte, 'L' length, 'd' distance"""
    bs, p, out = Bits(pay), 0, []
    while True:
        fin = bs.get(p, 1)
        lt, dt, p = header(bs, p)
        st = 0
        while True:
            k, v, p = dec(bs, lt, dt, p, st)
            if k == SPEC:
                break
            if k == LEN:
                out.append(("L", v - 253))
                st = 1
            elif k == DIST:
                out.append(("d", v - 0x7fff))
                st = 0
            else:
                out.append(("l", v))
                st = 0
        if fin:
            return out


def iters(L, d):
    n, done, deff = 0, 0, d
    while done < L:
        k = min(L - done, 16, deff)
        done += k
        n += 1
        if k == deff:
            deff *= 2
    return n


def run_block(tok, span=1024, lanes=64, exact=False, far_first=False):
    ae = sum(1 if k == "l" else v if k == "L" else 0 for k, v in tok)
    tok = tok + [("p", 0)] * (2 * lanes + 2)
    B, tp, steps, rounds, its = 0, 0, 0, 0, 0
    while B < ae:
        lanes_ = []
        for i in range(lanes):
            a, b, n = tok[tp + 2 * i], tok[tp + 2 * i + 1], tok[tp + 2 * i + 2]
            nl = (a[0] == "l") + (b[0] == "l")
            Lm = a[1] if a[0] == "L" else b[1] if b[0] == "L" else 0
            d = b[1] if a[0] == "L" else n[1] if b[0] == "L" else 0
            lanes_.append((nl, Lm, d, b[0] == "L"))
        O, acc, take = [], 0, []
        for nl, Lm, d, bl in lanes_:
            O.append(B + acc)
            take.append(acc < span and B + acc < ae)
            acc += nl + Lm
        nt = take.index(False) if False in take else lanes
        E = min(ae, O[nt - 1] + lanes_[nt - 1][0] + lanes_[nt - 1][1])
        ms = []  # (mO, Le, d)
        for i in range(nt):
            nl, Lm, d, bl = lanes_[i]
            if Lm:
                mO = O[i] + nl
                Le = min(Lm, ae - mO)
                if Le > 0:
                    ms.append((mO, Le, d))
        pend = list(range(len(ms)))
        first = True
        while pend:
            fr = ms[pend[0]][0]
            ready = []
            for idx, j in enumerate(pend):
                mO, Le, d = ms[j]
                s, se = mO - d, mO - d + min(Le, d)
                if exact or (far_first and first and d > NEAR):
                    ok = all(not (ms[q][0] < se and s < ms[q][0] + ms[q][1]) for q in pend if q != j)
                else:
                    pb = pend[:idx]
                    ok = se <= fr or not pb or ms[pb[-1]][0] + ms[pb[-1]][1] <= s
                if ok:
                    ready.append(j)
            rounds += 1
            its += max(iters(ms[j][1], ms[j][2]) for j in ready)
            pend = [j for j in pend if j not in ready]
            first = False
        steps += 1
        B = E
        tp = tp + 2 * nt + (1 if lanes_[nt - 1][3] else 0)
    return steps, rounds, its


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=30)
    ap.add_argument("--tile-mb", type=float, default=8)
    ap.add_argument("--span", type=int, default=1024)
    args = ap.parse_args()
    raw = synth.SynthBam(tile_mb=args.tile_mb).bytes().tobytes()
    pos, toks = 0, []
    while pos + 18 <= len(raw) and len(toks) < args.blocks:
        end = pos + (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
        pay = raw[pos + 18:end - 8]
        pos = end
        if len(pay) >= 1000:
            toks.append(block_tokens(pay))
    res = {}
    for name, kw in (("kernel_rule", {}), ("exact_rule", {"exact": True})):
        t = collections.Counter()
        for tk in toks:
            s, r, i = run_block(tk, span=args.span, **kw)
            t["steps"] += s
            t["rounds"] += r
            t["iters"] += i
        res[name] = {"steps": t["steps"], "rounds_per_step": round(t["rounds"] / t["steps"], 3),
                     "iters_per_step": round(t["iters"] / t["steps"], 3)}
    print(json.dumps({"blocks": len(toks), "span": args.span, **res}))


if __name__ == "__main__":
    main()

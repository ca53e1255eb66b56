#!/usr/bin/env python3
"""Pins bench.py's full-size parity digests with the CPU oracle (test infrastructure).

bench.py prints, for its full-check workload, two sharding-independent digests of the whole file's result:

* ``counts``: sha1[:16] of the packed full-check Counts vector (sbam.dist.pack_counts: per-flag totals, keys 1-2
  per flag, positions per key, readsBeforeError, close-call pairs, successes, TooFewFixedBlockBytes-only results,
  positions) — FullCheck.scala:141-191;
* ``splits``: sha1[:16] of the split rows (first record Pos, non-empty, records per split) of compute-splits at
  the bench's split size — CanLoadBam.scala:245-279, 281-334.

This script recomputes both with the oracle (oracle/oracle.c, the C restatement of the reference) over the exact
bytes bench.py generates (tools/synth.py with the same arguments), at full size, in the build container, and
writes them to tests/golden/bench_digests.json; bench.py sets ``parity.digest_pinned`` and requires equality for
``parity.ok`` when its workload has an entry.  A 10-80 GB file does not fit in host memory, so the oracle runs
over the file's segments (header blocks, each 64 MB tile, the unplaced tail — all block- and record-aligned):
segment k's positions are checked in the window u_k ++ u_k+1 ++ ... (at least 64 MB past the segment, or to the
true end of the stream), and a position whose evaluation reaches the window's end is counted (``hits``) — any hit
outside the last window fails the run, since that position's result could differ from the whole file's.
Hadoop splits are evaluated the same way: FindBlockStart on the compressed bytes from the split start,
FindRecordStart and the record chain in the window of the segment holding the split's first block.

    python tests/golden/make_bench_digests.py --size-gb 10            # bench.py's default N=1 line
    python tests/golden/make_bench_digests.py --size-gb 3.75 --world 8 # configs[2]: 30 GB, --gpus 8 --size-gb 3.75
    python tests/golden/make_bench_digests.py --size-gb 10 --level 0   # bench.py --level 0 (stored blocks)
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import oracle  # noqa: E402
import synth  # noqa: E402

OUT = os.path.join(HERE, "bench_digests.json")
HALO = 64 << 20  # uncompressed bytes a window extends past its segment (R = 10 chains of short reads: ~4 KB)
N_COUNT_WORDS = 19 + 21 * 19 + 21 + 21 * 128 + 19 * 19 + 3


def workload_key(s, args) -> dict:
    """What identifies the file and the run: the bytes (generator arguments and exact size) and the split size."""
    return {"file_bytes": int(s.size), "seed": args.seed, "tile_mb": args.tile_mb, "tiles": args.tiles,
            "read_len": args.read_len, "level": args.level, "split_mb": args.split_mb, "reads_to_check": 10}


def lib():
    L = oracle.lib()
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    L.or_counts_window.restype = None
    L.or_counts_window.argtypes = [vp, i64, vp, i32, i64, i64, i32, vp, vp, vp, vp, vp]
    L.or_find_record_start_window.restype = i64
    L.or_find_record_start_window.argtypes = [vp, i64, vp, i32, i64, i32, i64, vp]
    return L


def segments(s):
    """(compressed lo, hi, content id) of the file's block- and record-aligned pieces, in file order: the header
    blocks, every tile (a cycled tile repeats an earlier one's bytes: same id), the unplaced tail + EOF marker."""
    out = [(0, s.header.size, "header")]
    for k in range(s.copies):
        if s.distinct:
            lo, hi = int(s.tile_starts[k]), int(s.tile_starts[k + 1])
            cid = f"tile{k % len(s.tiles)}"
        else:
            lo, hi = s.header.size + k * s.tile.size, s.header.size + (k + 1) * s.tile.size
            cid = "tile0"
        out.append((lo, hi, cid))
    out.append((s.body, s.size, "tail"))
    return [x for x in out if x[1] > x[0]]


def block_table(d: np.ndarray):
    cap = d.size // 26 + 2
    st = np.zeros(cap, np.int64)
    cs, us, hs = (np.zeros(cap, np.int32) for _ in range(3))
    n = oracle.lib().or_metadata_stream(d.ctypes.data, d.size, 0, cap, st.ctypes.data, cs.ctypes.data,
                                        us.ctypes.data, hs.ctypes.data, None, None, None, None)
    if n < 0:
        raise ValueError("HeaderParseException inside a segment")
    return st[:n], cs[:n], us[:n], hs[:n]


def inflate(d, tab, threads):
    st, cs, us, hs = tab
    n = st.size
    uoff = np.zeros(n + 1, np.int64)
    uoff[1:] = np.cumsum(us.astype(np.int64))
    u = np.zeros(max(int(uoff[-1]), 1), np.uint8)
    cuts = np.linspace(0, n, max(1, min(threads, n)) + 1).astype(np.int64)

    def run(i):
        b0, b1 = int(cuts[i]), int(cuts[i + 1])
        if b1 <= b0:
            return
        out = u[int(uoff[b0]):]
        tot = oracle.lib().or_inflate_blocks(d.ctypes.data, b1 - b0, st[b0:b1].ctypes.data, cs[b0:b1].ctypes.data,
                                             us[b0:b1].ctypes.data, hs[b0:b1].ctypes.data, out.ctypes.data,
                                             int(uoff[b1] - uoff[b0]), None, None, None)
        if tot < 0:
            raise IOError("inflate failed")
    with ThreadPoolExecutor(len(cuts) - 1) as ex:
        list(ex.map(run, range(len(cuts) - 1)))
    return u[:int(uoff[-1])]


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-gb", type=float, default=10.0, help="compressed GB per GPU (bench.py --size-gb)")
    ap.add_argument("--world", type=int, default=1, help="bench.py --gpus (the file is world x size-gb)")
    ap.add_argument("--tile-mb", type=float, default=64.0)
    ap.add_argument("--tiles", type=int, default=16)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EEDBA11)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--level", type=int, default=6, help="zlib level of the synthetic blocks (bench.py --level)")
    ap.add_argument("--split-mb", type=float, default=2.0)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--halo-mb", type=float, default=HALO / (1 << 20))
    ap.add_argument("--out", default=OUT, help="digest database to update ('' = print only)")
    return ap


def pin(args) -> dict:
    """The oracle's digests for bench.py's workload `args` (see the module docstring)."""
    T = args.threads
    halo = int(args.halo_mb * (1 << 20))
    L = lib()
    t_all = time.time()
    s = synth.SynthBam.for_size(int(args.size_gb * 1e9 * args.world), tile_mb=args.tile_mb, seed=args.seed, threads=T,
                                read_len=args.read_len, level=args.level, distinct=args.tiles > 1,
                                cycle=max(args.tiles, 1))
    segs = segments(s)
    print(f"file {s.size} B, {s.n_records} records, {len(segs)} segments", flush=True)

    # block table of the whole file (MetadataStream per segment; every segment starts and ends on a block)
    starts, uoffs, seg_b0 = [], [np.zeros(1, np.int64)], []
    tabs = {}  # content id → block table (relative to the segment)
    nb = 0
    for lo, hi, cid in segs:
        if cid not in tabs:
            tabs[cid] = block_table(s.slice(lo, hi))
        st, cs, us, hs = tabs[cid]
        seg_b0.append(nb)
        starts.append(st + lo)
        uoffs.append(us.astype(np.int64))
        nb += st.size
    seg_b0.append(nb)
    start = np.concatenate(starts)
    uoff = np.cumsum(np.concatenate(uoffs))  # uoff[b] = stream offset of block b; uoff[nb] = stream length
    U = int(uoff[-1])
    seg_x = [int(uoff[b]) for b in seg_b0]
    print(f"{nb} blocks, {U} uncompressed bytes ({time.time() - t_all:.1f}s)", flush=True)

    # ContigLengths from the header segment (Header.scala:26-60, as BamFile does)
    u0 = inflate(s.slice(*segs[0][:2]), tabs[segs[0][2]], 1)
    lens = np.zeros(1 << 16, np.int64)
    end = np.zeros(1, np.int64)
    nref = int(oracle.lib().or_bam_header(u0.ctypes.data, u0.size, lens.ctypes.data, lens.size, end.ctypes.data))
    assert nref > 0

    # Hadoop splits → the segment of each split's first block
    split_size = int(args.split_mb * (1 << 20))
    hsplits = oracle.hadoop_splits(s.size, split_size)
    fbs = []
    for a, _ in hsplits:
        d = s.slice(a, min(s.size, a + (1 << 20)))
        out = np.zeros(1, np.int64)
        if oracle.lib().or_find_block_start(d.ctypes.data, d.size, 0, 5, out.ctypes.data) != 0:
            raise RuntimeError(f"HeaderSearchFailedException: {a}")
        fbs.append(a + int(out[0]))
    fbs = np.array(fbs, np.int64)

    counts = np.zeros(21 * 19, np.int64)
    npos = np.zeros(21, np.int64)
    rbe = np.zeros(21 * 128, np.int64)
    pair = np.zeros(19 * 19, np.int64)
    scal = np.zeros(3, np.int64)
    rows = np.zeros((len(hsplits), 4), np.int64)
    inflated = {}  # segment index → stream bytes (a rolling window)
    pool = ThreadPoolExecutor(T)

    def seg_u(k):
        if k not in inflated:
            lo, hi, cid = segs[k]
            inflated[k] = inflate(s.slice(lo, hi), tabs[cid], T)
        return inflated[k]

    blk_of_split = np.searchsorted(start, fbs)
    for k in range(len(segs)):
        t0 = time.time()
        parts, j = [seg_u(k)], k + 1
        while j < len(segs) and sum(p.size for p in parts) - parts[0].size < halo:
            parts.append(seg_u(j))
            j += 1
        final = j == len(segs)
        for old in [i for i in inflated if i < k]:
            del inflated[old]
        B = np.concatenate(parts) if len(parts) > 1 else parts[0]
        xs = seg_x[k]  # stream offset of B[0]
        n_here = parts[0].size
        # full check of segment k's positions (one or_counts_window per thread chunk; ctypes drops the GIL)
        cuts = np.linspace(0, n_here, T * 4 + 1).astype(np.int64)

        def one(i):
            c, npp, r, pr, sc = (np.zeros(21 * 19, np.int64), np.zeros(21, np.int64), np.zeros(21 * 128, np.int64),
                                 np.zeros(19 * 19, np.int64), np.zeros(3, np.int64))
            L.or_counts_window(B.ctypes.data, B.size, lens.ctypes.data, nref, int(cuts[i]), int(cuts[i + 1]), 10,
                               c.ctypes.data, npp.ctypes.data, r.ctypes.data, pr.ctypes.data, sc.ctypes.data)
            return c, npp, r, pr, sc
        seg_hits = 0
        for c, npp, r, pr, sc in pool.map(one, range(len(cuts) - 1)):
            counts += c
            npos += npp
            rbe += r
            pair += pr
            scal[:2] += sc[:2]
            seg_hits += int(sc[2])
        if seg_hits and not final:
            raise RuntimeError(f"segment {k}: {seg_hits} positions reached the window's end; widen HALO")
        # splits whose first block lies in segment k
        for i in np.nonzero((blk_of_split >= seg_b0[k]) & (blk_of_split < seg_b0[k + 1]))[0]:
            b = int(blk_of_split[i])
            assert int(start[b]) == int(fbs[i])
            x0 = int(uoff[b]) - xs
            hits = np.zeros(1, np.int64)
            x = int(L.or_find_record_start_window(B.ctypes.data, B.size, lens.ctypes.data, nref, x0, 10, 10_000_000,
                                                  hits.ctypes.data))
            if hits[0] and not final:
                raise RuntimeError(f"split {i}: FindRecordStart reached the window's end")
            if x < 0:
                raise RuntimeError(f"NoReadFoundException: {hsplits[i][0]}")
            be = int(np.searchsorted(start, hsplits[i][1], side="left"))
            x_end = (int(uoff[be]) if be < nb else U) - xs
            if x_end > B.size:
                raise RuntimeError(f"split {i}: its end lies past the window")
            cap = (x_end - x) // 36 + 2
            recs = np.zeros(cap, np.int64)
            n = int(oracle.lib().or_record_chain(B.ctypes.data, B.size, x, x_end, recs.ctypes.data, cap))
            if n:
                last = int(recs[n - 1])
                nxt = last + 4 + int(np.frombuffer(B[last:last + 4].tobytes(), "<i4")[0])
                if nxt < x_end and not final:
                    raise RuntimeError(f"split {i}: the record chain stopped at the window's end")
            xg = x + xs
            bx = int(np.searchsorted(uoff, xg, side="right")) - 1
            rows[i] = (int(start[bx]), xg - int(uoff[bx]), int(n > 0), n)
            if n == 0:
                raise RuntimeError(f"split {i} is empty: bench.py's empty-split row convention is not pinned here")
        print(f"segment {k + 1}/{len(segs)}: {n_here / 1e6:.0f} MB of positions, hits {seg_hits} "
              f"({'final window' if final else 'none allowed'}), {time.time() - t0:.1f}s", flush=True)
    pool.shutdown()

    totals = counts.reshape(21, 19).sum(0)
    by_key = counts.reshape(21, 19).copy()
    by_key[3:] = 0  # the GPU counts path keeps the per-flag table for keys 1-2 only (the report's close calls)
    packed = np.concatenate([totals, by_key.ravel(), npos, rbe, pair,
                             np.array([scal[0], scal[1], U], np.int64)]).astype(np.int64)
    assert packed.size == N_COUNT_WORDS
    assert int(scal[0]) == s.n_records and int(rows[:, 3].sum()) == s.n_records, "oracle self-check failed"
    dig = {"counts": hashlib.sha1(packed.tobytes()).hexdigest()[:16],
           "splits": hashlib.sha1(rows.ravel().tobytes()).hexdigest()[:16], "n_splits": len(hsplits)}
    entry = {"workload": workload_key(s, args), "digest": dig, "records": s.n_records, "n_success": int(scal[0]),
             "uncompressed_bytes": U, "made_by": f"tests/golden/make_bench_digests.py --size-gb {args.size_gb:g} "
             f"--world {args.world}" + (f" --level {args.level}" if args.level != 6 else ""),
             "oracle_wall_s": round(time.time() - t_all, 1), "threads": T}
    print(json.dumps(entry), flush=True)
    return entry


def main():
    args = parser().parse_args()
    entry = pin(args)
    if not args.out:
        return
    db = json.load(open(args.out)) if os.path.exists(args.out) else []
    db = [e for e in db if e["workload"] != entry["workload"]] + [entry]
    db.sort(key=lambda e: e["workload"]["file_bytes"])
    with open(args.out, "w") as fh:
        json.dump(db, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main()

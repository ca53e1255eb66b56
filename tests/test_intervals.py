"""loadBamIntervals: BAI chunk query and the interval-filtered record stream.

Pinned by LoadBAMTest.scala:47-102 on 2.bam + 2.bam.bai: "indexed all" (1:0-100000 → one chunk
0:5650-531725:0, 2450 records = 2500 minus 50 unmapped) and "indexed disjoint regions"
(1:13000-14000,1:60000-61000 → chunks 0:5650-314028:45444 and 439897:20150-439897:39777, 129 records, 1
partition at the default split size and 2 at MaxSplitSize(10000))."""
import os

import numpy as np
import pytest

from conftest import FIXTURES

CASES = [
    ("1:0-100000", [("0:5650", "531725:0")], 2450, None, 1),
    ("1:13000-14000,1:60000-61000", [("0:5650", "314028:45444"), ("439897:20150", "439897:39777")], 129, None, 1),
    ("1:13000-14000,1:60000-61000", [("0:5650", "314028:45444"), ("439897:20150", "439897:39777")], 129, 10000, 2),
]


def _bai():
    from sbam import bai
    return bai.parse_bai(open(os.path.join(FIXTURES, "2.bam.bai"), "rb").read())


def _query(loci):
    from sbam import bai
    return [(0 if c == "1" else -1, a + 1, e) for c, a, e in bai.parse_loci(loci)]


@pytest.mark.parametrize("loci,chunks,n,split,nparts", CASES)
def test_chunks_and_counts_on_oracle(loci, chunks, n, split, nparts, oracle_files):
    """Chunk list (htsjdk getFileSpan restated) and the filtered record count, with the record chains and
    reference spans computed on the CPU oracle's stream."""
    from sbam import bai
    got = bai.file_span(_bai(), _query(loci))
    assert [c.pos_str() for c in got] == chunks
    groups = bai.capped_cost_groups([c.size() for c in got], float(split or (32 << 20)))
    assert len(groups) == nparts
    o = oracle_files("2.bam")
    u = o.u.tobytes()
    st = np.asarray(o.start)

    def off(v):
        b, k = v >> 16, v & 0xffff
        i = int(np.searchsorted(st, b))
        return int(o.uoff[i]) + k if i < st.size and st[i] == b else o.L

    def i32(x):
        return int.from_bytes(u[x:x + 4], "little", signed=True)

    total = 0
    for c in got:
        x, end = off(c.start), off(c.end)
        while x < end:
            ri, pos, lrn, fnc = i32(x + 4), i32(x + 8), u[x + 12], i32(x + 16) & 0xffffffff
            nc, flag = fnc & 0xffff, fnc >> 16
            rl = sum(i32(x + 36 + lrn + 4 * k) >> 4 for k in range(nc)
                     if (i32(x + 36 + lrn + 4 * k) & 0xf) in (0, 2, 3, 7, 8))
            e = 0 if flag & 4 else pos + rl
            if ri == 0 and any(pos < b and e > a for _, a, b in bai.parse_loci(loci)):
                total += 1
            x += 4 + i32(x)
    assert total == n


@pytest.mark.gpu
@pytest.mark.parametrize("loci,chunks,n,split,nparts", CASES)
def test_load_bam_intervals(loci, chunks, n, split, nparts, gpu_files, oracle_files):
    g = gpu_files("2.bam")
    bai_bytes = open(os.path.join(FIXTURES, "2.bam.bai"), "rb").read()
    kw = {} if split is None else {"split_size": split}
    got_chunks, parts = g.load_bam_intervals(bai_bytes, loci, **kw)
    assert [c.pos_str() for c in got_chunks] == chunks
    assert len(parts) == nparts and sum(p.size for p in parts) == n
    offs = np.concatenate(parts)
    # every kept record is a real record start (the .records truth) and the spans match a host re-read
    truth = set(g.offset_of(__import__("sbam").Pos(*map(int, ln.split(","))))
                for ln in open(os.path.join(FIXTURES, "2.bam.records")))
    assert set(offs.tolist()) <= truth
    ri, st, en = g.record_spans(offs)
    assert np.all(ri == 0) and np.all(en >= st)

"""BASELINE configs[2] and configs[3] on one GPU.

configs[2] (full-check of a multi-GB Illumina-like BAM across 8 shards, exact verdict diff): sbam.dist.run_file
over a >= 4 GB file on disk as 8 byte-range shards (GpuShard: pread of [lo, owned_hi + halo), rank-0 header
parse, counts/bitmap checker + split records), combined like the 8-rank run's all_gather/all_reduce.  The
expected Counts and splits come from the CPU oracle on the same generator with 2, 3 and 4 tile copies: the file is
header | tile x k | unplaced tail | EOF, every middle tile contributes the same Counts (checked: C4 - C3 == C3 - C2),
so C_k = C3 + (k - 3)(C3 - C2); each split start maps into the 3-copy file at the same offset within its tile.
Reference: FullCheck.scala:141-191, CanLoadBam.scala:245-279, SplitRDD.scala:33-52.

configs[3] (loadReads streamed through HBM in windows): sbam.dist.WindowPipe (bench.py's --windows pipeline: two
contexts, sbam_load, the next window's staging on a loader thread) over W = 4 windows whose edges fall inside
records; partition sizes and every decoded column equal a single resident context's, and record offsets equal the
oracle's chains (CanLoadBam.scala:281-334).  SBAM_SCALE_GB sets the configs[2] size (default 4)."""
import copy
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

GB = float(os.environ.get("SBAM_SCALE_GB", "4"))
SPLIT = 2 << 20


def write_file(s, path, chunk=256 << 20):
    with open(path, "wb") as fh:
        for a in range(0, s.size, chunk):
            fh.write(s.slice(a, min(s.size, a + chunk)).tobytes())


def oracle_counts(o, threads=16, chunk=4 << 20):
    """(totals, by_key, positions, rbe, pair_hist, n_success) over the whole stream, chunked over threads."""
    from test_gpu_parity import pair_hist
    cuts = list(range(0, o.L, chunk)) + [o.L]

    def one(i):
        a, b = cuts[i], cuts[i + 1]
        c, npos, rbe, ns = o.counts_range(a, b)
        return c.sum(0), c, npos, rbe, pair_hist(o.check_full_range(a, b)), ns
    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(one, range(len(cuts) - 1)))
    return [sum(p[i] for p in parts) for i in range(6)]


def with_copies(s, k):
    t = copy.copy(s)
    t.copies = k
    t._sizes()
    return t


@pytest.mark.gpu
def test_configs2_eight_shards_exact(tmp_path):
    import oracle
    import synth
    from sbam import dist as sdist
    s = synth.SynthBam.for_size(int(GB * 1.01e9), tile_mb=8, threads=16)
    k, H, T = s.copies, s.header.size, s.tile.size
    assert s.size >= GB * 1e9 and k > 8
    path = str(tmp_path / "synth.bam")
    write_file(s, path)
    r = sdist.run_file(path, SPLIT, world=8, device=0)
    os.unlink(path)
    assert np.array_equal(r.contig_lengths, s.contig_lengths) and r.contig_lengths.size == 84

    # ---- expected Counts by extrapolating the oracle over 2, 3, 4 tile copies
    oc = {}
    for kk in (2, 3, 4):
        o = oracle.BamFile(with_copies(s, kk).bytes(), threads=16)
        oc[kk] = oracle_counts(o)
        if kk == 3:
            o3 = o
    for i in range(6):
        a, b, c = (np.asarray(oc[kk][i]) for kk in (4, 3, 2))
        assert np.array_equal(a - b, b - c), i  # every middle tile counts the same
    want = [np.asarray(oc[3][i]) + (k - 3) * (np.asarray(oc[3][i]) - np.asarray(oc[2][i])) for i in range(6)]
    got = r.counts
    assert np.array_equal(got["totals"], want[0])
    assert np.array_equal(got["by_key"][:3], want[1][:3])  # the report's close calls (keys 1-2); the counts path
    assert not got["by_key"][3:].any()                     # skips the per-flag table of keys >= 3
    assert np.array_equal(got["positions"], want[2])
    assert np.array_equal(got["reads_before_error"], want[3])
    assert np.array_equal(got["pair_hist"], want[4])
    assert got["n_success"] == int(want[5]) == s.n_records

    # ---- expected splits and partition sizes: each offset maps into the 3-copy file at the same place in its tile
    body = H + k * T

    def tiles_shift(x):  # tiles between x's place in the k-copy file and its image in the 3-copy file
        if x < H + T:
            return 0
        if x < body - T:
            return (x - H) // T - 1
        return k - 3
    R3 = o3.record_chain(o3.header_end, o3.L)
    assert R3.size == with_copies(s, 3).n_records

    def rec_index(x3, t):
        return int(np.searchsorted(R3, x3)) + t * s.tile_records
    firsts, sizes = [], []
    for a, e in sdist.hadoop_splits(s.size, SPLIT):
        t = tiles_shift(a)
        x = o3.find_record_start(o3.find_block_start(a - t * T))
        assert x is not None
        te = tiles_shift(e)
        xe = int(o3.uoff[o3.block_index_at_or_after(e - te * T)])
        n = max(0, rec_index(xe, te) - rec_index(x, t))
        sizes.append(n)
        if n:
            p = o3.pos_of(x)
            firsts.append((p.block_pos + t * T, p.offset))
    assert sum(sizes) == s.n_records
    assert r.partition_sizes == sizes
    assert [(sp.start.block_pos, sp.start.offset) for sp in r.splits] == firsts
    assert (r.splits[-1].end.block_pos, r.splits[-1].end.offset) == (s.size, 0)


@pytest.mark.gpu
def test_configs3_streamed_windows_equal_resident():
    import oracle
    import sbam
    import synth
    from sbam import dist as sdist
    s = synth.SynthBam(tile_mb=8, copies=6, threads=16)
    data = s.bytes()
    W = 4
    wplans = sdist.plan_shards(s.size, SPLIT, W)
    cols = tuple(sbam.RECORD_COLUMNS)
    got = []

    def run_window(sh):
        sizes, c = sh.load_columns(cols)
        st = sh.f.blocks()[0]
        return sizes, c, int(st[0]) if st.size else s.size

    pipe = sdist.WindowPipe(wplans, lambda lo, hi, j: s.slice(lo, hi), SPLIT, s.contig_lengths, 0, run_window)
    try:
        for _ in range(2):  # the second step reuses both contexts (sbam_load)
            got = pipe.step()
    finally:
        pipe.close()
    with sbam.BamFile(data, path="synth.bam") as f:
        want_sizes, want = f.load_records(SPLIT, columns=cols)
        edges_mid_record = 0
        sizes = np.concatenate([g[0] for g in got])
        assert np.array_equal(sizes, want_sizes) and int(sizes.sum()) == s.n_records
        i = 0
        for w, (sz, c, first_block) in enumerate(got):
            n = int(sz.sum())
            base = f.offset_of(sbam.Pos(first_block, 0))  # the window's stream starts at its first block
            for name in cols:
                exp = want[name][i:i + n]
                g = c[name] + base if name == "offset" else c[name]
                assert np.array_equal(g, exp), (w, name)
            if w > 0 and n:  # the window's first block starts inside a record
                edges_mid_record += int(want["offset"][i]) > base
            i += n
        assert edges_mid_record >= 1
    o = oracle.BamFile(data, threads=16)
    parts = oracle.load_reads_and_positions(o, SPLIT)
    assert [len(p) for p in parts] == want_sizes.tolist()
    assert np.array_equal(np.concatenate(parts), want["offset"])

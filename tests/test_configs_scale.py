"""BASELINE configs[2] and configs[3] on one GPU.

configs[2] (full-check of a multi-GB Illumina-like BAM across 8 shards, exact verdict diff): sbam.dist.run_file
over a >= 4 GB file on disk as 8 byte-range shards (GpuShard: pread of [lo, owned_hi + halo), rank-0 header
parse, counts/bitmap checker + split records), combined like the 8-rank run's all_gather/all_reduce.  The file has
no repeated tile (every 64 MB tile its own seed), and the expected Counts and splits come from one CPU-oracle run
over the whole file.  Reference: FullCheck.scala:141-191, CanLoadBam.scala:245-279, SplitRDD.scala:33-52.

configs[3] (loadReads streamed through HBM in windows): sbam.dist.WindowPipe (bench.py's --windows pipeline: two
contexts, sbam_load, the next window's staging on a loader thread) over W = 4 windows whose edges fall inside
records; partition sizes and every decoded column equal a single resident context's, and record offsets equal the
oracle's chains (CanLoadBam.scala:281-334).  SBAM_SCALE_GB sets the configs[2] size (default 4)."""
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


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_configs2_eight_shards_exact(tmp_path, distinct_synth):
    """configs[2] at 4 GB with no repeated tile: 8 byte-range shards from a file on disk, against ONE oracle run over
    the whole file (no extrapolation): Counts (totals, keys 1-2, positions per key, readsBeforeError, close-call
    pairs, successes), every split and every partition size."""
    import oracle
    from sbam import dist as sdist
    s = distinct_synth
    assert s.size >= GB * 1e9 and s.copies > 8
    path = str(tmp_path / "synth.bam")
    write_file(s, path)
    r = sdist.run_file(path, SPLIT, world=8, device=0)
    os.unlink(path)
    assert np.array_equal(r.contig_lengths, s.contig_lengths) and r.contig_lengths.size == 84

    o = oracle.BamFile(s.bytes(), threads=16)
    want = oracle_counts(o)
    got = r.counts
    assert np.array_equal(got["totals"], want[0])
    assert np.array_equal(got["by_key"][:3], want[1][:3])  # the report's close calls (keys 1-2); the counts path
    assert not got["by_key"][3:].any()                     # skips the per-flag table of keys >= 3
    assert np.array_equal(got["positions"], want[2])
    assert np.array_equal(got["reads_before_error"], want[3])
    assert np.array_equal(got["pair_hist"], want[4])
    assert got["n_success"] == int(want[5]) == s.n_records

    want_splits, parts = oracle.compute_splits(o, SPLIT)
    assert r.partition_sizes == [len(p) for p in parts] and sum(r.partition_sizes) == s.n_records
    assert [(sp.start.block_pos, sp.start.offset, sp.end.block_pos, sp.end.offset) for sp in r.splits] == \
        [(a.block_pos, a.offset, b.block_pos, b.offset) for a, b in want_splits]


@pytest.mark.gpu
@pytest.mark.parametrize("prefetch", [False, True])
def test_configs3_streamed_windows_equal_resident(prefetch):
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

    pipe = sdist.WindowPipe(wplans, lambda lo, hi, j: s.slice(lo, hi), SPLIT, s.contig_lengths, 0, run_window,
                            prefetch=prefetch)
    try:
        for _ in range(3):  # later steps reuse both contexts (sbam_load); with prefetch, window 0 loads early
            got = pipe.step()
        pipe.drop_prefetch()
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

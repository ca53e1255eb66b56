"""Long-read config (BASELINE.json configs[4]): ONT/PacBio-like records of 10–50 kb with
200–3000 CIGAR ops and names up to 63 characters, some larger than a 64 KiB BGZF block, so records span many
blocks, checker chains span many blocks, and shard edges fall mid-record.

The input is tools/synth_bam.c in long-read mode (read_len=0).  No reference fixture has such records, so the
expected results are the CPU oracle's (the oracle itself is pinned by the reference fixtures in
test_oracle.py); the generator's own record count is a second, independent check of the record chain."""
import numpy as np
import pytest

SPLITS = [64 * 1024, 256 * 1024, 1 << 20]


def _synth(tile_mb, copies):
    import synth
    return synth.SynthBam(tile_mb=tile_mb, copies=copies, read_len=0, threads=8)


@pytest.fixture(scope="module")
def long_file():
    """≈11 MB compressed / 25 MB uncompressed, two tile copies (the chain crosses a tile seam)."""
    import oracle
    s = _synth(4, 2)
    d = s.bytes()
    return s, d, oracle.BamFile(d, threads=8)


def _full_words_parallel(o, x0, x1, threads=8):
    from concurrent.futures import ThreadPoolExecutor
    cuts = np.linspace(x0, x1, threads + 1).astype(np.int64)
    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(lambda i: o.check_full_range(int(cuts[i]), int(cuts[i + 1])), range(threads)))
    return np.concatenate(parts)


def _record_fields(o, xs):
    u = o.u
    bs = np.array([int.from_bytes(u[x:x + 4].tobytes(), "little") for x in xs], np.int64)
    nc = np.array([int.from_bytes(u[x + 16:x + 18].tobytes(), "little") for x in xs], np.int64)
    lrn = np.array([int(u[x + 12]) for x in xs], np.int64)
    return bs, nc, lrn


def test_generator_shape(long_file):
    """The file has what the config asks for: many-op CIGARs, long names, records larger than a block."""
    s, d, o = long_file
    xs = o.record_chain(int(o.header_end), o.L)
    assert xs.size == s.n_records
    bs, nc, lrn = _record_fields(o, xs)
    assert (bs + 4 > 65536).sum() >= 3, "no record larger than a BGZF block"
    mapped = nc > 0
    assert nc[mapped].min() >= 200 and nc.max() <= 3000 and nc.max() > 1000
    assert lrn.max() <= 64 and lrn.min() >= 37


def test_oracle_checker_finds_every_record(long_file):
    s, d, o = long_file
    _, _, _, ns = o.counts_parallel(0, o.L, 10, 8)
    assert ns == s.n_records


def test_oracle_splits_cover_every_record(long_file):
    import oracle
    s, d, o = long_file
    for S in SPLITS:
        _, parts = oracle.compute_splits(o, S)
        assert sum(len(p) for p in parts) == s.n_records


@pytest.mark.gpu
class TestLongReadsGpu:
    @pytest.fixture(scope="class")
    def g(self, long_file):
        import sbam
        s, d, o = long_file
        f = sbam.BamFile(d, path="long.bam")
        yield f
        f.close()

    def test_blocks_and_bytes(self, g, long_file):
        s, d, o = long_file
        st, cs, us, uo = g.blocks()
        assert st.tolist() == o.start.tolist() and us.tolist() == o.usize.tolist()
        got = np.frombuffer(g.read_uncompressed(0, o.L), np.uint8)
        assert np.array_equal(got, o.u[:o.L])

    def test_full_words_every_position(self, g, long_file):
        s, d, o = long_file
        want = _full_words_parallel(o, 0, o.L)
        got = g.check_full_words(0, o.L)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: {got[bad[:5]]} vs {want[bad[:5]]}"

    @pytest.mark.parametrize("reads_to_check", [10, 2])
    def test_counts_by_key(self, g, long_file, reads_to_check):
        s, d, o = long_file
        c, npos, rbe, ns = o.counts_parallel(0, o.L, reads_to_check, 8)
        got = g.check_full_counts(0, o.L, reads_to_check, by_key=True)
        assert np.array_equal(got.by_key, c) and np.array_equal(got.positions, npos)
        assert np.array_equal(got.reads_before_error, rbe) and got.n_success == ns

    @pytest.mark.parametrize("reads_to_check", [10, 1])
    def test_counts_bit_sliced(self, g, long_file, reads_to_check):
        """The report-mode Counts (k_check_bits over the interior tiles).  Inside a long read's packed sequence every
        position reads n_cigar >= 0x1111 with valid ops (nibbles 1, 2, 4, 8), so the first invalid op lies thousands
        of ops on, often past the tile's window: the per-tile invalid-op table and the wave's scan past the window
        decide flag 15 there (before round 6 each such position read its ops one byte at a time: 8.4 s at 10 GB)."""
        s, d, o = long_file
        c, npos, rbe, ns = o.counts_parallel(0, o.L, reads_to_check, 8)
        got, bits = g.check_full_counts(0, o.L, reads_to_check, want_bitmap=True)
        assert np.array_equal(got.totals, c.sum(0)) and np.array_equal(got.by_key[:3], c[:3])
        assert np.array_equal(got.positions, npos) and np.array_equal(got.reads_before_error, rbe)
        assert got.n_success == ns and int(bits.sum()) == ns
        if reads_to_check == 10:
            assert np.array_equal(np.nonzero(bits)[0], o.record_chain(int(o.header_end), o.L))

    def test_eager_is_record_chain(self, g, long_file):
        s, d, o = long_file
        truth = o.record_chain(int(o.header_end), o.L)
        assert np.array_equal(np.nonzero(g.check_eager(0, g.uncompressed_size))[0], truth)

    @pytest.mark.parametrize("split_size", SPLITS)
    @pytest.mark.parametrize("bitmap", [False, True])
    def test_splits_and_partitions(self, g, long_file, split_size, bitmap):
        import oracle
        s, d, o = long_file
        want, parts = oracle.compute_splits(o, split_size)
        if bitmap:
            g.check_full_counts(0, g.uncompressed_size)
        got = g.compute_splits(split_size, use_success_bitmap=bitmap)
        assert [(x.start.block_pos, x.start.offset, x.end.block_pos, x.end.offset) for x in got] == \
            [(a.block_pos, a.offset, b.block_pos, b.offset) for a, b in want]
        assert g.partition_sizes(split_size) == [len(p) for p in parts]

    @pytest.mark.parametrize("world,split_size", [(2, 1 << 20), (3, 256 * 1024), (7, 64 * 1024)])
    def test_shards_with_small_halo(self, long_file, world, split_size):
        """Each shard loads its byte range plus a 64 KiB halo; records and chains that leave it make the shard
        grow its halo and re-run (sbam.dist.GpuShard).  The combined result equals the single-file oracle."""
        import oracle
        from sbam import dist as sdist
        s, d, o = long_file
        plans = sdist.plan_shards(s.size, split_size, world)
        results, grew = [], 0
        for p in plans:
            sh = sdist.GpuShard(p, s.slice, split_size, s.contig_lengths, halo=64 * 1024)
            try:
                results.append(sh.step())
                grew += sh.halo > 64 * 1024
            finally:
                sh.close()
        counts = np.sum([r.counts for r in results], axis=0)
        results = [sdist.ShardResult(counts if i == 0 else np.zeros_like(counts), r.first_block_pos,
                                     r.first_offset, r.nonempty, r.n_records) for i, r in enumerate(results)]
        splits, sizes, merged = sdist.combine(results, s.size)
        want, parts = oracle.compute_splits(o, split_size)
        assert [str(x) for x in splits] == [f"{a}-{b}" for a, b in want]
        assert sizes == [len(q) for q in parts]
        c, npos, rbe, ns = o.counts_parallel(0, o.L, 10, 8)
        u = sdist.unpack_counts(merged)
        assert np.array_equal(u["totals"], c.sum(0)) and np.array_equal(u["positions"], npos)
        assert u["n_success"] == ns == s.n_records
        assert grew >= 1, "no shard needed a larger halo: the test does not reach the halo path"

    @pytest.mark.parametrize("windows,split_size,prefetch", [(4, 256 * 1024, False), (6, 64 * 1024, False),
                                                          (3, 256 * 1024, True)])
    def test_window_pipe_halo_growth_reused_buffers(self, long_file, windows, split_size, prefetch):
        """sbam.dist.WindowPipe (bench --windows) with a 64 KiB halo over long reads: contexts grow their halo and
        re-read their range inside the pipe while the stager and loader threads reuse three staging buffers.  A halo
        retry must read private bytes (stage(lo, hi, None)), never a shared slot: the combined result equals the
        single-file oracle's for both steps (the second step reloads both contexts)."""
        import oracle
        from sbam import dist as sdist
        s, d, o = long_file
        bufs = [np.zeros(0, np.uint8) for _ in range(sdist.WindowPipe.NBUF)]

        def stage(lo, hi, k):
            hi = min(hi, s.size)
            if k is None:
                return s.slice(lo, hi)
            if bufs[k].size < hi - lo:
                bufs[k] = np.zeros(hi - lo, np.uint8)
            return s.slice(lo, hi, bufs[k][:hi - lo])

        wplans = sdist.plan_shards(s.size, split_size, windows)
        pipe = sdist.WindowPipe(wplans, stage, split_size, s.contig_lengths, 0, lambda sh: sh.step(),
                                halo=64 * 1024, prefetch=prefetch)
        want, parts = oracle.compute_splits(o, split_size)
        c, npos, rbe, ns = o.counts_parallel(0, o.L, 10, 8)
        try:
            for _ in range(3 if prefetch else 2):  # (an odd window count with prefetch alternates the contexts)
                results = pipe.step()
                counts = np.sum([r.counts for r in results], axis=0)
                results = [sdist.ShardResult(counts if i == 0 else np.zeros_like(counts), r.first_block_pos,
                                             r.first_offset, r.nonempty, r.n_records) for i, r in enumerate(results)]
                splits, sizes, merged = sdist.combine(results, s.size)
                assert [str(x) for x in splits] == [f"{a}-{b}" for a, b in want]
                assert sizes == [len(q) for q in parts]
                u = sdist.unpack_counts(merged)
                assert np.array_equal(u["totals"], c.sum(0)) and np.array_equal(u["positions"], npos)
                assert u["n_success"] == ns == s.n_records
            assert any(sh.halo > 64 * 1024 for sh in pipe.ctx), "no context grew its halo inside the pipe"
        finally:
            pipe.close()

"""HIP path (libsbam.so) vs the CPU oracle and the reference's goldens, on the reference's test BAMs.

Bit-exact for every byte / index / flag result.  Runs only on an MI355X (-m gpu)."""
import numpy as np
import pytest

from conftest import ALL_BAMS, INDEXED_BAMS, fixture_bytes, FIXTURES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ALL_BAMS)
def test_block_table(name, gpu_files, oracle_files):
    g, o = gpu_files(name), oracle_files(name)
    st, cs, us, uo = g.blocks()
    assert st.tolist() == o.start.tolist()
    assert cs.tolist() == o.csize.tolist()
    assert us.tolist() == o.usize.tolist()
    assert uo.tolist() == o.uoff[:-1].tolist()


@pytest.mark.parametrize("name", ALL_BAMS)
def test_inflate_bytes(name, gpu_files, oracle_files):
    g, o = gpu_files(name), oracle_files(name)
    assert g.uncompressed_size == o.L
    got = np.frombuffer(g.read_uncompressed(0, o.L), np.uint8)
    bad = np.nonzero(got != o.u[: o.L])[0]
    assert bad.size == 0, f"first mismatch at {bad[:5]}"


@pytest.mark.parametrize("name", ALL_BAMS)
def test_wave_decoder_covers_fixture_blocks(name, gpu_files):
    """Every block of the reference's BAMs (htsjdk/zlib dynamic-Huffman streams) is decoded by the wave-parallel
    decoder; none needs the exact per-lane fallback."""
    assert gpu_files(name).inflate_fallbacks() == 0


@pytest.mark.parametrize("name", ALL_BAMS)
def test_header(name, gpu_files, oracle_files):
    g, o = gpu_files(name), oracle_files(name)
    assert g.n_ref == o.nref
    assert g.contig_lengths.tolist() == o.lens[: o.nref].tolist()
    assert g.header_end == g.pos_of(o.header_end)


@pytest.mark.parametrize("name", ALL_BAMS)
def test_full_words_every_position(name, gpu_files, oracle_files):
    g, o = gpu_files(name), oracle_files(name)
    want = o.check_full_range(0, o.L)
    got = g.check_full_words(0, o.L)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: {got[bad[:5]]} vs {want[bad[:5]]}"


@pytest.mark.parametrize("name", INDEXED_BAMS)
def test_eager_matches_records(name, gpu_files):
    """eager.Checker true exactly at the .records positions (the indexed-checker truth)."""
    import oracle
    g = gpu_files(name)
    truth = np.array([g.offset_of(p) for p in oracle.parse_records_file(f"{FIXTURES}/{name}.records")])
    calls = g.check_eager(0, g.uncompressed_size)
    assert np.array_equal(np.nonzero(calls)[0], truth)


@pytest.mark.parametrize("name", ALL_BAMS)
@pytest.mark.parametrize("reads_to_check", [10, 1, 3])
@pytest.mark.parametrize("by_key", [False, True])
def test_full_counts(name, reads_to_check, by_key, gpu_files, oracle_files):
    g, o = gpu_files(name), oracle_files(name)
    counts, npos, rbe, nsucc = o.counts_range(0, o.L, reads_to_check)
    c, bits = g.check_full_counts(0, o.L, reads_to_check, want_bitmap=True, by_key=by_key)
    assert np.array_equal(c.totals, counts.sum(0))
    if by_key:
        assert np.array_equal(c.by_key, counts)
    else:
        assert np.array_equal(c.by_key[:3], counts[:3])
    assert np.array_equal(c.positions, npos)
    assert np.array_equal(c.reads_before_error, rbe)
    assert c.n_success == nsucc
    w = o.check_full_range(0, o.L, reads_to_check)
    assert np.array_equal(bits, (w & 0x80000000) != 0)
    assert np.array_equal(c.pair_hist, pair_hist(w))


def pair_hist(w):
    """Close-call pairs of the full-check report: key-2 results by (first flag, second flag), or (flag, flag)
    when the second non-zero field is readsBeforeError (FullCheck.scala:141-191)."""
    F = (w & 0x7ffff).astype(np.int64)
    k = (w >> 24) & 0x7f
    counted = ((w & 0x80000000) == 0) & ~((F == 1) & (k == 0))
    pop = np.zeros_like(F)
    for f in range(19):
        pop += (F >> f) & 1
    key2 = counted & (pop + (k > 0) == 2)
    out = np.zeros((19, 19), np.int64)
    for Fi in F[key2]:
        bits = [f for f in range(19) if (Fi >> f) & 1]
        out[bits[0], bits[1] if len(bits) > 1 else bits[0]] += 1
    return out


@pytest.mark.parametrize("name", ["2.bam", "5k.bam"])
def test_check_unaligned_ranges(name, gpu_files, oracle_files):
    """Sub-ranges with arbitrary (non 64-aligned) ends: words, counts, eager bitmap."""
    g, o = gpu_files(name), oracle_files(name)
    rng = np.random.default_rng(11)
    for _ in range(6):
        x0 = int(rng.integers(0, o.L - 1))
        x1 = int(min(o.L, x0 + rng.integers(1, 200000)))
        want = o.check_full_range(x0, x1)
        assert np.array_equal(g.check_full_words(x0, x1), want)
        c, bits = g.check_full_counts(x0, x1, want_bitmap=True)
        cnt, npos, _, ns = o.counts_range(x0, x1)
        assert np.array_equal(c.totals, cnt.sum(0)) and np.array_equal(c.positions, npos) and c.n_success == ns
        assert np.array_equal(bits, (want & 0x80000000) != 0)
        assert np.array_equal(g.check_eager(x0, x1), (want & 0x80000000) != 0)


def test_find_block_start_golden(gpu_files):
    # FindBlockStartTest.scala:9-16
    assert gpu_files("2.bam").find_block_start(26170) == 50249


@pytest.mark.parametrize("name", ALL_BAMS)
def test_find_block_starts_vs_oracle(name, gpu_files, oracle_files):
    g, o = gpu_files(name), oracle_files(name)
    rng = np.random.default_rng(7)
    qs = sorted(set(rng.integers(0, o.D, 200).tolist() + [0, 1, o.D - 1, o.D - 17, o.D - 18, o.D - 28]))
    got = g.find_block_starts(qs)
    want = [o.find_block_start(q) for q in qs]
    assert got.tolist() == want


def test_find_record_start_golden(gpu_files):
    # FindRecordStartTest.scala:16-26 (hadoop-bam says 311)
    from sbam import Pos
    assert gpu_files("1.bam").find_record_start(239479) == Pos(239479, 312)


def test_checker_points(gpu_files):
    # full/CheckerTest.scala:38-72
    from sbam import Pos, FLAG_NAMES
    g = gpu_files("2.bam")
    chk = g.full_checker()
    assert chk(Pos(439897, 52186)) == 0x80000000 | (10 << 24)  # Success(10)
    w = chk(Pos(0, 5649))
    assert [FLAG_NAMES[i] for i in range(19) if w & (1 << i)] == ["noReadName", "invalidCigarOp"]
    assert (w >> 24) & 0x7F == 0


@pytest.mark.parametrize("kb,expected", [
    (230, ["0:45846-239479:312", "239479:312-484396:25", "484396:25-597482:0"]),
    (240, ["0:45846-263656:191", "263656:191-508565:287", "508565:287-597482:0"]),
])
@pytest.mark.parametrize("bitmap", [False, True])
def test_compute_splits_golden(kb, expected, bitmap, gpu_files):
    # cli/src/test/scala/org/hammerlab/bam/spark/ComputeSplitsTest.scala:14-88
    g = gpu_files("1.bam")
    if bitmap:
        g.check_full_counts(0, g.uncompressed_size)
    assert [str(s) for s in g.compute_splits(kb * 1024, use_success_bitmap=bitmap)] == expected


@pytest.mark.parametrize("split_size,sizes", [
    (1000000, [2500]),
    (100000, [503, 414, 518, 421, 493, 151]),
    (20000, [96, 102, 105, 101, 99, 102, 101, 106, 0, 105, 105, 102, 104, 103, 104, 106, 104, 106, 0, 105,
             195, 101, 0, 99, 98, 99, 52]),
])
def test_partition_sizes_golden(split_size, sizes, gpu_files):
    # load/src/test/scala/org/hammerlab/bam/spark/load/LoadBAMTest.scala:24-45
    assert gpu_files("2.bam").partition_sizes(split_size) == sizes


def test_load_bam_1_count(gpu_files):
    # LoadBAMTest.scala "1.bam": loadBam(bam1, 300 KB).count == 4917
    assert sum(gpu_files("1.bam").partition_sizes(300 * 1024)) == 4917


def test_first_read_names(gpu_files):
    # LoadBAMChecks.scala:33-46
    import sbam
    parts = gpu_files("2.bam").load_reads_and_positions(100000)
    names = [sbam.read_name(r) for p in parts for (_, r) in p][:10]
    assert names == [
        "HWI-ST807:461:C2P0JACXX:4:2115:8592:79724", "HWI-ST807:461:C2P0JACXX:4:2115:8592:79724",
        "HWI-ST807:461:C2P0JACXX:4:1304:9505:89866", "HWI-ST807:461:C2P0JACXX:4:2311:6431:65669",
        "HWI-ST807:461:C2P0JACXX:4:1305:2342:51860", "HWI-ST807:461:C2P0JACXX:4:1305:2342:51860",
        "HWI-ST807:461:C2P0JACXX:4:1304:9505:89866", "HWI-ST807:461:C2P0JACXX:4:2311:6431:65669",
        "HWI-ST807:461:C2P0JACXX:4:1107:13461:64844", "HWI-ST807:461:C2P0JACXX:4:2203:17157:59976"]


@pytest.mark.parametrize("name", INDEXED_BAMS)
@pytest.mark.parametrize("split_kb", [20, 100, 2048])
def test_splits_and_partitions_vs_oracle(name, split_kb, gpu_files, oracle_files):
    import oracle
    g, o = gpu_files(name), oracle_files(name)
    S = split_kb * 1024
    try:
        want_splits, parts = oracle.compute_splits(o, S)
    except RuntimeError:
        with pytest.raises(Exception):
            g.compute_splits(S)
        return
    assert [(s.start.block_pos, s.start.offset, s.end.block_pos, s.end.offset) for s in g.compute_splits(S)] == \
        [(a.block_pos, a.offset, b.block_pos, b.offset) for a, b in want_splits]
    assert g.partition_sizes(S) == [len(p) for p in parts]


def test_sam_is_not_bam():
    # LoadSamAsBamFails.scala:11-18: HeaderParseException "Position 0: 64 != 31"
    import sbam
    sam = b"@HD\tVN:1.5\tSO:coordinate\n" * 10
    with pytest.raises(sbam.HeaderParseException, match=r"Position 0: 64 != 31"):
        sbam.BamFile(sam)


@pytest.mark.gpu
@pytest.mark.parametrize("name,window,kind", [("2.bam", 96 * 1024, "eager"), ("1.bam", 200 * 1024, "eager"),
                                              ("1.2203053-2211029.bam", 128 * 1024, "full")])
def test_lazy_block_checker_drop_in(tmp_path, name, window, kind):
    """sbam.checker.LazyBlockChecker, the MakeChecker drop-in (Checker.scala:23-25: built from the channel alone): the
    positions of every block in CallPartition's order (blocks.flatMap(PosIterator), CallPartition.scala:39-53) give
    the whole-file calls; each window of blocks costs one bulk call on first use."""
    import sbam
    from sbam import dist as sdist
    from sbam.checker import make_checker
    path = tmp_path / name
    path.write_bytes(fixture_bytes(name))
    with sbam.BamFile(fixture_bytes(name)) as f:
        want = f.check_eager() if kind == "eager" else f.check_full_words()
        st, cs, us, uo = f.blocks()
        lens = f.contig_lengths
    chk = make_checker(lens, kind=kind, window=window)(sdist.file_source(str(path)))
    rng = np.random.default_rng(7)
    for b in range(st.size):
        offs = np.arange(int(us[b])) if b % 4 == 0 else np.sort(rng.integers(0, int(us[b]), 200))
        got = [chk(sbam.Pos(int(st[b]), int(o))) for o in offs]
        assert got == [bool(want[uo[b] + o]) if kind == "eager" else int(want[uo[b] + o]) for o in offs], b
    assert 1 < chk.bulk_calls < st.size


@pytest.mark.gpu
def test_lazy_block_checker_windows_timed(tmp_path):
    """100+ lazy 4 MB windows through ONE kept context (sbam_load per window, no per-window context setup): the calls
    at sampled offsets of every block equal a resident whole-file check, only the last `keep` windows stay cached,
    and the ms per bulk call is printed (CallPartition.scala:35-53 calls Checker.apply per position of each block)."""
    import time
    import sbam
    import synth
    from sbam import dist as sdist
    from sbam.checker import LazyBlockChecker
    s = synth.SynthBam(tile_mb=220)
    path = tmp_path / "synth.bam"
    path.write_bytes(s.bytes().tobytes())
    with sbam.BamFile(s.bytes()) as f:
        want = f.check_eager()
        st, cs, us, uo = f.blocks()
    chk = LazyBlockChecker(*sdist.file_source(str(path)), s.contig_lengths, window=4 << 20)
    rng = np.random.default_rng(3)
    t0 = time.perf_counter()
    bad = 0
    for b in range(st.size):
        offs = rng.integers(0, int(us[b]), 16)
        got = np.array([chk(sbam.Pos(int(st[b]), int(o))) for o in offs])
        bad += int((got != want[uo[b] + offs].astype(bool)).sum())
        assert len(chk.windows) <= 2
    dt = time.perf_counter() - t0
    chk.close()
    assert bad == 0
    assert chk.bulk_calls >= 100
    print(f"lazy checker: {chk.bulk_calls} windows of 4 MB, {1e3 * dt / chk.bulk_calls:.2f} ms per bulk call "
          f"(incl. the host preads and lookups)")

"""Record decode (sbam_load_records): the partitions of loadReads / loadReadsAndPositions as record offsets, Pos
and fixed-field columns (CanLoadBam.scala:221-241, 281-334; RecordStream.scala:27-41).

Expected values: the CPU oracle's per-split record chains (oracle.load_reads_and_positions, pinned by
LoadBAMTest partition sizes and the .records files in test_oracle.py), the .records files themselves, and the
fixed fields read straight from the oracle's inflated stream.  Both device paths are covered: the serial chain
walk and the bitmap chain proof (use_success_bitmap after a full check), including a bitmap with false-positive
calls, where the proof must fail and the walk must take over."""
import numpy as np
import pytest

from conftest import FIXTURES, INDEXED_BAMS

pytestmark = pytest.mark.gpu

FIELDS = [("block_size", 0, np.int32), ("ref_id", 4, np.int32), ("pos", 8, np.int32), ("bin_mq_nl", 12, np.uint32),
          ("flag_nc", 16, np.uint32), ("l_seq", 20, np.int32), ("next_ref_id", 24, np.int32),
          ("next_pos", 28, np.int32), ("tlen", 32, np.int32)]


def expect(o, split_size):
    import oracle
    parts = oracle.load_reads_and_positions(o, split_size)
    offs = np.concatenate([p for p in parts] + [np.zeros(0, np.int64)]).astype(np.int64)
    return [len(p) for p in parts], offs


def check_columns(o, offs, cols):
    assert np.array_equal(cols["offset"], offs)
    for name, k, dt in FIELDS:
        want = np.array([int.from_bytes(o.u[x + k:x + k + 4].tobytes(), "little", signed=dt == np.int32)
                         for x in offs.tolist()], dt)
        assert np.array_equal(cols[name], want), name
    bp = np.array([o.pos_of(int(x)).block_pos for x in offs.tolist()], np.int64)
    bo = np.array([o.pos_of(int(x)).offset for x in offs.tolist()], np.int64)
    assert np.array_equal(cols["block_pos"], bp) and np.array_equal(cols["block_off"].astype(np.int64), bo)


@pytest.mark.parametrize("name", INDEXED_BAMS)
@pytest.mark.parametrize("split_kb", [20, 100, 2048])
@pytest.mark.parametrize("bitmap", [False, True, "eager"])
def test_load_records_vs_oracle(name, split_kb, bitmap, gpu_files, oracle_files):
    """bitmap: False = the chain walk; True = the full check's success bitmap; "eager" = the eager checker's calls
    (what the sharded loadReads uses, sbam.dist.shard_load)."""
    g, o = gpu_files(name), oracle_files(name)
    S = split_kb * 1024
    try:
        sizes, offs = expect(o, S)
    except RuntimeError:  # NoReadFoundException on this split size: the GPU path must raise too
        with pytest.raises(Exception):
            g.load_records(S)
        return
    if bitmap == "eager":
        g.check_eager_device(0, g.uncompressed_size)
    elif bitmap:
        g.check_full_counts(0, g.uncompressed_size)
    got_sizes, cols = g.load_records(S, use_success_bitmap=bool(bitmap))
    assert got_sizes.tolist() == sizes
    check_columns(o, offs, cols)


@pytest.mark.parametrize("name", INDEXED_BAMS)
def test_positions_are_records_file(name, gpu_files):
    """One split over the whole file: every record Pos of the .records sidecar, in order."""
    import oracle
    g = gpu_files(name)
    g.check_full_counts(0, g.uncompressed_size)
    _, cols = g.load_records(1 << 40, use_success_bitmap=True, columns=("block_pos", "block_off"))
    truth = oracle.parse_records_file(f"{FIXTURES}/{name}.records")
    assert list(zip(cols["block_pos"].tolist(), cols["block_off"].tolist())) == \
        [(p.block_pos, p.offset) for p in truth]


def test_proof_fails_on_false_positives(gpu_files, oracle_files):
    """A 0-record check calls every position true (Success(0)); the chain proof must reject that bitmap and the
    walk must still give the oracle's partitions."""
    g, o = gpu_files("2.bam"), oracle_files("2.bam")
    c = g.check_full_counts(0, g.uncompressed_size, reads_to_check=0)
    assert c.n_success > 2500, "the R=0 bitmap has no false positives; the test needs some"
    sizes, offs = expect(o, 100000)
    got_sizes, cols = g.load_records(100000, use_success_bitmap=True)
    assert got_sizes.tolist() == sizes
    check_columns(o, offs, cols)


def test_load_reads_bytes(gpu_files, oracle_files):
    """loadReadsAndPositions record bytes are the stream slices [x, x + 4 + block_size)."""
    import oracle
    g, o = gpu_files("1.bam"), oracle_files("1.bam")
    parts = g.load_reads_and_positions(230 * 1024)
    assert [len(p) for p in parts] == [len(p) for p in oracle.load_reads_and_positions(o, 230 * 1024)]
    for p in parts:
        for pos, rec in p[:50] + p[-50:]:
            x = o.offset_of(pos)
            bs = int.from_bytes(o.u[x:x + 4].tobytes(), "little")
            assert rec == o.u[x:x + 4 + bs].tobytes()


def test_long_reads(gpu_files):
    import oracle
    import sbam
    import synth
    s = synth.SynthBam(tile_mb=4, copies=2, read_len=0, threads=8)
    d = s.bytes()
    o = oracle.BamFile(d, threads=8)
    with sbam.BamFile(d, path="long.bam") as g:
        for S, bm in ((64 * 1024, False), (64 * 1024, True), (1 << 20, True)):
            if bm:
                g.check_full_counts(0, g.uncompressed_size)
            try:
                sizes, offs = expect(o, S)
            except RuntimeError:  # NoReadFoundException (a split starting past the last data block)
                with pytest.raises(sbam.NoReadFoundException):
                    g.load_records(S, use_success_bitmap=bm)
                continue
            got_sizes, cols = g.load_records(S, use_success_bitmap=bm)
            assert got_sizes.tolist() == sizes and sum(sizes) == s.n_records
            check_columns(o, offs, cols)


def test_synthetic_1gb_properties():
    """At 1 GB (no oracle pass): proof path == walk path, every record once, offsets chain by block_size."""
    import sbam
    import synth
    s = synth.SynthBam.for_size(int(1e9), tile_mb=64, threads=16)
    with sbam.BamFile(s.bytes(), path="synth.bam") as g:
        S = 2 << 20
        sw, cw = g.load_records(S, columns=("offset", "block_size"))
        g.check_full_counts(0, g.uncompressed_size)
        sp, cp = g.load_records(S, use_success_bitmap=True, columns=("offset", "block_size"))
        assert np.array_equal(sw, sp) and np.array_equal(cw["offset"], cp["offset"])
        assert int(sp.sum()) == s.n_records
        g.check_eager_device(0, g.uncompressed_size)  # the eager calls' bitmap proves the same chains
        se, ce = g.load_records(S, use_success_bitmap=True, columns=("offset", "block_size"))
        assert np.array_equal(sw, se) and np.array_equal(cw["offset"], ce["offset"])
        off, bs = cp["offset"], cp["block_size"].astype(np.int64)
        assert np.array_equal(off[1:], off[:-1] + 4 + bs[:-1])


@pytest.mark.parametrize("R", [1, 2, 10])
@pytest.mark.parametrize("split_kb", [20, 1 << 20])
def test_last_pass0_hop_inside_range(R, split_kb):
    """ADVICE r05 (k_p0_links' last list entry): 100 zero bytes after the last record of 2.bam, inside its last data
    block.  The last true record is then the list's last PASS0 site and its hop lands inside the checked range on a
    position that is not a PASS0 site (zeros fail record 0: noReadName).  RecordStream walks through the zeros as
    25 four-byte records (block_size 0), so a loadReads that trusted the eager bitmap there would miss them: the last
    entry must count as a missing link, the chain proof must run and fail, and the walk must give the oracle's
    partitions.  Under the round-4 rule (last entry always linked) the proof was skipped for R = 1."""
    import oracle
    import sbam
    from test_eager_wave import bgzf
    base = oracle.BamFile(open(f"{FIXTURES}/2.bam", "rb").read())
    blob = bgzf(base.u[:base.L].tobytes() + b"\x00" * 100)
    o = oracle.BamFile(blob)
    S = split_kb * 1024
    parts = oracle.load_reads_and_positions(o, S, reads_to_check=R)
    sizes = [len(p) for p in parts]
    offs = np.concatenate(parts).astype(np.int64)
    assert np.array_equal(offs[-25:], o.L - 100 + 4 * np.arange(25))  # the zero "records" are in the partitions
    with sbam.BamFile(blob, path="zeros_tail.bam") as g:
        g.check_eager_device(0, g.uncompressed_size, R)
        got_sizes, cols = g.load_records(S, reads_to_check=R, use_success_bitmap=True)
        assert got_sizes.tolist() == sizes
        check_columns(o, offs, cols)

"""CPU oracle pinned against the reference's own fixtures and golden outputs (no GPU)."""
import re

import numpy as np
import pytest

from conftest import ALL_BAMS, FIXTURES, GOLDEN, INDEXED_BAMS


@pytest.mark.parametrize("name", INDEXED_BAMS)
def test_blocks_file(name, oracle_files):
    """MetadataStream == the .blocks sidecar (IndexBlocksTest.scala:8-14)."""
    import oracle
    o = oracle_files(name)
    assert list(zip(o.start.tolist(), o.csize.tolist(), o.usize.tolist())) == \
        oracle.parse_blocks_file(f"{FIXTURES}/{name}.blocks")


@pytest.mark.parametrize("name", INDEXED_BAMS)
def test_checker_truth_is_records_file(name, oracle_files):
    """Success at exactly the .records positions, every uncompressed offset (indexed.Checker truth)."""
    import oracle
    o = oracle_files(name)
    w = o.check_full_range(0, o.L)
    truth = [o.offset_of(p) for p in oracle.parse_records_file(f"{FIXTURES}/{name}.records")]
    assert np.nonzero(w & oracle.W_SUCCESS)[0].tolist() == truth


def _totals(path):
    sec = open(path).read().split("Total error counts:")[1]
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"(\w+):\s+(\d+)", sec)}


def _close_calls(path):
    m = re.search(r"of (\d+) positions where exactly two checks failed", open(path).read())
    return int(m.group(1)) if m else 0


@pytest.mark.parametrize("golden,bam,blocks", [
    ("2.bam", "2.bam", None),
    ("1.bam", "1.bam", None),
    ("1.noblocks.bam", "1.bam", None),
    ("2.bam.first", "2.bam", lambda f: [0]),          # -i 0
    ("2.bam.second", "2.bam", lambda f: [1]),         # -i 26169
    ("2.bam.200k", "2.bam", lambda f: [b for b in range(f.nblocks) if f.start[b] < 200 * 1024]),  # -i 0-200k
])
def test_full_check_goldens(golden, bam, blocks, oracle_files):
    """cli/src/test/resources/output/full-check/* 'Total error counts' and close-call counts (FullCheckTest)."""
    import oracle
    o = oracle_files(bam)
    counts = np.zeros((21, 19), np.int64)
    npos = np.zeros(21, np.int64)
    for b in (range(o.nblocks) if blocks is None else blocks(o)):
        c, n, _, _ = o.counts_range(int(o.uoff[b]), int(o.uoff[b + 1]))
        counts += c
        npos += n
    tot = counts.sum(0)
    want = _totals(f"{GOLDEN}/full-check/{golden}")
    got = {oracle.FLAG_NAMES[i]: int(tot[i]) for i in range(1, 19)}
    for k, v in got.items():
        assert v == want.get(k, 0), k
    assert npos[1] == 0  # "No positions where only one check failed"
    assert npos[2] == _close_calls(f"{GOLDEN}/full-check/{golden}")


def test_check_bam_false_positive_flags(oracle_files):
    """output/check-bam/1.bam: hadoop-bam's 5 false positives, full-checker flags."""
    import oracle
    o = oracle_files("1.bam")
    for p in ["39374:30965", "239479:311", "484396:46507", "508565:56574", "533464:49472"]:
        b, off = (int(x) for x in p.split(":"))
        w = o.check_full(o.offset_of(oracle.Pos(b, off)))
        assert oracle.flags_of(w) == ["tooLargeReadPos", "tooLargeNextReadPos", "emptyReadName", "invalidCigarOp"]


def test_checker_points(oracle_files):
    """full/CheckerTest.scala:38-72."""
    import oracle
    o = oracle_files("2.bam")
    assert o.check_full(o.offset_of(oracle.Pos(439897, 52186))) == 0x80000000 | (10 << 24)
    w = o.check_full(o.offset_of(oracle.Pos(0, 5649)))
    assert oracle.flags_of(w) == ["noReadName", "invalidCigarOp"] and (w >> 24) & 0x7F == 0
    # @1006167:15243 is past 2.bam's end; on 5k.bam it is the last block − 4 B: tooFewFixedBlockBytes
    o5 = oracle_files("5k.bam")
    assert o5.check_full(o5.offset_of(oracle.Pos(1006167, 15243))) == 1


def test_find_block_and_record_start(oracle_files):
    """FindBlockStartTest.scala:9-16, FindRecordStartTest.scala:16-26."""
    assert oracle_files("2.bam").find_block_start(26170) == 50249
    o = oracle_files("1.bam")
    assert str(o.pos_of(o.find_record_start(239479))) == "239479:312"


def test_header(oracle_files):
    """ByteStreamTest.scala:14-43 (84 refs, first record Pos(0,5650) of 2.bam); 5k.bam header alone in block 0."""
    o = oracle_files("2.bam")
    assert o.nref == 84 and str(o.pos_of(o.header_end)) == "0:5650"
    assert o.lens[0] == 249250621
    assert str(oracle_files("5k.bam").pos_of(oracle_files("5k.bam").header_end)) == "2454:0"


@pytest.mark.parametrize("kb,expected", [
    (230, ["0:45846-239479:312", "239479:312-484396:25", "484396:25-597482:0"]),
    (240, ["0:45846-263656:191", "263656:191-508565:287", "508565:287-597482:0"]),
])
def test_compute_splits(kb, expected, oracle_files):
    """ComputeSplitsTest.scala:14-88, CompareTest.scala:42-55."""
    import oracle
    splits, _ = oracle.compute_splits(oracle_files("1.bam"), kb * 1024)
    assert [f"{a}-{b}" for a, b in splits] == expected


def test_compare_115k(oracle_files):
    """CompareTest.scala:72-83: spark-bam split 239479:312-361204:42 at 115KB."""
    import oracle
    splits, _ = oracle.compute_splits(oracle_files("1.bam"), 115 * 1024)
    assert "239479:312-361204:42" in [f"{a}-{b}" for a, b in splits]


@pytest.mark.parametrize("split_size,sizes", [
    (1000000, [2500]),
    (100000, [503, 414, 518, 421, 493, 151]),
    (20000, [96, 102, 105, 101, 99, 102, 101, 106, 0, 105, 105, 102, 104, 103, 104, 106, 104, 106, 0, 105,
             195, 101, 0, 99, 98, 99, 52]),
])
def test_partition_sizes(split_size, sizes, oracle_files):
    """LoadBAMTest.scala:24-45."""
    import oracle
    assert [len(p) for p in oracle.load_reads_and_positions(oracle_files("2.bam"), split_size)] == sizes


def test_load_bam_1_count(oracle_files):
    import oracle
    assert sum(len(p) for p in oracle.load_reads_and_positions(oracle_files("1.bam"), 300 * 1024)) == 4917


def test_hadoop_splits_rule():
    import oracle
    # seqdoop splits in ComputeSplitsTest: 0-235520, 235520-471040, 471040-597482 at 230k
    assert oracle.hadoop_splits(597482, 230 * 1024) == [(0, 235520), (235520, 471040), (471040, 597482)]
    assert oracle.hadoop_splits(110, 100) == [(0, 110)]
    assert oracle.hadoop_splits(111, 100) == [(0, 100), (100, 111)]
    assert oracle.hadoop_splits(0, 100) == []


def test_sam_header_parse_exception():
    """LoadSamAsBamFails.scala:15-17: HeaderParseException 'Position 0: 64 != 31'."""
    import oracle
    with pytest.raises(ValueError, match=r"Position 0: 64 != 31"):
        oracle.BamFile(b"@HD\tVN:1.5\n" * 4)


def test_synthetic_generator_chain_is_checker_truth():
    """tools/synth_bam.c output: checker successes == record chain (no false calls) across tile seams."""
    import oracle
    import synth
    s = synth.SynthBam(tile_mb=1, copies=3, threads=4)
    o = oracle.BamFile(s.bytes())
    w = o.check_full_range(0, o.L)
    chain = o.record_chain(o.header_end, o.L)
    assert len(chain) == s.n_records
    assert np.array_equal(np.nonzero(w & oracle.W_SUCCESS)[0], chain)

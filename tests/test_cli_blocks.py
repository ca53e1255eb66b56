"""check-blocks -s, index-blocks and index-records drop-ins against the reference's
goldens and sidecar fixtures.

check-blocks: the expected texts are CheckBlocksTest.scala's ("1.bam spark-bam" is the `-s` case; "2.bam" and
"1.block-aligned.bam" ran eager vs hadoop-bam there, with no mismatched block, so eager vs the indexed records
prints the same text — the sidecar for 1.block-aligned.bam is written by our own index-records).
index-blocks / index-records: IndexBlocksTest / IndexRecordsTest compare with 2.bam.blocks / 2.bam.records;
here every record-indexed fixture's sidecars are reproduced."""
import os
import shutil

import numpy as np
import pytest

from conftest import FIXTURES, GOLDEN, INDEXED_BAMS
from test_cli import OracleBam


def _golden(name):
    return open(os.path.join(GOLDEN, "check-blocks", name)).read()


def _records(path, f):
    return np.array([f.offset_of(tuple(int(v) for v in ln.split(","))) for ln in open(path) if ln.strip()],
                    np.int64)


def test_hist_stats_lines_check_blocks_goldens():
    """Stats.fromHist formatting (N, μ/σ, med/mad, elems with v×c and …, interpolated percentiles) from the
    blocks' first-read offsets that the .blocks/.records sidecars imply."""
    from sbam.cli import hist_stats_lines
    for bam, golden in (("1.bam", "1.bam-s"), ("2.bam", "2.bam")):
        starts = [int(ln.split(",")[0]) for ln in open(os.path.join(FIXTURES, bam + ".blocks")) if ln.strip()]
        firsts = {}
        for ln in open(os.path.join(FIXTURES, bam + ".records")):
            b, o = (int(v) for v in ln.split(","))
            firsts.setdefault(b, o)
        hist = {}
        for s in starts:
            hist[firsts[s]] = hist.get(firsts[s], 0) + 1
        want = _golden(golden).split("\n")[3:12]
        assert hist_stats_lines(list(hist.items())) == want


class _OracleBlocks(OracleBam):
    def __init__(self, data):
        super().__init__(data)
        self.file_size = len(data)


@pytest.mark.parametrize("bam,golden", [("1.bam", "1.bam-s"), ("2.bam", "2.bam")])
def test_check_blocks_logic(bam, golden):
    """check-blocks -s report assembly on the oracle backend."""
    from sbam import Pos, cli
    data = open(os.path.join(FIXTURES, bam), "rb").read()
    f = _OracleBlocks(data)
    truth = [f.offset_of(Pos(*(int(v) for v in ln.split(",")))) for ln in open(os.path.join(FIXTURES, bam + ".records"))]
    text = "\n".join(cli.check_blocks_lines(f, np.asarray(truth, np.int64), 10)) + "\n"
    assert text == _golden(golden)


def test_check_blocks_mismatch_format():
    """The mismatch branch (CheckBlocks.scala:160-190): with 1.bam's record 239479:312 removed from the indexed
    truth, the eager checker's first read of that block (239479:312) and the truth's next one differ."""
    from sbam import Pos, cli
    data = open(os.path.join(FIXTURES, "1.bam"), "rb").read()
    f = _OracleBlocks(data)
    lines = [ln for ln in open(os.path.join(FIXTURES, "1.bam.records")) if ln.strip() != "239479,312"]
    truth = [f.offset_of(Pos(*(int(v) for v in ln.split(",")))) for ln in lines]
    out = cli.check_blocks_lines(f, np.asarray(truth, np.int64), 10)
    assert out[0] == "First read-position mismatched in 1 of 25 BGZF blocks"
    assert out[2] == "25871 of 597482 (0.043300049206503294) compressed positions would lead to bad splits"
    assert out[-2:] == ["1 mismatched blocks:", "\t239479 (prev block size: 25871):\t239479:312\t239479:" +
                        out[-1].rsplit(":", 1)[1]]


def test_index_blocks_logic():
    from sbam import cli
    for bam in INDEXED_BAMS:
        data = open(os.path.join(FIXTURES, bam), "rb").read()
        got = cli.index_blocks_lines(OracleBam(data))
        assert got == [ln.strip() for ln in open(os.path.join(FIXTURES, bam + ".blocks")) if ln.strip()], bam


@pytest.mark.gpu
@pytest.mark.parametrize("bam", INDEXED_BAMS)
def test_index_sidecars(bam, tmp_path):
    """index-blocks / index-records reproduce the reference's .blocks / .records files byte for byte."""
    from sbam import cli
    for cmd, ext in (("index-blocks", ".blocks"), ("index-records", ".records")):
        out = tmp_path / (bam + ext)
        assert cli.main([cmd, os.path.join(FIXTURES, bam), str(out)]) == 0
        assert out.read_text() == open(os.path.join(FIXTURES, bam + ext)).read(), (bam, cmd)


@pytest.mark.gpu
@pytest.mark.parametrize("bam,golden", [("1.bam", "1.bam-s"), ("2.bam", "2.bam"),
                                        ("1.block-aligned.bam", "1.block-aligned.bam")])
def test_check_blocks_report(bam, golden, tmp_path):
    from sbam import cli
    path = tmp_path / bam
    shutil.copy(os.path.join(FIXTURES, bam), path)
    rec = os.path.join(FIXTURES, bam + ".records")
    if os.path.exists(rec):
        shutil.copy(rec, str(path) + ".records")
    else:  # no sidecar in the reference: write it with index-records first
        assert cli.main(["index-records", str(path), str(path) + ".records"]) == 0
    out = tmp_path / "out.txt"
    assert cli.main(["check-blocks", "-s", str(path), str(out)]) == 0
    assert out.read_text() == _golden(golden)


@pytest.mark.gpu
@pytest.mark.parametrize("bam,golden,window", [("1.bam", "1.bam-s", 100 * 1024), ("2.bam", "2.bam", 64 * 1024),
                                               ("1.block-aligned.bam", "1.block-aligned.bam", 256 * 1024)])
def test_check_blocks_through_read_start_finders(bam, golden, window, tmp_path):
    """check-blocks' callPartition (CheckBlocks.scala:37-56) run through the drop-in ReadStartFinders: the GPU-backed
    LazyBlockChecker's nextReadStart (eager.Checker, eager/Checker.scala:127-162) against IndexedChecker's
    (indexed.Checker over the `.records` set), block by block with small windows so the walks cross windows; the
    report equals the reference's CheckBlocksTest text, and nextReadStart at sampled positions equals the truth's."""
    from sbam import Pos, cli, dist as sdist
    from sbam.checker import IndexedChecker, LazyBlockChecker
    path = tmp_path / bam
    shutil.copy(os.path.join(FIXTURES, bam), path)
    rec = os.path.join(FIXTURES, bam + ".records")
    if not os.path.exists(rec):
        rec = str(path) + ".records"
        assert cli.main(["index-records", str(path), rec]) == 0
    import sbam
    with sbam.BamFile(open(path, "rb").read()) as f:
        st, cs, us, uo = f.blocks()
        lens = f.contig_lengths
    blocks = [(int(a), int(b)) for a, b in zip(st, cs)]  # (Blocks(): the BGZF block metadata, file order)
    truth = IndexedChecker.from_records_file(rec)
    eager = LazyBlockChecker(*sdist.file_source(str(path)), lens, window=window)
    try:
        text = "\n".join(cli.check_blocks_report(blocks, eager.next_read_start, truth.next_read_start,
                                                 os.path.getsize(path), 10)) + "\n"
        assert text == _golden(golden)
        assert eager.bulk_calls > 1
        rng = np.random.default_rng(11)
        for b in rng.choice(len(blocks), min(len(blocks), 12), replace=False):
            start, _ = blocks[int(b)]
            for o in np.sort(rng.integers(0, int(us[int(b)]), 8)):
                p = Pos(start, int(o))
                assert eager.next_read_start(p) == truth.next_read_start(p), (bam, p)
                got = eager.next_read_start_with_delta(p)
                if got is not None:  # the delta counts positions (bytes of the uncompressed stream) passed over
                    q, d = got
                    assert eager.next_read_start(p, max_read_size=d) is None
                    assert eager.next_read_start(p, max_read_size=d + 1) == q
        last = blocks[-1][0]
        assert eager.next_read_start(Pos(last, int(us[-1]) - 1)) == truth.next_read_start(Pos(last, int(us[-1]) - 1))
    finally:
        eager.close()

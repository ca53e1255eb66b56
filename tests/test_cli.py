"""CLI drop-ins (sbam.cli) against the reference's golden outputs, verbatim.

full-check: cli/src/test/resources/output/full-check/* with the arguments of FullCheckTest.scala:12-68 (all
`-l 10`).  compute-splits -s: the lines ComputeSplitsTest.scala:14-30 pins (the timing line is matched by
shape, as the reference's `l"... ${d}ms"` matcher does).  The formatting helpers are checked on CPU; the
report runs need libsbam.so on a GPU."""
import os
import re
import shutil

import pytest

from conftest import FIXTURES, GOLDEN


def test_format_bytes_and_sizes():
    from sbam.cli import format_bytes, parse_bytes, parse_ranges
    assert [format_bytes(n) for n in (597454, 531725, 221910, 26169, 24080)] == \
        ["583K", "519K", "217K", "25.6K", "23.5K"]
    assert parse_bytes("230k") == 230 * 1024 and parse_bytes("2m") == 2 << 20 and parse_bytes("100") == 100
    assert parse_ranges("0-200k") == [(0, 204800)] and parse_ranges("26169") == [(26169, 26170)]


def test_stats_lines_compute_splits_test():
    # ComputeSplitsTest.scala:18-22 ("eager 230KB") and :73-77 ("compare 240KB")
    from sbam.cli import stats_lines
    assert stats_lines([224301, 244822, 113078]) == [
        "N: 3, μ/σ: 194067/57877.4, med/mad: 224301/20521",
        " elems: 224301 244822 113078",
        "sorted: 113078 224301 244822"]
    assert stats_lines([248438, 244941, 88822])[0] == "N: 3, μ/σ: 194067/74433.1, med/mad: 244941/3497"
    assert stats_lines([242083, 253302, 134922])[0] == "N: 3, μ/σ: 210102.3/53357.5, med/mad: 242083/11219"


def test_split_length():
    from sbam import Pos, Split
    from sbam.cli import split_length
    assert split_length(Split(Pos(0, 45846), Pos(239479, 312))) == 224301
    assert split_length(Split(Pos(239479, 312), Pos(484396, 25))) == 244822


class OracleBam:
    """sbam.BamFile-shaped view of a file on the CPU oracle: runs the report logic without a GPU (test
    backend only; the CLI itself always opens libsbam.so)."""

    def __init__(self, data):
        import oracle
        self.o = oracle.BamFile(data)
        self.uncompressed_size = self.o.L
        self.loads_to_eof = True

    def blocks(self):
        return self.o.start, self.o.csize, self.o.usize, self.o.uoff[:-1]

    def check_full_counts(self, x0, x1, R=10, want_bitmap=False, by_key=False):
        import numpy as np
        import sbam
        from test_gpu_parity import pair_hist
        c, npos, rbe, ns = self.o.counts_range(x0, x1, R)
        w = self.o.check_full_range(x0, x1, R)
        C = sbam.Counts(c.sum(0), c, npos, rbe, pair_hist(w), x1 - x0, ns, int(np.sum(w == 1)))
        return (C, (w & 0x80000000) != 0) if want_bitmap else C

    def check_full_words(self, x0, x1, R=10):
        return self.o.check_full_range(x0, x1, R)

    def check_eager(self, x0, x1, R=10):
        return (self.o.check_full_range(x0, x1, R) & 0x80000000) != 0

    def read_uncompressed(self, x, n):
        return self.o.u[x:x + n].tobytes()

    def pos_of(self, x):
        import sbam
        p = self.o.pos_of(x)
        return sbam.Pos(p.block_pos, p.offset)

    def offset_of(self, p):
        return self.o.offset_of(p)


CASES = [
    ("1.bam", "1.bam", ["-m", "200k"]),
    ("1.noblocks.bam", "1.bam", ["-m", "200k"]),
    ("2.bam.first", "2.bam", ["-i", "0"]),
    ("2.bam.second", "2.bam", ["-i", "26169"]),
    ("2.bam.200k", "2.bam", ["-i", "0-200k", "-m", "100k"]),
    ("2.bam", "2.bam", []),
]


@pytest.mark.parametrize("golden,bam,args", CASES)
def test_full_check_report_logic(golden, bam, args):
    """The report assembly on the oracle backend reproduces every full-check golden verbatim."""
    from sbam import cli
    data = open(os.path.join(FIXTURES, bam), "rb").read()
    ranges = cli.parse_ranges(args[args.index("-i") + 1]) if "-i" in args else None
    records = os.path.join(FIXTURES, bam + ".records") if golden != "1.noblocks.bam" else None
    rep = cli.FullCheckReport(OracleBam(data), data, records, 10, ranges)
    assert "\n".join(rep.lines()) + "\n" == open(os.path.join(GOLDEN, "full-check", golden)).read()


@pytest.mark.gpu
@pytest.mark.parametrize("golden,bam,args", CASES)
def test_full_check_report(golden, bam, args, tmp_path):
    from sbam import cli
    src = os.path.join(FIXTURES, bam)
    path = tmp_path / bam
    shutil.copy(src, path)
    if golden != "1.noblocks.bam":  # bam1Unindexed: the same file without its .records / .blocks sidecars
        shutil.copy(src + ".records", str(path) + ".records")
    out = tmp_path / "out.txt"
    assert cli.main(["full-check", "-l", "10", *args, str(path), str(out)]) == 0
    want = open(os.path.join(GOLDEN, "full-check", golden)).read()
    assert out.read_text() == want


@pytest.mark.gpu
@pytest.mark.parametrize("m,split_lines,stats", [
    ("230k", ["0:45846-239479:312", "239479:312-484396:25", "484396:25-597482:0"],
     "N: 3, μ/σ: 194067/57877.4, med/mad: 224301/20521"),
    ("240k", ["0:45846-263656:191", "263656:191-508565:287", "508565:287-597482:0"],
     "N: 3, μ/σ: 194067/74433.1, med/mad: 244941/3497"),
])
def test_compute_splits_report(m, split_lines, stats, tmp_path):
    from sbam import cli
    out = tmp_path / "out.txt"
    assert cli.main(["compute-splits", "-s", "-m", m, os.path.join(FIXTURES, "1.bam"), str(out)]) == 0
    lines = out.read_text().split("\n")
    assert re.fullmatch(r"Get spark-bam splits: \d+ms", lines[0])
    assert lines[1:4] == ["", "Split-size distribution:", stats]
    assert lines[6:] == ["", "3 splits:"] + ["\t" + s for s in split_lines] + ["", ""]


def test_check_bam_logic():
    """check-bam -s summary on the oracle backend: CheckBamTest.scala "eager 1.bam" (no false calls)."""
    from sbam import cli
    data = open(os.path.join(FIXTURES, "1.bam"), "rb").read()
    rep = cli.FullCheckReport(OracleBam(data), data, os.path.join(FIXTURES, "1.bam.records"), 10)
    assert rep.check_bam_lines() == CHECK_BAM_EAGER_1


CHECK_BAM_EAGER_1 = ["1608257 uncompressed positions", "583K compressed", "Compression ratio: 2.69", "4917 reads",
                     "All calls matched!"]


@pytest.mark.gpu
def test_check_bam_report(tmp_path):
    # CheckBamTest.scala:40-50 ("eager 1.bam", -m 200k)
    from sbam import cli
    path = tmp_path / "1.bam"
    shutil.copy(os.path.join(FIXTURES, "1.bam"), path)
    shutil.copy(os.path.join(FIXTURES, "1.bam.records"), str(path) + ".records")
    out = tmp_path / "out.txt"
    assert cli.main(["check-bam", "-s", "-m", "200k", str(path), str(out)]) == 0
    assert out.read_text() == "\n".join(CHECK_BAM_EAGER_1) + "\n"


@pytest.mark.gpu
def test_count_reads_report(tmp_path):
    # CountReadsTest.scala:10-20: 4917 reads in 1.bam at 240k
    from sbam import cli
    out = tmp_path / "out.txt"
    assert cli.main(["count-reads", "-m", "240k", os.path.join(FIXTURES, "1.bam"), str(out)]) == 0
    lines = out.read_text().split("\n")
    assert re.fullmatch(r"spark-bam read-count time: \d+", lines[0])
    assert lines[2] == "spark-bam found 4917 reads"


def test_split_size_defaults_follow_hadoop():
    """-m unset: compute-splits / count-reads use the FileSystem's split size (SplitSize.scala:10-17; the local FS
    block is 32 MiB), check-blocks 2 MB; a larger -m is capped at the FS block (FileInputFormat.computeSplitSize).
    The cap and the local default come from Hadoop, outside the reference tree: parity unpinned."""
    import sbam
    from sbam import cli
    assert sbam.effective_split_size(None) == 32 << 20
    assert sbam.effective_split_size(2 << 20) == 2 << 20
    assert sbam.effective_split_size(64 << 20) == 32 << 20
    assert sbam.effective_split_size(64 << 20, fs_block_size=128 << 20) == 64 << 20
    import argparse
    seen = {}
    orig = argparse.ArgumentParser.parse_args

    def capture(self, argv=None, ns=None):
        a = orig(self, argv, ns)
        seen[a.cmd] = a.max_split_size
        raise SystemExit(0)
    argparse.ArgumentParser.parse_args = capture
    try:
        for cmd in ("compute-splits", "count-reads", "check-blocks"):
            try:
                cli.main([cmd, "x.bam"])
            except SystemExit:
                pass
    finally:
        argparse.ArgumentParser.parse_args = orig
    assert seen == {"compute-splits": None, "count-reads": None, "check-blocks": 2 << 20}


@pytest.mark.gpu
@pytest.mark.parametrize("cmd", ["compute-splits", "count-reads"])
def test_cli_sharded_ranks_match_single(tmp_path, cmd):
    """`--gpus 2` starts two ranks (torch.distributed.run; gloo on GPU 0 to rehearse on one card) that run
    sbam.dist.run_file: the report equals the single-GPU one (timing line aside)."""
    import subprocess
    import sys
    from conftest import ROOT
    src = os.path.join(ROOT, "tests", "fixtures", "2.bam")
    one, two = tmp_path / "one.txt", tmp_path / "two.txt"
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "spark-bam_amd"))
    base = [sys.executable, "-m", "sbam.cli", cmd, "-m", "100000", src]
    subprocess.run(base + [str(one)], check=True, env=env, timeout=100)
    subprocess.run(base + [str(two), "--gpus", "2", "--dist-backend", "gloo", "--device", "0"], check=True, env=env,
                   timeout=100)
    a, b = one.read_text().split("\n"), two.read_text().split("\n")
    assert a[1:] == b[1:] and len(a) > 3


@pytest.mark.parametrize("golden,bam,args", CASES)
def test_full_check_parts_merge_in_file_order(golden, bam, args):
    """full-check --gpus N / --windows W assemble the report from per-shard parts (sbam.cli.merge_parts): Counts
    summed, the sampled close calls and the truth comparison concatenated in file order and cut to the limit.  The
    blocks split into three contiguous shards on the oracle backend give every golden verbatim."""
    import numpy as np
    from sbam import cli
    data = open(os.path.join(FIXTURES, bam), "rb").read()
    ranges = cli.parse_ranges(args[args.index("-i") + 1]) if "-i" in args else None
    records = os.path.join(FIXTURES, bam + ".records") if golden != "1.noblocks.bam" else None
    ob = OracleBam(data)
    nb = ob.blocks()[0].size
    parts = []
    for a, b in ((0, nb // 3), (nb // 3, 2 * nb // 3), (2 * nb // 3, nb)):
        m = np.zeros(nb, bool)
        m[a:b] = True
        parts.append(cli.FullCheckReport(ob, data, records, 10, ranges, blocks=m).parts())
    merged = cli.merge_parts(parts, 10)
    assert "\n".join(cli.full_check_lines(merged, 10)) + "\n" == open(os.path.join(GOLDEN, "full-check", golden)).read()


@pytest.mark.gpu
@pytest.mark.parametrize("golden,bam,args", [CASES[0], CASES[4], CASES[5]])
@pytest.mark.parametrize("mode", [["--gpus", "2", "--dist-backend", "gloo", "--device", "0"], ["--windows", "3"]])
def test_full_check_sharded_matches_golden(tmp_path, golden, bam, args, mode):
    """full-check over byte-range shards (sbam.dist.full_check_file): two ranks (torch.distributed.run; gloo on GPU 0
    to rehearse on one card) or three windows one after another on one GPU — the report equals the golden."""
    import subprocess
    import sys
    from conftest import ROOT
    path = tmp_path / bam
    shutil.copy(os.path.join(FIXTURES, bam), path)
    shutil.copy(os.path.join(FIXTURES, bam + ".records"), str(path) + ".records")
    out = tmp_path / "out.txt"
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "spark-bam_amd"))
    subprocess.run([sys.executable, "-m", "sbam.cli", "full-check", "-l", "10", *args, *mode, str(path), str(out)],
                   check=True, env=env, timeout=200)
    assert out.read_text() == open(os.path.join(GOLDEN, "full-check", golden)).read()

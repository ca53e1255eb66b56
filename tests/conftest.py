import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

FIXTURES = os.path.join(ROOT, "tests", "fixtures")
GOLDEN = os.path.join(ROOT, "tests", "golden")

# The reference's record-indexed test BAMs (test_bams/src/main/resources, cli/src/test/resources/slice)
INDEXED_BAMS = ["1.bam", "2.bam", "5k.bam", "1.2203053-2211029.bam", "2.100-1000.bam"]
ALL_BAMS = INDEXED_BAMS + ["1.block-aligned.bam"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsbam.so)")


def fixture_bytes(name):
    with open(os.path.join(FIXTURES, name), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def oracle_files():
    import oracle
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = oracle.BamFile(fixture_bytes(name))
        return cache[name]
    return get


@pytest.fixture(scope="session")
def gpu_files():
    import sbam
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = sbam.BamFile(fixture_bytes(name), path=name)
        return cache[name]
    yield get
    for f in cache.values():
        f.close()


@pytest.fixture(scope="session")
def distinct_synth():
    """A multi-GB synthetic Illumina-like BAM (the bench generator) with NO repeated tile: every 64 MB tile has its
    own seed (tools/synth.py distinct=True).  SBAM_SCALE_GB sets the size (default 4).  Shared by the at-scale tests."""
    import synth
    gb = float(os.environ.get("SBAM_SCALE_GB", "4"))
    s = synth.SynthBam.for_size(int(gb * 1.01e9), tile_mb=64, threads=16, distinct=True)
    digests = {hash(t[:1 << 16].tobytes()) for t in s.tiles[: s.copies]}
    assert len(digests) == s.copies, "a tile repeats"
    return s

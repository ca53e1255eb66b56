"""The eager record-0 pass (k_eager_wave, one wave per interior tile) against the oracle on inputs that stress its
paths: a tile where every position survives the refIdx / nextRefIdx prefilter (a 45 KB run of zero bytes inside a
record: more than the wave's 128-entry survivor queue holds, so the queue runs in rounds), survivors at the tile's
last positions (whose nextRefIdx lies in the 64 B the wave loads past the tile), and the plain fixtures.  eager.Checker =
eager/Checker.scala:24-126; its calls equal full.Checker's success bit (both are "the first R records pass")."""
import os
import struct
import zlib

import numpy as np
import pytest

from conftest import FIXTURES


def bgzf(u: bytes, chunk: int = 65280) -> bytes:
    """BGZF blocks (RFC 1952 members with the BC extra field, zlib level 6) of `u`, then the EOF marker block."""
    out = []
    for i in range(0, len(u), chunk):
        p = u[i:i + chunk]
        co = zlib.compressobj(6, zlib.DEFLATED, -15, 8)
        data = co.compress(p) + co.flush()
        hdr = b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<HBBHH", 6, 66, 67, 2, 18 + len(data) + 8 - 1)
        out.append(hdr + data + struct.pack("<II", zlib.crc32(p), len(p)))
    co = zlib.compressobj(6, zlib.DEFLATED, -15, 8)
    data = co.compress(b"") + co.flush()
    hdr = b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<HBBHH", 6, 66, 67, 2, 18 + len(data) + 8 - 1)
    out.append(hdr + data + struct.pack("<II", 0, 0))
    return b"".join(out)


def zero_record(l_seq: int = 30000) -> bytes:
    """A valid BAM record (contig 0, one l_seq-M op) whose sequence and qualities are all zero bytes."""
    name = b"zeros\x00"
    body = struct.pack("<iiBBHHHiiii", 0, 100, len(name), 0, 4680, 1, 0, l_seq, -1, -1, 0) + name
    body += struct.pack("<I", (l_seq << 4) | 0) + b"\x00" * ((l_seq + 1) // 2) + b"\x00" * l_seq
    return struct.pack("<i", len(body)) + body


@pytest.fixture(scope="module")
def zero_run_bam():
    import oracle
    data = open(os.path.join(FIXTURES, "2.bam"), "rb").read()
    o = oracle.BamFile(data)
    u = o.u[:o.L].tobytes()
    recs = [ln.split(",") for ln in open(os.path.join(FIXTURES, "2.bam.records")) if ln.strip()]
    at = o.offset_of(oracle.Pos(int(recs[len(recs) // 3][0]), int(recs[len(recs) // 3][1])))
    u2 = u[:at] + zero_record() + zero_record(4001) + u[at:]
    blob = bgzf(u2)
    return blob, oracle.BamFile(blob), at


def test_zero_run_file_is_valid_for_the_oracle(zero_run_bam):
    blob, o, at = zero_run_bam
    w = o.check_full_range(at, at + 200)
    assert w[0] & 0x80000000  # the zero-run record is a true record start


@pytest.mark.gpu
def test_eager_zero_run_survivor_rounds(zero_run_bam):
    import sbam
    blob, o, at = zero_run_bam
    with sbam.BamFile(blob, path="zeros.bam") as g:
        assert g.uncompressed_size == o.L
        want = (o.check_full_range(0, o.L) & 0x80000000) != 0
        got = g.check_eager(0, o.L)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, f"{bad.size} mismatches, first {bad[:8]}"
        # every range start/end alignment the interior tiling can see around the zero run
        for x0 in (at - 8192 * 3 - 17, at - 1, at + 5):
            for x1 in (at + 64000 + 333, o.L - 300000):
                got = g.check_eager(x0, x1)
                assert np.array_equal(got, want[x0:x1]), (x0, x1)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["1.bam", "5k.bam", "1.2203053-2211029.bam"])
def test_eager_every_offset_unaligned_ranges(name):
    """Calls over ranges whose interior tiles start at every residue of the 16-B pieces equal the whole-file calls."""
    import sbam
    import oracle
    data = open(os.path.join(FIXTURES, name), "rb").read()
    o = oracle.BamFile(data)
    want = (o.check_full_range(0, o.L) & 0x80000000) != 0
    with sbam.BamFile(data) as g:
        assert np.array_equal(g.check_eager(0, o.L), want)
        for x0 in (1, 15, 63, 64, 1000, 8191, 8193):
            assert np.array_equal(g.check_eager(x0, o.L), want[x0:]), x0

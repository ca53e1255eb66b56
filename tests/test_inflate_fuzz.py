"""Inflate fuzz at scale: 100 000 BGZF blocks of mixed inputs (BAM slices, text, random bytes,
runs, DNA, binned qualities, mixtures), raw-deflated by Python's zlib at levels 0-9 × {default, filtered,
Huffman-only, RLE, fixed} × memLevel 1-9 × window 2^9-2^15, sizes 1 B-65 280 B; every block's GPU output against the
CRC32 and ISIZE of its own footer (zlib's output: Stream.scala:49-54 inflates with java.util.zip.Inflater).  The
corpus builder is tools/inflate_fuzz.py (its log with the wave decoder's path counts is under profiles/r05/)."""
import os

import pytest


def test_fuzz_corpus_shape():
    """A small corpus on the CPU: every block parses back (BSIZE chain), ISIZE matches, the EOF block ends it."""
    import struct
    import zlib
    import inflate_fuzz
    data, meta = inflate_fuzz.make_corpus(300, seed=3, workers=2, per_task=100)
    pos, n = 0, 0
    while pos < len(data):
        end = pos + struct.unpack("<H", data[pos + 16:pos + 18])[0] + 1
        crc, isz = struct.unpack("<II", data[end - 8:end])
        payload = zlib.decompressobj(-15).decompress(data[pos + 18:end - 8])
        assert len(payload) == isz and zlib.crc32(payload) == crc
        pos, n = end, n + 1
    assert n == len(meta) + 1 and isz == 0
    assert {m[1] for m in meta} == set(range(10)) and len({m[2] for m in meta}) == 5


@pytest.mark.gpu
def test_inflate_fuzz_100k_blocks():
    import inflate_fuzz
    n = int(os.environ.get("SBAM_FUZZ_BLOCKS", "100000"))
    data, meta = inflate_fuzz.make_corpus(n, seed=1, workers=16)
    res = inflate_fuzz.check(data, meta)
    print(res)
    assert res["blocks"] == n  # (the empty EOF block ends the block stream: MetadataStream.scala:23-54)
    assert res["mismatches"] == 0, res["first_mismatches"]

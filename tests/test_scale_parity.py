"""configs[2]-style verdict diff at scale: on a multi-GB synthetic BAM resident on the GPU, the full checker's
result word at every offset of randomly sampled block runs equals the CPU oracle's, the oracle inflating those
blocks itself from the compressed bytes (an independent stream); 4096 sampled blocks inflate to the CRC32 and
ISIZE their BGZF footers store; and the eager and full checks agree at every offset and call exactly the
generated records.  The file has no repeated tile (conftest.distinct_synth); SBAM_SCALE_GB sets the size (default
4)."""
import os

import numpy as np
import pytest

GB = float(os.environ.get("SBAM_SCALE_GB", "4"))


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_sampled_verdicts_at_scale(distinct_synth):
    import oracle
    import sbam
    s = distinct_synth  # no repeated tile: the 48 sampled runs come from different tiles
    data = s.bytes()
    lens = np.asarray(s.contig_lengths, np.int64)
    with sbam.BamFile(data, path="synth.bam") as g:
        st, cs, us, uo = g.blocks()
        rng = np.random.default_rng(0x5EED)
        picks = np.sort(rng.choice(st.size - 40, 48, replace=False))
        tiles = {int(np.searchsorted(s.tile_starts, int(st[b]), side="right")) for b in picks.tolist()}
        assert len(tiles) >= 24, "samples concentrated in few tiles"
        compared = 0
        for b in picks.tolist():
            # 24 whole blocks as an independent BGZF stream; positions of the first 8 are compared (their
            # record-0 reads reach at most 36 + 255 + 4·65535 bytes, ~4 blocks; chains of real records ~4 KB)
            o = oracle.BamFile(data[int(st[b]):int(st[b + 24])])
            o.lens[:lens.size] = lens
            o.nref = lens.size
            x1 = int(uo[b + 8] - uo[b])
            want = o.check_full_range(0, x1)
            got = g.check_full_words(int(uo[b]), int(uo[b]) + x1)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (b, bad[:5], got[bad[:5]], want[bad[:5]])
            compared += x1
        assert compared > 48 * 8 * 60000
        # inflate at scale: each sampled block's bytes match the CRC32 its BGZF footer stores (the reference never
        # checks it, but a correct inflate reproduces it), and its size the footer's ISIZE
        import zlib
        for b in np.sort(rng.choice(st.size, 4096, replace=False)).tolist():
            end = int(st[b]) + int(cs[b])
            crc, isize = (int.from_bytes(data[end - 8 + k:end - 4 + k].tobytes(), "little") for k in (0, 4))
            raw = g.read_uncompressed(int(uo[b]), int(us[b]))
            assert len(raw) == isize and zlib.crc32(raw) == crc, b
        # eager and full checks agree at every offset, and call exactly the generated records
        L = g.uncompressed_size
        eager = g.check_eager(0, L)
        c, full = g.check_full_counts(0, L, want_bitmap=True)
        assert np.array_equal(eager, full) and int(eager.sum()) == c.n_success == s.n_records

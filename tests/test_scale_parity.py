"""configs[2]-style verdict diff at scale: on a multi-GB synthetic BAM resident on the GPU, the full checker's
result word at every offset of randomly sampled block runs equals the CPU oracle's, the oracle inflating those
blocks itself from the compressed bytes (an independent stream).  The bench's full-size properties (records ==
checker calls == generator count) cover the rest of the file.  SBAM_SCALE_GB sets the size (default 4)."""
import os

import numpy as np
import pytest

GB = float(os.environ.get("SBAM_SCALE_GB", "4"))


@pytest.mark.gpu
def test_sampled_verdicts_at_scale():
    import oracle
    import sbam
    import synth
    s = synth.SynthBam.for_size(int(GB * 1e9), tile_mb=64, threads=16)
    data = s.bytes()
    lens = np.asarray(s.contig_lengths, np.int64)
    with sbam.BamFile(data, path="synth.bam") as g:
        st, cs, us, uo = g.blocks()
        rng = np.random.default_rng(0x5EED)
        picks = np.sort(rng.choice(st.size - 40, 48, replace=False))
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

"""Bit-exact parity on the bench's own data shape: a synthetic Illumina-like BAM (tools/synth_bam.c, the
bench generator at a small size: 150 bp pairs over the 84 GRCh37 contigs, zlib-6, records straddling blocks).
The fixtures pin the reference's semantics; this pins the GPU kernels on the workload the bench measures —
every interior-tile fast path and the per-key counting — against the CPU oracle at every offset."""
import numpy as np
import pytest

from test_gpu_parity import pair_hist


@pytest.fixture(scope="module")
def synth_file():
    import oracle
    import synth
    s = synth.SynthBam.for_size(int(20e6), tile_mb=8, threads=16)
    data = s.bytes()
    o = oracle.BamFile(data, threads=16)
    return s, data, o


def test_oracle_finds_every_generated_record(synth_file):
    s, _, o = synth_file
    assert o.nref == len(s.contig_lengths)
    assert o.counts_range(0, o.L)[3] == s.n_records


@pytest.mark.gpu
def test_synthetic_every_offset_and_counts(synth_file):
    import sbam
    s, data, o = synth_file
    with sbam.BamFile(data, path="synth.bam") as g:
        assert g.uncompressed_size == o.L
        assert g.read_uncompressed(0, o.L) == o.u[:o.L].tobytes()
        assert g.inflate_fallbacks() == 0  # every block through the wave-parallel decoder
        w = o.check_full_range(0, o.L)
        got = g.check_full_words(0, o.L)
        bad = np.flatnonzero(got != w)
        assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: {got[bad[:5]]} vs {w[bad[:5]]}"
        counts, npos, rbe, nsucc = o.counts_range(0, o.L)
        c, bits = g.check_full_counts(0, o.L, want_bitmap=True)
        assert np.array_equal(c.totals, counts.sum(0))
        assert np.array_equal(c.by_key[:3], counts[:3])
        assert np.array_equal(c.positions, npos)
        assert np.array_equal(c.reads_before_error, rbe)
        assert c.n_success == nsucc == s.n_records
        assert np.array_equal(bits, (w & 0x80000000) != 0)
        assert np.array_equal(c.pair_hist, pair_hist(w))
        assert np.array_equal(g.check_eager(0, o.L), (w & 0x80000000) != 0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["many_contigs", "many_contigs_short", "reads_to_check_0"])
def test_counts_general_paths(synth_file, case):
    """Past the bit-sliced interior pass's LDS table of contig lengths (n_ref > 4096: the rare length probes read the
    device table, round 5) and with reads_to_check = 0 (the general k_check<MODE_COUNTS, 0> over every tile), against
    the oracle: 5000 contigs (the 84 real ones, then 4916 more, so refIdx values up to 4999 become in-range; "short":
    lengths 1-999, so refPos > length fires on many of them) and R = 0."""
    import sbam
    s, data, o = synth_file
    R = 0 if case == "reads_to_check_0" else 10
    lens, nref = o.lens, o.nref
    try:
        if case.startswith("many_contigs"):
            rng = np.random.default_rng(7)
            extra = rng.integers(1, 1000 if case.endswith("short") else 1 << 31, 5000 - o.nref).astype(np.int64)
            o.lens = np.zeros(1 << 16, np.int64)
            o.lens[:nref] = lens[:nref]
            o.lens[nref:5000] = extra
            o.nref = 5000
        x1 = min(o.L, 6_000_000)
        counts, npos, rbe, nsucc = o.counts_range(0, x1, R)
        w = o.check_full_range(0, x1, R)
        with sbam.BamFile(data, path="synth.bam", contig_lengths=o.lens[:o.nref]) as g:
            c, bits = g.check_full_counts(0, x1, reads_to_check=R, want_bitmap=True)
            assert np.array_equal(c.totals, counts.sum(0))
            assert np.array_equal(c.by_key[:3], counts[:3])
            assert np.array_equal(c.positions, npos)
            assert np.array_equal(c.reads_before_error, rbe)
            assert c.n_success == nsucc
            assert np.array_equal(bits, (w & 0x80000000) != 0)
    finally:
        o.lens, o.nref = lens, nref

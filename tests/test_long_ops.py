"""Op arrays longer than 64 ops (round 6): the checkers' invalid-op search past the first 64 ops of a position's
CIGAR — the per-tile table (next_bad_in_window), the first-invalid-op bytes, the scans past the tile's window
(k_check_bits: the whole wave, scan_past_window; k_check: one lane, cached per wave) and k_eager_wave's
wave-read CIGARs (ops_bad_wave) — against the oracle, on hand-built records inserted into the reference's 2.bam:

* a true record with 3000 valid CIGAR ops, and one whose op 2000 is invalid (full/Checker.scala's CIGAR loop:
  flag 15 deep inside a long array, and a failing record in the chains around it);
* a record whose packed sequence is 40 KB of 0x12 bytes (valid op codes; every position there reads n_cigar = 0x1212
  = 4626 ops, 18.5 KB of reach) followed by valid quality bytes and then invalid ones at offsets staggered across the
  four residue classes — so that positions find their first invalid op inside their window, just past it, or many
  windows on, and the answer differs by class;
* a record whose sequence is 200 KB of 0x88 bytes (n_cigar = 0x8888 = 34 952 ops, 140 KB of reach: positions at its
  start find no invalid op within their array at all, and the wave's scan runs past its 256 KiB reach).

Expected values are the oracle's (pinned by the reference's fixtures in test_oracle.py)."""
import os
import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import FIXTURES
from test_eager_wave import bgzf


def record(name: bytes, ops, seq: bytes, qual: bytes, l_seq: int) -> bytes:
    name = name + b"\x00"
    body = struct.pack("<iiBBHHHiiii", 0, 100, len(name), 30, 4680, len(ops), 0, l_seq, -1, -1, 0) + name
    body += b"".join(struct.pack("<I", op) for op in ops) + seq + qual
    return struct.pack("<i", len(body)) + body


def staggered_tail(n_valid: int) -> bytes:
    """n_valid valid quality bytes (0x11), then invalid ones (0x19) at offsets 0, 5, 10, 15 of a 20-byte tail (one per
    residue class, each class's first invalid op at a different distance), then ordinary qualities (0x1e: invalid)."""
    tail = bytearray(b"\x11" * 20)
    for k in (0, 5, 10, 15):
        tail[k] = 0x19
    return b"\x11" * n_valid + bytes(tail)


@pytest.fixture(scope="module")
def long_ops_bam():
    import oracle
    data = open(os.path.join(FIXTURES, "2.bam"), "rb").read()
    o = oracle.BamFile(data)
    u = o.u[:o.L].tobytes()
    recs = [ln.split(",") for ln in open(os.path.join(FIXTURES, "2.bam.records")) if ln.strip()]
    at = o.offset_of(oracle.Pos(int(recs[len(recs) // 3][0]), int(recs[len(recs) // 3][1])))
    m1 = (1 << 4) | 0  # 1M
    ok = record(b"long_cigar_ok", [m1] * 3000, b"\x11" * 1500, b"\x1e" * 3000, 3000)
    bad_ops = [m1] * 3000
    bad_ops[2000] = (1 << 4) | 9  # op code 9 > Checker.MAX_CIGAR_OP
    bad = record(b"long_cigar_bad", bad_ops, b"\x11" * 1500, b"\x1e" * 3000, 3000)
    q1 = staggered_tail(30001)
    seq_run = record(b"seq_run_0x12", [(80000 << 4) | 0], b"\x12" * 40000, q1 + b"\x1e" * (80000 - len(q1)), 80000)
    q2 = staggered_tail(7)
    far_run = record(b"seq_run_0x88", [(400000 << 4) | 0], b"\x88" * 200000, q2 + b"\x1e" * (400000 - len(q2)), 400000)
    u2 = u[:at] + ok + bad + seq_run + far_run + u[at:]
    blob = bgzf(u2)
    ob = oracle.BamFile(blob)
    return blob, ob, at


def _words(o, x0, x1, R=10, threads=8):
    cuts = np.linspace(x0, x1, threads + 1).astype(np.int64)
    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(lambda i: o.check_full_range(int(cuts[i]), int(cuts[i + 1]), R), range(threads)))
    return np.concatenate(parts)


@pytest.fixture(scope="module")
def words10(long_ops_bam):
    blob, o, at = long_ops_bam
    return _words(o, 0, o.L)


def test_oracle_sees_the_long_arrays(long_ops_bam):
    """The inserted records do what the docstring says, per the oracle: the 3000-op record passes record 0 and the
    one with an invalid op 2000 fails flag 15; across the valid run's last 18 KB (where the arrays reach its end) both
    outcomes of flag 15 occur."""
    blob, o, at = long_ops_bam
    w = o.check_full_range(at, at + 1, 1)
    assert w[0] & 0x80000000
    bad_at = at + 4 + int.from_bytes(o.u[at:at + 4].tobytes(), "little")
    assert o.check_full_range(bad_at, bad_at + 1, 1)[0] & (1 << 15)
    seq_at = bad_at + 4 + int.from_bytes(o.u[bad_at:bad_at + 4].tobytes(), "little")
    w = o.check_full_range(seq_at + 40000, seq_at + 70000, 1)
    f15 = (w & (1 << 15)) != 0
    assert f15.any() and (~f15).any()


@pytest.mark.gpu
class TestLongOpsGpu:
    @pytest.fixture(scope="class")
    def g(self, long_ops_bam):
        import sbam
        blob, o, at = long_ops_bam
        f = sbam.BamFile(blob, path="long_ops.bam")
        assert f.uncompressed_size == o.L
        yield f
        f.close()

    @pytest.mark.parametrize("reads_to_check", [10, 1])
    def test_words_every_offset(self, g, long_ops_bam, words10, reads_to_check):
        blob, o, at = long_ops_bam
        want = words10 if reads_to_check == 10 else _words(o, 0, o.L, reads_to_check)
        got = g.check_full_words(0, o.L, reads_to_check)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: {got[bad[:5]]} vs {want[bad[:5]]}"

    @pytest.mark.parametrize("by_key", [False, True])
    def test_counts(self, g, long_ops_bam, words10, by_key):
        blob, o, at = long_ops_bam
        c, npos, rbe, ns = o.counts_parallel(0, o.L, 10, 8)
        got, bits = g.check_full_counts(0, o.L, 10, want_bitmap=True, by_key=by_key)
        assert np.array_equal(got.totals, c.sum(0))
        assert np.array_equal(got.by_key if by_key else got.by_key[:3], c if by_key else c[:3])
        assert np.array_equal(got.positions, npos) and np.array_equal(got.reads_before_error, rbe)
        assert got.n_success == ns
        assert np.array_equal(bits, (words10 & 0x80000000) != 0)

    def test_eager_calls(self, g, long_ops_bam, words10):
        blob, o, at = long_ops_bam
        want = (words10 & 0x80000000) != 0
        got = g.check_eager(0, o.L)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, f"{bad.size} mismatches, first {bad[:8]}"

"""Inflate edge cases: BGZF files whose payloads cover every DEFLATE shape zlib emits (stored, fixed and
dynamic Huffman blocks, Huffman-only, RLE, overlapping copies of every period up to 48, matches that reach
back 32 KiB) plus corrupted and mis-sized payloads, checked against the oracle's zlib inflate
(Inflater.inflate(buf, 0, ISIZE) semantics of bgzf/src/main/scala/org/hammerlab/bgzf/block/Stream.scala:31-71).

The files are built here from Python's zlib (no reference fixtures cover these shapes; the reference's own
BGZF goldens are exercised by test_gpu_parity)."""
import struct
import zlib

import numpy as np
import pytest

EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def bgzf_block(payload: bytes, isize: int) -> bytes:
    bsize = 18 + len(payload) + 8 - 1
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize)
    return hdr + payload + struct.pack("<II", 0, isize & 0xffffffff)


def deflate(data: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
    return c.compress(data) + c.flush()


def sample_inputs(seed: int):
    r = np.random.default_rng(seed)
    out = []
    out.append(r.integers(0, 256, 60000, dtype=np.uint8).tobytes())                 # incompressible
    out.append(b"A" * 60000)                                                          # dist-1 run, 258-B matches
    for period in (2, 3, 5, 7, 13, 16, 17, 31, 40, 41, 47, 48, 64, 200):             # overlapping copies
        unit = r.integers(0, 256, period, dtype=np.uint8).tobytes()
        out.append((unit * (60000 // period + 1))[:60000])
    text = b" ".join(b"SYN:1:FC:%d:%d:%d" % tuple(r.integers(0, 9999, 3)) for _ in range(4000))
    out.append(text[:60000])
    # BAM-like: qualities with runs, 2-bit bases, far repeats (up to 32 KiB back)
    q = r.choice(np.frombuffer(b"#+5?EJ", np.uint8), 30000).tobytes()
    far = r.integers(0, 256, 20000, dtype=np.uint8).tobytes()
    out.append((q[:20000] + far + q[:5000] + far[:15000])[:60000])
    out.append(b"x")
    return out  # (an empty payload would end the stream: MetadataStream.scala:23-54)


SHAPES = [(6, zlib.Z_DEFAULT_STRATEGY), (0, zlib.Z_DEFAULT_STRATEGY), (1, zlib.Z_DEFAULT_STRATEGY),
          (9, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_FILTERED), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE),
          (6, zlib.Z_FIXED)]


def build_file(seed: int, corrupt: int = 0, size_jitter: bool = False):
    """A BGZF file of many blocks; `corrupt` flips that many random payload bits in ONE block."""
    r = np.random.default_rng(seed + 1000)
    blocks = []
    for i, data in enumerate(sample_inputs(seed)):
        level, strat = SHAPES[(i + seed) % len(SHAPES)]
        p = bytearray(deflate(data, level, strat))
        isize = len(data)
        blocks.append([p, isize])
    if corrupt:
        b = int(r.integers(0, len(blocks)))
        p = blocks[b][0]
        if len(p):
            for _ in range(corrupt):
                k = int(r.integers(0, len(p) * 8))
                p[k >> 3] ^= 1 << (k & 7)
    if size_jitter:
        b = int(r.integers(0, len(blocks)))
        blocks[b][1] = max(0, blocks[b][1] + int(r.choice([-100, -1, 1, 7])))
    return b"".join(bgzf_block(bytes(p), n) for p, n in blocks) + EOF_BLOCK


def oracle_result(data: bytes):
    import oracle
    try:
        f = oracle.BamFile(data)
    except IOError as e:
        return ("error", str(e))
    return ("ok", f.u[: f.L].tobytes())


def gpu_result(data: bytes):
    import sbam
    g = sbam.BamFile(data, inflate=False)
    try:
        n = g.inflate()
    except sbam.InflateException as e:
        g.close()
        return ("error", str(e))
    out = g.read_uncompressed(0, n)
    g.close()
    return ("ok", out)


def test_oracle_roundtrips_every_shape():
    data = build_file(0)
    kind, out = oracle_result(data)
    assert kind == "ok"
    assert out == b"".join(sample_inputs(0))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_inflate_shapes_bit_exact(seed):
    data = build_file(seed)
    assert gpu_result(data) == oracle_result(data)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(24))
def test_inflate_mis_sized_isize(seed):
    data = build_file(seed, size_jitter=True)
    assert gpu_result(data) == oracle_result(data)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_inflate_corrupted_payloads(seed):
    data = build_file(seed, corrupt=1 + seed % 4)
    assert gpu_result(data) == oracle_result(data)


def stored_chain(p: bytes) -> bool:
    """Whether a raw DEFLATE stream is only stored blocks from its first bit to a final block (RFC 1951 3.2.4) —
    the payloads k_inflate_stored copies."""
    pos = 0  # bit position
    while True:
        if (pos >> 3) >= len(p):
            return False
        hb = (p[pos >> 3] | (p[(pos >> 3) + 1] << 8 if (pos >> 3) + 1 < len(p) else 0)) >> (pos & 7)
        if (hb >> 1) & 3:
            return False
        byp = (pos + 3 + 7) >> 3
        if byp + 4 > len(p):
            return False
        ln, nln = struct.unpack("<HH", p[byp:byp + 4])
        if ln ^ 0xffff != nln or byp + 4 + ln > len(p):
            return False
        if hb & 1:
            return True
        pos = (byp + 4 + ln) * 8


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_wave_decoder_takes_every_compressed_block(seed):
    """Fixed, dynamic, Huffman-only and RLE blocks are decoded by the wave-parallel decoder, and payloads that are only
    stored blocks (level 0; incompressible data at any level) are copied by k_inflate_stored; only a payload whose
    first DEFLATE block is stored but which goes on with Huffman blocks takes the per-lane exact decoder (round 6;
    before, every payload starting with a stored block did).  The bytes: test_inflate_shapes_bit_exact."""
    import sbam
    data = build_file(seed)
    exact = 0
    for i, raw in enumerate(sample_inputs(seed)):
        level, strat = SHAPES[(i + seed) % len(SHAPES)]
        p = deflate(raw, level, strat)
        exact += ((p[0] >> 1) & 3) == 0 and not stored_chain(p)  # first block's BTYPE stored, not all stored
    g = sbam.BamFile(data, inflate=False)
    try:
        g.inflate()
        assert g.inflate_fallbacks() == exact
    finally:
        g.close()


def stored_block(data: bytes, final: bool) -> bytes:
    """One byte-aligned stored DEFLATE block (the header's 5 padding bits are zero)."""
    return bytes([1 if final else 0]) + struct.pack("<HH", len(data), len(data) ^ 0xffff) + data


def stored_shape_blocks(seed):
    """(payload, ISIZE) pairs of stored-block payloads that zlib inflates to exactly ISIZE bytes."""
    r = np.random.default_rng(seed)
    blocks = []
    for n in (1, 15, 16, 17, 1000, 4096, 65480, int(r.integers(2, 65480))):  # (BSIZE is a u16: <= 65510 stored bytes)
        x = r.integers(0, 256, n, dtype=np.uint8).tobytes()
        blocks.append((deflate(x, 0), n))
    x = r.integers(0, 256, 65000, dtype=np.uint8).tobytes()
    blocks.append((stored_block(x[:40001], False) + stored_block(x[40001:], True), 65000))
    for _ in range(6):  # chains of small stored blocks, some empty
        parts = [r.integers(0, 256, int(r.integers(0, 40)), dtype=np.uint8).tobytes()
                 for _ in range(int(r.integers(2, 60)))]
        blocks.append((b"".join(stored_block(x, i == len(parts) - 1) for i, x in enumerate(parts)),
                       sum(len(x) for x in parts)))
    x = r.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    blocks.append((b"".join(stored_block(x[i:i + 30], i + 30 >= 3000) for i in range(0, 3000, 30)), 3000))  # 100
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    hx = b"ACGT" * 2000
    blocks.append((c.compress(hx) + c.flush(zlib.Z_SYNC_FLUSH) + stored_block(x[:777], True), len(hx) + 777))
    good = stored_block(x[:500], True)
    blocks.append((good, 500))
    blocks.append((good + b"\x17\x42", 500))  # trailing bytes after the final block (zlib ignores them)
    return blocks, good


def test_stored_shapes_oracle():
    blocks, _ = stored_shape_blocks(0)
    kind, out = oracle_result(b"".join(bgzf_block(p, n) for p, n in blocks) + EOF_BLOCK)
    assert kind == "ok" and len(out) == sum(n for _, n in blocks)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_stored_payload_shapes(seed):
    """Payloads of stored blocks against zlib: level 0 of sizes up to a full BGZF block (one or two stored blocks), chains of
    many small and zero-length stored blocks (every alignment of a block edge against the output's 16-B chunks), a
    stored block after a sync-flushed Huffman block (the exact decoder), and the cases the copy must hand to the exact
    decoder: LEN != ~NLEN, data past the payload, no final block, ISIZE other than the chain's bytes, trailing bytes
    after the final block, more stored blocks than the copy lists (64)."""
    blocks, good = stored_shape_blocks(seed)
    data = b"".join(bgzf_block(p, n) for p, n in blocks) + EOF_BLOCK
    assert gpu_result(data) == oracle_result(data)
    bad = [(good[:3] + bytes([good[3] ^ 1]) + good[4:], 500),  # NLEN
           (good[:-1], 500),                                     # data past the payload
           (stored_block(good[5:], False), 500),                 # no final block
           (good, 499), (good, 501), (good, 0)]                  # ISIZE other than the chain's bytes
    for p, n in bad:
        data = b"".join(bgzf_block(q, m) for q, m in blocks[:3] + [(p, n)] + blocks[3:5]) + EOF_BLOCK
        assert gpu_result(data) == oracle_result(data), (p[:8], n)


@pytest.mark.gpu
@pytest.mark.parametrize("n_blocks", [300, 1500])
def test_scan_many_small_blocks(n_blocks):
    """The one-pass BGZF scan keeps up to 512 candidates per 1 MiB chunk; more (blocks under 2 KiB, here ~40 B) take
    the exact two-pass path.  Both give the oracle's block table and bytes (Header.make / MetadataStream)."""
    import sbam
    r = np.random.default_rng(n_blocks)
    datas = [r.integers(0, 4, int(r.integers(1, 40)), dtype=np.uint8).tobytes() for _ in range(n_blocks)]
    data = b"".join(bgzf_block(deflate(x), len(x)) for x in datas) + EOF_BLOCK
    assert oracle_result(data) == ("ok", b"".join(datas))
    assert gpu_result(data) == ("ok", b"".join(datas))
    g = sbam.BamFile(data, inflate=False)
    try:
        starts = g.blocks()[0]
        want = np.cumsum([0] + [len(bgzf_block(deflate(x), len(x))) for x in datas[:-1]])
        assert np.array_equal(starts, want)
    finally:
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("gap", [4099, 1021])
def test_scan_fake_headers_every_alignment(gap):
    """Stored blocks whose payloads hold a BGZF header pattern every `gap` bytes (Header.make's bytes 0-3 and
    12-14), over > 2 MiB so that the fake candidates fall at every position of a lane's 32 and across the 1 MiB
    scan chunks (gap 1021: > 512 candidates per chunk, the exact two-pass path).  MetadataStream follows BSIZE
    from block 0, so the block table and bytes must equal the oracle's."""
    import sbam
    r = np.random.default_rng(gap)
    fake = b"\x1f\x8b\x08\x04" + bytes(8) + b"BC\x02" + b"\x00\xff\x00"
    datas = []
    for i in range(40):
        x = bytearray(r.integers(0, 256, int(r.integers(50000, 65000)), dtype=np.uint8).tobytes())
        for o in range(int(r.integers(0, gap)), len(x) - len(fake), gap):
            x[o:o + len(fake)] = fake
        datas.append(bytes(x))
    blocks = [bgzf_block(deflate(x, 0), len(x)) for x in datas]
    data = b"".join(blocks) + EOF_BLOCK
    assert len(data) > 2 << 20
    assert oracle_result(data) == ("ok", b"".join(datas))
    assert gpu_result(data) == ("ok", b"".join(datas))
    g = sbam.BamFile(data, inflate=False)
    try:
        assert np.array_equal(g.blocks()[0], np.cumsum([0] + [len(b) for b in blocks[:-1]]))
    finally:
        g.close()


# ---- a hand-placed fixed-Huffman stream: a round boundary of the wave decoder between a length and its distance --
class _BitWriter:
    def __init__(self):
        self.bits = []

    def put(self, v: int, n: int):  # n bits of v, LSB first (header fields, extra bits)
        self.bits += [(v >> i) & 1 for i in range(n)]

    def code(self, c: int, n: int):  # a Huffman code, MSB first
        self.bits += [(c >> (n - 1 - i)) & 1 for i in range(n)]

    def lit(self, b: int):
        assert b < 144
        self.code(0x30 + b, 8)

    def len258(self):
        self.code(0xC0 + 5, 8)  # symbol 285, no extra bits

    def dist(self, d: int):
        if d == 1:
            self.code(0, 5)
        else:
            assert d == 32768
            self.code(29, 5)
            self.put(d - 24577, 13)

    def tobytes(self) -> bytes:
        b = self.bits + [0] * (-len(self.bits) % 8)
        return bytes(sum(b[i + j] << j for j in range(8)) for i in range(0, len(b), 8))


def straddle_stream(distance_ok: bool):
    """One final fixed-Huffman block whose first 64 x 544-bit round ends inside a 258-byte length symbol, with
    32768 <= bytes out (including that match) < 32768 + 258; its distance (the next round's first symbol, decoded
    in the distance state with the pending length) reaches exactly back to the block start (valid) or one byte
    further (zlib: "invalid distance too far back").  The wave decoder's "no distance can reach past the start"
    shortcut must still check it (the round starts in the distance state)."""
    B = 3 + 64 * 544  # bit of the first round's end, from the payload start
    for n_m in range(100, 128):
        for n9 in range(0, 8):  # 9-bit literals (144..255) shift the bit count by one each
            rest = B - 8 - 11 - 13 * n_m - 9 * n9
            if rest < 0:
                continue
            n8 = rest // 8 + (1 if rest % 8 else 0)  # pos_c in [B - 8, B - 1]
            pos_c = 11 + 13 * n_m + 9 * n9 + 8 * n8
            out_after = 1 + 258 * n_m + n9 + n8 + 258
            if B - 8 <= pos_c < B and 32768 <= out_after < 32768 + 258 and out_after - 258 < 32768:
                w = _BitWriter()
                w.put(1, 1)
                w.put(1, 2)
                w.lit(65)
                for _ in range(n_m):
                    w.len258()
                    w.dist(1)
                for i in range(n9):
                    w.code(0x190 + (i % 100), 9)  # literal 144 + i
                for i in range(n8):
                    w.lit(33 + i % 90)
                assert len(w.bits) == pos_c
                w.len258()
                start = out_after - 258
                if distance_ok:
                    # the furthest valid distance from this match start: back to byte 0 (d = start <= 32767)
                    w.code(29 if start > 24576 else 28, 5)
                    w.put(start - (24577 if start > 24576 else 16385), 13 if start > 24576 else 13)
                else:
                    w.dist(32768)  # 32768 > start: too far back
                w.code(0, 7)  # end of block
                return w.tobytes(), out_after
    raise AssertionError("no layout")


def straddle_file(distance_ok: bool) -> bytes:
    payload, n = straddle_stream(distance_ok)
    return bgzf_block(payload, n) + EOF_BLOCK


def test_oracle_straddle_distance():
    kind, out = oracle_result(straddle_file(True))
    assert kind == "ok" and len(out) == straddle_stream(True)[1]
    kind, msg = oracle_result(straddle_file(False))
    assert kind == "error" and msg.startswith("Expected %d decompressed bytes" % straddle_stream(False)[1]), msg


@pytest.mark.gpu
@pytest.mark.parametrize("distance_ok", [True, False])
def test_inflate_round_boundary_distance(distance_ok):
    data = straddle_file(distance_ok)
    assert gpu_result(data) == oracle_result(data)


@pytest.mark.gpu
@pytest.mark.parametrize("arena_mb", ["", "256"])
@pytest.mark.parametrize("kind", ["stored", "huffman_then_stored", "huffman_only"])
def test_token_arena_growth(kind, arena_mb, monkeypatch):
    """Blocks whose tokens outgrow the main token regions (1 B per output byte): a stored block after Huffman output
    (the exact decoder, which always writes into the arena) and Huffman-only blocks (1 token = 2 B per byte: the wave
    decoder moves them into the arena).  32 MiB of them exceed the default arena (1/16 of the output + 1 MiB), so the
    first inflate overflows and the host grows the arena and inflates again; the bytes equal zlib's either way.
    Level-0 payloads (only stored blocks) need no tokens at all since round 6: k_inflate_stored copies them."""
    import sbam
    r = np.random.default_rng(11)
    n, size = 512, 65498
    if kind == "stored":
        datas = [r.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(n)]
        pays = [deflate(x, 0) for x in datas]
    elif kind == "huffman_then_stored":  # a sync-flushed Huffman block, then the rest as one final stored block
        datas = [b"ACGT" * 64 + r.integers(0, 256, size - 256, dtype=np.uint8).tobytes() for _ in range(n)]
        pays = []
        for x in datas:
            c = zlib.compressobj(6, zlib.DEFLATED, -15)
            pays.append(c.compress(x[:256]) + c.flush(zlib.Z_SYNC_FLUSH) + stored_block(x[256:], True))
    else:
        datas = [r.integers(0, 16, size, dtype=np.uint8).tobytes() for _ in range(n)]
        pays = [deflate(x, 6, zlib.Z_HUFFMAN_ONLY) for x in datas]
    data = b"".join(bgzf_block(p, len(x)) for p, x in zip(pays, datas)) + EOF_BLOCK
    monkeypatch.setenv("SBAM_ARENA_MB", arena_mb)  # "" = the default (1/16 of the output: grown once)
    kind_, out = gpu_result(data)
    assert kind_ == "ok"
    bad = [i for i in range(n) if out[i * size:(i + 1) * size] != datas[i]]
    assert not bad, (len(bad), bad[:8], len(out))
    g = sbam.BamFile(data, inflate=False)
    try:
        g.inflate()
        assert g.inflate_fallbacks() == (n if kind == "huffman_then_stored" else 0)
    finally:
        g.close()

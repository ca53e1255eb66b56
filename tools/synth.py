"""Synthetic BAM workloads for bench.py and the large-size tests (SURVEY §8(d) config specs).

A synthetic file is   header blocks | tile × k | unplaced tail | EOF marker   where a tile is a run of records
cut into 65498-byte payloads compressed at zlib level 6 (tools/synth_bam.c) that visits all 84 contigs, and the
tail is the unplaced pairs (refID = pos = -1) a coordinate-sorted WGS BAM ends with (short reads only).  Tile
and tail end on record boundaries, so the record chain runs through every seam; any byte range of the file can be produced without
materialising the whole file (``SynthBam.slice``), which is how each rank builds its shard + halo."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libsynth.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.synth_header.restype = i64
        L.synth_header.argtypes = [ctypes.POINTER(vp)]
        L.synth_tile.restype = i64
        L.synth_tile.argtypes = [ctypes.c_uint64, i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp),
                                 ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.synth_unplaced.restype = i64
        L.synth_unplaced.argtypes = L.synth_tile.argtypes
        L.synth_contigs.argtypes = [ctypes.POINTER(ctypes.c_int32), vp]
        L.synth_free.argtypes = [vp]
        L.synth_eof.restype = vp
        _lib = L
    return _lib


def _take(p, n) -> np.ndarray:
    a = np.frombuffer(ctypes.string_at(p, n), np.uint8).copy()
    lib().synth_free(p)
    return a


def tile_seed(seed: int, k: int) -> int:
    """Seed of tile k of a distinct-tile file (tile 0 keeps `seed`)."""
    return (seed + k * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF


class SynthBam:
    """`distinct=False`: one tile repeated `copies` times (the bench input: any byte range is cheap to produce).
    `distinct=True`: `copies` different tiles (tile k from tile_seed(seed, k), generated in parallel), so a multi-GB
    file has no repeated tile — the large-size parity tests compare it with full oracle runs."""

    def __init__(self, tile_mb: float = 64.0, copies: int = 1, read_len: int = 150, seed: int = 0x5EEDBA11,
                 level: int = 6, threads: int = 16, unplaced_mb: float | None = None, distinct: bool = False,
                 cycle: int = 0):
        L = lib()
        p = ctypes.c_void_p()
        n = L.synth_header(ctypes.byref(p))
        self.header = _take(p, n)
        self.seed, self.read_len, self.level, self.tile_mb, self.threads = seed, read_len, level, tile_mb, threads
        nrec, ulen = ctypes.c_int64(0), ctypes.c_int64(0)
        n = L.synth_tile(seed, int(tile_mb * 3 * 2 ** 20), read_len, level, threads, ctypes.byref(p),
                         ctypes.byref(nrec), ctypes.byref(ulen))
        self.tile = _take(p, n)
        self.eof = np.frombuffer(ctypes.string_at(L.synth_eof(), 28), np.uint8).copy()
        self.tile_records = nrec.value
        self.tile_u = ulen.value
        if unplaced_mb is None:
            unplaced_mb = min(1.0, tile_mb / 4) if read_len else 0.0
        self.tail = np.zeros(0, np.uint8)
        self.tail_records = 0
        if unplaced_mb > 0:
            n = L.synth_unplaced(seed, int(unplaced_mb * 3 * 2 ** 20), read_len, level, threads, ctypes.byref(p),
                                 ctypes.byref(nrec), ctypes.byref(ulen))
            self.tail = _take(p, n)
            self.tail_records = nrec.value
        self.distinct = distinct
        self.cycle = cycle  # distinct: tile k is tiles[k % cycle] (0: every tile its own seed)
        self.tiles = [self.tile]
        self.tiles_records = [self.tile_records]
        self.copies = copies
        if distinct:
            self._make_tiles(self._ntiles(copies))
        self._sizes()
        nr = ctypes.c_int32(0)
        lens = np.zeros(128, np.int64)
        L.synth_contigs(ctypes.byref(nr), lens.ctypes.data)
        self.contig_lengths = lens[: nr.value]

    def _ntiles(self, copies: int) -> int:
        return min(copies, self.cycle) if self.cycle > 0 else copies

    def _make_tiles(self, k: int):
        """Tiles 1 .. k-1 of a distinct-tile file, one generator call per worker thread (ctypes releases the GIL)."""
        from concurrent.futures import ThreadPoolExecutor
        L = lib()

        def one(i):
            p = ctypes.c_void_p()
            nrec, ulen = ctypes.c_int64(0), ctypes.c_int64(0)
            n = L.synth_tile(tile_seed(self.seed, i), int(self.tile_mb * 3 * 2 ** 20), self.read_len, self.level, 1,
                             ctypes.byref(p), ctypes.byref(nrec), ctypes.byref(ulen))
            return _take(p, n), nrec.value
        with ThreadPoolExecutor(self.threads) as ex:
            got = list(ex.map(one, range(len(self.tiles), k)))
        self.tiles += [t for t, _ in got]
        self.tiles_records += [r for _, r in got]

    @staticmethod
    def for_size(target_bytes: int, tile_mb: float = 64.0, **kw) -> "SynthBam":
        distinct = kw.pop("distinct", False)
        s = SynthBam(tile_mb=tile_mb, copies=1, **kw)
        s.copies = max(1, round((target_bytes - s.header.size - s.tail.size - 28) / s.tile.size))
        if distinct:
            s.distinct = True
            s._make_tiles(s._ntiles(s.copies))
        s._sizes()
        return s

    def _sizes(self):
        if self.distinct:
            nt = len(self.tiles)
            sz = np.array([self.tiles[k % nt].size for k in range(self.copies)], np.int64)
            self.tile_starts = self.header.size + np.concatenate([[0], np.cumsum(sz)])
            self.body = int(self.tile_starts[-1])
            self.n_records = int(sum(self.tiles_records[k % nt] for k in range(self.copies))) + self.tail_records
        else:
            self.body = self.header.size + self.copies * self.tile.size  # where the unplaced tail starts
            self.n_records = self.copies * self.tile_records + self.tail_records
        self.size = self.body + self.tail.size + 28

    def slice(self, lo: int, hi: int, out: np.ndarray | None = None) -> np.ndarray:
        """File bytes [lo, hi) (hi clamped to the file size)."""
        hi = min(hi, self.size)
        out = np.empty(hi - lo, np.uint8) if out is None else out
        H, T = self.header.size, self.tile.size
        pos = lo
        while pos < hi:
            if pos < H:
                n = min(hi, H) - pos
                out[pos - lo: pos - lo + n] = self.header[pos: pos + n]
            elif pos < self.body:
                if self.distinct:
                    k = int(np.searchsorted(self.tile_starts, pos, side="right")) - 1
                    tile, o = self.tiles[k % len(self.tiles)], pos - int(self.tile_starts[k])
                else:
                    k, o = divmod(pos - H, T)
                    tile = self.tile
                n = min(hi - pos, tile.size - o)
                out[pos - lo: pos - lo + n] = tile[o: o + n]
            elif pos < self.body + self.tail.size:
                o = pos - self.body
                n = min(hi - pos, self.tail.size - o)
                out[pos - lo: pos - lo + n] = self.tail[o: o + n]
            else:
                o = pos - self.body - self.tail.size
                n = hi - pos
                out[pos - lo: pos - lo + n] = self.eof[o: o + n]
            pos += n
        return out

    def bytes(self) -> np.ndarray:
        return self.slice(0, self.size)


def bgzf_blocks(raw: bytes):
    """(start, size, ISIZE) of every BGZF block of `raw` (BSIZE at +16, ISIZE in the last 4 bytes)."""
    out, pos = [], 0
    while pos + 18 <= len(raw):
        n = (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
        out.append((pos, n, int.from_bytes(raw[pos + n - 4:pos + n], "little")))
        pos += n
    return out


class TiledBam(SynthBam):
    """A real BAM's data blocks repeated to a target size behind its header block (bench.py --real): the header block,
    then the data blocks (every block after the header block up to the EOF marker) k times, then the EOF marker.  The
    file must have a header-only first block and data blocks that start and end on record boundaries — true of the
    reference's test_bams/src/main/resources/5k.bam (tests/fixtures/5k.bam: block 0 is the header, its .records file
    starts every one of blocks 1..49 at offset 0), so the tiled stream is a valid BAM of real htsjdk-written
    records whose record chain runs through every seam."""

    def __init__(self, path: str, target_bytes: int):  # (SynthBam's generator is not used)
        import zlib
        raw = open(path, "rb").read()
        blocks = bgzf_blocks(raw)
        assert blocks[-1][2] == 0, "no EOF marker block"
        h0, hn, _ = blocks[0]
        self.header = np.frombuffer(raw[h0:h0 + hn], np.uint8).copy()
        d0, d1 = blocks[1][0], blocks[-1][0]
        self.tile = np.frombuffer(raw[d0:d1], np.uint8).copy()
        self.eof = np.frombuffer(raw[d1:d1 + blocks[-1][1]], np.uint8).copy()
        self.tail = np.zeros(0, np.uint8)
        self.tail_records = 0
        # header (Header.scala:26-60) and the records of one tile, from zlib
        hx = raw[h0 + 18:h0 + hn - 8]
        u = zlib.decompressobj(-15).decompress(hx)
        p = 8 + int.from_bytes(u[4:8], "little")
        n_ref = int.from_bytes(u[p:p + 4], "little")
        p += 4
        lens = []
        for _ in range(n_ref):
            ln = int.from_bytes(u[p:p + 4], "little")
            lens.append(int.from_bytes(u[p + 4 + ln:p + 8 + ln], "little", signed=True))
            p += 8 + ln
        assert p == len(u), "the first block must hold exactly the header"
        self.contig_lengths = np.array(lens, np.int64)
        ut = b"".join(zlib.decompressobj(-15).decompress(raw[s + 18:s + n - 8]) for s, n, _ in blocks[1:-1])
        x, nrec = 0, 0
        while x < len(ut):
            x += 4 + int.from_bytes(ut[x:x + 4], "little")
            nrec += 1
        assert x == len(ut), "the data blocks must end on a record boundary"
        self.tile_records, self.tile_u = nrec, len(ut)
        self.seed, self.read_len, self.level, self.tile_mb, self.threads = 0, -1, -1, self.tile.size / 2 ** 20, 1
        self.distinct, self.cycle = False, 0
        self.tiles, self.tiles_records = [self.tile], [nrec]
        self.copies = max(1, round((target_bytes - self.header.size - 28) / self.tile.size))
        self.path = path
        self._sizes()

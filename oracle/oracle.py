"""Python face of the CPU oracle (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only as
the checker.  It wraps oracle/build/liboracle.so (oracle.c, the C restatement of the reference's
BGZF / checker / record-chain functions) and restates in Python the small host-side pieces of the
reference that are plain control flow:

* Hadoop FileInputFormat split rule used through hammerlab ``FileSplits.asJava``
  (load/src/main/scala/org/hammerlab/bam/spark/load/CanLoadBam.scala:182,291; SPLIT_SLOP = 1.1);
* ``CanLoadBam.loadReadsAndPositions`` / ``loadSplitsAndReads`` split assembly
  (CanLoadBam.scala:245-334): FindBlockStart → FindRecordStart → records with Pos < (end, 0),
  first Pos of every non-empty partition, ``sliding2(Pos(fileSize, 0))``;
* ``full-check`` Counts folding (cli/.../check/full/FullCheck.scala:141-191).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from bisect import bisect_right
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

FLAG_NAMES = [  # bit order: check/src/main/scala/org/hammerlab/bam/check/full/error/Flags.scala:201-223
    "tooFewFixedBlockBytes", "negativeReadIdx", "tooLargeReadIdx", "negativeReadPos", "tooLargeReadPos",
    "negativeNextReadIdx", "tooLargeNextReadIdx", "negativeNextReadPos", "tooLargeNextReadPos",
    "tooFewBytesForReadName", "nonNullTerminatedReadName", "nonASCIIReadName", "noReadName", "emptyReadName",
    "tooFewBytesForCigarOps", "invalidCigarOp", "emptyMappedCigar", "emptyMappedSeq",
    "tooFewRemainingBytesImplied",
]
W_SUCCESS = 0x80000000

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, u8p, vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p
        L.or_metadata_stream.restype = i64
        L.or_metadata_stream.argtypes = [vp, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp]
        L.or_find_block_start.restype = ctypes.c_int
        L.or_find_block_start.argtypes = [vp, i64, i64, i32, vp]
        L.or_inflate_blocks.restype = i64
        L.or_inflate_blocks.argtypes = [vp, i64, vp, vp, vp, vp, vp, i64, vp, vp, vp]
        L.or_bam_header.restype = i32
        L.or_bam_header.argtypes = [vp, i64, vp, i32, vp]
        L.or_check_full.restype = ctypes.c_uint32
        L.or_check_full.argtypes = [vp, i64, vp, i32, i64, i32]
        L.or_check_full_range.restype = None
        L.or_check_full_range.argtypes = [vp, i64, vp, i32, i64, i64, i32, vp]
        L.or_counts_range.restype = None
        L.or_counts_range.argtypes = [vp, i64, vp, i32, i64, i64, i32, vp, vp, vp, vp]
        L.or_find_record_start.restype = i64
        L.or_find_record_start.argtypes = [vp, i64, vp, i32, i64, i32, i64]
        L.or_record_chain.restype = i64
        L.or_record_chain.argtypes = [vp, i64, i64, i64, vp, i64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a is not None else None


@dataclass(frozen=True, order=True)
class Pos:
    """bgzf/src/main/scala/org/hammerlab/bgzf/Pos.scala:12-41."""
    block_pos: int
    offset: int

    def __str__(self):
        return f"{self.block_pos}:{self.offset}"


class BamFile:
    """A BGZF/BAM file opened on the CPU oracle: block table, inflated stream, header."""

    def __init__(self, data: bytes | np.ndarray, threads: int = 1):
        self.d = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        self.D = int(self.d.size)
        cap = self.D // 26 + 2
        start = np.zeros(cap, np.int64)
        csize = np.zeros(cap, np.int32)
        usize = np.zeros(cap, np.int32)
        hsize = np.zeros(cap, np.int32)
        ep, ei, ea, ee = (np.zeros(1, np.int64), np.zeros(1, np.int32), np.zeros(1, np.int32), np.zeros(1, np.int32))
        n = lib().or_metadata_stream(_p(self.d), self.D, 0, cap, _p(start), _p(csize), _p(usize), _p(hsize),
                                     _p(ep), _p(ei), _p(ea), _p(ee))
        if n < 0:
            raise ValueError(f"Position {int(ei[0])}: {int(ea[0])} != {int(ee[0])}")
        self.nblocks = int(n)
        self.start, self.csize, self.usize, self.hsize = start[:n], csize[:n], usize[:n], hsize[:n]
        self.uoff = np.zeros(n + 1, np.int64)
        self.uoff[1:] = np.cumsum(self.usize.astype(np.int64))
        self.L = int(self.uoff[-1])
        self.u = np.zeros(max(self.L, 1), np.uint8)
        self._inflate(threads)
        self.lens = np.zeros(1 << 16, np.int64)
        end = np.zeros(1, np.int64)
        nref = lib().or_bam_header(_p(self.u), self.L, _p(self.lens), self.lens.size, _p(end))
        self.nref = int(nref) if nref >= 0 else 0
        self.header_end = int(end[0]) if nref >= 0 else 0

    def _inflate(self, threads: int):
        """zlib inflate of every block; `threads` > 1 splits the block list across threads (ctypes drops the GIL)."""
        n = self.nblocks
        chunks = np.linspace(0, n, max(1, min(threads, n)) + 1).astype(np.int64)

        def run(b0, b1):
            eb, ef = np.zeros(1, np.int64), np.zeros(1, np.int64)
            uo = np.zeros(max(b1 - b0, 1), np.int64)
            out = self.u[int(self.uoff[b0]):]
            tot = lib().or_inflate_blocks(_p(self.d), b1 - b0, _p(self.start[b0:b1]), _p(self.csize[b0:b1]),
                                          _p(self.usize[b0:b1]), _p(self.hsize[b0:b1]), out.ctypes.data,
                                          int(self.uoff[b1] - self.uoff[b0]), _p(uo), _p(eb), _p(ef))
            if tot < 0:
                b = b0 + int(eb[0])
                raise IOError(f"Expected {int(self.usize[b])} decompressed bytes, found {int(ef[0])}")
        if len(chunks) <= 2:
            run(0, n)
        else:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(len(chunks) - 1) as ex:
                list(ex.map(lambda i: run(int(chunks[i]), int(chunks[i + 1])), range(len(chunks) - 1)))

    def counts_parallel(self, x0: int, x1: int, reads_to_check: int = 10, threads: int = 1):
        """counts_range split over `threads` threads (summed)."""
        from concurrent.futures import ThreadPoolExecutor
        cuts = np.linspace(x0, x1, max(1, threads) + 1).astype(np.int64)
        with ThreadPoolExecutor(max(1, threads)) as ex:
            parts = list(ex.map(lambda i: self.counts_range(int(cuts[i]), int(cuts[i + 1]), reads_to_check),
                                range(len(cuts) - 1)))
        c = sum(p[0] for p in parts)
        return c, sum(p[1] for p in parts), sum(p[2] for p in parts), sum(p[3] for p in parts)

    # ---- Pos <-> flat uncompressed offset (UncompressedBytes.scala:17-19; ByteStreamTest.scala:45-53)
    def pos_of(self, x: int) -> Pos:
        b = int(np.searchsorted(self.uoff[1:], x, side="right"))
        if b >= self.nblocks:
            return Pos(self.end_block_pos(), 0)
        return Pos(int(self.start[b]), int(x - self.uoff[b]))

    def end_block_pos(self) -> int:
        return int(self.start[-1] + self.csize[-1]) if self.nblocks else 0

    def offset_of(self, p: Pos) -> int:
        b = int(np.searchsorted(self.start, p.block_pos))
        if b >= self.nblocks or int(self.start[b]) != p.block_pos:
            raise KeyError(p)
        return int(self.uoff[b]) + p.offset

    def block_index_at_or_after(self, compressed_off: int) -> int:
        return int(np.searchsorted(self.start, compressed_off, side="left"))

    # ---- checker
    def check_full(self, x: int, reads_to_check: int = 10) -> int:
        return int(lib().or_check_full(_p(self.u), self.L, _p(self.lens), self.nref, x, reads_to_check))

    def check_full_range(self, x0: int, x1: int, reads_to_check: int = 10) -> np.ndarray:
        out = np.zeros(max(x1 - x0, 0), np.uint32)
        lib().or_check_full_range(_p(self.u), self.L, _p(self.lens), self.nref, x0, x1, reads_to_check, _p(out))
        return out

    def counts_range(self, x0: int, x1: int, reads_to_check: int = 10):
        counts = np.zeros(21 * 19, np.int64)
        npos = np.zeros(21, np.int64)
        rbe = np.zeros(21 * 128, np.int64)
        ns = np.zeros(1, np.int64)
        lib().or_counts_range(_p(self.u), self.L, _p(self.lens), self.nref, x0, x1, reads_to_check,
                              _p(counts), _p(npos), _p(rbe), _p(ns))
        return counts.reshape(21, 19), npos, rbe.reshape(21, 128), int(ns[0])

    def find_block_start(self, start: int, blocks_to_check: int = 5) -> int:
        out = np.zeros(1, np.int64)
        rc = lib().or_find_block_start(_p(self.d), self.D, start, blocks_to_check, _p(out))
        if rc != 0:
            raise RuntimeError(f"HeaderSearchFailedException: {start}")
        return int(out[0])

    def find_record_start(self, block_start: int, reads_to_check: int = 10, max_read_size: int = 10_000_000):
        """FindRecordStart.withDelta from Pos(block_start, 0); returns flat offset or None."""
        b = self.block_index_at_or_after(block_start)
        if b >= self.nblocks or int(self.start[b]) != block_start:
            return None  # EOF-marker block / past the stream: empty stream, None
        x0 = int(self.uoff[b])
        x = lib().or_find_record_start(_p(self.u), self.L, _p(self.lens), self.nref, x0, reads_to_check,
                                       max_read_size)
        return None if x < 0 else int(x)

    def record_chain(self, x0: int, x_end: int) -> np.ndarray:
        cap = max((x_end - x0) // 36 + 2, 2)
        out = np.zeros(cap, np.int64)
        n = lib().or_record_chain(_p(self.u), self.L, x0, x_end, _p(out), cap)
        return out[:n]

    def x_end_of(self, end_compressed: int) -> int:
        """Flat offset of Pos(end, 0): first block whose start >= end (records with Pos < (end,0))."""
        b = self.block_index_at_or_after(end_compressed)
        return int(self.uoff[b]) if b < self.nblocks else self.L


def hadoop_splits(size: int, split_size: int):
    """FileInputFormat.getSplits rule (SPLIT_SLOP = 1.1) as used via hammerlab FileSplits."""
    out, off, rem = [], 0, size
    while rem / split_size > 1.1:
        out.append((off, off + split_size))
        off += split_size
        rem -= split_size
    if rem > 0:
        out.append((off, size))
    return out


def load_reads_and_positions(f: BamFile, split_size: int, blocks_to_check=5, reads_to_check=10,
                             max_read_size=10_000_000):
    """Per Hadoop split: list of record flat offsets (CanLoadBam.scala:281-334)."""
    parts = []
    for (start, end) in hadoop_splits(f.D, split_size):
        bs = f.find_block_start(start, blocks_to_check)
        x = f.find_record_start(bs, reads_to_check, max_read_size)
        if x is None:
            raise RuntimeError(f"NoReadFoundException: {start}")
        parts.append(f.record_chain(x, f.x_end_of(end)))
    return parts


def compute_splits(f: BamFile, split_size: int, **kw):
    """loadSplitsAndReads splits (CanLoadBam.scala:245-279)."""
    parts = load_reads_and_positions(f, split_size, **kw)
    firsts = [f.pos_of(int(p[0])) for p in parts if len(p)]
    ends = firsts[1:] + [Pos(f.D, 0)]
    return list(zip(firsts, ends)), parts


def flags_of(word: int):
    return [FLAG_NAMES[i] for i in range(19) if word & (1 << i)]


def parse_blocks_file(path):
    rows = [tuple(int(v) for v in l.split(",")) for l in open(path) if l.strip()]
    return rows


def parse_records_file(path):
    return [Pos(*(int(v) for v in l.split(","))) for l in open(path) if l.strip()]

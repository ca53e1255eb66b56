"""sbam — host-side mirror of spark-bam's split/check/decode API over the MI355X C-ABI (libsbam.so).

Names, argument meaning and error behaviour follow the reference:

* ``Pos`` / ``Split``                         bgzf/.../Pos.scala:12-41, check/.../bam/spark/Split.scala:9-13
* ``BamFile.find_block_start``                bgzf/.../block/FindBlockStart.scala:8-36
* ``BamFile.find_record_start``               check/.../bam/spark/FindRecordStart.scala:11-63
* ``BamFile.eager_checker`` / ``full_checker``  check/.../check/{eager,full}/Checker.scala (Checker[Call].apply)
* ``BamFile.load_splits_and_reads`` etc.      load/.../spark/load/CanLoadBam.scala:173-382
* exceptions ``HeaderParseException``, ``HeaderSearchFailedException``, ``NoReadFoundException``,
  ``InflateException`` carry the reference's message text.

Everything computes on the GPU through ``libsbam.so``; there is no CPU fallback: importing this module
without the built library raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SBAM_LIB", os.path.join(_HERE, "..", "build", "libsbam.so"))

SBAM_OK = 0
ERR_HEADER_PARSE, ERR_HEADER_SEARCH, ERR_INFLATE, ERR_NO_READ_FOUND, ERR_NOT_BAM, ERR_ARG, ERR_HIP, ERR_STATE, \
    ERR_HALO = range(1, 10)

FLAG_NAMES = [  # check/src/main/scala/org/hammerlab/bam/check/full/error/Flags.scala:201-223
    "tooFewFixedBlockBytes", "negativeReadIdx", "tooLargeReadIdx", "negativeReadPos", "tooLargeReadPos",
    "negativeNextReadIdx", "tooLargeNextReadIdx", "negativeNextReadPos", "tooLargeNextReadPos",
    "tooFewBytesForReadName", "nonNullTerminatedReadName", "nonASCIIReadName", "noReadName", "emptyReadName",
    "tooFewBytesForCigarOps", "invalidCigarOp", "emptyMappedCigar", "emptyMappedSeq",
    "tooFewRemainingBytesImplied",
]
WORD_SUCCESS = 0x80000000
WORD_HALO = 0x00800000

# Defaults (bgzf/.../block/package.scala:20-21, check/.../check/package.scala:17-18,28-29)
BGZF_BLOCKS_TO_CHECK = 5
READS_TO_CHECK = 10
MAX_READ_SIZE = 10_000_000
# Hadoop's local FileSystem block size (fs.local.block.size default): what a split size falls back to when
# -m/--max-split-size is unset (check/.../args/SplitSize.scala:10-17: "default to underlying FileSystem's value").
LOCAL_FS_BLOCK_SIZE = 32 << 20


def effective_split_size(max_split_size: Optional[int] = None, fs_block_size: int = LOCAL_FS_BLOCK_SIZE) -> int:
    """The split size Hadoop's FileInputFormat uses: computeSplitSize(blockSize, minSize=1, maxSize) =
    max(1, min(maxSize, blockSize)), with maxSize = the FS block size when -m is unset (SplitSize.scala:10-17).
    The FS-block cap comes from Hadoop, outside the reference tree: parity unpinned (no golden splits a file into
    pieces larger than 32 MiB)."""
    m = fs_block_size if max_split_size is None else int(max_split_size)
    return max(1, min(m, fs_block_size))


class SbamError(Exception):
    code = 0


class HeaderParseException(SbamError):
    code = ERR_HEADER_PARSE


class HeaderSearchFailedException(SbamError):
    code = ERR_HEADER_SEARCH


class InflateException(IOError, SbamError):
    code = ERR_INFLATE


class NoReadFoundException(SbamError):
    code = ERR_NO_READ_FOUND


class HaloException(SbamError):
    code = ERR_HALO


_EXC = {c.code: c for c in (HeaderParseException, HeaderSearchFailedException, InflateException,
                            NoReadFoundException, HaloException)}


class _Pos(ctypes.Structure):
    _fields_ = [("block_pos", ctypes.c_int64), ("offset", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class _Split(ctypes.Structure):
    _fields_ = [("start", _Pos), ("end", _Pos)]


class _Error(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("idx", ctypes.c_int32), ("actual", ctypes.c_int64),
                ("expected", ctypes.c_int64), ("position", ctypes.c_int64), ("message", ctypes.c_char * 512)]


class _Counts(ctypes.Structure):
    _fields_ = [("totals", ctypes.c_int64 * 19), ("counts", ctypes.c_int64 * (21 * 19)), ("positions", ctypes.c_int64 * 21),
                ("reads_before_error", ctypes.c_int64 * (21 * 128)), ("pair_hist", ctypes.c_int64 * (19 * 19)),
                ("n_positions", ctypes.c_int64), ("n_success", ctypes.c_int64),
                ("n_too_few_fixed", ctypes.c_int64), ("n_halo", ctypes.c_int64)]


class _SplitArgs(ctypes.Structure):
    _fields_ = [("split_size", ctypes.c_int64), ("bgzf_blocks_to_check", ctypes.c_int32),
                ("reads_to_check", ctypes.c_int32), ("max_read_size", ctypes.c_int32),
                ("use_success_bitmap", ctypes.c_int32)]


class _RecordColumns(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("offset", "block_pos", "block_off", "block_size", "ref_id", "pos",
                                               "bin_mq_nl", "flag_nc", "l_seq", "next_ref_id", "next_pos", "tlen")]


RECORD_COLUMNS = {"offset": np.int64, "block_pos": np.int64, "block_off": np.int32, "block_size": np.int32,
                  "ref_id": np.int32, "pos": np.int32, "bin_mq_nl": np.uint32, "flag_nc": np.uint32,
                  "l_seq": np.int32, "next_ref_id": np.int32, "next_pos": np.int32, "tlen": np.int32}


EXPORTS = [  # every symbol include/sbam.h declares
    "sbam_open", "sbam_close", "sbam_load", "sbam_reserve", "sbam_last_error", "sbam_set_path", "sbam_reset", "sbam_version", "sbam_find_block_starts", "sbam_scan_blocks",
    "sbam_get_blocks", "sbam_inflate", "sbam_inflate_fallbacks", "sbam_read_uncompressed", "sbam_pos_to_offset", "sbam_offset_to_pos",
    "sbam_header", "sbam_set_contig_lengths", "sbam_check_eager", "sbam_check_full_words", "sbam_check_full_counts",
    "sbam_find_record_start", "sbam_file_splits", "sbam_split_records", "sbam_compute_splits",
    "sbam_record_offsets", "sbam_record_spans", "sbam_load_records", "sbam_get_record_columns", "sbam_record_columns_device",
    "sbam_last_kernel_ms",
]

_lib = None


def source_digest() -> str:
    """Digest of the kernel and C-ABI sources libsbam.so is built from: ties committed profiles (PMC traffic) to
    the kernel build they were measured on."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(_HERE, "..", "csrc")
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".hip", ".cpp", ".h")):
            with open(os.path.join(csrc, name), "rb") as fh:
                h.update(name.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def load_library(path: str = LIB_PATH):
    """Load libsbam.so; raises (no fallback) when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"libsbam.so not built at {path}: run `make -C spark-bam_amd` (no CPU fallback exists)")
    L = ctypes.CDLL(os.path.abspath(path))
    vp, i64, i32, P = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER
    sig = {
        "sbam_open": (ctypes.c_int, [ctypes.c_int, vp, i64, i64, i64, P(vp)]),
        "sbam_close": (None, [vp]),
        "sbam_last_error": (P(_Error), [vp]),
        "sbam_set_path": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "sbam_reset": (ctypes.c_int, [vp]),
        "sbam_version": (ctypes.c_char_p, []),
        "sbam_find_block_starts": (ctypes.c_int, [vp, vp, i64, i32, vp]),
        "sbam_scan_blocks": (ctypes.c_int, [vp, P(i64)]),
        "sbam_get_blocks": (ctypes.c_int, [vp, vp, vp, vp, vp, i64]),
        "sbam_inflate": (ctypes.c_int, [vp, P(i64)]),
        "sbam_inflate_fallbacks": (ctypes.c_int, [vp, P(i64)]),
        "sbam_read_uncompressed": (ctypes.c_int, [vp, i64, i64, vp]),
        "sbam_pos_to_offset": (ctypes.c_int, [vp, _Pos, P(i64)]),
        "sbam_offset_to_pos": (ctypes.c_int, [vp, i64, P(_Pos)]),
        "sbam_header": (ctypes.c_int, [vp, P(i32), vp, i32, P(_Pos)]),
        "sbam_set_contig_lengths": (ctypes.c_int, [vp, i32, vp]),
        "sbam_check_eager": (ctypes.c_int, [vp, i64, i64, i32, vp]),
        "sbam_check_full_words": (ctypes.c_int, [vp, i64, i64, i32, vp]),
        "sbam_check_full_counts": (ctypes.c_int, [vp, i64, i64, i32, i32, P(_Counts), vp]),
        "sbam_find_record_start": (ctypes.c_int, [vp, i64, i32, i32, P(i32), P(_Pos), P(i32)]),
        "sbam_file_splits": (ctypes.c_int, [i64, i64, vp, vp, i64, P(i64)]),
        "sbam_split_records": (ctypes.c_int, [vp, P(_SplitArgs), i64, i64, vp, vp, vp]),
        "sbam_compute_splits": (ctypes.c_int, [vp, P(_SplitArgs), vp, i64, P(i64)]),
        "sbam_record_offsets": (ctypes.c_int, [vp, i64, i64, vp, i64, P(i64)]),
        "sbam_load": (ctypes.c_int, [vp, vp, i64, i64, i64]),
        "sbam_reserve": (ctypes.c_int, [vp, i64, i64, i64, i64]),
        "sbam_record_spans": (ctypes.c_int, [vp, vp, i64, vp, vp, vp]),
        "sbam_load_records": (ctypes.c_int, [vp, P(_SplitArgs), i64, i64, vp, P(i64)]),
        "sbam_get_record_columns": (ctypes.c_int, [vp, i64, i64, P(_RecordColumns)]),
        "sbam_record_columns_device": (ctypes.c_int, [vp, P(_RecordColumns), P(i64)]),
        "sbam_last_kernel_ms": (ctypes.c_double, [vp, ctypes.c_char_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


@dataclass(frozen=True, order=True)
class Pos:
    """Virtual position (bgzf/src/main/scala/org/hammerlab/bgzf/Pos.scala:12-41)."""
    block_pos: int
    offset: int

    def __str__(self):
        return f"{self.block_pos}:{self.offset}"

    def to_htsjdk(self) -> int:
        return (self.block_pos << 16) | self.offset

    @staticmethod
    def from_htsjdk(v: int) -> "Pos":
        return Pos(v >> 16, v & 0xFFFF)

    def minus(self, other: "Pos", ratio: float = 3.0) -> float:
        """Pos.- with EstimatedCompressionRatio (Pos.scala:17-22)."""
        return float(max(0, self.block_pos - other.block_pos + int((self.offset - other.offset) / ratio)))


@dataclass(frozen=True)
class Split:
    """check/src/main/scala/org/hammerlab/bam/spark/Split.scala:9-13."""
    start: Pos
    end: Pos

    def length(self, ratio: float = 3.0) -> float:
        return self.end.minus(self.start, ratio)

    def __str__(self):
        return f"{self.start}-{self.end}"


def _pos(p: _Pos) -> Pos:
    return Pos(int(p.block_pos), int(p.offset))


@dataclass
class Counts:
    """full-check reductions (check/.../full/error/Counts.scala; FullCheck.scala:141-191)."""
    totals: np.ndarray  # [19] per flag over every counted position ("Total error counts")
    by_key: np.ndarray  # [21, 19]: keys 1-2 always; every key when computed with by_key=True
    positions: np.ndarray  # [21]
    reads_before_error: np.ndarray  # [21, 128]
    pair_hist: np.ndarray  # [19, 19]
    n_positions: int
    n_success: int
    n_too_few_fixed: int

    def total_error_counts(self) -> dict:
        t = self.totals
        return {FLAG_NAMES[i]: int(t[i]) for i in range(19)}


def n_hadoop_splits(file_size: int, split_size: int) -> int:
    """len(hadoop_splits(...)) without building the list (a 10 GB file has ~5000 splits)."""
    n = ctypes.c_int64(0)
    load_library().sbam_file_splits(file_size, split_size, None, None, 0, ctypes.byref(n))
    return int(n.value)


def hadoop_splits(file_size: int, split_size: int):
    """FileInputFormat split rule (through libsbam.sbam_file_splits)."""
    L = load_library()
    n = ctypes.c_int64(0)
    L.sbam_file_splits(file_size, split_size, None, None, 0, ctypes.byref(n))
    s = np.zeros(n.value, np.int64)
    e = np.zeros(n.value, np.int64)
    L.sbam_file_splits(file_size, split_size, _ptr(s), _ptr(e), n.value, ctypes.byref(n))
    return list(zip(s.tolist(), e.tolist()))


class BamFile:
    """One BAM file (or a shard of one) resident on one GPU — the per-task channel of the reference
    (load/.../spark/load/Channels.scala:15-26) with the hot path behind it."""

    def __init__(self, data, device: int = 0, base_offset: int = 0, file_size: Optional[int] = None,
                 path: str = "<bytes>", inflate: bool = True, contig_lengths: Optional[Sequence[int]] = None):
        self.L = load_library()
        buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        self._buf = np.ascontiguousarray(buf)
        self.path = path
        self.base_offset = base_offset
        self.file_size = int(file_size if file_size is not None else base_offset + self._buf.size)
        self.ctx = ctypes.c_void_p()
        rc = self.L.sbam_open(device, _ptr(self._buf), self._buf.size, base_offset, self.file_size,
                              ctypes.byref(self.ctx))
        self._check(rc)
        self._check(self.L.sbam_set_path(self.ctx, str(path).encode()))
        self.n_blocks = self._scan()
        self.uncompressed_size = None
        self.n_ref = None
        self.contig_lengths = None
        self.header_end = None
        if inflate:
            self.inflate()
            if contig_lengths is not None:
                self.set_contig_lengths(contig_lengths)
            elif base_offset == 0:
                self.header()

    # ---- plumbing
    def _check(self, rc):
        if rc == SBAM_OK:
            return
        e = self.L.sbam_last_error(self.ctx).contents if self.ctx else None
        msg = e.message.decode() if e else f"sbam error {rc}"
        raise _EXC.get(rc, SbamError)(msg)

    def close(self):
        if self.ctx:
            self.L.sbam_close(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, data, base_offset: int = 0, file_size: Optional[int] = None):
        """sbam_load: make another byte range resident in this context (allocations kept, stages dropped).
        `data` (numpy uint8, possibly a view of pinned host memory) must stay alive while loading."""
        buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        self._buf = np.ascontiguousarray(buf)
        file_size = int(file_size if file_size is not None else base_offset + self._buf.size)
        # the context drops its contig lengths when the range may hold a different header (sbam_load)
        drop = base_offset == 0 or file_size != self.file_size
        self.base_offset = base_offset
        self.file_size = file_size
        self._check(self.L.sbam_load(self.ctx, _ptr(self._buf), self._buf.size, base_offset, self.file_size))
        if drop:
            self.n_ref = self.contig_lengths = self.header_end = None
        self.n_blocks = None
        self.uncompressed_size = None

    def reserve(self, comp_bytes: int, n_blocks: int, ubytes: int, n_records: int = 0):
        """sbam_reserve: size the device buffers for windows up to these sizes, so no later load reallocates.  A
        buffer that grows drops the context's stages (their device data is gone); an inflated stream this object
        had is then inflated again from the resident bytes (a dropped block scan needs nothing here: the library
        re-runs it on its next use, ensure_blocks)."""
        had_stream = self.uncompressed_size is not None
        self._check(self.L.sbam_reserve(self.ctx, int(comp_bytes), int(n_blocks), int(ubytes), int(n_records)))
        if had_stream and self.L.sbam_read_uncompressed(self.ctx, 0, 0, None) == ERR_STATE:
            self.n_blocks = self._scan()
            self.inflate()

    @property
    def loads_to_eof(self) -> bool:
        """Whether the resident bytes reach the end of the file (else a scan past them is a halo miss)."""
        return self.base_offset + self._buf.size >= self.file_size

    def reset(self):
        """Drop derived stages (keeps the resident compressed bytes and allocations)."""
        self._check(self.L.sbam_reset(self.ctx))
        self.n_blocks = None
        self.uncompressed_size = None

    def run(self, contig_lengths: Optional[Sequence[int]] = None):
        """Scan → inflate → header/contig lengths from the resident compressed bytes."""
        self.n_blocks = self._scan()
        self.inflate()
        if contig_lengths is not None:
            self.set_contig_lengths(contig_lengths)
        elif self.base_offset == 0:
            self.header()

    def kernel_ms(self, name: str) -> float:
        return float(self.L.sbam_last_kernel_ms(self.ctx, name.encode()))

    # ---- BGZF
    def _scan(self) -> int:
        n = ctypes.c_int64(0)
        self._check(self.L.sbam_scan_blocks(self.ctx, ctypes.byref(n)))
        return n.value

    def blocks(self):
        """(start, compressedSize, uncompressedSize, uncompressedOffset) arrays (IndexBlocks.scala:40-44)."""
        n = self.n_blocks
        st, cs, us, uo = (np.zeros(n, np.int64), np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int64))
        self._check(self.L.sbam_get_blocks(self.ctx, _ptr(st), _ptr(cs), _ptr(us), _ptr(uo), n))
        return st, cs, us, uo

    def find_block_starts(self, starts: Sequence[int], bgzf_blocks_to_check: int = BGZF_BLOCKS_TO_CHECK):
        q = np.asarray(starts, np.int64)
        out = np.zeros(q.size, np.int64)
        self._check(self.L.sbam_find_block_starts(self.ctx, _ptr(q), q.size, bgzf_blocks_to_check, _ptr(out)))
        return out

    def find_block_start(self, start: int, bgzf_blocks_to_check: int = BGZF_BLOCKS_TO_CHECK) -> int:
        """FindBlockStart.apply (FindBlockStart.scala:8-36)."""
        return int(self.find_block_starts([start], bgzf_blocks_to_check)[0])

    def inflate(self) -> int:
        n = ctypes.c_int64(0)
        self._check(self.L.sbam_inflate(self.ctx, ctypes.byref(n)))
        self.uncompressed_size = n.value
        return n.value

    def inflate_fallbacks(self) -> int:
        """Blocks the last inflate decoded on the exact per-lane path instead of the wave-parallel one."""
        n = ctypes.c_int64(0)
        self._check(self.L.sbam_inflate_fallbacks(self.ctx, ctypes.byref(n)))
        return n.value

    def read_uncompressed(self, off: int, length: int) -> bytes:
        out = np.zeros(length, np.uint8)
        self._check(self.L.sbam_read_uncompressed(self.ctx, off, length, _ptr(out)))
        return out.tobytes()

    def offset_of(self, pos: Pos) -> int:
        o = ctypes.c_int64(0)
        self._check(self.L.sbam_pos_to_offset(self.ctx, _Pos(pos.block_pos, pos.offset, 0), ctypes.byref(o)))
        return o.value

    def pos_of(self, off: int) -> Pos:
        p = _Pos()
        self._check(self.L.sbam_offset_to_pos(self.ctx, off, ctypes.byref(p)))
        return _pos(p)

    # ---- header
    def header(self):
        n = ctypes.c_int32(0)
        lens = np.zeros(1 << 16, np.int64)
        end = _Pos()
        self._check(self.L.sbam_header(self.ctx, ctypes.byref(n), _ptr(lens), lens.size, ctypes.byref(end)))
        self.n_ref = n.value
        self.contig_lengths = lens[: n.value].copy()
        self.header_end = _pos(end)
        return self.n_ref, self.contig_lengths, self.header_end

    def set_contig_lengths(self, lens: Sequence[int]):
        a = np.asarray(lens, np.int64)
        self._check(self.L.sbam_set_contig_lengths(self.ctx, a.size, _ptr(a)))
        self.n_ref, self.contig_lengths = int(a.size), a.copy()

    # ---- checkers
    def check_eager(self, x0: int = 0, x1: Optional[int] = None, reads_to_check: int = READS_TO_CHECK) -> np.ndarray:
        """eager.Checker at every offset of [x0, x1) → bool array."""
        x1 = self.uncompressed_size if x1 is None else x1
        words = np.zeros((x1 - x0 + 63) // 64 + 1, np.uint64)
        self._check(self.L.sbam_check_eager(self.ctx, x0, x1, reads_to_check, _ptr(words)))
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        return bits[: x1 - x0].astype(bool)

    def check_eager_device(self, x0: int = 0, x1: Optional[int] = None,
                           reads_to_check: int = READS_TO_CHECK) -> None:
        """check_eager leaving the success bitmap on the device (the split computation reads it there)."""
        x1 = self.uncompressed_size if x1 is None else x1
        self._check(self.L.sbam_check_eager(self.ctx, x0, x1, reads_to_check, None))

    def check_full_words(self, x0: int = 0, x1: Optional[int] = None,
                         reads_to_check: int = READS_TO_CHECK) -> np.ndarray:
        """full.Checker result words (sbam.h layout) for every offset of [x0, x1)."""
        x1 = self.uncompressed_size if x1 is None else x1
        out = np.zeros(max(x1 - x0, 1), np.uint32)
        self._check(self.L.sbam_check_full_words(self.ctx, x0, x1, reads_to_check, _ptr(out)))
        return out[: x1 - x0]

    def check_full_counts(self, x0: int = 0, x1: Optional[int] = None, reads_to_check: int = READS_TO_CHECK,
                          want_bitmap: bool = False, by_key: bool = False):
        x1 = self.uncompressed_size if x1 is None else x1
        c = _Counts()
        bm = np.zeros((x1 - x0 + 63) // 64 + 1, np.uint64) if want_bitmap else None
        self._check(self.L.sbam_check_full_counts(self.ctx, x0, x1, reads_to_check, 1 if by_key else 0,
                                                  ctypes.byref(c), _ptr(bm)))
        counts = Counts(np.ctypeslib.as_array(c.totals).copy(),
                        np.ctypeslib.as_array(c.counts).reshape(21, 19).copy(),
                        np.ctypeslib.as_array(c.positions).copy(),
                        np.ctypeslib.as_array(c.reads_before_error).reshape(21, 128).copy(),
                        np.ctypeslib.as_array(c.pair_hist).reshape(19, 19).copy(),
                        int(c.n_positions), int(c.n_success), int(c.n_too_few_fixed))
        if want_bitmap:
            bits = np.unpackbits(bm.view(np.uint8), bitorder="little")[: x1 - x0].astype(bool)
            return counts, bits
        return counts

    def eager_checker(self, reads_to_check: int = READS_TO_CHECK):
        """Checker[Boolean] (check/.../check/Checker.scala:7-9) backed by a bulk GPU bitmap, the
        indexed.Checker precedent (check/.../check/indexed/Checker.scala:12-27)."""
        bits = self.check_eager(0, self.uncompressed_size, reads_to_check)
        return lambda pos: bool(bits[self.offset_of(pos)])

    def full_checker(self, reads_to_check: int = READS_TO_CHECK):
        words = self.check_full_words(0, self.uncompressed_size, reads_to_check)
        return lambda pos: int(words[self.offset_of(pos)])

    def find_record_start_with_delta(self, block_start: int, reads_to_check: int = READS_TO_CHECK,
                                     max_read_size: int = MAX_READ_SIZE):
        """FindRecordStart.withDelta from Pos(block_start, 0): (Pos, delta) or None."""
        found, p, d = ctypes.c_int32(0), _Pos(), ctypes.c_int32(0)
        self._check(self.L.sbam_find_record_start(self.ctx, block_start, reads_to_check, max_read_size,
                                                  ctypes.byref(found), ctypes.byref(p), ctypes.byref(d)))
        return (_pos(p), d.value) if found.value else None

    def find_record_start(self, block_start: int, reads_to_check: int = READS_TO_CHECK,
                          max_read_size: int = MAX_READ_SIZE) -> Pos:
        """FindRecordStart.apply: raises NoReadFoundException on None (FindRecordStart.scala:11-28)."""
        r = self.find_record_start_with_delta(block_start, reads_to_check, max_read_size)
        if r is None:
            raise NoReadFoundException(
                f"Failed to find a valid read-start in {max_read_size} attempts in {self.path} from {block_start}")
        return r[0]

    # ---- splits / records (CanLoadBam)
    def _args(self, split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, use_bitmap):
        return _SplitArgs(split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, 1 if use_bitmap else 0)

    def split_records(self, split_size: int, first: int = 0, count: Optional[int] = None,
                      bgzf_blocks_to_check: int = BGZF_BLOCKS_TO_CHECK, reads_to_check: int = READS_TO_CHECK,
                      max_read_size: int = MAX_READ_SIZE, use_success_bitmap: bool = False):
        """Per Hadoop split: (first record Pos, non-empty?, record count)."""
        bp, off, nonempty, n = self.split_records_arrays(split_size, first, count, bgzf_blocks_to_check,
                                                         reads_to_check, max_read_size, use_success_bitmap)
        return [(Pos(int(bp[i]), int(off[i])), bool(nonempty[i]), int(n[i])) for i in range(bp.size)]

    def split_records_arrays(self, split_size: int, first: int = 0, count: Optional[int] = None,
                             bgzf_blocks_to_check: int = BGZF_BLOCKS_TO_CHECK, reads_to_check: int = READS_TO_CHECK,
                             max_read_size: int = MAX_READ_SIZE, use_success_bitmap: bool = False):
        """split_records as arrays (first record block_pos, offset, non-empty, record count): no per-split
        Python objects (a 10 GB file has ~5000 splits)."""
        ns = n_hadoop_splits(self.file_size, split_size)
        count = ns - first if count is None else count
        fp = np.zeros(max(count, 1), dtype=[("block_pos", "<i8"), ("offset", "<i4"), ("reserved", "<i4")])
        fd = np.zeros(max(count, 1), np.int32)
        nr = np.zeros(max(count, 1), np.int64)
        a = self._args(split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, use_success_bitmap)
        self._check(self.L.sbam_split_records(self.ctx, ctypes.byref(a), first, count, fp.ctypes.data,
                                              _ptr(fd), _ptr(nr)))
        return (fp["block_pos"][:count].copy(), fp["offset"][:count].astype(np.int64), fd[:count] != 0,
                nr[:count].copy())

    def partition_sizes(self, split_size: int, **kw) -> List[int]:
        """records.partitionSizes of sc.loadReads / loadBam (LoadBAMTest.scala:24-45)."""
        return [n for (_, _, n) in self.split_records(split_size, **kw)]

    def compute_splits(self, split_size: int, bgzf_blocks_to_check: int = BGZF_BLOCKS_TO_CHECK,
                       reads_to_check: int = READS_TO_CHECK, max_read_size: int = MAX_READ_SIZE,
                       use_success_bitmap: bool = False) -> List[Split]:
        """loadSplitsAndReads(...).splits (CanLoadBam.scala:245-279)."""
        a = self._args(split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, use_success_bitmap)
        cap = n_hadoop_splits(self.file_size, split_size) + 1
        out = (_Split * cap)()
        n = ctypes.c_int64(0)
        self._check(self.L.sbam_compute_splits(self.ctx, ctypes.byref(a), ctypes.addressof(out), cap,
                                               ctypes.byref(n)))
        return [Split(_pos(out[i].start), _pos(out[i].end)) for i in range(n.value)]

    def record_offsets(self, x0: int, x_end: int) -> np.ndarray:
        cap = max((x_end - x0) // 36 + 2, 2)
        out = np.zeros(cap, np.int64)
        n = ctypes.c_int64(0)
        self._check(self.L.sbam_record_offsets(self.ctx, x0, x_end, _ptr(out), cap, ctypes.byref(n)))
        return out[: n.value]

    def load_records(self, split_size: int, first: int = 0, count: Optional[int] = None,
                     bgzf_blocks_to_check: int = BGZF_BLOCKS_TO_CHECK, reads_to_check: int = READS_TO_CHECK,
                     max_read_size: int = MAX_READ_SIZE, use_success_bitmap: bool = False,
                     columns: Optional[Sequence[str]] = tuple(RECORD_COLUMNS)):
        """Records of Hadoop splits [first, first+count) decoded on the GPU (sbam_load_records): returns
        (partition sizes, {column: ndarray}) with the records of all those splits concatenated in split order.
        `columns=None` leaves the columns on the device (count only)."""
        ns = n_hadoop_splits(self.file_size, split_size)
        count = ns - first if count is None else count
        sizes = np.zeros(max(count, 1), np.int64)
        n = ctypes.c_int64(0)
        a = self._args(split_size, bgzf_blocks_to_check, reads_to_check, max_read_size, use_success_bitmap)
        self._check(self.L.sbam_load_records(self.ctx, ctypes.byref(a), first, count, _ptr(sizes), ctypes.byref(n)))
        sizes = sizes[:count]
        if columns is None:
            return sizes, {}
        cols = {k: np.zeros(n.value, RECORD_COLUMNS[k]) for k in columns}
        rc = _RecordColumns(**{k: v.ctypes.data for k, v in cols.items()})
        self._check(self.L.sbam_get_record_columns(self.ctx, 0, n.value, ctypes.byref(rc)))
        return sizes, cols

    def record_spans(self, offsets: np.ndarray):
        """(ref_id, start, end) of the records at `offsets`: [getStart - 1, getEnd) as CanLoadBam.region uses it
        (unmapped: end 0)."""
        offs = np.ascontiguousarray(offsets, np.int64)
        n = offs.size
        r, a, b = (np.zeros(n, np.int32) for _ in range(3))
        self._check(self.L.sbam_record_spans(self.ctx, _ptr(offs), n, _ptr(r), _ptr(a), _ptr(b)))
        return r, a, b

    def _vpos_offset(self, v: int) -> int:
        """Stream offset of an htsjdk virtual offset (block << 16 | offset); a block at or past the end of the
        stream (the EOF marker) maps to the stream end."""
        st, _, us, uo = self.blocks()
        b, o = v >> 16, v & 0xffff
        i = int(np.searchsorted(st, b))
        if i < st.size and int(st[i]) == b:
            return int(uo[i]) + min(o, int(us[i]))
        if i >= st.size:
            return self.uncompressed_size
        raise SbamError(f"no BGZF block at {b}")

    def load_bam_intervals(self, bai: bytes, loci: str, split_size: int = 32 << 20, ratio: float = 3.0):
        """sc.loadBamIntervals (CanLoadBam.scala:59-138): the BAI chunks overlapping `loci` (htsjdk getFileSpan,
        sbam.bai), grouped into partitions by estimated size (cappedCostGroups), and per chunk the records from
        chunk.start while Pos < chunk.end whose [getStart - 1, getEnd) intersects the loci.  Record chains and
        reference spans run on the GPU (sbam_record_offsets, sbam_record_spans).  Returns (chunks, partitions):
        partitions = per partition, the record stream offsets kept, in file order.  (The MaxSplitSize default of
        32 MiB is hammerlab's, outside the reference tree: parity unpinned.)"""
        from sbam import bai as B
        from sbam.cli import header_names
        refs = B.parse_bai(bai)
        names = header_names(self)
        q = []
        for contig, a, e in B.parse_loci(loci):
            ri = names.index(contig) if contig in names else -1
            q.append((ri, a + 1, e if e is not None else 0))  # toHtsJDKIntervals: 1-based closed
        chunks = B.file_span(refs, q)
        groups = B.capped_cost_groups([c.size(ratio) for c in chunks], float(split_size))
        want = [(names.index(c) if c in names else -2, a, e) for c, a, e in B.parse_loci(loci)]
        parts = []
        for g in groups:
            kept = []
            for ci in g:
                c = chunks[ci]
                offs = self.record_offsets(self._vpos_offset(c.start), self._vpos_offset(c.end))
                if offs.size == 0:
                    continue
                ri, st, en = self.record_spans(offs)
                m = np.zeros(offs.size, bool)
                for r, a, e in want:
                    m |= (ri == r) & (st < (e if e is not None else 1 << 31)) & (en > a)
                kept.append(offs[m])
            parts.append(np.concatenate(kept) if kept else np.zeros(0, np.int64))
        return chunks, parts

    def load_reads_and_positions(self, split_size: int, **kw):
        """loadReadsAndPositions: per partition, list of (Pos, record bytes) (CanLoadBam.scala:281-334).  Record
        offsets and Pos come from sbam_load_records; each partition's bytes are one contiguous stream slice."""
        sizes, c = self.load_records(split_size, columns=("offset", "block_pos", "block_off", "block_size"), **kw)
        parts, i = [], 0
        for n in sizes.tolist():
            recs = []
            if n:
                off, bs = c["offset"][i:i + n], c["block_size"][i:i + n]
                x0, x1 = int(off[0]), int(off[-1]) + 4 + int(bs[-1])
                raw = self.read_uncompressed(x0, x1 - x0)
                for j in range(n):
                    o = int(off[j]) - x0
                    recs.append((Pos(int(c["block_pos"][i + j]), int(c["block_off"][i + j])), raw[o:o + 4 + int(bs[j])]))
            parts.append(recs)
            i += n
        return parts

    def load_reads(self, split_size: int, **kw):
        """sc.loadReads (CanLoadBam.scala:348-352): per partition, list of record bytes."""
        return [[r for (_, r) in p] for p in self.load_reads_and_positions(split_size, **kw)]


def read_name(record: bytes) -> str:
    """read_name field of a BAM record (bytes starting at block_size)."""
    lrn = record[12]
    return record[36:36 + lrn - 1].decode()

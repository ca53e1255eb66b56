"""Drop-in `MakeChecker` shape over the GPU path (check/src/main/scala/org/hammerlab/bam/check/Checker.scala:7-25).

The reference builds one checker per partition from the channel alone (`MakeChecker[Call, C] extends
(CachingChannel[SeekableByteChannel] ⇒ C)`, built before the partition's blocks are iterated:
cli/src/main/scala/org/hammerlab/bam/check/CallPartition.scala:35-37) and then calls `apply(pos)` at every
position of its blocks (PosIterator).  `LazyBlockChecker` keeps exactly that contract: construction takes the byte
source (the channel) and nothing about the partition; the first `apply(pos)` in a block the cache does not cover makes
ONE bulk GPU call over that block and the blocks after it (a window of compressed bytes), and caches their calls; every
later `apply` in those blocks is a bit (or word) lookup — the shape of the reference's own bulk-precomputed
`indexed.Checker` (check/.../check/indexed/Checker.scala:12-27).  A window whose checked chains run past its bytes
(HALO: long records) doubles and retries.  INTEGRATION.md shows the same class on the JVM (Panama).

The eager kind is also the reference's `ReadStartFinder` (check/.../check/ReadStartFinder.scala:5-11; eager.Checker
mixes it in, eager/Checker.scala:18-22, 128-162): `next_read_start(pos)` walks the uncompressed positions from `pos`
over the cached calls, block after block (filling windows as it goes), for at most `max_read_size` positions — what
check-blocks' `callPartition` asks of both of its checkers (cli/.../check/blocks/CheckBlocks.scala:37-56).
`IndexedChecker` is the other side of that comparison: indexed.Checker over a `.records` set."""
from __future__ import annotations

from collections import OrderedDict
import bisect
from typing import Callable, Dict, Iterable, Optional, Sequence, Tuple

import numpy as np

import sbam


class NoDataBlock(sbam.SbamError):
    """The block chain has no block with data at a position: the EOF marker, an empty block (MetadataStream stops
    there) or a position that is not a block start."""


class LazyBlockChecker:
    """eager.Checker (`kind="eager"`: apply → bool, eager/Checker.scala:24-126) or full.Checker (`kind="full"`: apply →
    the sbam.h result word, full/Checker.scala:22-184), computed a window of blocks at a time on first use.

    One device context serves every window (opened on the first miss, refilled by sbam_load afterwards: no stream
    creation, allocation or free per window), and only the calls of the last `keep` windows stay cached: a
    partition's positions arrive in file order (PosIterator over its blocks), so older windows are not asked again —
    and a revisited one is simply recomputed."""

    def __init__(self, source: Callable[[int, int], np.ndarray], file_size: int, contig_lengths: Sequence[int],
                 reads_to_check: int = sbam.READS_TO_CHECK, window: int = 4 << 20, device: int = 0,
                 kind: str = "eager", keep: int = 2):
        assert kind in ("eager", "full") and keep >= 1
        self.source, self.file_size = source, int(file_size)
        self.contig_lengths = np.asarray(contig_lengths, np.int64)
        self.R, self.window, self.device, self.kind, self.keep = reads_to_check, int(window), device, kind, keep
        self.windows: "OrderedDict[int, Dict[int, np.ndarray]]" = OrderedDict()  # window start → {block start → calls}
        self.cache: Dict[int, np.ndarray] = {}  # block start → calls at offsets 0 .. usize-1 (the kept windows)
        self.next_block: Dict[int, int] = {}     # block start → the next block's start (start + compressed size)
        self.bulk_calls = 0                      # GPU windows computed (one per cache miss, plus HALO retries)
        self.f: Optional[sbam.BamFile] = None

    def _load(self, lo: int, hi: int):
        data = self.source(lo, hi)
        if self.f is None:
            self.f = sbam.BamFile(data, device=self.device, base_offset=lo, file_size=self.file_size, inflate=False)
        else:
            self.f.load(data, base_offset=lo, file_size=self.file_size)
        return self.f

    def _fill(self, block_pos: int):
        win = self.window
        while True:
            lo, hi = block_pos, min(self.file_size, block_pos + win)
            self.bulk_calls += 1
            f = self._load(lo, hi)
            f.run(contig_lengths=self.contig_lengths)
            st, cs, us, uo = f.blocks()
            if st.size == 0 or int(st[0]) != block_pos:
                raise NoDataBlock(f"no BGZF block starts at {block_pos}")
            # the blocks of the first half of the window (all of them when it reaches EOF): the second half is the
            # halo their chains read
            end = hi if f.loads_to_eof else lo + (hi - lo) // 2
            nb = max(1, int(np.searchsorted(st + cs, end, side="right")))
            x1 = int(uo[nb - 1]) + int(us[nb - 1])
            try:
                calls = (f.check_eager(0, x1, self.R) if self.kind == "eager" else
                         f.check_full_words(0, x1, self.R))
            except sbam.HaloException:
                if hi >= self.file_size:
                    raise
                win *= 2
                continue
            blocks = {int(st[b]): calls[int(uo[b]): int(uo[b]) + int(us[b])] for b in range(nb)}
            self.windows[lo] = blocks
            while len(self.windows) > self.keep:
                for k in self.windows.popitem(last=False)[1]:
                    self.cache.pop(k, None)
                    self.next_block.pop(k, None)
            self.cache.update(blocks)
            self.next_block.update({int(st[b]): int(st[b]) + int(cs[b]) for b in range(nb)})
            return

    def apply(self, pos: sbam.Pos):
        calls = self.cache.get(pos.block_pos)
        if calls is None:
            self._fill(pos.block_pos)
            calls = self.cache[pos.block_pos]
        v = calls[pos.offset]
        return bool(v) if self.kind == "eager" else int(v)

    __call__ = apply

    def _calls(self, block_pos: int, first: bool) -> Optional[np.ndarray]:
        """The calls of the block at block_pos; None when the block chain (followed from an earlier block) has no
        further block with data there: the EOF marker, an empty block or the file's end (MetadataStream stops)."""
        calls = self.cache.get(block_pos)
        if calls is None:
            if not first and block_pos >= self.file_size:
                return None
            try:
                self._fill(block_pos)
            except NoDataBlock:  # (only this: a HIP, inflate or halo error on a later window still raises)
                if first:
                    raise
                return None
            calls = self.cache[block_pos]
        return calls

    def next_read_start_with_delta(self, start: sbam.Pos,
                                   max_read_size: int = sbam.MAX_READ_SIZE) -> Optional[Tuple[sbam.Pos, int]]:
        """eager.Checker.nextReadStartWithDelta (eager/Checker.scala:133-162): the first position at or after `start`
        whose call is true, with the number of positions passed over; None after `max_read_size` positions, or when
        the uncompressed stream ends (the end of the file, or an empty block: MetadataStream stops there)."""
        if self.kind != "eager":
            raise TypeError("ReadStartFinder is eager.Checker's (full.Checker has no nextReadStart)")
        bp, off, idx = int(start.block_pos), int(start.offset), 0
        while idx < max_read_size:
            if bp >= self.file_size:
                return None
            calls = self._calls(bp, first=idx == 0 and bp == int(start.block_pos))
            if calls is None or calls.size == 0:
                return None
            n = int(calls.size)
            if off >= n:  # Pos(block, usize) is the next block's start (UncompressedBytes' curPos)
                off -= n
                bp = self.next_block[bp]
                continue
            seg = calls[off: off + min(n - off, max_read_size - idx)]
            hit = np.flatnonzero(seg)
            if hit.size:
                return sbam.Pos(bp, off + int(hit[0])), idx + int(hit[0])
            idx += seg.size
            off = n
        return None

    def next_read_start(self, start: sbam.Pos, max_read_size: int = sbam.MAX_READ_SIZE) -> Optional[sbam.Pos]:
        """ReadStartFinder.nextReadStart (ReadStartFinder.scala:5-11; eager/Checker.scala:127-131)."""
        r = self.next_read_start_with_delta(start, max_read_size)
        return None if r is None else r[0]

    nextReadStart = next_read_start

    def close(self):
        """The partition is done (CallPartition's .finish(close)): release the device context."""
        if self.f is not None:
            self.f.close()
            self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class IndexedChecker:
    """indexed.Checker (check/src/main/scala/org/hammerlab/bam/check/indexed/Checker.scala:12-27): the calls of a
    known set of record starts (a `.records` sidecar) — apply(pos) is membership, nextReadStart the first member at or
    after `pos`.  It is the truth side of check-blocks' comparison (CheckBlocks.scala:80-91)."""

    def __init__(self, read_positions: Iterable[sbam.Pos]):
        self.positions = sorted(set(read_positions))
        self._set = set(self.positions)

    @classmethod
    def from_records_file(cls, path: str) -> "IndexedChecker":
        """A `.records` sidecar: one `blockPos,offset` line per record (IndexRecords.scala:36-90)."""
        out = []
        for ln in open(path):
            if ln.strip():
                b, o = ln.split(",")
                out.append(sbam.Pos(int(b), int(o)))
        return cls(out)

    def apply(self, pos: sbam.Pos) -> bool:
        return pos in self._set

    __call__ = apply

    def next_read_start(self, start: sbam.Pos, max_read_size: int = sbam.MAX_READ_SIZE) -> Optional[sbam.Pos]:
        i = bisect.bisect_left(self.positions, start)
        return self.positions[i] if i < len(self.positions) else None

    nextReadStart = next_read_start


def make_checker(contig_lengths: Sequence[int], reads_to_check: int = sbam.READS_TO_CHECK, kind: str = "eager",
                 window: int = 4 << 20, device: int = 0):
    """`MakeChecker`: channel → Checker.  `channel` = (source(lo, hi) → bytes, file size), e.g. sbam.dist.file_source."""
    def make(channel) -> LazyBlockChecker:
        source, size = channel
        return LazyBlockChecker(source, size, contig_lengths, reads_to_check, window, device, kind)
    return make

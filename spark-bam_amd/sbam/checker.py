"""Drop-in `MakeChecker` shape over the GPU path (check/src/main/scala/org/hammerlab/bam/check/Checker.scala:7-25).

The reference builds one checker per partition from the channel alone (`MakeChecker[Call, C] extends
(CachingChannel[SeekableByteChannel] ⇒ C)`, built before the partition's blocks are iterated:
cli/src/main/scala/org/hammerlab/bam/check/CallPartition.scala:35-37) and then calls `apply(pos)` at every
position of its blocks (PosIterator).  `LazyBlockChecker` keeps exactly that contract: construction takes the byte
source (the channel) and nothing about the partition; the first `apply(pos)` in a block the cache does not cover makes
ONE bulk GPU call over that block and the blocks after it (a window of compressed bytes), and caches their calls; every
later `apply` in those blocks is a bit (or word) lookup — the shape of the reference's own bulk-precomputed
`indexed.Checker` (check/.../check/indexed/Checker.scala:12-27).  A window whose checked chains run past its bytes
(HALO: long records) doubles and retries.  INTEGRATION.md shows the same class on the JVM (Panama)."""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable, Dict, Optional, Sequence

import numpy as np

import sbam


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
                raise sbam.SbamError(f"no BGZF block starts at {block_pos}")
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
            self.cache.update(blocks)
            return

    def apply(self, pos: sbam.Pos):
        calls = self.cache.get(pos.block_pos)
        if calls is None:
            self._fill(pos.block_pos)
            calls = self.cache[pos.block_pos]
        v = calls[pos.offset]
        return bool(v) if self.kind == "eager" else int(v)

    __call__ = apply

    def close(self):
        """The partition is done (CallPartition's .finish(close)): release the device context."""
        if self.f is not None:
            self.f.close()
            self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def make_checker(contig_lengths: Sequence[int], reads_to_check: int = sbam.READS_TO_CHECK, kind: str = "eager",
                 window: int = 4 << 20, device: int = 0):
    """`MakeChecker`: channel → Checker.  `channel` = (source(lo, hi) → bytes, file size), e.g. sbam.dist.file_source."""
    def make(channel) -> LazyBlockChecker:
        source, size = channel
        return LazyBlockChecker(source, size, contig_lengths, reads_to_check, window, device, kind)
    return make

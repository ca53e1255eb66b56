"""BAI index and the interval query of `loadBamIntervals`.

Reference: `CanLoadBam.loadBamIntervals` (load/src/main/scala/org/hammerlab/bam/spark/load/CanLoadBam.scala:59-138)
asks htsjdk for the file span of the query intervals (`getIntevalChunks`, :387-421 →
`BAMFileReader.getFileSpan`), groups the chunks into partitions by estimated size (`cappedCostGroups`, :84-92),
and streams each chunk's records from `chunk.start` while `Pos < chunk.end`, keeping those whose
`[getStart - 1, getEnd)` region intersects the intervals (:107-135, `region` :423-431).

The htsjdk pieces restated here (htsjdk ~2.9, a third-party dependency absent from /root/reference):
  * BAI layout (SAM spec §5.2; also the reference's own reader, check/.../bam/index/Index.scala:60-90):
    "BAI\\1", n_ref, then per reference n_bin × (bin u32, n_chunk, n_chunk × (beg u64, end u64)), n_intv ×
    ioffset u64; bin 37450 is the metadata pseudo-bin;
  * GenomicIndexUtil.regionToBins(start, end) over 1-based closed coordinates (0 / negative = open);
  * LinearIndex.getMinimumOffset(start): the 16 kb window of start - 1;
  * Chunk.optimizeChunkList(chunks, minOffset): sort; drop chunks ending at or before minOffset; coalesce a
    chunk into the previous one when they overlap (block address, then in-block offset) or are adjacent
    (one's end == the other's start);
  * BAMFileSpan.merge over the intervals' spans: optimizeChunkList(all chunks, 0).
Pinned by LoadBAMTest "indexed all" / "indexed disjoint regions" (chunk lists and record counts for 2.bam);
other shapes (several references, empty bins) follow the same rules but are parity unpinned."""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

METADATA_BIN = 37450
LIDX_SHIFT = 14


@dataclass(frozen=True, order=True)
class Chunk:
    """Index.Chunk (check/.../bam/index/Index.scala:53-57): virtual offsets [start, end)."""
    start: int  # htsjdk virtual offset: block address << 16 | in-block offset
    end: int

    @staticmethod
    def block(v: int) -> int:
        return v >> 16

    @staticmethod
    def off(v: int) -> int:
        return v & 0xffff

    def overlaps(self, other: "Chunk") -> bool:
        if self == other:
            return True
        left, right = (self, other) if self < other else (other, self)
        lb, rb = Chunk.block(left.end), Chunk.block(right.start)
        if lb != rb:
            return lb > rb
        return Chunk.off(left.end) > Chunk.off(right.start)

    def adjacent(self, other: "Chunk") -> bool:
        return self.end == other.start or self.start == other.end

    def size(self, ratio: float = 3.0) -> float:
        """Chunk.size = end - start as Pos (bgzf/.../Pos.scala:17-22): Δblock + Δoffset / ratio."""
        return (Chunk.block(self.end) - Chunk.block(self.start)) + (Chunk.off(self.end) - Chunk.off(self.start)) / ratio

    def pos_str(self) -> Tuple[str, str]:
        return (f"{Chunk.block(self.start)}:{Chunk.off(self.start)}", f"{Chunk.block(self.end)}:{Chunk.off(self.end)}")


@dataclass
class Reference:
    bins: Dict[int, List[Chunk]]
    ioffsets: List[int]


def parse_bai(data: bytes) -> List[Reference]:
    if data[:4] != b"BAI\x01":
        raise IOError("Bad BAI magic")
    p = 4
    (n_ref,) = struct.unpack_from("<i", data, p)
    p += 4
    refs = []
    for _ in range(n_ref):
        (n_bin,) = struct.unpack_from("<i", data, p)
        p += 4
        bins: Dict[int, List[Chunk]] = {}
        for _ in range(n_bin):
            b, n_chunk = struct.unpack_from("<Ii", data, p)
            p += 8
            cs = [Chunk(*struct.unpack_from("<QQ", data, p + 16 * k)) for k in range(n_chunk)]
            p += 16 * n_chunk
            bins[b] = cs
        (n_intv,) = struct.unpack_from("<i", data, p)
        p += 4
        ioff = list(struct.unpack_from(f"<{n_intv}Q", data, p))
        p += 8 * n_intv
        refs.append(Reference(bins, ioff))
    return refs


def region_to_bins(start: int, end: int) -> Optional[List[int]]:
    """GenomicIndexUtil.regionToBins: 1-based closed [start, end]."""
    mx = 0x1FFFFFFF
    s = 0 if start <= 0 else (start - 1) & mx
    e = mx if end <= 0 else (end - 1) & mx
    if s > e:
        return None
    out = [0]
    for base, sh in ((1, 26), (9, 23), (73, 20), (585, 17), (4681, 14)):
        out.extend(range(base + (s >> sh), base + (e >> sh) + 1))
    return out


def min_offset(ref: Reference, start: int) -> int:
    s = 0 if start <= 0 else start - 1
    w = s >> LIDX_SHIFT
    return ref.ioffsets[w] if w < len(ref.ioffsets) else 0


def optimize_chunks(chunks: Sequence[Chunk], min_off: int) -> List[Chunk]:
    out: List[Chunk] = []
    for c in sorted(chunks):
        if c.end <= min_off:
            continue
        if not out:
            out.append(c)
            continue
        last = out[-1]
        if not last.overlaps(c) and not last.adjacent(c):
            out.append(c)
        elif c.end > last.end:
            out[-1] = Chunk(last.start, c.end)
    return out


def span_overlapping(refs: Sequence[Reference], ref_idx: int, start: int, end: int) -> List[Chunk]:
    """AbstractBAMFileIndex.getSpanOverlapping → BinningIndexContent.getChunksOverlapping."""
    if ref_idx < 0 or ref_idx >= len(refs) or not refs[ref_idx].bins:
        return []
    ref = refs[ref_idx]
    bins = region_to_bins(start, end)
    if bins is None:
        return []
    chunks = [c for b in bins if b != METADATA_BIN for c in ref.bins.get(b, ())]
    if not chunks:
        return []
    return optimize_chunks(chunks, min_offset(ref, start))


def file_span(refs: Sequence[Reference], query: Sequence[Tuple[int, int, int]]) -> List[Chunk]:
    """BAMFileReader.getFileSpan: merge of the intervals' spans. query = (ref index, 1-based start, end)."""
    chunks = [c for r, s, e in query for c in span_overlapping(refs, r, s, e)]
    return optimize_chunks(chunks, 0)


def parse_loci(s: str) -> List[Tuple[str, int, Optional[int]]]:
    """LociSet text (`1:13000-14000,1:60000-61000`): contig, 0-based start, exclusive end (None = contig end)."""
    out = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if ":" in part:
            contig, rng = part.rsplit(":", 1)
            a, b = rng.split("-", 1)
            out.append((contig, int(a), int(b)))
        else:
            out.append((part, 0, None))
    return out


def capped_cost_groups(costs: Sequence[float], cap: float) -> List[List[int]]:
    """magic_rdds cappedCostGroups: consecutive elements, a group closes before the element that would push
    its cost past `cap` (an element costlier than `cap` is a group of its own)."""
    groups: List[List[int]] = []
    cur: List[int] = []
    tot = 0.0
    for i, c in enumerate(costs):
        if cur and tot + c > cap:
            groups.append(cur)
            cur, tot = [], 0.0
        cur.append(i)
        tot += c
    if cur:
        groups.append(cur)
    return groups

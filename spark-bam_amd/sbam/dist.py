"""Multi-GPU driver: one process per GPU, byte-range shards of one BAM, tiny collectives.

Shard planning follows the reference's partitioning (one task per Hadoop FileSplit,
load/.../spark/load/SplitRDD.scala:33-52): rank r owns a contiguous run of Hadoop splits; it loads the
compressed bytes of those splits plus a halo (records and 10-record checker chains straddle shard edges),
starts its BGZF stream at FindBlockStart(first split start) and stops checking at the block where rank
r+1 starts.  The only cross-GPU traffic is what Spark's driver does with tiny data:

* ``all_gather`` of each split's first-record Pos / non-empty flag / record count
  (``mapPartitions(first).collect``, CanLoadBam.scala:262-271);
* ``all_reduce(sum)`` of the full-check Counts table (``reduceByKey(_ |+| _)``, FullCheck.scala:160-168).

A chain that leaves the loaded bytes reports HALO; the shard doubles its halo and re-runs (adaptive halo
for long reads).  ``compute`` is pluggable so the distributed logic is testable on CPU (gloo) with a
CPU-side per-shard function; production uses ``GpuShard``.

``run_file`` is the file-level driver: rank 0 parses the BAM header and broadcasts ContigLengths
(CanLoadBam.scala:179-180: the driver reads the header once and ships it to every task), every rank preads
only its own byte range + halo, and without a process group the same shards run one after another on this
process's GPU (a file larger than one GPU's HBM, or a one-GPU rehearsal of an N-GPU run).  ``WindowPipe`` streams
one rank's range through two contexts in windows (CanLoadBam.scala:281-334 at more than HBM per GPU).
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

N_COUNT_WORDS = 19 + 21 * 19 + 21 + 21 * 128 + 19 * 19 + 3


def hadoop_splits(file_size: int, split_size: int):
    """FileInputFormat rule (SPLIT_SLOP 1.1), same arithmetic as sbam_file_splits."""
    out, off, rem = [], 0, file_size
    while rem / split_size > 1.1:
        out.append((off, off + split_size))
        off += split_size
        rem -= split_size
    if rem > 0:
        out.append((off, file_size))
    return out


@dataclass
class ShardPlan:
    rank: int
    world: int
    split_first: int  # first Hadoop split index owned
    split_count: int
    lo: int  # first compressed byte owned (start of the first owned split)
    owned_hi: int  # start of the next rank's first split (or file size)
    file_size: int

    def load_range(self, halo: int):
        return self.lo, min(self.file_size, self.owned_hi + halo)


def plan_shards(file_size: int, split_size: int, world: int) -> List[ShardPlan]:
    sp = hadoop_splits(file_size, split_size)
    ns = len(sp)
    plans = []
    for r in range(world):
        i0, i1 = r * ns // world, (r + 1) * ns // world
        lo = sp[i0][0] if i0 < ns else file_size
        hi = sp[i1][0] if i1 < ns else file_size
        plans.append(ShardPlan(r, world, i0, i1 - i0, lo, hi, file_size))
    return plans


@dataclass
class ShardResult:
    counts: np.ndarray  # int64[N_COUNT_WORDS] (by_key, positions, rbe, pair, n_success, n_tff, n_positions)
    first_block_pos: np.ndarray  # int64[split_count]
    first_offset: np.ndarray  # int64[split_count]
    nonempty: np.ndarray  # int64[split_count]
    n_records: np.ndarray  # int64[split_count]


def pack_counts(c) -> np.ndarray:
    return np.concatenate([c.totals, c.by_key.ravel(), c.positions, c.reads_before_error.ravel(), c.pair_hist.ravel(),
                           np.array([c.n_success, c.n_too_few_fixed, c.n_positions], np.int64)]).astype(np.int64)


def unpack_counts(v: np.ndarray) -> dict:
    o = 0
    out = {}
    for name, n, shape in (("totals", 19, (19,)), ("by_key", 21 * 19, (21, 19)), ("positions", 21, (21,)),
                           ("reads_before_error", 21 * 128, (21, 128)), ("pair_hist", 19 * 19, (19, 19))):
        out[name] = v[o:o + n].reshape(shape)
        o += n
    out["n_success"], out["n_too_few_fixed"], out["n_positions"] = (int(x) for x in v[o:o + 3])
    return out


def shard_pass(f, p: ShardPlan, split_size: int, R: int = 10) -> ShardResult:
    """One shard's hot path once its stream is inflated (``f``: sbam.BamFile over the shard's bytes, or any
    object with the same methods): full check of the positions of the blocks the shard owns (from its first
    block to the block where the next shard starts), then the owned Hadoop splits' first records and counts."""
    if p.owned_hi >= p.file_size:
        x1 = f.uncompressed_size
    else:
        st, _, _, uo = f.blocks()
        nb = f.find_block_start(p.owned_hi)
        b = int(np.searchsorted(st, nb))
        x1 = int(uo[b]) if b < st.size else f.uncompressed_size
    counts = f.check_full_counts(0, x1, R)
    if p.split_count:
        bp, off, nonempty, n = f.split_records_arrays(split_size, first=p.split_first, count=p.split_count,
                                                      reads_to_check=R, use_success_bitmap=True)
    else:
        bp = off = nonempty = n = np.zeros(0, np.int64)
    return ShardResult(pack_counts(counts), bp.astype(np.int64), off.astype(np.int64), nonempty.astype(np.int64),
                       n.astype(np.int64))


def shard_load(f, p: ShardPlan, split_size: int, R: int = 10, use_success_bitmap: bool = False,
               eager_proof: bool = True) -> np.ndarray:
    """One shard's loadReads: the owned Hadoop splits' records decoded into device columns
    (sbam_load_records; CanLoadBam.scala:281-334); returns the partition sizes.

    eager_proof: first run the eager checker over the shard (its calls' bitmap stays on the device) so that the
    splits' record chains come from that bitmap once sbam_load_records has proved it — every set bit from a
    split's first record hops (block_size) to the next set bit — instead of one lane walking each split's chain
    record by record (twice: counts, then offsets).  The records are the same either way: a bitmap that fails
    the proof falls back to the walk."""
    if not p.split_count:
        return np.zeros(0, np.int64)
    if eager_proof and not use_success_bitmap:
        f.check_eager_device(0, f.uncompressed_size, R)
        use_success_bitmap = True
    sizes, _ = f.load_records(split_size, first=p.split_first, count=p.split_count, reads_to_check=R,
                              use_success_bitmap=use_success_bitmap, columns=None)
    return sizes


class GpuShard:
    """Per-rank GPU work for one shard: scan → inflate → full check (owned positions) → split records."""

    def __init__(self, plan: ShardPlan, source: Callable[[int, int], np.ndarray], split_size: int,
                 contig_lengths: Sequence[int], device: int = 0, halo: int = 2 << 20, reads_to_check: int = 10):
        import sbam
        self.sbam = sbam
        self.plan, self.source, self.split_size = plan, source, split_size
        self.contig_lengths = np.asarray(contig_lengths, np.int64)
        self.device, self.halo, self.R = device, halo, reads_to_check
        self.f = None
        self.retries = 0  # halo retries so far (each grows the halo 4x and re-runs the shard)
        self._open()

    def _open(self):
        lo, hi = self.plan.load_range(self.halo)
        if self.f is not None:
            self.f.close()
        self.f = self.sbam.BamFile(self.source(lo, hi), device=self.device, base_offset=lo,
                                   file_size=self.plan.file_size, inflate=False)
        self._reserved = 0  # a new context (WindowPipe._reserve sizes it again)

    def reload(self, plan: ShardPlan, data: np.ndarray, source: Optional[Callable[[int, int], np.ndarray]] = None):
        """Stream the next byte-range window through this shard's context (sbam_load: device allocations are
        kept): `data` = the bytes of plan.load_range(self.halo).  `source` replaces the byte source a halo retry
        reads from (it must not hand back a buffer another window is being staged into)."""
        self.plan = plan
        if source is not None:
            self.source = source
        lo, _ = plan.load_range(self.halo)
        self.f.load(data, base_offset=lo, file_size=plan.file_size)

    def _once(self) -> ShardResult:
        self.f.reset()
        self.f.run(contig_lengths=self.contig_lengths)
        return shard_pass(self.f, self.plan, self.split_size, self.R)

    def run_with(self, fn):
        """Any per-shard work fn(f, plan) on the shard's inflated stream, with the halo retry of step()."""
        def once():
            self.f.reset()
            self.f.run(contig_lengths=self.contig_lengths)
            return fn(self.f, self.plan)
        return self._retry(once)

    def _retry(self, fn):
        while True:
            try:
                return fn()
            except self.sbam.HaloException:
                if self.plan.load_range(self.halo)[1] >= self.plan.file_size:
                    raise
                self.halo *= 4
                self.retries += 1
                # the grown range goes into the same context (sbam_load keeps its device allocations and only grows
                # the ones the larger range needs), so a retry costs one H2D copy and the re-run, not a new context
                lo, hi = self.plan.load_range(self.halo)
                self.f.load(self.source(lo, hi), base_offset=lo, file_size=self.plan.file_size)

    def step(self) -> ShardResult:
        """compute-splits + full-check of the shard."""
        return self._retry(self._once)

    def load_step(self) -> np.ndarray:
        """loadReads of the shard: scan → inflate → FindBlockStart/FindRecordStart → record chains → columns."""
        def once():
            self.f.reset()
            self.f.run(contig_lengths=self.contig_lengths)
            return shard_load(self.f, self.plan, self.split_size, self.R)
        return self._retry(once)

    def load_columns(self, columns: Sequence[str]):
        """load_step with the decoded record columns copied out: (partition sizes, {column: ndarray})."""
        def once():
            self.f.reset()
            self.f.run(contig_lengths=self.contig_lengths)
            p = self.plan
            if not p.split_count:
                return np.zeros(0, np.int64), {k: np.zeros(0, self.sbam.RECORD_COLUMNS[k]) for k in columns}
            self.f.check_eager_device(0, self.f.uncompressed_size, self.R)  # (shard_load's eager_proof)
            return self.f.load_records(self.split_size, first=p.split_first, count=p.split_count,
                                       reads_to_check=self.R, use_success_bitmap=True, columns=columns)
        return self._retry(once)

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None


def combine(results: Sequence[ShardResult], file_size: int):
    """Rank-0 assembly of gathered shard results → (Split list, partition sizes, merged counts)."""
    from sbam import Pos, Split
    firsts, sizes = [], []
    counts = np.zeros(N_COUNT_WORDS, np.int64)
    for r in results:
        counts += r.counts
        for b, o, ne, n in zip(r.first_block_pos, r.first_offset, r.nonempty, r.n_records):
            sizes.append(int(n))
            if ne:
                firsts.append(Pos(int(b), int(o)))
    ends = firsts[1:] + [Pos(file_size, 0)]
    return [Split(a, b) for a, b in zip(firsts, ends)], sizes, counts


def gather_results(res: ShardResult, plans: Sequence[ShardPlan], device=None) -> Optional[List[ShardResult]]:
    """all_gather of per-shard results (fixed-size int64 rows) + all_reduce of counts via torch.distributed.
    Returns the per-rank list on every rank (counts of each entry are the merged totals on rank 0's row)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    maxs = max(p.split_count for p in plans)
    row = np.zeros(4 * maxs, np.int64)
    k = len(res.n_records)
    for j, a in enumerate((res.first_block_pos, res.first_offset, res.nonempty, res.n_records)):
        row[j * maxs: j * maxs + k] = a
    t = torch.from_numpy(row)
    c = torch.from_numpy(res.counts.copy())
    if device is not None:
        t, c = t.to(device), c.to(device)
    out = torch.empty(world * row.size, dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(out, t)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    out = out.cpu().numpy().reshape(world, 4, maxs)
    merged = c.cpu().numpy()
    results = []
    for r, p in enumerate(plans):
        n = p.split_count
        results.append(ShardResult(merged if r == 0 else np.zeros_like(merged), out[r, 0, :n], out[r, 1, :n],
                                   out[r, 2, :n], out[r, 3, :n]))
    return results


# ---- file-level driver ----------------------------------------------------------------------------------------

# HBM per compressed byte of one loaded range (DESIGN.md §Data layout): the compressed bytes, the uncompressed
# stream (r per byte, r = uncompressed / compressed), the decoder's main token regions (r: 1 B per uncompressed byte),
# the success bitmap (r / 8), the token arena, plus block tables, candidates and the checker's lists (< 0.05).
# The arena's default is 1/16 B per uncompressed byte, but a block whose tokens outgrow its main region (more than
# (ISIZE + 16) / 2 tokens: stored blocks, Huffman-only or RLE streams — fewer than 2 output bytes per token) takes
# 2 B per uncompressed byte there (sbam_inflate grows the arena to what the blocks asked for and decodes again).  The
# compression ratio does not tell such blocks apart (Huffman-only over a 4-letter alphabet compresses 4:1), so
# bgzf_sample_stats counts the DEFLATE tokens of a few sampled blocks.


def hbm_bytes_per_compressed_byte(ratio: float, arena_frac: float = 0.0) -> float:
    """Device bytes a loaded range needs per compressed byte at compression ratio `ratio`: the compressed bytes, and
    per uncompressed byte the stream (1), the main token regions (1), the success bitmap (1/8) and the token arena
    (the default 1/16, or 2 B per byte of the `arena_frac` of the output in blocks that need it, whichever is more);
    block tables and scratch ~0.05."""
    arena = max(0.0625, 2.0 * arena_frac * 1.125)
    return 1.0 + ratio * (1.0 + 1.0 + 0.125 + arena) + 0.05


def _first_header(raw: bytes) -> int:
    """Offset of the first BGZF header (magic 1f 8b 08 04, 'BC' at +12) in `raw`, or -1 (a range may start inside
    a block)."""
    pos = 0
    while True:
        pos = raw.find(b"\x1f\x8b\x08\x04", pos)
        if pos < 0 or raw[pos + 12:pos + 14] == b"BC":
            return pos
        pos += 1


_CL_ORDER = (16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15)
_LEN_EXTRA = [0] * 8 + [k // 4 - 1 for k in range(8, 28)] + [0]
_DIST_EXTRA = [0] * 4 + [k // 2 - 1 for k in range(4, 30)]


def _huff_table(lengths):
    """15-bit lookup table of a canonical code (stream bits LSB first): entry = symbol << 4 | length (0 = no code)."""
    tab = [0] * 32768
    code, nxt, cnt = 0, [0] * 16, [0] * 16
    for l in lengths:
        cnt[l] += 1
    cnt[0] = 0
    for l in range(1, 16):
        code = (code + cnt[l - 1]) << 1
        nxt[l] = code
    for sym, l in enumerate(lengths):
        if l:
            c = nxt[l]
            nxt[l] += 1
            r = int(format(c, f"0{l}b")[::-1], 2)
            e = (sym << 4) | l
            for j in range(r, 32768, 1 << l):
                tab[j] = e
    return tab


def deflate_token_count(payload: bytes, limit: int = 1 << 20) -> int:
    """Tokens (literals + lengths + distances, the decoder's u16 stream) of a raw DEFLATE stream, or -1 when it does not
    parse; stops after `limit` output bytes.  (RFC 1951; used only to budget HBM for the token arena.)"""
    n = len(payload)
    pos = 0          # next byte to enter the bit buffer
    bb = bc = 0      # bit buffer (LSB first) and its count

    def need(k):
        nonlocal pos, bb, bc
        while bc < k:
            bb |= (payload[pos] if pos < n else 0) << bc
            pos += 1
            bc += 8

    def bits(k):
        nonlocal bb, bc
        need(k)
        v = bb & ((1 << k) - 1)
        bb >>= k
        bc -= k
        return v

    def sym(tab):
        nonlocal bb, bc
        need(15)
        e = tab[bb & 32767]
        if not e:
            raise ValueError
        bb >>= e & 15
        bc -= e & 15
        return e >> 4

    tokens = out = 0
    try:
        while out < limit:
            fin, typ = bits(1), bits(2)
            if typ == 0:
                bb >>= bc & 7
                bc -= bc & 7
                ln = bits(16)
                bits(16)
                tokens += ln
                out += ln
                inbuf = bc // 8  # whole bytes already in the bit buffer (bc is a multiple of 8 here)
                if ln >= inbuf:
                    bb = bc = 0
                    pos += ln - inbuf
                else:
                    bb >>= 8 * ln
                    bc -= 8 * ln
            elif typ in (1, 2):
                if typ == 1:
                    ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                    dl = [5] * 30
                else:
                    hlit, hdist, hclen = bits(5) + 257, bits(5) + 1, bits(4) + 4
                    cl = [0] * 19
                    for i in range(hclen):
                        cl[_CL_ORDER[i]] = bits(3)
                    ctab = _huff_table(cl)
                    lens = []
                    while len(lens) < hlit + hdist:
                        s_ = sym(ctab)
                        if s_ < 16:
                            lens.append(s_)
                        elif s_ == 16:
                            lens += [lens[-1]] * (3 + bits(2))
                        else:
                            lens += [0] * ((3 + bits(3)) if s_ == 17 else (11 + bits(7)))
                    ll, dl = lens[:hlit], lens[hlit:hlit + hdist]
                ltab, dtab = _huff_table(ll), _huff_table(dl)
                while True:
                    s_ = sym(ltab)
                    if s_ < 256:
                        tokens += 1
                        out += 1
                    elif s_ == 256:
                        break
                    else:
                        k = s_ - 257
                        base = (k + 3) if k < 8 else 258 if k == 28 else (((4 | (k & 3)) << _LEN_EXTRA[k]) + 3)
                        out += base + bits(_LEN_EXTRA[k])
                        d = sym(dtab)
                        bits(_DIST_EXTRA[d])
                        tokens += 2
                    if out >= limit:
                        break
            else:
                return -1
            if fin:
                break
    except (ValueError, IndexError):
        return -1
    return tokens


def bgzf_sample_stats(source: Callable[..., np.ndarray], size: int, sample: int = 8 << 20,
                      token_blocks: int = 12) -> Tuple[float, float]:
    """(uncompressed / compressed, share of the uncompressed bytes in blocks whose tokens outgrow the main token
    region) over the BGZF blocks of the first `sample` bytes (the block chain from the first header: BSIZE at +16,
    ISIZE in the block's last 4 bytes — Header.scala, the footer); the token share from `token_blocks` blocks spread
    over the sample (a block that does not parse counts as an arena block); (3.0, 0.0) when nothing parses."""
    buf = source(0, min(size, sample))
    raw = buf.tobytes()
    pos = _first_header(raw)
    if pos < 0:
        return 3.0, 0.0
    comp = unc = 0
    blocks = []
    while pos + 18 <= len(raw) and raw[pos] == 0x1F and raw[pos + 1] == 0x8B:
        bsize = raw[pos + 16] | (raw[pos + 17] << 8)
        end = pos + bsize + 1
        if end > len(raw):
            break
        isz = int.from_bytes(raw[end - 4:end], "little")
        unc += isz
        comp += bsize + 1
        blocks.append((pos, end, isz))
        pos = end
    if not (comp and unc):
        return 3.0, 0.0
    picks = sorted({int(i) for i in np.linspace(0, len(blocks) - 1, min(token_blocks, len(blocks)))})
    tot = big = 0
    for i in picks:
        st, end, isz = blocks[i]
        xlen = raw[st + 10] | (raw[st + 11] << 8)
        t = deflate_token_count(raw[st + 12 + xlen:end - 8], isz)
        tot += isz
        big += isz if (t < 0 or t > (isz + 16) // 2) else 0
    return unc / comp, (big / tot if tot else 0.0)


def bgzf_ratio(source: Callable[..., np.ndarray], size: int, sample: int = 8 << 20) -> float:
    """Uncompressed / compressed bytes over the BGZF blocks of the first `sample` bytes (bgzf_sample_stats)."""
    return bgzf_sample_stats(source, size, sample)[0]


def bgzf_buffer_stats(buf: np.ndarray) -> Tuple[float, float]:
    """(uncompressed / compressed, compressed bytes per block) over the BGZF block chain from the first header in
    `buf` (as bgzf_ratio); (3.0, 65536.0) when nothing parses."""
    raw = buf[: 8 << 20].tobytes()
    pos = 0
    while True:
        pos = raw.find(b"\x1f\x8b\x08\x04", pos)
        if pos < 0 or raw[pos + 12:pos + 14] == b"BC":
            break
        pos += 1
    comp = unc = nb = 0
    while pos >= 0 and pos + 18 <= len(raw) and raw[pos] == 0x1F and raw[pos + 1] == 0x8B:
        end = pos + (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
        if end > len(raw):
            break
        unc += int.from_bytes(raw[end - 4:end], "little")
        comp += end - pos
        nb += 1
        pos = end
    return (unc / comp, comp / nb) if comp and unc else (3.0, 65536.0)


def auto_windows(size: int, source: Callable[..., np.ndarray], free_bytes: int, contexts: int = 2,
                 headroom: float = 0.8) -> int:
    """Windows for a `size`-byte range so that `contexts` loaded windows (WindowPipe keeps two) fit in `headroom` of
    `free_bytes` of HBM, from the file's measured compression ratio (with 10 % margin) and the share of its output in
    low-ratio blocks, whose tokens may take the arena at 2 B per byte (stored / Huffman-only inputs)."""
    ratio, arena_frac = bgzf_sample_stats(source, size)
    per_byte = hbm_bytes_per_compressed_byte(1.1 * ratio, arena_frac)
    need = size * per_byte * contexts
    return max(1, int(np.ceil(need / (headroom * free_bytes))))


def device_free_bytes(device: int) -> int:
    import torch
    return int(torch.cuda.mem_get_info(device)[0])


def file_source(path: str) -> Tuple[Callable[..., np.ndarray], int]:
    """(source, file size) for a BAM on disk: source(lo, hi[, out]) preads bytes [lo, hi) into a new (or the given)
    uint8 array — a rank touches only its own byte range, never the whole file."""
    size = os.path.getsize(path)

    def source(lo: int, hi: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        hi = min(hi, size)
        buf = np.empty(hi - lo, np.uint8) if out is None else out[: hi - lo]
        mv = memoryview(buf)
        fd = os.open(path, os.O_RDONLY)
        try:
            got = 0
            while got < hi - lo:
                n = os.preadv(fd, [mv[got: min(hi - lo, got + (1 << 30))]], lo + got)
                if n <= 0:
                    raise IOError(f"{path}: short read at {lo + got}")
                got += n
        finally:
            os.close(fd)
        return buf

    return source, size


def read_contig_lengths(source: Callable[[int, int], np.ndarray], file_size: int, device: int = 0,
                        probe: int = 1 << 20) -> np.ndarray:
    """ContigLengths from the header at the start of the file (ContigLengths.scala:20-37 via htsjdk's header
    reader): the first `probe` bytes are inflated on the GPU and parsed (sbam_header); a header longer than the
    probe doubles it."""
    import sbam
    hi = min(file_size, probe)
    while True:
        try:
            with sbam.BamFile(source(0, hi), device=device, file_size=file_size, inflate=False) as f:
                f.inflate()
                return f.header()[1]
        except sbam.SbamError as e:
            if "truncated header" not in str(e) or hi >= file_size:
                raise
            hi = min(file_size, 2 * hi)


def broadcast_lengths(lens: Optional[np.ndarray], device=None) -> np.ndarray:
    """Rank 0's ContigLengths to every rank (the reference broadcasts the header's lengths to its tasks)."""
    import torch
    import torch.distributed as dist
    n = torch.tensor([0 if lens is None else len(lens)], dtype=torch.int64, device=device)
    dist.broadcast(n, src=0)
    t = torch.zeros(int(n.item()), dtype=torch.int64, device=device)
    if dist.get_rank() == 0:
        t.copy_(torch.from_numpy(np.asarray(lens, np.int64)))
    dist.broadcast(t, src=0)
    return t.cpu().numpy()


@dataclass
class RunResult:
    splits: list  # [sbam.Split] (compute-splits)
    partition_sizes: List[int]  # records per Hadoop split
    counts: dict  # merged full-check Counts (unpack_counts)
    contig_lengths: np.ndarray


def _dist_ready() -> bool:
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()
    except ImportError:
        return False


def run_file(path, split_size: Optional[int] = None, world: Optional[int] = None, device: Optional[int] = None,
             halo: int = 2 << 20, reads_to_check: int = 10, coll_device=None,
             open_shard: Optional[Callable[[ShardPlan, Callable, int, np.ndarray], object]] = None,
             read_header: Optional[Callable[[Callable, int, int], np.ndarray]] = None) -> RunResult:
    """full-check + compute-splits of one BAM over byte-range shards (FullCheck.scala:141-191 with the splits of
    CanLoadBam.scala:245-279).  `path`: a file name, or a (source, file_size) pair.

    In a torch.distributed process group (RCCL on GPUs; gloo to rehearse) the shards are the ranks: rank 0 reads
    the header and broadcasts ContigLengths, each rank preads [lo, owned_hi + halo) of its own shard, and the
    results meet in one all_gather + one all_reduce (gather_results); every rank returns the whole result.
    Without a process group, `world` shards (default 1) run one after another on `device`.
    `open_shard(plan, source, split_size, contig_lengths)` / `read_header(source, size, device)` replace the GPU
    shard and header reader (CPU tests)."""
    import sbam
    split_size = sbam.effective_split_size(split_size)
    source, size = file_source(path) if isinstance(path, (str, os.PathLike)) else path
    grouped = _dist_ready()  # in a process group the collectives run even at world size 1 (RCCL exercised)
    if grouped:
        import torch.distributed as dist
        world, rank = dist.get_world_size(), dist.get_rank()
        ranks = [rank]
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", 0))
    else:
        world, rank = world or 1, 0
        ranks = list(range(world))
        device = 0 if device is None else device
    read_header = read_header or read_contig_lengths
    lens = read_header(source, size, device) if rank == 0 else None
    if grouped:
        lens = broadcast_lengths(lens, coll_device)
    if open_shard is None:
        def open_shard(plan, src, ss, cl):
            return GpuShard(plan, src, ss, cl, device=device, halo=halo, reads_to_check=reads_to_check)
    plans = plan_shards(size, split_size, world)
    results = []
    for r in ranks:
        sh = open_shard(plans[r], source, split_size, lens)
        try:
            results.append(sh.step())
        finally:
            sh.close()
    if grouped:
        results = gather_results(results[0], plans, device=coll_device)
    splits, sizes, counts = combine(results, size)
    return RunResult(splits, sizes, unpack_counts(counts), np.asarray(lens, np.int64))


def owned_blocks(f, p: ShardPlan) -> np.ndarray:
    """Block mask of the blocks shard `p` owns in its context `f`: from its first block up to the block where the next
    shard's stream starts (FindBlockStart of that shard's first split), as shard_pass does."""
    st = f.blocks()[0]
    if p.owned_hi >= p.file_size:
        return np.ones(st.size, bool)
    b = int(np.searchsorted(st, f.find_block_start(p.owned_hi)))
    m = np.zeros(st.size, bool)
    m[:b] = True
    return m


def read_header_names(source, file_size: int, device: int = 0, probe: int = 1 << 20):
    """(ContigLengths, contig names) from the header at the start of the file (bam/header/Header.scala:26-60)."""
    import sbam
    from sbam.cli import header_names
    hi = min(file_size, probe)
    while True:
        try:
            with sbam.BamFile(source(0, hi), device=device, file_size=file_size, inflate=False) as f:
                f.inflate()
                return f.header()[1], header_names(f)
        except sbam.SbamError as e:
            if "truncated header" not in str(e) or hi >= file_size:
                raise
            hi = min(file_size, 2 * hi)


def _pack_parts_counts(q) -> np.ndarray:
    return np.concatenate([q.totals, q.by_key.ravel(), q.positions, q.rbe.ravel(), q.pair.ravel(),
                           np.array([q.n_positions, q.compressed], np.int64)]).astype(np.int64)


def full_check_file(path, limit: int = 10, ranges=None, reads_to_check: int = 10, world: Optional[int] = None,
                    device: Optional[int] = None, halo: int = 2 << 20, coll_device=None,
                    records_path: Optional[str] = None, split_size: int = 2 << 20):
    """`full-check` over byte-range shards (FullCheck.scala:88-323 with Blocks' partitions, Blocks.scala:141-207).
    Each shard full-checks the blocks it owns and samples its first `limit` close calls of keys 1 and 2 (and its
    disagreements with the `.records` truth) as PosMetadata lines — the next record of a sampled position may lie in
    the halo, which grows when needed.  In a process group (RCCL on GPUs) rank 0 reads the header and broadcasts the
    contig lengths (device tensor) and names; the Counts meet in one all_reduce on `coll_device` (reduceByKey,
    FullCheck.scala:160-168) and the sampled lines in one all_gather_object (the driver's take(limit)).  Without a
    process group, `world` shards run one after another on `device` (a file larger than HBM in windows).
    Returns the merged sbam.cli.FullCheckParts on every rank."""
    import sbam
    from sbam.cli import FullCheckParts, FullCheckReport, merge_parts
    source, size = file_source(path) if isinstance(path, (str, os.PathLike)) else path
    grouped = _dist_ready()  # in a process group the collectives run even at world size 1 (RCCL exercised)
    if grouped:
        import torch.distributed as dist
        world, rank = dist.get_world_size(), dist.get_rank()
        ranks = [rank]
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", 0))
    else:
        world, rank = world or 1, 0
        ranks = list(range(world))
        device = 0 if device is None else device
    lens, names = read_header_names(source, size, device) if rank == 0 else (None, None)
    if grouped:
        import torch.distributed as dist
        lens = broadcast_lengths(lens, coll_device)
        box = [names]
        dist.broadcast_object_list(box, src=0, device=coll_device)
        names = box[0]
    plans = plan_shards(size, split_size, world)
    parts = []
    for r in ranks:
        sh = GpuShard(plans[r], source, split_size, lens, device=device, halo=halo, reads_to_check=reads_to_check)
        try:
            parts.append(sh.run_with(lambda f, p: FullCheckReport(
                f, None, records_path, limit, ranges, reads_to_check, blocks=owned_blocks(f, p),
                names=names).parts()))
        finally:
            sh.close()
    if grouped:
        import torch
        import torch.distributed as dist
        mine = parts[0]
        c = torch.from_numpy(_pack_parts_counts(mine))
        if coll_device is not None:
            c = c.to(coll_device)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        v = c.cpu().numpy()
        lists = [None] * world
        dist.all_gather_object(lists, (mine.close, mine.truth))
        o = 0
        fields = []
        for n, shape in ((19, (19,)), (21 * 19, (21, 19)), (21, (21,)), (21 * 128, (21, 128)), (19 * 19, (19, 19))):
            fields.append(v[o:o + n].reshape(shape))
            o += n
        parts = [FullCheckParts(*fields, int(v[o]), int(v[o + 1]), close, truth) if i == 0 else
                 FullCheckParts(*(np.zeros_like(x) for x in fields), 0, 0, close, truth)
                 for i, (close, truth) in enumerate(lists)]
    return merge_parts(parts, limit)


class WindowPipe:
    """A rank's byte range streamed through two contexts in W windows (`wplans`: the windows' ShardPlans): while
    window w computes on one context, a loader thread copies window w+1's bytes into the other (sbam_load's host →
    device copy) and a stager thread stages window w+2 into host memory (`stage(lo, hi, k)` into staging buffer
    k).  Windows are numbered across steps (g = step · W + w): window g uses context g mod 2 and staging buffer
    g mod 3, so the pipeline runs on from one step into the next — the last window of a step computes while the
    next step's window 0 is copied (`prefetch=True`; `drop_prefetch()` discards one that no step will use).
    Without a pending prefetch a step starts with window 0 loaded in the foreground.  `run_window(shard)` is the
    per-window work (GpuShard.step / load_step / anything on shard.f).  Buffer k is restaged only after the copy
    that read it has finished (window g+2 reuses window g-1's buffer, whose copy ended before window g-1 computed)."""
    NBUF = 3

    def __init__(self, wplans, stage, split_size, contig_lengths, device, run_window, halo: int = 2 << 20,
                 prefetch: bool = False):
        from concurrent.futures import ThreadPoolExecutor
        self.wplans, self.stage, self.split_size = wplans, stage, split_size
        self.contig_lengths, self.device, self.run_window, self.halo = contig_lengths, device, run_window, halo
        self.prefetch = prefetch
        self.loader = ThreadPoolExecutor(max_workers=1)
        self.stager = ThreadPoolExecutor(max_workers=1)
        self.ctx = [None, None]
        self._inflight = []   # loader futures of the running step
        self.g = 0            # global number of the next step's window 0
        self._next = None     # (load future of window g, {g': staged future}) carried over from the last step

    def _range(self, g):
        sh = self.ctx[g % 2]
        return self.wplans[g % len(self.wplans)].load_range(sh.halo if sh is not None else self.halo)

    def _stage(self, g):
        lo, hi = self._range(g)
        return lo, hi, self.stage(lo, hi, g % self.NBUF)

    def _load(self, g, staged):
        wp = self.wplans[g % len(self.wplans)]
        j, k = g % 2, g % self.NBUF
        lo, hi, buf = staged.result()
        if (lo, hi) != self._range(g):  # the context's halo grew since staging: stage again
            lo, hi = self._range(g)
            buf = self.stage(lo, hi, k)
        src = self._source(lo, hi, buf)
        if self.ctx[j] is None:
            self.ctx[j] = GpuShard(wp, src, self.split_size, self.contig_lengths, device=self.device, halo=self.halo)
        else:
            self.ctx[j].reload(wp, buf, src)
        self._reserve(self.ctx[j], buf)
        return self.ctx[j]

    def _reserve(self, sh, buf):
        """Size a context once for the largest window of the plan (device buffers are grow-only: a context that
        first meets a larger window than before would hipFree + hipMalloc tens of GB inside a timed step), from the
        compression ratio and block size of the staged bytes (+12 %)."""
        comp = max(p.load_range(sh.halo)[1] - p.load_range(sh.halo)[0] for p in self.wplans)
        if getattr(sh, "_reserved", 0) >= comp:
            return
        ratio, per_block = bgzf_buffer_stats(buf)
        U = int(comp * ratio * 1.12) + (1 << 20)
        sh.f.reserve(comp, int(comp / per_block * 1.12) + 1024, U, U // 200)
        sh._reserved = comp

    def _source(self, lo, hi, buf):
        """The byte source of one loaded window: its staged bytes for its own range; any other range (a halo retry)
        is staged into a private buffer, never into a shared staging slot."""
        def src(a, b):
            return buf if (a, b) == (lo, hi) else self.stage(a, b, None)
        return src

    def drop_prefetch(self):
        """Wait for and discard a prefetched window 0 (the next step then loads it in the foreground)."""
        if self._next is not None:
            fut, staged = self._next
            fut.result()
            for f in staged.values():
                f.result()
            self._next = None  # window self.g is loaded again (same context) by the next step

    def step(self) -> list:
        W = len(self.wplans)
        g0 = self.g
        if self._next is not None:
            fut, staged = self._next
            self._next = None
        else:
            staged = {g: self.stager.submit(self._stage, g) for g in range(g0, g0 + min(2, W))}
            fut = None
        try:
            return self._windows(g0, W, staged, fut)
        except BaseException:
            # a failed window (a non-halo error, or a halo retry that reached EOF): drain the loads and stagings still
            # in flight — they drive the other context and the staging buffers — so that a retried step starts clean
            for f in ([fut] if fut is not None else []) + list(staged.values()) + list(self._inflight):
                try:
                    f.result()
                except BaseException:
                    pass
            self._inflight = []
            self._next = None
            raise

    def _windows(self, g0, W, staged, fut) -> list:
        self._inflight = []
        out = []
        sh = self._load(g0, staged[g0]) if fut is None else None
        dbg = os.environ.get("SBAM_PIPE_DEBUG")
        for w in range(W):
            g = g0 + w
            t0 = time.perf_counter()
            if sh is None:
                sh = fut.result()
            if dbg:
                print(f"[pipe] window {g}: waited {1e3 * (time.perf_counter() - t0):.1f} ms for its load", file=sys.stderr)
            last = w + 1 == W
            if not last or self.prefetch:
                if g + 1 not in staged:
                    staged[g + 1] = self.stager.submit(self._stage, g + 1)
                fut = self.loader.submit(self._load, g + 1, staged[g + 1])
                self._inflight.append(fut)
            if (w + 2 < W or self.prefetch) and g + 2 not in staged:
                staged[g + 2] = self.stager.submit(self._stage, g + 2)
            t1 = time.perf_counter()
            out.append(self.run_window(sh))
            if dbg:
                print(f"[pipe] window {g}: ran {1e3 * (time.perf_counter() - t1):.1f} ms", file=sys.stderr)
            sh = None
        self.g = g0 + W
        if self.prefetch:
            self._next = (fut, {k: v for k, v in staged.items() if k >= self.g})
        return out

    def close(self):
        self.loader.shutdown()
        self.stager.shutdown()
        for sh in self.ctx:
            if sh is not None:
                sh.close()
        self.ctx = [None, None]

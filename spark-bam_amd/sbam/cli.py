"""spark-bam CLI drop-ins over the GPU path: `full-check`, `check-bam -s`, `check-blocks -s`, `compute-splits -s`,
`count-reads`, `index-blocks`, `index-records`.

    python -m sbam.cli full-check [-l LIMIT] [-m SPLIT] [-i RANGES] [-r READS] [--gpus N | --windows W] BAM [OUT]
    python -m sbam.cli check-bam -s [-l LIMIT] [-m SPLIT] [-i RANGES] BAM [OUT]
    python -m sbam.cli check-blocks -s [-l LIMIT] BAM [OUT]
    python -m sbam.cli index-blocks BAM [OUT]
    python -m sbam.cli index-records BAM [OUT]
    python -m sbam.cli compute-splits [-s] [-l LIMIT] [-m SPLIT] BAM [OUT]
    python -m sbam.cli count-reads [-m SPLIT] BAM [OUT]

Report text follows the reference apps line for line, so the goldens of cli/src/test/resources/output/ diff
verbatim (tests/test_cli.py):
  * full-check: FullCheck.scala:141-322, the CheckerApp summary (CheckerApp.scala:140-222) when a `.records`
    sidecar is present, PosMetadata / NextRecord (check/PosMetadata.scala, NextRecord.scala), Counts.lines
    (check/.../full/error/Counts.scala:59-127);
  * check-bam -s: eager/CheckBam.scala + the CheckerApp comparison with the `.records` truth;
  * check-blocks -s: blocks/CheckBlocks.scala (eager vs indexed first read per block);
  * index-blocks / index-records: bgzf/.../index/IndexBlocks.scala, check/.../bam/index/IndexRecords.scala (the
    `.blocks` / `.records` sidecars);
  * compute-splits: ComputeSplits.scala:56-68 (-s: spark-bam splits only; hadoop-bam comparison is out of scope);
  * count-reads: compare/CountReads.scala:80-100, spark-bam side only.
Counting, checking and splitting all run through libsbam.so (sbam.BamFile); this module only formats."""
from __future__ import annotations

import argparse
import math
import os
import sys
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

import sbam
from sbam import FLAG_NAMES, Pos

RATIO = 3.0  # EstimatedCompressionRatio default (bgzf/.../EstimatedCompressionRatio.scala)


# ---- small formatting helpers ----------------------------------------------------------------------------
def parse_bytes(s: str) -> int:
    """hammerlab Bytes arguments: 230k, 2m, 1g (binary multiples), or a plain byte count."""
    s = s.strip().lower()
    mult = {"k": 1 << 10, "m": 1 << 20, "g": 1 << 30, "t": 1 << 40}
    if s and s[-1] == "b":
        s = s[:-1]
    if s and s[-1] in mult:
        return int(float(s[:-1]) * mult[s[-1]])
    return int(s)


def format_bytes(n: int) -> str:
    """Bytes.format as the goldens show it: three significant digits of the binary unit (25.6K, 217K, 583K)."""
    units = "KMGTPE"
    if n < 1024:
        return f"{n}B"
    v, u = float(n), -1
    while v >= 1024 and u < len(units) - 1:
        v /= 1024
        u += 1
    s = f"{v:.0f}" if v >= 100 else f"{v:.1f}" if v >= 10 else f"{v:.2f}"
    return s + units[u]


def parse_ranges(s: str) -> List[Tuple[int, int]]:
    """-i ranges of compressed block starts: `0`, `26169`, `0-200k`, comma-separated ([lo, hi) each; a single
    value N is the point range [N, N+1))."""
    out = []
    for part in s.split(","):
        part = part.strip()
        if "-" in part:
            a, b = part.split("-", 1)
            out.append((parse_bytes(a), parse_bytes(b)))
        else:
            v = parse_bytes(part)
            out.append((v, v + 1))
    return out


def show_flags(F: int) -> str:
    return ",".join(FLAG_NAMES[i] for i in range(19) if F >> i & 1)


def count_lines(pairs: Sequence[Tuple[str, int]], include_zeros: bool, hide_tff: bool,
                reads_before_error: Optional[Sequence[Tuple[int, int]]] = None) -> List[str]:
    """Counts.lines (Counts.scala:80-127): fields sorted by value, descending, ties in field order (stable)."""
    rows = [(k, str(v)) for k, v in sorted(pairs, key=lambda kv: -kv[1])
            if (v > 0 or include_zeros) and (k != "tooFewFixedBlockBytes" or not hide_tff)]
    if reads_before_error:
        rows.append(("readsBeforeError", " ".join(f"{r}ⅹ{n}" for r, n in sorted(reads_before_error))))
    if not rows:
        return []
    mk = max(len(k) for k, _ in rows)
    mv = max(len(v) for _, v in rows)
    return [f"{' ' * (mk - len(k))}{k}:\t{' ' * (mv - len(v))}{v}" for k, v in rows]


def print_limited(out: List[str], items: Sequence[str], total: Optional[int], header: str, trunc_header,
                  limit: int, indent: str = ""):
    """hammerlab cli `print(...)`: header, then at most `limit` indented items and `…` when truncated."""
    n_total = len(items) if total is None else total
    if n_total > limit:
        out.append(indent + trunc_header(limit))
        out.extend(indent + "\t" + x for x in items[:limit])
        out.append(indent + "\t…")
    else:
        out.append(indent + header)
        out.extend(indent + "\t" + x for x in items)


# ---- record display (PosMetadata.showRecord over htsjdk SAMRecord.toString) -------------------------------
def show_record(rec: bytes, contig_names: Sequence[str]) -> str:
    ref = int.from_bytes(rec[4:8], "little", signed=True)
    pos = int.from_bytes(rec[8:12], "little", signed=True)
    lrn = rec[12]
    flag = int.from_bytes(rec[18:20], "little")
    l_seq = int.from_bytes(rec[20:24], "little", signed=True)
    name = rec[36:36 + max(lrn - 1, 0)].decode("latin-1")
    s = name
    if flag & 1:
        s += " 1/2" if flag & 0x40 else " 2/2"
    s += f" {l_seq}b"
    unmapped = bool(flag & 4)
    s += " unmapped read" if unmapped else " aligned read"  # SAMRecord.toString minus its trailing '.'
    start = pos + 1  # getStart: 1-based alignment start
    where = f"{contig_names[ref] if 0 <= ref < len(contig_names) else ref}:{start}"
    if unmapped and start >= 0 and 0 <= ref < len(contig_names):
        s += f" (placed at {where})"
    elif not unmapped:
        s += f" @ {where}"
    return s


# ---- full-check ----------------------------------------------------------------------------------------------
@dataclass
class FullCheckParts:
    """One byte range's share of a full-check report (the whole file, or one shard of `full-check --gpus N`):
    Counts, the first `limit` close calls of keys 1 and 2 as PosMetadata lines, and the comparison with the
    `.records` truth.  Parts of consecutive ranges merge in file order (merge_parts) — Spark's reduceByKey of Counts
    and the driver's take(limit) of the sampled positions (FullCheck.scala:141-191, CheckerApp.scala:140-222)."""
    totals: np.ndarray      # (19,)
    by_key: np.ndarray      # (21, 19): keys 1-2 exact (the report prints only those)
    positions: np.ndarray   # (21,)
    rbe: np.ndarray         # (21, 128) readsBeforeError by key
    pair: np.ndarray        # (19, 19) close-call flag pairs
    n_positions: int
    compressed: int
    close: dict             # key -> PosMetadata lines of the first `limit` positions with that key
    truth: Optional[dict]   # {"tp", "fp": [(F, PosMetadata line or None)], "fn": [Pos text]} with a .records file


def merge_parts(parts: Sequence[FullCheckParts], limit: int) -> FullCheckParts:
    """Shards in file order → one report's parts (counts summed, sampled lines concatenated and cut to `limit`)."""
    def add(name):
        return sum(getattr(q, name) for q in parts)
    close = {k: [ln for q in parts for ln in q.close.get(k, [])][:limit] for k in (1, 2)}
    truth = None
    if parts and all(q.truth is not None for q in parts):
        fp = [x for q in parts for x in q.truth["fp"]]
        truth = {"tp": sum(q.truth["tp"] for q in parts), "fp": fp,
                 "fn": [x for q in parts for x in q.truth["fn"]]}
    return FullCheckParts(add("totals"), add("by_key"), add("positions"), add("rbe"), add("pair"),
                          add("n_positions"), add("compressed"), close, truth)


def truth_lines(n_positions: int, compressed: int, tp: int, fps: Sequence[Tuple[int, Optional[str]]],
                fns: Sequence[str], limit: int) -> List[str]:
    """CheckerApp.scala:140-222: positions, compressed size, ratio, reads, then the comparison of the calls with the
    `.records` truth (lines, false-positive flags histogram and sites, false-negative positions)."""
    ratio = n_positions / compressed if compressed else float("nan")
    out = [f"{n_positions} uncompressed positions", f"{format_bytes(compressed)} compressed",
           "Compression ratio: %.2f" % ratio, f"{tp + len(fns)} reads"]
    if not fps and not fns:
        out.append("All calls matched!")
        return out
    out += [f"{len(fps)} false positives, {len(fns)} false negatives", ""]
    if fps:
        hist = {}
        for F, _ in fps:
            hist[F] = hist.get(F, 0) + 1
        rows = sorted(hist.items(), key=lambda kv: -kv[1])
        print_limited(out, [f"{n}:\t{show_flags(F)}" for F, n in rows], None,
                      "False-positive-site flags histogram:", lambda _: "False-positive-site flags histogram:", limit)
        out.append("")
        items = [ln for _, ln in fps[:limit]]
        print_limited(out, items, len(fps), "False positives with succeeding read info:",
                      lambda n: f"{n} of {len(fps)} false positives with succeeding read info::", limit)
    if fns:
        print_limited(out, list(fns[:limit]), len(fns), f"{len(fns)} false negatives:",
                      lambda n: f"{n} of {len(fns)} false negatives:", limit)
    return out


def full_check_lines(p: FullCheckParts, limit: int) -> List[str]:
    """FullCheck.scala:141-322 report text from (merged) parts."""
    out = []
    if p.truth is not None:
        fp, fn = p.truth["fp"], p.truth["fn"]
        if fp or fn:  # FullCheck.scala:108-114: a full-check call disagreeing with the records is an error
            raise RuntimeError(f"{len(fp)} false positives, {len(fn)} false negatives against the .records truth")
        out += truth_lines(p.n_positions, p.compressed, p.truth["tp"], fp, fn, limit) + [""]
    field_names = FLAG_NAMES[:19]

    def pairs(vec):
        return [(field_names[i], int(vec[i])) for i in range(19)]

    npos = p.positions
    if npos[1] > 0:  # critical (key-1) section, FullCheck.scala:230-258
        out.append("Critical error counts (true negatives where only one check failed):")
        out += ["\t" + l for l in count_lines(pairs(p.by_key[1]), False, False)]
        out.append("")
        n1 = int(npos[1])
        print_limited(out, p.close[1], n1, f"{n1} critical positions:",
                      lambda n: f"{n} of {n1} critical positions:", limit)
    else:
        out.append("No positions where only one check failed")
    out.append("")
    if npos[2] > 0:  # close calls (key 2), FullCheck.scala:262-306
        n2 = int(npos[2])
        print_limited(out, p.close[2], n2, f"{n2} positions where exactly two checks failed:",
                      lambda n: f"{n} of {n2} positions where exactly two checks failed:", limit)
        out.append("")
        hist = []
        for i in range(19):
            for j in range(19):
                if p.pair[i, j]:
                    hist.append((int(p.pair[i, j]), (1 << i) | (1 << j)))
        hist.sort(key=lambda t: -t[0])  # stable: reduceByKey output order is not pinned beyond the counts
        if hist and hist[0][0] > 1:
            print_limited(out, [f"{n}:\t{show_flags(F)}" for n, F in hist], None, "Histogram:",
                          lambda _: "Histogram:", limit, indent="\t")
            out.append("")
        out.append("\tPer-flag totals:")
        out += ["\t\t" + l for l in count_lines(pairs(p.by_key[2]), False, False)]
        out.append("")
    else:
        out += ["No positions where exactly two checks failed", ""]
    rb = [(k, int(p.rbe[:, k].sum())) for k in range(1, 128) if p.rbe[:, k].sum()]
    out.append("Total error counts:")
    out += ["\t" + l for l in count_lines(pairs(p.totals), True, True, rb)]
    out.append("")
    return out


class FullCheckReport:
    """full-check over the blocks selected by `ranges` (None = whole file) of one context.  `blocks` (a block-index
    mask) restricts it further to the blocks a shard owns; `names` = the header's contig names (a shard's stream
    does not start at the header)."""

    def __init__(self, f: sbam.BamFile, data: Optional[bytes], records_path: Optional[str], limit: int = 10,
                 ranges: Optional[List[Tuple[int, int]]] = None, reads_to_check: int = 10,
                 blocks: Optional[np.ndarray] = None, names: Optional[List[str]] = None):
        self.f, self.data, self.limit, self.R = f, data, limit, reads_to_check
        st, cs, us, uo = f.blocks()
        sel = np.ones(st.size, bool) if ranges is None else \
            np.any([(st >= lo) & (st < hi) for lo, hi in ranges], axis=0)
        if blocks is not None:
            sel &= blocks
        self.block_starts = set(st[sel].tolist())
        self.runs = self._runs(np.nonzero(sel)[0], uo, us)
        self.compressed = int(cs[sel].astype(np.int64).sum())
        self.records_path = records_path
        self.names = header_names(f) if names is None else names

    @staticmethod
    def _runs(idx, uo, us):
        """contiguous block-index runs → uncompressed [x0, x1) ranges"""
        runs = []
        for b in idx.tolist():
            x0, x1 = int(uo[b]), int(uo[b]) + int(us[b])
            if runs and runs[-1][1] == x0:
                runs[-1][1] = x1
            else:
                runs.append([x0, x1])
        return [(a, b) for a, b in runs]

    def close_calls(self, key: int, want: int) -> List[Tuple[int, int]]:
        """First `want` positions (file order) whose result has exactly `key` non-zero fields."""
        got = []
        if want <= 0:
            return got
        chunk = 1 << 24
        for x0, x1 in self.runs:
            for a in range(x0, x1, chunk):
                b = min(x1, a + chunk)
                w = self.f.check_full_words(a, b, self.R)
                F = (w & 0x7ffff).astype(np.uint32)
                kk = (w >> 24) & 0x7f
                pop = np.zeros(F.size, np.int64)
                for i in range(19):
                    pop += (F >> i) & 1
                counted = ((w & 0x80000000) == 0) & ~((F == 1) & (kk == 0))
                hit = np.nonzero(counted & (pop + (kk > 0) == key))[0]
                for h in hit[: want - len(got)].tolist():
                    got.append((a + h, int(w[h])))
                if len(got) >= want:
                    return got
        return got

    def pos_metadata(self, x: int, w: int) -> str:
        p = self.f.pos_of(x)
        nxt = self.next_record(x)
        if nxt is None:
            desc = "no next record"
        else:
            y, delta = nxt
            bs = int.from_bytes(self.f.read_uncompressed(y, 4), "little", signed=True)
            desc = f"{delta} before {show_record(self.f.read_uncompressed(y, 4 + bs), self.names)}"
        return f"{p}:\t{desc}. Failing checks: {show_flags(w & 0x7ffff)}"

    def next_record(self, x: int, max_read_size: int = 10_000_000):
        """FindRecordStart.withDelta(pos) (FindRecordStart.scala:30-63): first eager-true offset >= x.  A search that
        runs past a shard's loaded bytes raises HaloException (the shard grows its halo and re-runs)."""
        L = self.f.uncompressed_size
        lim = min(L, x + max_read_size)
        a, step = x, 1 << 20
        while a < lim:
            b = min(lim, a + step)
            calls = self.f.check_eager(a, b, self.R)
            hit = np.nonzero(calls)[0]
            if hit.size:
                return a + int(hit[0]), a + int(hit[0]) - x
            a = b
        if lim < x + max_read_size and not getattr(self.f, "loads_to_eof", True):
            raise sbam.HaloException(f"next record after {x} lies past the loaded bytes")
        return None

    def truth(self) -> set:
        """The `.records` positions (IndexRecords.scala) inside this report's blocks, as stream offsets."""
        out = set()
        for line in open(self.records_path):
            if line.strip():
                b, o = (int(v) for v in line.split(","))
                if b in self.block_starts:
                    out.add(self.f.offset_of(Pos(b, o)))
        return out

    def compare(self, calls_bits):
        """(tp, false-positive offsets, false-negative offsets) of the calls against the `.records` truth."""
        truth = self.truth()
        tp, fps, fns = 0, [], []
        for x0, bits in calls_bits:
            called = set((x0 + np.nonzero(bits)[0]).tolist())
            expected = {t for t in truth if x0 <= t < x0 + bits.size}
            tp += len(called & expected)
            fps += sorted(called - expected)
            fns += sorted(expected - called)
        return tp, fps, fns

    def truth_part(self, calls_bits) -> dict:
        tp, fps, fns = self.compare(calls_bits)
        words = {x: int(self.f.check_full_words(x, x + 1, self.R)[0]) for x in fps}
        fp = [(words[x] & 0x7ffff, self.pos_metadata(x, words[x]) if i < self.limit else None)
              for i, x in enumerate(fps)]
        return {"tp": tp, "fp": fp, "fn": [str(self.f.pos_of(x)) for x in fns]}

    def check_bam_lines(self) -> List[str]:
        """check-bam -s (eager/CheckBam.scala, vsIndexed): the eager checker at every position of the selected
        blocks against the `.records` truth."""
        calls_bits = [(x0, self.f.check_eager(x0, x1, self.R)) for x0, x1 in self.runs]
        n_positions = sum(x1 - x0 for x0, x1 in self.runs)
        t = self.truth_part(calls_bits)
        return truth_lines(n_positions, self.compressed, t["tp"], t["fp"], t["fn"], self.limit)

    def parts(self) -> FullCheckParts:
        """The full checker over every position of the selected blocks (Counts by the bit-sliced counts path: keys
        1-2 per flag, positions per key, pairs, readsBeforeError, totals) plus the sampled close calls."""
        by_key = np.zeros((21, 19), np.int64)
        npos = np.zeros(21, np.int64)
        totals = np.zeros(19, np.int64)
        rbe = np.zeros((21, 128), np.int64)
        pair = np.zeros((19, 19), np.int64)
        n_positions = 0
        calls_bits = []
        has_truth = bool(self.records_path) and os.path.exists(self.records_path)
        for x0, x1 in self.runs:
            c, bits = self.f.check_full_counts(x0, x1, self.R, want_bitmap=True)
            by_key += c.by_key
            npos += c.positions
            totals += c.totals
            rbe += c.reads_before_error
            pair += c.pair_hist
            n_positions += x1 - x0
            calls_bits.append((x0, bits))
        close = {k: [self.pos_metadata(x, w) for x, w in self.close_calls(k, min(self.limit, int(npos[k])))]
                 for k in (1, 2)}
        truth = self.truth_part(calls_bits) if has_truth else None
        return FullCheckParts(totals, by_key, npos, rbe, pair, n_positions, self.compressed, close, truth)

    def lines(self) -> List[str]:
        return full_check_lines(self.parts(), self.limit)


def header_names(f: sbam.BamFile) -> List[str]:
    """Contig names from the BAM header in the device stream (check/.../bam/header/Header.scala:26-60)."""
    u = f.read_uncompressed(0, min(f.uncompressed_size, 1 << 20))
    if u[:4] != b"BAM\x01":
        return []
    lt = int.from_bytes(u[4:8], "little")
    p = 8 + lt
    n = int.from_bytes(u[p:p + 4], "little")
    p += 4
    names = []
    for _ in range(n):
        ln = int.from_bytes(u[p:p + 4], "little")
        names.append(u[p + 4:p + 4 + ln - 1].decode("latin-1"))
        p += 4 + ln + 4
    return names


# ---- compute-splits / count-reads ------------------------------------------------------------------------
def split_length(s: sbam.Split) -> int:
    """Split.length = Pos.-(end, start) (bgzf/.../Pos.scala:17-22), then .toInt in ComputeSplits."""
    return int(max(0, s.end.block_pos - s.start.block_pos + math.trunc((s.end.offset - s.start.offset) / RATIO)))


def _num(v: float) -> str:
    r = round(v, 1)
    return str(int(r)) if r == int(r) else f"{r:.1f}"


def stats_lines(xs: Sequence[int]) -> List[str]:
    """hammerlab Stats for a small sample (the form ComputeSplitsTest pins): N, mean/population σ,
    median/MAD, elements and sorted elements.  (Stats' histogram form for large N is not pinned by any
    reference fixture.)"""
    a = np.asarray(xs, np.float64)
    n = a.size
    if n == 0:
        return ["N: 0"]
    mean = a.mean()
    sd = math.sqrt(((a - mean) ** 2).mean())
    med = float(np.median(a))
    mad = float(np.median(np.abs(a - med)))
    return [f"N: {n}, μ/σ: {_num(mean)}/{_num(sd)}, med/mad: {_num(med)}/{_num(mad)}",
            " elems: " + " ".join(str(int(v)) for v in xs),
            "sorted: " + " ".join(str(int(v)) for v in sorted(xs))]


def compute_splits_lines(f: sbam.BamFile, split_size: int, limit: int) -> List[str]:
    t = time.perf_counter()
    splits = f.compute_splits(split_size)
    return splits_report(splits, int((time.perf_counter() - t) * 1e3), limit)


def splits_report(splits, ms: int, limit: int) -> List[str]:
    """ComputeSplits.scala:56-68 report text for a list of splits found in `ms` milliseconds."""
    out = [f"Get spark-bam splits: {ms}ms", "", "Split-size distribution:"]
    out += stats_lines([split_length(s) for s in splits])
    out.append("")
    items = [str(s) for s in splits]
    print_limited(out, items, None, f"{len(splits)} splits:", lambda n: f"First {n} of {len(splits)} splits:", limit)
    out.append("")
    return out


def count_reads_lines(f: sbam.BamFile, split_size: int) -> List[str]:
    t = time.perf_counter()
    n = sum(f.partition_sizes(split_size))
    return count_report(n, int((time.perf_counter() - t) * 1e3))


def count_report(n: int, ms: int) -> List[str]:
    """CountReads.scala:80-100 report text (spark-bam side)."""
    return [f"spark-bam read-count time: {ms}", "", f"spark-bam found {n} reads", ""]


def spawn_ranks(n: int, argv: Sequence[str]) -> int:
    """`--gpus N` outside torchrun: N ranks of this command under torch.distributed.run (one per GPU), started
    before this process touches a GPU."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = pkg + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "-m", "sbam.cli"] + list(argv)
    return subprocess.call(cmd, env=env)


def sharded_lines(a) -> Optional[List[str]]:
    """compute-splits / count-reads / full-check over byte-range shards, one rank per GPU (sbam.dist.run_file /
    full_check_file: rank 0 reads the header, each rank preads its shard, the results meet in tiny collectives).
    Returns the report on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    from sbam import dist as sdist
    local = int(os.environ.get("LOCAL_RANK", 0)) if a.device is None else a.device
    torch.cuda.set_device(local)
    if a.dist_backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        coll = torch.device("cuda", local)
    else:  # gloo: rehearse N ranks on one GPU (--device), small collectives on the host
        dist.init_process_group(a.dist_backend)
        coll = None
    try:
        if a.cmd == "full-check":
            parts = sdist.full_check_file(a.bam, a.print_limit, a.intervals, a.reads_to_check, device=local,
                                          coll_device=coll, records_path=a.bam + ".records")
            return full_check_lines(parts, a.print_limit) if dist.get_rank() == 0 else None
        t = time.perf_counter()
        r = sdist.run_file(a.bam, sbam.effective_split_size(a.max_split_size), device=local, coll_device=coll)
        ms = int((time.perf_counter() - t) * 1e3)
        if dist.get_rank() != 0:
            return None
        if a.cmd == "compute-splits":
            return splits_report(r.splits, ms, a.print_limit)
        return count_report(sum(r.partition_sizes), ms)
    finally:
        dist.destroy_process_group()


# ---- check-blocks -s / index-blocks / index-records ------------------------------------------------------------
def _jround(v: float) -> int:
    """java.lang.Math.round: floor(x + 0.5)."""
    return int(math.floor(v + 0.5))


def hist_stats_lines(hist: Sequence[Tuple[int, int]]) -> List[str]:
    """hammerlab Stats.fromHist with Show[Double] = math.round (CheckBlocks.scala:135-150): N, mean/population σ,
    median/MAD; the (value, count) entries in value order (`v×c` for repeats, first 10 … last 10 past 20
    entries); percentiles by linear interpolation at rank p(N+1)/100, printed for the p whose rank lies in
    [1, N].  Pinned by the CheckBlocksTest goldens (N = 25); other sizes are parity unpinned."""
    hist = sorted((int(v), int(c)) for v, c in hist if c > 0)
    vals = np.repeat(np.array([v for v, _ in hist], np.float64), [c for _, c in hist])
    n = vals.size
    if n == 0:
        return ["N: 0"]
    mean = vals.mean()
    sd = math.sqrt(((vals - mean) ** 2).mean())
    med = float(np.median(vals))
    mad = float(np.median(np.abs(vals - med)))
    out = [f"N: {n}, μ/σ: {_jround(mean)}/{_jround(sd)}, med/mad: {_jround(med)}/{_jround(mad)}"]
    ent = [str(v) if c == 1 else f"{v}×{c}" for v, c in hist]
    if len(ent) > 20:
        ent = ent[:10] + ["…"] + ent[-10:]
    out.append(" elems: " + " ".join(ent))
    for p in (1, 5, 10, 25, 50, 75, 90, 95, 99):
        r = p * (n + 1) / 100.0
        if r < 1 or r > n:
            continue
        i = int(math.floor(r)) - 1
        v = vals[i] + (r - 1 - i) * (vals[min(i + 1, n - 1)] - vals[i])
        out.append(f"{p:>4}:\t{_jround(v)}")
    return out


def _next_start(sorted_offs: np.ndarray, x: int) -> Optional[int]:
    i = int(np.searchsorted(sorted_offs, x))
    return int(sorted_offs[i]) if i < sorted_offs.size else None


def check_blocks_lines(f: sbam.BamFile, truth_offsets: np.ndarray, limit: int,
                       reads_to_check: int = sbam.READS_TO_CHECK) -> List[str]:
    """check-blocks -s (cli/.../check/blocks/CheckBlocks.scala:37-190): per BGZF block, the eager checker's
    nextReadStart(Pos(start, 0)) (GPU bitmap) against the indexed checker's (the `.records` truth,
    check/.../indexed/Checker.scala:12-27); blocks whose answers differ, weighted by the previous block's
    compressed size, and the histogram of the blocks' first-read offsets."""
    st, cs, us, uo = f.blocks()
    L = f.uncompressed_size
    eager = np.flatnonzero(f.check_eager(0, L, reads_to_check)).astype(np.int64)
    truth = np.sort(np.asarray(truth_offsets, np.int64))
    by_start = {int(st[b]): int(uo[b]) for b in range(st.size)}

    def finder(offs):
        def next_read_start(p: sbam.Pos) -> Optional[sbam.Pos]:
            x = _next_start(offs, by_start[p.block_pos] + p.offset)
            return None if x is None else f.pos_of(x)
        return next_read_start

    blocks = [(int(st[b]), int(cs[b])) for b in range(st.size)]
    return check_blocks_report(blocks, finder(eager), finder(truth), f.file_size, limit)


def check_blocks_report(blocks: Sequence[Tuple[int, int]], next1: Callable[[sbam.Pos], Optional[sbam.Pos]],
                        next2: Callable[[sbam.Pos], Optional[sbam.Pos]], size: int, limit: int) -> List[str]:
    """CheckBlocks.callPartition + run (CheckBlocks.scala:37-190) over (start, compressedSize) blocks in file order and
    two ReadStartFinders' nextReadStart (e.g. sbam.checker.LazyBlockChecker and IndexedChecker): the report text."""
    bad, offs = [], {}
    for b, (start, _) in enumerate(blocks):
        p1, p2 = next1(sbam.Pos(start, 0)), next2(sbam.Pos(start, 0))
        off = p1.offset if p1 is not None and p1.block_pos == start else None
        offs[off] = offs.get(off, 0) + 1
        if (str(p1) if p1 else None) != (str(p2) if p2 else None):
            bad.append((start, p1, p2, blocks[b - 1][1] if b > 0 else 1))
    n_blocks = len(blocks)
    out: List[str] = []

    def offsets_info():
        keys = set(offs)
        if keys == {None, 0}:
            out.extend(["", f"{offs[0]} blocks start with a read, {offs[None]} blocks didn't contain a read"])
        elif keys == {0}:
            out.extend(["", "All blocks start with reads"])
        else:
            out.extend(["", f"Offsets of blocks' first reads ({offs.get(None, 0)} blocks didn't contain a read "
                            "start):"])
            out.extend(hist_stats_lines([(k, v) for k, v in offs.items() if k is not None]))

    if not bad:
        out.append(f"First read-position matched in {n_blocks} BGZF blocks totaling {format_bytes(size)}B "
                   "(compressed)")
        offsets_info()
    else:
        wc = sum(w for *_, w in bad)
        out += [f"First read-position mismatched in {len(bad)} of {n_blocks} BGZF blocks", "",
                f"{wc} of {size} ({repr(wc / size)}) compressed positions would lead to bad splits"]
        offsets_info()
        out.append("")
        items = [f"{s} (prev block size: {w}):\t{p1 if p1 else '-'}\t{p2 if p2 else '-'}" for s, p1, p2, w in bad]
        print_limited(out, items, None, f"{len(bad)} mismatched blocks:",
                      lambda n: f"{n} of {len(bad)} mismatched blocks:", limit)
    return out


def index_blocks_lines(f: sbam.BamFile) -> List[str]:
    """IndexBlocks (bgzf/.../index/IndexBlocks.scala:24-45): `start,compressedSize,uncompressedSize` per block of
    the MetadataStream (which stops at the first empty block), from the GPU header scan."""
    st, cs, us, _ = f.blocks()
    return [f"{a},{b},{c}" for a, b, c in zip(st.tolist(), cs.tolist(), us.tolist())]


def index_records_lines(f: sbam.BamFile) -> List[str]:
    """IndexRecords (check/.../bam/index/IndexRecords.scala:36-90, PosStream): `blockPos,offset` of every record
    start from the end of the BAM header, chained by block_size (PosStream.scala:14-22).  PosStream emits a
    record's Pos once its 4-byte block_size is read and drops the rest lazily, so a truncated last record is
    still listed and ends the stream.  (A negative block_size, which PosStream would step over by 4 bytes, ends
    the listing here: parity unpinned, no fixture has one.)"""
    f.header()
    L = f.uncompressed_size
    x0 = f.offset_of(f.header_end)
    offs = [int(x) for x in f.record_offsets(x0, L)]
    x = x0
    if offs:
        x = offs[-1] + 4 + int.from_bytes(f.read_uncompressed(offs[-1], 4), "little", signed=True)
    if x + 4 <= L and int.from_bytes(f.read_uncompressed(x, 4), "little", signed=True) >= 0:
        offs.append(x)  # truncated last record
    return [str(f.pos_of(x)).replace(":", ",") for x in offs]


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="sbam.cli")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("full-check", "check-bam", "check-blocks", "compute-splits", "count-reads", "index-blocks",
                 "index-records"):
        p = sub.add_parser(name)
        p.add_argument("-l", "--print-limit", type=int, default=10)
        # check-blocks defaults to 2 MB (blocks/CheckBlocks.scala via Blocks.scala:64); compute-splits and
        # count-reads to the FileSystem's split size (args/SplitSize.scala:10-17)
        p.add_argument("-m", "--max-split-size", type=parse_bytes, default=(2 << 20) if name == "check-blocks" else None)
        p.add_argument("bam")
        p.add_argument("out", nargs="?")
        if name in ("full-check", "check-bam"):
            p.add_argument("-i", "--intervals", type=parse_ranges, default=None)
            p.add_argument("-r", "--reads-to-check", type=int, default=10)
        if name in ("compute-splits", "check-bam", "check-blocks"):
            p.add_argument("-s", "--spark-bam", action="store_true")
        if name == "full-check":
            p.add_argument("--windows", type=int, default=1,
                           help="byte-range shards run one after another on one GPU (files larger than HBM); "
                                "0 = as many as the file's size, compression ratio and free HBM need")
        if name in ("compute-splits", "count-reads", "full-check"):
            p.add_argument("--gpus", type=int, default=1, help="byte-range shards, one rank per GPU")
            p.add_argument("--dist-backend", default="nccl", help="nccl (RCCL); gloo to rehearse ranks on one GPU")
            p.add_argument("--device", type=int, default=None, help="GPU of every rank (default LOCAL_RANK)")
    a = ap.parse_args(argv)
    if getattr(a, "gpus", 1) > 1:
        if "WORLD_SIZE" not in os.environ:
            return spawn_ranks(a.gpus, sys.argv[1:] if argv is None else argv)
        lines = sharded_lines(a)
        if lines is not None:
            text = "\n".join(lines) + "\n"
            if a.out:
                open(a.out, "w").write(text)
            else:
                sys.stdout.write(text)
        return 0
    dev = getattr(a, "device", None) or 0
    if a.cmd == "full-check" and a.windows == 0:
        from sbam import dist as sdist
        src, size = sdist.file_source(a.bam)
        # the budget leaves room for halo retries: a window's halo can grow 4x per HaloException (2 -> 8 -> 32 MiB
        # of compressed bytes and beyond), each compressed byte costing hbm_bytes_per_compressed_byte in HBM
        margin = int(sdist.hbm_bytes_per_compressed_byte(3.3) * (128 << 20))
        a.windows = sdist.auto_windows(size, src, max(1, sdist.device_free_bytes(dev) - margin), contexts=1)
    if a.cmd == "full-check" and a.windows > 1:
        from sbam import dist as sdist
        parts = sdist.full_check_file(a.bam, a.print_limit, a.intervals, a.reads_to_check, world=a.windows,
                                      device=dev, records_path=a.bam + ".records")
        text = "\n".join(full_check_lines(parts, a.print_limit)) + "\n"
        if a.out:
            open(a.out, "w").write(text)
        else:
            sys.stdout.write(text)
        return 0
    data = open(a.bam, "rb").read()
    with sbam.BamFile(data, path=a.bam, device=dev) as f:
        if a.cmd == "full-check":
            rep = FullCheckReport(f, data, a.bam + ".records", a.print_limit, a.intervals, a.reads_to_check)
            lines = rep.lines()
        elif a.cmd == "check-bam":
            rep = FullCheckReport(f, data, a.bam + ".records", a.print_limit, a.intervals, a.reads_to_check)
            if not os.path.exists(rep.records_path):
                raise SystemExit(f"check-bam -s needs the indexed records {rep.records_path} (index-records)")
            lines = rep.check_bam_lines()
        elif a.cmd == "check-blocks":
            rp = a.bam + ".records"
            if not a.spark_bam or not os.path.exists(rp):
                raise SystemExit("check-blocks runs as -s (spark-bam eager checker vs the indexed records "
                                 f"{rp}); the hadoop-bam comparison is out of scope")
            truth = [f.offset_of(Pos(*(int(v) for v in ln.split(",")))) for ln in open(rp) if ln.strip()]
            lines = check_blocks_lines(f, np.asarray(truth, np.int64), a.print_limit)
        elif a.cmd == "index-blocks":
            lines = index_blocks_lines(f)
        elif a.cmd == "index-records":
            lines = index_records_lines(f)
        elif a.cmd == "compute-splits":
            lines = compute_splits_lines(f, sbam.effective_split_size(a.max_split_size), a.print_limit)
        else:
            lines = count_reads_lines(f, sbam.effective_split_size(a.max_split_size))
    text = "\n".join(lines) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    else:
        sys.stdout.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Inflate fuzz corpus: BGZF blocks of mixed inputs compressed by Python's zlib over every level,
strategy, memLevel and window size, checked block by block against the CRC32 / ISIZE of their own footers after the
GPU inflate (k_inflate_wave, k_inflate_slow, k_inflate_resolve).  The reference inflates each block with
java.util.zip.Inflater (bgzf/src/main/scala/org/hammerlab/bgzf/block/Stream.scala:49-54); a BGZF footer's CRC32 is
that inflate's expected output, so a matching CRC is parity with zlib for valid streams.

    inflate_fuzz.py [--blocks N] [--seed S] [--workers W] [--json]

With SBAM_LIB pointing at the wave-statistics build (make -C spark-bam_amd EXTRA=-DSBAM_WAVE_STATS
BUILD=build_stats) it also reports how the wave decoder's rare paths were exercised: lanes that re-decoded in phase B
(modes R / F), rounds with a mode-F lane, lanes with more than 64 / 96 tokens (the tails past the register tokens),
rounds with a stop.  The corpus is generated in worker processes (the GPU box gives a job 16 host threads)."""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import time
import zlib
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402

STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]
KINDS = ["bam", "text", "random", "runs", "dna", "quals", "mixed"]


def deflate(payload: bytes, level: int, strategy: int, mem: int, wbits: int) -> bytes:
    co = zlib.compressobj(level, zlib.DEFLATED, -wbits, mem, strategy)
    return co.compress(payload) + co.flush()


def bgzf_block(payload: bytes, level: int, strategy: int, mem: int, wbits: int) -> bytes:
    data = deflate(payload, level, strategy, mem, wbits)
    hdr = b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<HBBHH", 6, 66, 67, 2, 18 + len(data) + 8 - 1)
    return hdr + data + struct.pack("<II", zlib.crc32(payload), len(payload))


def _payload(rng: np.random.Generator, kind: str, n: int, bam: np.ndarray) -> bytes:
    if kind == "bam":  # a slice of a synthetic BAM's uncompressed stream
        a = int(rng.integers(0, bam.size - n))
        return bam[a:a + n].tobytes()
    if kind == "text":
        words = [b"chr%d" % i for i in range(1, 23)] + [b"ACGT", b"read", b"\t", b"\n", b"60M", b"*", b"=", b"0"]
        out = bytearray()
        while len(out) < n:
            out += words[int(rng.integers(0, len(words)))]
        return bytes(out[:n])
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "runs":
        out = bytearray()
        while len(out) < n:
            out += bytes([int(rng.integers(0, 256))]) * int(rng.integers(1, 700))
        return bytes(out[:n])
    if kind == "dna":
        return np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)].tobytes()
    if kind == "quals":  # binned qualities with runs
        q = np.frombuffer(b"#+5?FFFFF:", np.uint8)[rng.integers(0, 10, n)]
        return q.tobytes()
    # mixed: pieces of the other kinds
    out = bytearray()
    while len(out) < n:
        k = KINDS[int(rng.integers(0, len(KINDS) - 1))]
        out += _payload(rng, k, min(n - len(out), int(rng.integers(1, 4096))), bam)
    return bytes(out[:n])


def _make(args):
    seed, count, bam_bytes = args
    rng = np.random.default_rng(seed)
    bam = np.frombuffer(bam_bytes, np.uint8)
    blocks, meta = [], []
    for _ in range(count):
        kind = KINDS[int(rng.integers(0, len(KINDS)))]
        r = rng.random()
        n = int(rng.integers(1, 64)) if r < 0.1 else int(rng.integers(64, 4096)) if r < 0.6 else \
            int(rng.integers(4096, 32768)) if r < 0.92 else int(rng.integers(32768, 65281)) if r < 0.97 else 65280
        level = int(rng.integers(0, 10))
        strat = STRATEGIES[int(rng.integers(0, len(STRATEGIES)))]
        mem = int(rng.integers(1, 10))
        wbits = int(rng.integers(9, 16))
        p = _payload(rng, kind, n, bam)
        while len(deflate(p, level, strat, mem, wbits)) + 26 > 65536:  # BSIZE is a u16: shorten incompressible input
            p = p[: len(p) * 7 // 8]
        n = len(p)
        blocks.append(bgzf_block(p, level, strat, mem, wbits))
        meta.append((kind, level, strat, mem, wbits, n))
    return b"".join(blocks), meta


def bgzf_inflate(raw: bytes) -> bytes:
    """The uncompressed stream of a BGZF file (Python zlib, block by block: BSIZE at +16)."""
    out, pos = [], 0
    while pos + 18 <= len(raw):
        end = pos + (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
        xlen = raw[pos + 10] | (raw[pos + 11] << 8)
        out.append(zlib.decompressobj(-15).decompress(raw[pos + 12 + xlen:end - 8]))
        pos = end
    return b"".join(out)


def make_corpus(n_blocks: int, seed: int = 1, workers: int = 16, per_task: int = 2000):
    """(BGZF bytes ending in the EOF marker block, per-block metadata): n_blocks blocks, no empty block before the
    end (the block stream stops at the first empty block: MetadataStream)."""
    import synth
    ub = bgzf_inflate(synth.SynthBam(tile_mb=16.0, seed=seed).bytes().tobytes())
    tasks = [(seed * 1_000_003 + i, min(per_task, n_blocks - i * per_task), ub)
             for i in range((n_blocks + per_task - 1) // per_task)]
    with ProcessPoolExecutor(max_workers=workers) as ex:
        parts = list(ex.map(_make, tasks))
    data = b"".join(p[0] for p in parts) + bgzf_block(b"", 6, 0, 8, 15)
    meta = [m for p in parts for m in p[1]]
    return data, meta


def check(data: bytes, meta) -> dict:
    """Inflate the corpus on the GPU; per block, CRC32 and ISIZE of its output against its footer."""
    import sbam
    f = sbam.BamFile(data, inflate=False, path="fuzz.bgzf")
    t0 = time.perf_counter()
    f.inflate()
    dt = time.perf_counter() - t0
    st, cs, us, uo = f.blocks()
    u = np.frombuffer(f.read_uncompressed(0, f.uncompressed_size), np.uint8)
    raw = np.frombuffer(data, np.uint8)
    bad = []
    for b in range(st.size):
        e = int(st[b]) + int(cs[b])
        crc, isz = struct.unpack("<II", raw[e - 8:e].tobytes())
        if int(us[b]) != isz or zlib.crc32(u[int(uo[b]):int(uo[b]) + isz]) != crc:
            bad.append(b)
    out = {"blocks": int(st.size), "expected_blocks": len(meta),  # (the EOF marker ends the stream: not a block)
           "uncompressed_bytes": int(f.uncompressed_size),
           "mismatches": len(bad), "first_mismatches": [(int(b), meta[b] if b < len(meta) else None) for b in bad[:10]],
           "exact_path_blocks": f.inflate_fallbacks(), "inflate_wall_s": round(dt, 3),
           "decode_ms": round(f.kernel_ms("inflate_decode"), 3), "resolve_ms": round(f.kernel_ms("inflate_resolve"), 3)}
    kinds = {}
    for m in meta:
        kinds[m[0]] = kinds.get(m[0], 0) + 1
    out["by_kind"] = kinds
    out["by_level"] = {lv: sum(1 for m in meta if m[1] == lv) for lv in range(10)}
    out["by_strategy"] = {str(s): sum(1 for m in meta if m[2] == s) for s in STRATEGIES}
    L = sbam.load_library()
    if hasattr(L, "sbam_debug_wave_stats"):  # the wave-statistics build: how often the rare paths ran
        import ctypes
        fn = L.sbam_debug_wave_stats
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
        buf = (ctypes.c_ulonglong * 40)()
        fn(buf, 1)
        f.reset()
        f._scan()
        f.inflate()
        fn(buf, 1)
        v = list(buf)
        out["wave_stats"] = {n: int(v[i]) for i, n in (
            (6, "rounds"), (14, "lanes"), (15, "lanes_phaseB_modeR_or_F"), (23, "rounds_any_modeF"),
            (16, "lanes_gt64_tokens"), (17, "lanes_gt96_tokens"), (19, "rounds_any_phaseB"),
            (22, "rounds_with_stop"), (9, "headers"))}
    f.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=100_000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--workers", type=int, default=min(16, os.cpu_count() or 1))
    a = ap.parse_args()
    t0 = time.perf_counter()
    data, meta = make_corpus(a.blocks, a.seed, a.workers)
    gen = time.perf_counter() - t0
    res = check(data, meta)
    res["corpus_bytes"] = len(data)
    res["generate_s"] = round(gen, 1)
    print(json.dumps(res), flush=True)
    return 0 if res["mismatches"] == 0 and res["blocks"] == res["expected_blocks"] else 1


if __name__ == "__main__":
    sys.exit(main())

"""Multi-process path on CPU (gloo, world size 2 and 3): shard planning, per-shard pass, all_gather /
all_reduce and rank-0 assembly reproduce the single-process splits, partition sizes and Counts.  The per-shard
compute is the CPU oracle behind the same interface the GPU shard uses (sbam.dist.shard_pass)."""
import os
import socket

import numpy as np
import pytest

from conftest import FIXTURES, fixture_bytes


class OracleShard:
    """sbam.BamFile-shaped view of one shard on the CPU oracle (test backend for shard_pass)."""

    def __init__(self, o, lo):
        import oracle
        self.o, self.oracle = o, oracle
        b0 = o.block_index_at_or_after(o.find_block_start(lo)) if lo > 0 else 0
        self.b0 = b0
        self.x_base = int(o.uoff[b0])
        self.uncompressed_size = o.L - self.x_base

    def blocks(self):
        o, b0 = self.o, self.b0
        return o.start[b0:], o.csize[b0:], o.usize[b0:], o.uoff[b0:-1] - self.x_base

    def find_block_start(self, q):
        return self.o.find_block_start(q)

    def check_full_counts(self, x0, x1, R):
        import sbam
        c, npos, rbe, ns = self.o.counts_range(self.x_base + x0, self.x_base + x1, R)
        w = self.o.check_full_range(self.x_base + x0, self.x_base + x1, R)
        tff = int(np.sum(w == 1))
        return sbam.Counts(c.sum(0), c, npos, rbe, np.zeros((19, 19), np.int64), x1 - x0, ns, tff)

    def split_records(self, split_size, first, count, reads_to_check, use_success_bitmap):
        import sbam
        o = self.o
        out = []
        for (start, end) in self.oracle.hadoop_splits(o.D, split_size)[first:first + count]:
            x = o.find_record_start(o.find_block_start(start), reads_to_check)
            chain = o.record_chain(x, o.x_end_of(end))
            p = o.pos_of(x)
            out.append((sbam.Pos(p.block_pos, p.offset), len(chain) > 0, len(chain)))
        return out

    def split_records_arrays(self, split_size, first, count, reads_to_check, use_success_bitmap):
        recs = self.split_records(split_size, first, count, reads_to_check, use_success_bitmap)
        return (np.array([r[0].block_pos for r in recs], np.int64), np.array([r[0].offset for r in recs], np.int64),
                np.array([r[1] for r in recs], bool), np.array([r[2] for r in recs], np.int64))


def _worker(rank, world, port, name, split_size, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from sbam import dist as sdist
    o = oracle.BamFile(fixture_bytes(name))
    plans = sdist.plan_shards(o.D, split_size, world)
    res = sdist.shard_pass(OracleShard(o, plans[rank].lo), plans[rank], split_size, 10)
    gathered = sdist.gather_results(res, plans)
    if rank == 0:
        splits, sizes, counts = sdist.combine(gathered, o.D)
        q.put(([str(s) for s in splits], sizes, counts.tolist()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name,split_size", [("2.bam", 100000), ("1.bam", 230 * 1024), ("5k.bam", 150000)])
def test_sharded_equals_single(world, name, split_size):
    import multiprocessing as mp
    import oracle
    from sbam import dist as sdist
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, name, split_size, q)) for r in range(world)]
    for p in ps:
        p.start()
    splits, sizes, counts = q.get(timeout=120)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    o = oracle.BamFile(fixture_bytes(name))
    want, parts = oracle.compute_splits(o, split_size)
    assert splits == [f"{a}-{b}" for a, b in want]
    assert sizes == [len(p) for p in parts]
    c, npos, rbe, ns = o.counts_range(0, o.L)
    u = sdist.unpack_counts(np.array(counts, np.int64))
    assert np.array_equal(u["totals"], c.sum(0))
    assert np.array_equal(u["positions"], npos) and u["n_success"] == ns


def test_plan_covers_every_split_once():
    from sbam import dist as sdist
    for world in (1, 2, 3, 8):
        plans = sdist.plan_shards(10_000_000, 1 << 20, world)
        idx = [i for p in plans for i in range(p.split_first, p.split_first + p.split_count)]
        assert idx == list(range(len(sdist.hadoop_splits(10_000_000, 1 << 20))))
        assert plans[0].lo == 0 and plans[-1].owned_hi == 10_000_000
        for a, b in zip(plans, plans[1:]):
            assert a.owned_hi == b.lo


class OracleShardRunner:
    """run_file's shard interface (step/close) on the CPU oracle."""

    def __init__(self, plan, source, split_size, contig_lengths):
        import oracle
        self.o = oracle.BamFile(source(0, plan.file_size).tobytes())
        assert list(self.o.lens[: self.o.nref]) == list(contig_lengths)
        self.plan, self.split_size = plan, split_size

    def step(self):
        from sbam import dist as sdist
        return sdist.shard_pass(OracleShard(self.o, self.plan.lo), self.plan, self.split_size, 10)

    def close(self):
        pass


def oracle_header(source, size, device):
    import oracle
    o = oracle.BamFile(source(0, size).tobytes())
    return o.lens[: o.nref].copy()


def _expected(name, split_size):
    import oracle
    o = oracle.BamFile(fixture_bytes(name))
    want, parts = oracle.compute_splits(o, split_size)
    c, npos, rbe, ns = o.counts_range(0, o.L)
    return [f"{a}-{b}" for a, b in want], [len(p) for p in parts], c.sum(0), npos, ns


def _run_file_worker(rank, world, port, path, split_size, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sbam import dist as sdist
    seen = []

    def header(source, size, device):
        seen.append(rank)
        return oracle_header(source, size, device)
    r = sdist.run_file(path, split_size, open_shard=OracleShardRunner, read_header=header)
    q.put((rank, [str(s) for s in r.splits], r.partition_sizes, r.counts["totals"].tolist(),
           r.counts["n_success"], r.contig_lengths.tolist(), seen))
    dist.destroy_process_group()


@pytest.mark.parametrize("name,split_size", [("2.bam", 100000), ("1.bam", 230 * 1024)])
def test_run_file_gloo_world2(tmp_path, name, split_size):
    """run_file over a file on disk in a world-2 gloo group: only rank 0 reads the header, the ContigLengths reach
    rank 1 by broadcast, each rank preads its own range, and both ranks return the single-process result."""
    import multiprocessing as mp
    path = tmp_path / name
    path.write_bytes(fixture_bytes(name))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run_file_worker, args=(r, 2, port, str(path), split_size, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted([q.get(timeout=120) for _ in range(2)])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    splits, sizes, totals, npos, ns = _expected(name, split_size)
    for rank, sp, sz, tot, nsucc, lens, seen in got:
        assert sp == splits and sz == sizes and tot == totals.tolist() and nsucc == ns
        assert seen == ([0] if rank == 0 else [])
        assert lens == got[0][5]


def test_run_file_sequential_shards(tmp_path):
    """Without a process group, run_file runs `world` shards one after another (one GPU, or here the oracle)."""
    from sbam import dist as sdist
    path = tmp_path / "5k.bam"
    path.write_bytes(fixture_bytes("5k.bam"))
    splits, sizes, totals, npos, ns = _expected("5k.bam", 150000)
    for world in (1, 3):
        r = sdist.run_file(str(path), 150000, world=world, open_shard=OracleShardRunner, read_header=oracle_header)
        assert [str(s) for s in r.splits] == splits and r.partition_sizes == sizes
        assert np.array_equal(r.counts["totals"], totals) and r.counts["n_success"] == ns
        assert np.array_equal(r.counts["positions"], npos)


def test_file_source_preads_ranges(tmp_path):
    from sbam import dist as sdist
    data = fixture_bytes("2.bam")
    path = tmp_path / "2.bam"
    path.write_bytes(data)
    src, size = sdist.file_source(str(path))
    assert size == len(data)
    for lo, hi in ((0, 10), (1000, 70000), (size - 5, size + 100)):
        assert src(lo, hi).tobytes() == data[lo:min(hi, size)]
    out = np.zeros(200, np.uint8)
    assert src(50, 150, out).tobytes() == data[50:150]


def _run_file_gpu_worker(rank, world, port, path, split_size, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sbam import dist as sdist
    r = sdist.run_file(path, split_size, device=0)
    q.put((rank, [str(s) for s in r.splits], r.partition_sizes, r.counts["totals"].tolist(), r.counts["n_success"],
           r.counts["positions"].tolist()))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name,split_size", [("2.bam", 100000), ("5k.bam", 150000)])
def test_run_file_gloo_world2_gpu_shards(tmp_path, name, split_size):
    """The world-2 run through GpuShard (both ranks on GPU 0, gloo collectives): pread shards, rank-0 header,
    broadcast ContigLengths, all_gather/all_reduce — the single-process oracle result on every rank."""
    import multiprocessing as mp
    path = tmp_path / name
    path.write_bytes(fixture_bytes(name))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run_file_gpu_worker, args=(r, 2, port, str(path), split_size, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted([q.get(timeout=100) for _ in range(2)])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    splits, sizes, totals, npos, ns = _expected(name, split_size)
    for rank, sp, sz, tot, nsucc, pos in got:
        assert sp == splits and sz == sizes and tot == totals.tolist() and nsucc == ns and pos == npos.tolist()


def _rccl_worker(port, path, split_size, golden, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from sbam import cli
        from sbam import dist as sdist
        assert dist.get_backend() == "nccl"
        lens = sdist.broadcast_lengths(np.arange(84, dtype=np.int64) * 7 + 1, dev)
        r = sdist.run_file(path, split_size, device=0, coll_device=dev)
        parts = sdist.full_check_file(path, 10, None, 10, device=0, coll_device=dev, records_path=path + ".records")
        text = "\n".join(cli.full_check_lines(parts, 10)) + "\n"
        q.put((lens.tolist(), [str(s) for s in r.splits], r.partition_sizes, r.counts["totals"].tolist(),
               r.counts["n_success"], text == golden))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_collectives_single_rank(tmp_path):
    """The RCCL path (backend "nccl" = RCCL on ROCm) on device tensors, in a one-rank group on GPU 0: broadcast_lengths,
    run_file's all_gather_into_tensor + all_reduce (gather_results) and full_check_file's all_reduce,
    all_gather_object and broadcast_object_list — the collectives the 8-GPU runs use (CanLoadBam.scala:262-271,
    FullCheck.scala:160-168).  Results equal the single-process oracle's splits/Counts and the full-check golden."""
    import multiprocessing as mp
    from conftest import FIXTURES, GOLDEN
    name, split_size = "2.bam", 100000
    path = tmp_path / name
    path.write_bytes(fixture_bytes(name))
    (tmp_path / (name + ".records")).write_bytes(open(os.path.join(FIXTURES, name + ".records"), "rb").read())
    golden = open(os.path.join(GOLDEN, "full-check", name)).read()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), str(path), split_size, golden, q))
    p.start()
    lens, sp, sz, tot, nsucc, golden_ok = q.get(timeout=150)
    p.join(60)
    assert p.exitcode == 0
    assert lens == (np.arange(84) * 7 + 1).tolist()
    splits, sizes, totals, npos, ns = _expected(name, split_size)
    assert sp == splits and sz == sizes and tot == totals.tolist() and nsucc == ns
    assert golden_ok


def test_hbm_budget_and_auto_windows():
    """HBM per compressed byte (DESIGN.md §Data layout) from the file's measured BGZF ratio; a range that starts
    inside a block finds the first header; auto_windows fits two contexts in 80 % of the free bytes."""
    from sbam import dist as sdist
    src, size = sdist.file_source(os.path.join(FIXTURES, "2.bam"))
    r = sdist.bgzf_ratio(src, size)
    assert 2.9 < r < 3.2
    assert abs(sdist.bgzf_ratio(lambda lo, hi: src(lo + 1000, hi + 1000), size - 1000) - r) < 0.05
    per = sdist.hbm_bytes_per_compressed_byte(1.1 * r)
    assert abs(per - (1 + 1.1 * r * 2.1875 + 0.05)) < 1e-9
    assert sdist.bgzf_sample_stats(src, size)[1] < 0.05  # zlib-6 BAM blocks: the arena's default share
    need = size * per * 2
    assert sdist.auto_windows(size, src, int(need / 0.8) + 1) == 1
    assert sdist.auto_windows(size, src, int(need / 0.8 / 3) + 1) == 3


def _bgzf_block(payload: bytes, level: int, strategy: int = 0) -> bytes:
    """One BGZF block (RFC 1952 member with the BC extra field) of `payload`, raw-deflated at `level`."""
    import struct
    import zlib
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    data = co.compress(payload) + co.flush()
    bsize = 18 + len(data) + 8 - 1
    hdr = b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<HBBHH", 6, 66, 67, 2, bsize)
    return hdr + data + struct.pack("<II", zlib.crc32(payload), len(payload))


def test_auto_windows_budgets_arena_for_stored_blocks():
    """stored and Huffman-only blocks need 2 B of token arena per uncompressed byte, so auto_windows
    budgets them (bgzf_sample_stats' low-ratio share) instead of the 1/16 default, and picks more windows than the
    same ratio at the default would."""
    import zlib
    from sbam import dist as sdist
    rng = np.random.default_rng(5)
    raw = rng.integers(0, 4, 60000, dtype=np.uint8).tobytes()
    stored = b"".join(_bgzf_block(raw, 0) for _ in range(40))
    huff = b"".join(_bgzf_block(raw, 6, zlib.Z_HUFFMAN_ONLY) for _ in range(40))
    for blob in (stored, huff):
        buf = np.frombuffer(blob, np.uint8)
        src = (lambda b: lambda lo, hi: b[lo:hi])(buf)
        r, frac = sdist.bgzf_sample_stats(src, buf.size)
        assert frac == 1.0
        per = sdist.hbm_bytes_per_compressed_byte(1.1 * r, frac)
        assert per > sdist.hbm_bytes_per_compressed_byte(1.1 * r) + 2.0 * 1.1 * r
        free = int(buf.size * per * 2 / 0.8 / 2) + 1  # room for half of what the worst case needs
        assert sdist.auto_windows(buf.size, src, free) == 2
    # the token counter: one token per byte for stored and Huffman-only streams; zlib-6 matches take two tokens each
    import zlib as z
    for level, strat in ((0, 0), (6, z.Z_HUFFMAN_ONLY)):
        co = z.compressobj(level, z.DEFLATED, -15, 9, strat)
        assert sdist.deflate_token_count(co.compress(raw) + co.flush()) == len(raw)
    text = b"".join(b"read%07d\tACGTTGCA\n" % i for i in range(3000))
    co = z.compressobj(6, z.DEFLATED, -15, 8, 0)
    t = sdist.deflate_token_count(co.compress(text) + co.flush())
    assert 0 < t < len(text) // 2 and t % 1 == 0
    assert sdist.deflate_token_count(b"\xff\xff\xff") == -1  # block type 3

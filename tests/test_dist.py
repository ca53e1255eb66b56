"""Multi-process path on CPU (gloo, world size 2 and 3): shard planning, per-shard pass, all_gather /
all_reduce and rank-0 assembly reproduce the single-process splits, partition sizes and Counts.  The per-shard
compute is the CPU oracle behind the same interface the GPU shard uses (sbam.dist.shard_pass)."""
import os
import socket

import numpy as np
import pytest

from conftest import fixture_bytes


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

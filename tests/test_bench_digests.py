"""The full-size parity pins of bench.py (tests/golden/bench_digests.json).

tests/golden/make_bench_digests.py runs the CPU oracle over bench.py's exact synthetic file in segments (the file
does not fit in host memory at 10-80 GB).  Here the same script, on a small file with windows narrower than a tile,
must give the digests of ONE whole-file oracle run (oracle.BamFile over all bytes: Counts by or_counts_range, pair
histogram from the words, oracle.compute_splits) — so the segmenting changes nothing.  Then the committed pins
must be well-formed and cover bench.py's headline (configs[1]: 10 GB on one GPU) and configs[2] (30 GB over 8)."""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import make_bench_digests as mbd  # noqa: E402


def whole_file_digests(s, split_size):
    import oracle
    from test_gpu_parity import pair_hist
    o = oracle.BamFile(s.bytes(), threads=8)
    c, npos, rbe, ns = o.counts_parallel(0, o.L, 10, 8)
    words = o.check_full_range(0, o.L)
    tff = int((((words & 0x80000000) == 0) & ((words & 0x7ffff) == 1) & (((words >> 24) & 0x7f) == 0)).sum())
    by_key = c.copy()
    by_key[3:] = 0
    packed = np.concatenate([c.sum(0), by_key.ravel(), npos, rbe.ravel(), pair_hist(words).ravel(),
                             np.array([ns, tff, o.L], np.int64)]).astype(np.int64)
    splits, parts = oracle.compute_splits(o, split_size)
    rows = []
    for p in parts:
        fp = o.pos_of(int(p[0]))
        rows.append((fp.block_pos, fp.offset, 1, len(p)))
    rows = np.array(rows, np.int64)
    return {"counts": hashlib.sha1(packed.tobytes()).hexdigest()[:16],
            "splits": hashlib.sha1(rows.ravel().tobytes()).hexdigest()[:16], "n_splits": len(parts)}


@pytest.mark.parametrize("level", [6, 0])
def test_segmented_pin_equals_whole_file_oracle(level):
    """level 0: bench.py --level 0's stored blocks (one pin per level)."""
    import synth
    args = argparse.Namespace(size_gb=0.03, world=2, tile_mb=4.0, tiles=3, seed=0x5EEDBA11, read_len=150,
                              split_mb=1.0, threads=8, halo_mb=2.0, out="", level=level)
    got = mbd.pin(args)
    assert got["workload"]["level"] == level
    s = synth.SynthBam.for_size(int(args.size_gb * 1e9 * args.world), tile_mb=args.tile_mb, seed=args.seed, threads=8,
                                read_len=150, level=level, distinct=True, cycle=args.tiles)
    assert got["workload"]["file_bytes"] == s.size and s.copies > args.tiles  # cycled tiles, several windows
    assert got["digest"] == whole_file_digests(s, int(args.split_mb * (1 << 20)))


def test_committed_pins_cover_the_headline_workloads():
    db = json.load(open(os.path.join(GOLDEN, "bench_digests.json")))
    by_size = {}
    for e in db:
        w = e["workload"]
        assert set(e["digest"]) == {"counts", "splits", "n_splits"} and e["n_success"] == e["records"]
        assert (w["seed"], w["tile_mb"], w["tiles"], w["read_len"], w["split_mb"]) == (0x5EEDBA11, 64.0, 16, 150, 2.0)
        assert w["level"] in (0, 1, 6)
        by_size[e["made_by"]] = e
    made = " ".join(by_size)
    assert "--size-gb 10 --world 1" in made  # configs[1]: bench.py's N=1 line
    assert "--size-gb 3.75 --world 8" in made  # configs[2]: bench.py --gpus 8 --size-gb 3.75 (30 GB)

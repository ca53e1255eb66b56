#!/usr/bin/env python3
"""Diagnostic: cProfile of the bench step's host side (sbam.dist.GpuShard.step over a resident synthetic shard, the
bench's default workload at --size-gb) — where the host time between and inside the device work goes."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]
import synth  # noqa: E402
from sbam import dist as sdist  # noqa: E402

size = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
s = synth.SynthBam.for_size(int(size * 1e9), tile_mb=64.0, distinct=True, cycle=16, threads=16)
plan = sdist.plan_shards(s.size, 2 << 20, 1)[0]
sh = sdist.GpuShard(plan, s.slice, 2 << 20, s.contig_lengths)
sh.step()
t = time.perf_counter()
for _ in range(3):
    sh.step()
print("step ms", (time.perf_counter() - t) / 3 * 1e3)
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    sh.step()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)

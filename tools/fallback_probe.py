#!/usr/bin/env python3
"""Diagnostic: which edge-case payload (tests/test_inflate_streams.py shapes) the wave decoder hands to the
per-lane fallback: one single-block BGZF file per payload, fallback count each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import sbam  # noqa: E402
from test_inflate_streams import EOF_BLOCK, SHAPES, bgzf_block, deflate, sample_inputs  # noqa: E402

for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    for i, raw in enumerate(sample_inputs(seed)):
        level, strat = SHAPES[(i + seed) % len(SHAPES)]
        p = deflate(raw, level, strat)
        data = bgzf_block(p, len(raw)) + EOF_BLOCK
        g = sbam.BamFile(data, inflate=False)
        g.inflate()
        fb = g.inflate_fallbacks()
        g.close()
        if fb and ((p[0] >> 1) & 3) != 0:
            print(f"seed {seed} input {i}: level {level} strategy {strat} len {len(raw)} btype {(p[0] >> 1) & 3} "
                  f"payload {len(p)} -> fallback", flush=True)
print("done")

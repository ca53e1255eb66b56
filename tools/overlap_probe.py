#!/usr/bin/env python3
"""Experiment: how much of scan+inflate on one stream overlaps a full check on another.  Two library contexts
over the same synthetic BAM (each with its own HIP stream); context B is inflated once, then timed:
  seq  — A: reset + scan + inflate, then B: full check (one after the other);
  conc — the same two calls from two host threads at once (ctypes releases the GIL).
Prints one JSON line of wall-clock ms."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-gb", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import sbam
    import synth
    s = synth.SynthBam.for_size(int(args.size_gb * 1e9), tile_mb=64.0)
    data = s.bytes()
    a = sbam.BamFile(data, inflate=False)
    b = sbam.BamFile(data, inflate=False)
    for f in (a, b):
        f.reset()
        f.run(contig_lengths=s.contig_lengths)
    U = b.uncompressed_size

    def inflate_a():
        a.reset()
        a.run(contig_lengths=s.contig_lengths)

    def check_b():
        b.check_full_counts(0, U)

    inflate_a()
    check_b()
    res = {"seq": [], "conc": [], "inflate_only": [], "check_only": []}
    for _ in range(args.reps):
        t0 = time.perf_counter()
        inflate_a()
        t1 = time.perf_counter()
        check_b()
        t2 = time.perf_counter()
        res["inflate_only"].append((t1 - t0) * 1e3)
        res["check_only"].append((t2 - t1) * 1e3)
        res["seq"].append((t2 - t0) * 1e3)
        th = [threading.Thread(target=inflate_a), threading.Thread(target=check_b)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        res["conc"].append((time.perf_counter() - t0) * 1e3)
    out = {k: round(float(np.median(v)), 2) for k, v in res.items()}
    out["size_gb"] = round(s.size / 1e9, 3)
    out["kernels_a"] = {k: round(a.kernel_ms(k), 2) for k in ("scan", "inflate_decode", "inflate_resolve")}
    out["kernels_b"] = {"check_full": round(b.kernel_ms("check_full"), 2)}
    print(json.dumps(out), flush=True)
    a.close()
    b.close()


if __name__ == "__main__":
    main()

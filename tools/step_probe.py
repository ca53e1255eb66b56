#!/usr/bin/env python3
"""Experiment: host wall time of each phase of one bench step (sbam/dist.py GpuShard._once + shard_pass), to
find time outside the kernels.  Prints one JSON line of median ms per phase."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-gb", type=float, default=10.0)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--torch", action="store_true", help="initialise torch.cuda first, as bench.py does")
    args = ap.parse_args()
    if args.torch:
        import torch
        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    import synth
    from sbam import dist as sdist
    s = synth.SynthBam.for_size(int(args.size_gb * 1e9), tile_mb=64.0)
    split = 2 << 20
    plan = sdist.plan_shards(s.size, split, 1)[0]
    shard = sdist.GpuShard(plan, s.slice, split, s.contig_lengths, device=0)
    shard.step()
    f = shard.f
    ph = {}

    def t(name, fn):
        t0 = time.perf_counter()
        r = fn()
        ph.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
        return r

    for _ in range(args.steps):
        t0 = time.perf_counter()
        t("reset", f.reset)
        t("scan_blocks", lambda: setattr(f, "n_blocks", f._scan()))
        t("inflate", f.inflate)
        t("contigs", lambda: f.set_contig_lengths(s.contig_lengths))
        t("blocks_d2h", f.blocks)
        U = f.uncompressed_size
        t("check_full_counts", lambda: f.check_full_counts(0, U, 10))
        t("split_records", lambda: f.split_records(split, first=plan.split_first, count=plan.split_count,
                                                   reads_to_check=10, use_success_bitmap=True))
        ph.setdefault("step_total", []).append((time.perf_counter() - t0) * 1e3)
    out = {k: round(float(np.median(v)), 2) for k, v in ph.items()}
    out["kernels"] = {k: round(f.kernel_ms(k), 2) for k in ("scan", "chain", "inflate", "check_full", "find_record",
                                                          "records")}
    print(json.dumps(out), flush=True)
    shard.close()


if __name__ == "__main__":
    main()

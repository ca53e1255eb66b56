#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot kernels from rocprofv3 --pmc passes (one counter group per pass, as the
MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE cannot share a pass).

    traffic_pmc.py OUT.json FETCH_DIR WRITE_DIR [--sq-dir D ...] [--size-gb G] [--seed S] [--tile-mb T]

FETCH_DIR / WRITE_DIR hold p_counter_collection.csv of a `--pmc FETCH_SIZE` and a `--pmc WRITE_SIZE` run of
tools/bench_kernels.py on the bench workload.  Values are KB per dispatch; per kernel the median dispatch is
kept.  Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE is doubled — gfx950 tallies each
128-B request at 64 B for 16-B/lane reads, which is how every one of these kernels reads; WRITE_SIZE is exact
for 16-B/lane stores and is used as reported.  FETCH counts Infinity-Cache hits too (memory-side requests).  --sq-dir adds the SQ instruction/cycle counters
of further passes (SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVE_CYCLES, ...) per dispatch, as reported
(instruction counts are per wave: one VALU instruction = 64 lane-ops)."""
import argparse
import csv
import json
import os
import statistics
from collections import defaultdict

KERNELS = {"k_check_bits": "sbam::k_check_bits", "k_check<0, 0>": "sbam::k_check<0, 0>", "k_check<0, 2>": "sbam::k_check<0, 2>",
           "k_p0_links": "sbam::k_p0_links", "k_p0_list": "sbam::k_p0_list", "k_p0_count": "sbam::k_p0_count",
           "k_inflate_decode": "sbam::k_inflate_wave", "k_inflate_slow": "sbam::k_inflate_slow",
           "k_inflate_resolve": "sbam::k_inflate_resolve<12>", "k_check<1, 0>": "sbam::k_check<1, 0>",
           "k_check<1, 1>": "sbam::k_check<1, 1>", "k_check<1, 2>": "sbam::k_check<1, 2>",
           "k_chains": "sbam::k_chains",
           "k_scan_count": "sbam::k_scan_count", "k_scan_write": "sbam::k_scan_write", "k_scan_slots": "sbam::k_scan_slots",
           "k_scan_slots_wide": "sbam::k_scan_slots_wide<32>",
           "k_scan_compact": "sbam::k_scan_compact",
           "k_record_counts": "sbam::k_record_counts", "k_eager_wave": "sbam::k_eager_wave"}


def per_dispatch(d, counter, scale=1024.0):
    """Median per dispatch of `counter` per kernel (FETCH/WRITE_SIZE are KB: scale to bytes)."""
    vals = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "p_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        for k, prefix in KERNELS.items():
            if name == prefix:
                vals[k].append(float(r["Counter_Value"]) * scale)
    return {k: statistics.median(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def counters_in(d):
    return sorted({r["Counter_Name"] for r in csv.DictReader(open(os.path.join(d, "p_counter_collection.csv")))})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--sq-dir", action="append", default=[])
    ap.add_argument("--size-gb", type=float, default=10.0)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EEDBA11)
    ap.add_argument("--tile-mb", type=float, default=64.0)
    ap.add_argument("--tiles", type=int, default=16)
    a = ap.parse_args()
    fetch, nf = per_dispatch(a.fetch_dir, "FETCH_SIZE")
    write, nw = per_dispatch(a.write_dir, "WRITE_SIZE")
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "spark-bam_amd"))
    import sbam
    out = {"workload": {"size_gb": a.size_gb, "seed": a.seed, "tile_mb": a.tile_mb, "tiles": a.tiles},
           "source_digest": sbam.source_digest(),
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes of tools/bench_kernels.py; "
                     "median dispatch; FETCH x2 (gfx950 64-B tally of 128-B requests), WRITE as reported",
           "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        f2 = 2.0 * fetch[k]
        out["kernels"][k] = {"fetch_size_reported": fetch[k], "fetch_bytes": f2, "write_bytes": write[k],
                             "hbm_bytes_per_launch": int(f2 + write[k]), "dispatches": [nf[k], nw[k]]}
    for d in a.sq_dir:
        for cn in counters_in(d):
            v, _ = per_dispatch(d, cn, 1.0)
            for k, x in v.items():
                out["kernels"].setdefault(k, {})[cn] = x
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out["kernels"]))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel microbenchmark on a synthetic BAM resident in HBM: scan, inflate, full check (report and
by-key modes), eager check, split records.  Prints one JSON line of average device ms (HIP events on the
library stream) plus algorithmic GB/s.  Used for A/B experiments and rocprofv3 --pmc passes."""
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
    ap.add_argument("--size-gb", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="scan,inflate,check_full,check_eager,splits")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--tiles", type=int, default=16, help="distinct tiles cycled (bench.py's default input)")
    args = ap.parse_args()
    import sbam
    import synth
    s = synth.SynthBam.for_size(int(args.size_gb * 1e9), tile_mb=min(64.0, args.size_gb * 300), read_len=args.read_len,
                                distinct=args.tiles > 1, cycle=max(args.tiles, 1))
    data = s.bytes()
    f = sbam.BamFile(data, inflate=False)
    f.reset()
    f.run(contig_lengths=s.contig_lengths)
    U = f.uncompressed_size
    only = args.only.split(",")
    out = {"size_gb": round(s.size / 1e9, 3), "uncompressed_gb": round(U / 1e9, 3)}
    ms = {}

    def timed(name, fn, kern):
        fn()
        t = []
        for _ in range(args.reps):
            fn()
            t.append(f.kernel_ms(kern))
        ms[name] = round(float(np.median(t)), 3)

    if "scan" in only or "inflate" in only:
        def scan_inflate():
            f.reset()
            f.run(contig_lengths=s.contig_lengths)
        scan_inflate()
        tt = {"scan": [], "inflate": [], "inflate_decode": [], "inflate_resolve": []}
        for _ in range(args.reps):
            scan_inflate()
            for k in tt:
                tt[k].append(f.kernel_ms(k))
        for k in tt:
            ms[k] = round(float(np.median(tt[k])), 3)
        out["inflate_fallbacks"] = int(f.inflate_fallbacks())  # blocks the exact decoder took
        if hasattr(f.L, "sbam_debug_inflate_pieced"):  # blocks whose first DEFLATE block went through the lane regions
            import ctypes
            n = ctypes.c_int64(0)
            if f.L.sbam_debug_inflate_pieced(f.ctx, ctypes.byref(n)) == 0:
                out["inflate_pieced"] = int(n.value)
    if "check_full" in only:
        timed("check_full", lambda: f.check_full_counts(0, U), "check_full")
        c = f.check_full_counts(0, U)
        out["n_success_ok"] = bool(c.n_success == s.n_records)
    if "check_bykey" in only:
        timed("check_bykey", lambda: f.check_full_counts(0, U, by_key=True), "check_full")
    if "check_eager" in only:
        timed("check_eager", lambda: f.check_eager(0, U), "check_eager")
        p0 = []
        for _ in range(args.reps):  # the record-0 pass alone (k_eager_wave + boundary tiles), bitmap left on the device
            f.check_eager_device(0, U)
            p0.append(f.kernel_ms("check_eager_pass0"))
        ms["check_eager_pass0"] = round(float(np.median(p0)), 3)
    if "splits" in only:
        f.check_full_counts(0, U)
        t0 = time.perf_counter()
        parts = f.partition_sizes(2 << 20, use_success_bitmap=True)
        ms["splits_wall"] = round((time.perf_counter() - t0) * 1e3, 3)
        out["records_ok"] = bool(sum(parts) == s.n_records)
    st, cs, us, uo = f.blocks()
    C = int(cs.astype(np.int64).sum())
    gbs = {}
    if "inflate" in ms:
        gbs["inflate"] = round((C + U) / ms["inflate"] / 1e6, 2)
    for k in ("check_full", "check_bykey", "check_eager", "check_eager_pass0"):
        if k in ms:
            gbs[k] = round((U + U / 8) / ms[k] / 1e6, 2)
    out.update({"ms": ms, "alg_GBps": gbs})
    print(json.dumps(out), flush=True)
    f.close()


if __name__ == "__main__":
    main()

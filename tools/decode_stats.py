#!/usr/bin/env python3
"""Diagnostic: cycle attribution inside k_inflate_decode (build with EXTRA=-DSBAM_DEC_STATS into
spark-bam_amd/build_stats, run with SBAM_LIB pointing at it).  Prints per-wave averages."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-gb", type=float, default=4.0)
    args = ap.parse_args()
    import numpy as np
    import sbam
    import synth
    s = synth.SynthBam.for_size(int(args.size_gb * 1e9), tile_mb=64.0)
    f = sbam.BamFile(s.bytes(), inflate=False)
    f.inflate()
    L = sbam.load_library()
    L.sbam_debug_decode_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    st = np.zeros(16, np.uint64)
    L.sbam_debug_decode_stats(st.ctypes.data, 1)
    f.reset()
    f.run(contig_lengths=s.contig_lengths)
    L.sbam_debug_decode_stats(st.ctypes.data, 0)
    nwaves = 256 * 4 if f.n_blocks >= 65536 else (f.n_blocks + 255) // 256 * 4
    names = ["top(next/park)", "epoch", "chain_with_hdr", "chain_decode_only", "done", "iterations",
             "iters_with_hdr", "lane_iters_decoding", "lane_iters_parked", "total_cycles"]
    out = {n: float(st[i]) / nwaves for i, n in enumerate(names)}
    it = out["iterations"]
    out["cycles_per_iteration"] = out["total_cycles"] / it
    out["decoding_lanes_per_iteration"] = out["lane_iters_decoding"] / it
    out["parked_lanes_per_iteration"] = out["lane_iters_parked"] / it
    out["ms"] = {k: f.kernel_ms(k) for k in ("inflate_decode", "inflate_resolve")}
    out["blocks"] = int(f.n_blocks)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}))


if __name__ == "__main__":
    main()

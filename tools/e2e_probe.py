#!/usr/bin/env python3
"""Diagnostic: where the pinned-host step (bench.py e2e_h2d) spends its time.  Times, on a 10 GB synthetic file:
the plain pinned H2D copy of one window, one window's load (sbam_load) + compute alone, and the pipelined step
(sbam.dist.WindowPipe) for W windows.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]


def main():
    import torch
    import numpy as np
    import synth
    from sbam import dist as sdist
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    split = 2 << 20
    s = synth.SynthBam.for_size(int(10e9), tile_mb=64.0)
    host = torch.empty(s.size, dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    s.slice(0, s.size, hv)
    out = {"windows": W, "file_gb": round(s.size / 1e9, 3)}
    # plain H2D of one window's bytes
    n = s.size // W
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        dev.copy_(host[:n], non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        dev.copy_(host[:n], non_blocking=True)
    torch.cuda.synchronize()
    out["h2d_window_ms"] = round((time.perf_counter() - t) / 3 * 1e3, 2)
    out["h2d_gbs"] = round(n / ((time.perf_counter() - t) / 3) / 1e9, 2)
    del dev
    wplans = sdist.plan_shards(s.size, split, W)
    times = {"load": [], "run": []}

    def stage(lo, hi, j):
        return hv[lo:hi]

    def run_window(sh):
        t0 = time.perf_counter()
        r = sh.step()
        times["run"].append((time.perf_counter() - t0) * 1e3)
        return r

    pipe = sdist.WindowPipe(wplans, stage, split, s.contig_lengths, 0, run_window)
    pipe.step()
    torch.cuda.synchronize()
    times["run"].clear()
    t = time.perf_counter()
    pipe.step()
    torch.cuda.synchronize()
    out["pipelined_step_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    out["run_window_ms"] = [round(x, 2) for x in times["run"]]
    # serial: load then run, per window
    ser = []
    for w in range(W):
        t0 = time.perf_counter()
        sh = pipe._load(w, 0)
        t1 = time.perf_counter()
        sh.step()
        t2 = time.perf_counter()
        ser.append((round((t1 - t0) * 1e3, 2), round((t2 - t1) * 1e3, 2)))
    out["serial_load_run_ms"] = ser
    pipe.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

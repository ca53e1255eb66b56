#!/usr/bin/env python3
"""bench.py — compressed-BAM GB/s for compute-splits + full-check on MI355X (BASELINE.json `metric`).

Workload (configs[1]/[2] of BASELINE.json): a synthetic Illumina-like BAM (150 bp paired
reads, zlib level 6, htsjdk-style 65498-B payloads, records straddling blocks; tools/synth_bam.c) of
--size-gb compressed bytes PER GPU.  One step = the whole hot path over the whole file from compressed bytes
resident in HBM:

    BGZF header scan → block chain → inflate every block → full checker at every uncompressed offset
    (Counts + success bitmap) → per Hadoop split (2 MiB): FindBlockStart → FindRecordStart → record chain
    → split assembly (+ all_gather of split starts / all_reduce of Counts when N > 1)

N > 1: one process per GPU (torch.distributed, RCCL), rank r owns a contiguous run of Hadoop splits of an
N × size-gb file (weak scaling) and loads only its byte range + halo (sbam/dist.py).

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel (largest average device time),
measured with HIP events on the library's stream over the timed steps; `cpu_baseline` times the CPU oracle
(oracle/, a C restatement of the reference — the Scala/Spark reference cannot run on this image) on a
bounded sample of the same generator on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def measured_traffic(kernel: str, args):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes (tools/traffic_pmc.py →
    profiles/*/traffic.json), when they were taken on this same workload; else None.  FETCH_SIZE is doubled
    for the kernels' 16-B/lane streaming reads (MI355X_MICROARCH.md, HBM/rocprofv3: gfx950 tallies each
    128-B request at 64 B); WRITE_SIZE is used as reported."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("workload") != {"size_gb": args.size_gb, "seed": args.seed, "tile_mb": args.tile_mb}:
            continue
        k = t.get("kernels", {}).get(kernel)
        if k:
            return {"hbm_bytes_per_launch": k["hbm_bytes_per_launch"], "source": os.path.relpath(path, ROOT)}
    return None


def cpu_baseline(sample_mb: float, threads: int, split_size: int, seed: int):
    """Oracle (C restatement of the reference algorithm) on a bounded sample of the same synthetic stream:
    zlib inflate + full checker at every position + compute-splits, `threads` host threads."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import synth
    s = synth.SynthBam.for_size(int(sample_mb * 1e6), tile_mb=min(64.0, sample_mb), seed=seed, threads=threads)
    data = s.bytes()
    t0 = time.perf_counter()
    f = oracle.BamFile(data, threads=threads)
    _, _, _, nsucc = f.counts_parallel(0, f.L, 10, threads)
    splits, parts = oracle.compute_splits(f, split_size)
    wall = time.perf_counter() - t0
    assert nsucc == s.n_records and sum(len(p) for p in parts) == s.n_records, "oracle sample self-check failed"
    return {"value": round(data.size / wall / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"first {data.size / 1e6:.1f} MB compressed ({f.L / 1e6:.1f} MB uncompressed, {s.n_records} records) "
                      f"of the same synthetic generator: zlib inflate + full check of every offset + "
                      f"compute-splits @ {split_size >> 20} MiB, {wall:.2f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size-gb", type=float, default=10.0, help="compressed GB per GPU")
    ap.add_argument("--split-mb", type=float, default=2.0)
    ap.add_argument("--tile-mb", type=float, default=64.0)
    ap.add_argument("--threads", type=int, default=16, help="host threads (generator, CPU baseline)")
    ap.add_argument("--cpu-sample-mb", type=float, default=2000.0,
                    help="compressed MB of the same synthetic file timed on the CPU oracle (~10 s at 16 threads)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EEDBA11)
    ap.add_argument("--workload", choices=["full-check", "load-reads"], default="full-check",
                    help="full-check: BASELINE metric (compute-splits + full-check); load-reads: configs[3] "
                         "(FindBlockStart → FindRecordStart → record chains → decoded columns)")
    ap.add_argument("--windows", type=int, default=1,
                    help="byte-range windows per GPU: streams a shard larger than HBM through one device "
                         "(two contexts: window w+1's host staging and PCIe copy overlap window w's kernels; "
                         "both inside the timed step)")
    ap.add_argument("--read-len", type=int, default=150, help="0 = long-read config (configs[4])")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, the product path); gloo only to rehearse N ranks on one GPU (--device)")
    ap.add_argument("--device", type=int, default=None, help="GPU index (default LOCAL_RANK)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0)) if args.device is None else args.device
    import torch
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        dist = None
    dev = torch.device("cuda", local)
    cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # collective tensors

    import sbam
    import synth
    from sbam import dist as sdist

    split_size = int(args.split_mb * (1 << 20))
    t = time.time()
    s = synth.SynthBam.for_size(int(args.size_gb * 1e9 * world), tile_mb=args.tile_mb, seed=args.seed,
                                threads=args.threads, read_len=args.read_len)
    W = max(1, args.windows)
    plans = sdist.plan_shards(s.size, split_size, world)  # rank-level plans (what all_gather sees)
    plan = plans[rank]
    wplans = sdist.plan_shards(s.size, split_size, world * W)[rank * W:(rank + 1) * W]
    shard = sdist.GpuShard(plan, s.slice, split_size, s.contig_lengths, device=local) if W == 1 else None
    log(f"[rank {rank}] synthetic file {s.size / 1e9:.2f} GB ({s.n_records} records), shard "
        f"[{plan.lo}, {plan.owned_hi}) splits {plan.split_first}+{plan.split_count} in {W} window(s), "
        f"workload {args.workload}, setup {time.time() - t:.1f}s")
    kernels = ("scan", "chain", "inflate", "inflate_decode", "inflate_resolve", "check_full", "check_pass0",
               "check_chains", "find_record", "records", "load_records")
    last = {}

    def run_window(sh):
        if args.workload == "load-reads":
            sizes = sh.load_step()
            z = np.zeros(len(sizes), np.int64)
            r = sdist.ShardResult(np.zeros(sdist.N_COUNT_WORDS, np.int64), z, z, (sizes > 0).astype(np.int64),
                                  sizes.astype(np.int64))
        else:
            r = sh.step()
        ms = {k: max(sh.f.kernel_ms(k), 0.0) for k in kernels}
        last.update(U=int(sh.f.uncompressed_size), blocks=sh.f.blocks(), f=sh.f)
        return r, ms

    # --windows W: a shard larger than HBM streams through two contexts (sbam_load keeps their allocations):
    # while one computes window w, a loader thread fills pinned host memory with window w+1 (the synthetic
    # file's slice, copied by `threads` workers) and copies it to the other context's device buffer.
    loader = fill_pool = None
    if W > 1:
        from concurrent.futures import ThreadPoolExecutor
        loader, fill_pool = ThreadPoolExecutor(max_workers=1), ThreadPoolExecutor(max_workers=args.threads)
        wshards, pinned = [None, None], [None, None]

        def fill(buf, lo, hi):
            n, k = hi - lo, args.threads
            step_b = -(-n // k)
            futs = [fill_pool.submit(s.slice, lo + a, lo + min(n, a + step_b), buf[a:min(n, a + step_b)])
                    for a in range(0, n, step_b)]
            for fu in futs:
                fu.result()

        def load(w, j):  # window w into context slot j (slots alternate per load, so W may be odd)
            wp = wplans[w]
            sh = wshards[j]
            lo, hi = wp.load_range(sh.halo if sh is not None else 2 << 20)
            if pinned[j] is None or pinned[j].numel() < hi - lo:
                pinned[j] = torch.empty(int((hi - lo) * 1.05), dtype=torch.uint8, pin_memory=True)
            buf = pinned[j].numpy()[:hi - lo]
            fill(buf, lo, hi)
            if sh is None:
                wshards[j] = sdist.GpuShard(wp, lambda a, b: buf if (a, b) == (lo, hi) else s.slice(a, b), split_size,
                                            s.contig_lengths, device=local)
            else:
                sh.reload(wp, buf)
            return wshards[j]

        pending = {"w": 0, "seq": 0, "fut": loader.submit(load, 0, 0)}

    def step():
        if W == 1:
            res, ms = run_window(shard)
        else:
            parts, ms = [], {k: 0.0 for k in kernels}
            U, nb = 0, 0
            for w in range(W):
                assert pending["w"] == w
                sh = pending["fut"].result()
                nxt = (w + 1) % W  # the next window (of this step or the next one) loads while this one runs
                pending["seq"] += 1
                pending.update(w=nxt, fut=loader.submit(load, nxt, pending["seq"] % 2))
                try:
                    r, m = run_window(sh)
                    U += last["U"]
                    nb += last["blocks"][0].size
                finally:
                    last.pop("f", None)
                parts.append(r)
                for k in kernels:
                    ms[k] += m[k]
            last.update(U=U, nblocks=nb)
            res = sdist.ShardResult(np.sum([r.counts for r in parts], axis=0),
                                    *(np.concatenate([getattr(r, a) for r in parts]) for a in
                                      ("first_block_pos", "first_offset", "nonempty", "n_records")))
        if world > 1 and args.workload == "full-check":
            sdist.gather_results(res, plans, device=cdev)
        return res, ms

    def sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    res = None
    for _ in range(args.warmup):
        res, _ = step()
    tot_ms = {k: 0.0 for k in kernels}
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ts = time.perf_counter()
        res, ms = step()
        log(f"[rank {rank}] step {i}: {(time.perf_counter() - ts) * 1e3:.1f} ms (host wall)")
        for k in kernels:
            tot_ms[k] += ms[k]
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # --- size-independent parity properties of the last step (full sizes; fixtures cover exactness)
    counts = sdist.unpack_counts(res.counts)
    n_rec = int(res.n_records.sum())
    if args.workload == "load-reads":  # no checker pass in this workload: the record count is the property
        counts["n_success"] = n_rec
    ok_local = counts["n_success"] == int(res.n_records.sum()) if world == 1 else True
    if world > 1:
        v = torch.tensor([counts["n_success"], n_rec], dtype=torch.int64, device=cdev)
        dist.all_reduce(v)
        tot_succ, tot_rec = (int(x) for x in v.tolist())
    else:
        tot_succ, tot_rec = counts["n_success"], n_rec
    parity = {"records": tot_rec, "expected_records": s.n_records, "checker_true": tot_succ,
              "ok": bool(tot_rec == s.n_records and tot_succ == s.n_records and ok_local)}
    if not parity["ok"]:
        log(f"[rank {rank}] PARITY PROPERTY FAILED: {parity}")

    # --- roofline of the dominant kernel (this rank's shard; per launch).  Candidates are single kernels:
    # k_check<0, 1> (record-0 pass over the interior tiles: reads U, writes the U/8 PASS0 bitmap), k_inflate_decode (reads the C payload;
    # its token stream is an internal intermediate) and k_inflate_resolve (writes U; tokens internal).
    U = last["U"]
    if W == 1:
        st, cs, us, uo = last["blocks"]
        comp_payload = int(cs.astype(np.int64).sum())
        nblocks = int(st.size)
    else:  # per-window launches; the roofline uses the summed window times and bytes
        comp_payload = plan.owned_hi - plan.lo
        nblocks = last["nblocks"]
    avg = {k: tot_ms[k] / args.steps for k in kernels}
    alg = {"check_pass0": U + U // 8, "inflate_decode": comp_payload, "inflate_resolve": U}
    names = {"check_pass0": "k_check<0, 1>", "inflate_decode": "k_inflate_decode", "inflate_resolve": "k_inflate_resolve"}
    if args.workload == "load-reads":
        del alg["check_pass0"]
    dom = max(alg, key=lambda k: avg[k])
    achieved = alg[dom] / (avg[dom] * 1e-3) / 1e9 if avg[dom] > 0 else 0.0
    traffic = measured_traffic(names[dom], args) if (args.read_len == 150 and W == 1) else None

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.workload == "full-check" and args.read_len == 150:
            try:
                cpu = cpu_baseline(args.cpu_sample_mb, args.threads, split_size, args.seed)
            except Exception as e:  # reported, never substituted for the GPU number
                log(f"cpu baseline failed: {e!r}")
        value = s.size * args.steps / elapsed / 1e9
        fc = args.workload == "full-check"
        line = {
            "metric": "compressed BAM GB/s for compute-splits + full-check (whole node, 1/2/4/8 GPU)" if fc else
                      "compressed BAM GB/s for loadReads record decode (whole node, 1/2/4/8 GPU)",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (tools/synth_bam.c: %s, zlib-6 BGZF, seed %#x)" % (
                "150bp paired Illumina-like" if args.read_len == 150 else "long-read 10-50 kb" if args.read_len == 0
                else f"{args.read_len} bp", args.seed),
            "config": {"workload": ("Synthetic %.0f GB %s BAM per GPU: " % (
                                   args.size_gb, "Illumina-like" if args.read_len == 150 else
                                   "long-read" if args.read_len == 0 else f"{args.read_len} bp")) +
                                   ("compute-splits @ %g MiB + full-check of every uncompressed offset" % args.split_mb
                                    if fc else "loadReads @ %g MiB splits: records decoded into device columns"
                                    % args.split_mb),
                       "file_gb": round(s.size / 1e9, 3), "uncompressed_gb_per_gpu": round(U / 1e9, 3),
                       "records": s.n_records, "blocks_per_gpu": nblocks, "split_mb": args.split_mb,
                       "windows_per_gpu": W, "parallelism": f"shard{world}"},
            "uncompressed_gbps": round(U * world * args.steps / elapsed / 1e9, 3),
            "kernel_ms": {k: round(v, 3) for k, v in avg.items()},
            "roofline": {"bound": "hbm", "kernel": names[dom], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic["hbm_bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "algorithmic_bytes": alg[dom], "avg_launch_ms": round(avg[dom], 3)},
            "stage_rooflines": {k: {"achieved": round(alg[k] / (avg[k] * 1e-3) / 1e9, 2) if avg[k] > 0 else None,
                                    "algorithmic_bytes": alg[k], "avg_launch_ms": round(avg[k], 3)} for k in alg},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if shard is not None:
        shard.close()
    if loader is not None:
        pending["fut"].result()
        loader.shutdown()
        fill_pool.shutdown()
        for sh in wshards:
            if sh is not None:
                sh.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

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
N × size-gb file (weak scaling) and loads only its byte range + halo (sbam/dist.py).  `--gpus N` without a
torchrun environment spawns the N ranks itself (torch.distributed.run) before anything touches the GPU.

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel (largest average device time),
measured with HIP events on the library's stream over the timed steps; `e2e_h2d` is the same step from
pinned host memory (host → device copies inside the timed step, overlapped with the kernels of the previous
window); `cpu_baseline` times the CPU oracle (oracle/, a C restatement of the reference — the Scala/Spark
reference cannot run on this image) on a bounded sample of the same generator on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torchrun: launch N ranks (one per GPU) with torch.distributed.run and return
    its exit code.  This process has not imported torch, so no GPU has been touched before the children start."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[launcher] {' '.join(cmd)}")
    return subprocess.call(cmd)


def host_cores():
    """(threads the host side may use, CPUs the machine shows).  A GPU box's process gets a share of a larger
    machine: OMP_NUM_THREADS (16 there) is that share; os.cpu_count() is the whole machine."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(aff, share) if share > 0 else aff), (os.cpu_count() or aff)


def measured_traffic(kernel: str, args):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes (tools/traffic_pmc.py →
    profiles/*/traffic.json), when they were taken on this same workload AND the same kernel build (the
    library's source digest); else None.  FETCH_SIZE is doubled for the kernels' 16-B/lane streaming reads
    (MI355X_MICROARCH.md, HBM/rocprofv3: gfx950 tallies each 128-B request at 64 B); WRITE_SIZE as reported."""
    import glob
    import sbam
    digest = sbam.source_digest()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("workload") != {"size_gb": args.size_gb, "seed": args.seed, "tile_mb": args.tile_mb,
                                 "tiles": args.tiles}:
            continue
        if t.get("source_digest") != digest:
            continue
        k = t.get("kernels", {}).get(kernel)
        if k:
            return {"hbm_bytes_per_launch": k["hbm_bytes_per_launch"], "source": os.path.relpath(path, ROOT)}
    return None


def copy_peak(dev) -> dict:
    """Measured HBM copy peak on this GPU: tools/hbm_peak.hip (16-B nontemporal loads/stores, 4 in flight per lane,
    grid-stride) over 4 GiB device to device, read + write bytes / kernel time; the best of a few grid sizes."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libhbmpeak.so"))
    lib.hbm_copy_peak.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double)]
    n = 4 << 30
    best = None
    for nt in (0, 1):
        for grid in (2048, 8192, 32768):
            ms = ctypes.c_double(0.0)
            rc = lib.hbm_copy_peak(dev.index or 0, n, 10, grid, nt, ctypes.byref(ms))
            if rc == 0 and ms.value > 0 and (best is None or ms.value < best[2]):
                best = (grid, nt, ms.value)
    if best is None:
        raise RuntimeError("hbm_copy_peak failed")
    return {"value": round(2 * n / (best[2] * 1e-3) / 1e9, 1), "unit": "GB/s", "bytes": 2 * n,
            "how": f"tools/hbm_peak.hip: global_load/store_dwordx4 copy of 4 GiB device->device "
                   f"({'nontemporal' if best[1] else 'plain'}), read+write bytes / kernel time, 10 reps, "
                   f"best of grids 2048/8192/32768 x 256 and plain/nontemporal: {best[0]}"}


REAL_BAM = os.path.join(ROOT, "tests", "fixtures", "5k.bam")  # the reference's test_bams/src/main/resources/5k.bam


def make_file(args, target_bytes: int, threads: int, tile_mb: float = None):
    """The bench input: the synthetic generator (tools/synth_bam.c at zlib level --level), or with --real a real
    BAM's data blocks tiled to the target size behind its header block (synth.TiledBam)."""
    import synth
    if args.real:
        return synth.TiledBam(args.real, target_bytes)
    return synth.SynthBam.for_size(target_bytes, tile_mb=args.tile_mb if tile_mb is None else tile_mb, seed=args.seed,
                                   threads=threads, read_len=args.read_len, level=args.level,
                                   distinct=args.tiles > 1, cycle=max(args.tiles, 1))


def data_desc(args, s) -> str:
    if args.real:
        return (f"real: the data blocks of {os.path.relpath(args.real, ROOT)} (the reference's test BAM, htsjdk-written) "
                f"tiled {s.copies} times behind its header block")
    return "synthetic (tools/synth_bam.c: %s, zlib-%d BGZF, seed %#x, %s)" % (
        "150bp paired Illumina-like" if args.read_len == 150 else "long-read 10-50 kb" if args.read_len == 0
        else f"{args.read_len} bp", args.level, args.seed,
        f"a cycle of {min(args.tiles, s.copies)} distinct {args.tile_mb:g} MB tiles" if args.tiles > 1
        else f"one {args.tile_mb:g} MB tile repeated")


def pinned_digest(args, s):
    """The CPU oracle's digests of this exact file and split size (tests/golden/bench_digests.json, written by
    tests/golden/make_bench_digests.py at full size), or None when this workload was not pinned."""
    if args.real or args.contigs or args.workload != "full-check":
        return None
    key = {"file_bytes": int(s.size), "seed": args.seed, "tile_mb": args.tile_mb, "tiles": args.tiles,
           "read_len": args.read_len, "level": args.level, "split_mb": args.split_mb, "reads_to_check": 10}
    try:
        db = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")))
    except (OSError, ValueError):
        return None
    for e in db:
        if e["workload"] == key:
            return e
    return None


def cpu_baseline(args, sample_mb: float, threads: int, split_size: int):
    """Oracle (C restatement of the reference algorithm) on a bounded sample of the same input stream:
    zlib inflate + full checker at every position + compute-splits, `threads` host threads."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    s = make_file(args, int(sample_mb * 1e6), threads, tile_mb=min(64.0, sample_mb))
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


def cpu_baseline_load_reads(args, sample_mb: float, threads: int, split_size: int):
    """Oracle on a bounded sample for the loadReads workload (configs[3]): zlib inflate (`threads` host threads)
    then, per Hadoop split, FindBlockStart → FindRecordStart → the record chain (CanLoadBam.scala:281-334).  The
    oracle stops at record offsets (no field decode into columns), so the CPU side does less work than the GPU."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    s = make_file(args, int(sample_mb * 1e6), threads, tile_mb=min(64.0, sample_mb))
    data = s.bytes()
    t0 = time.perf_counter()
    f = oracle.BamFile(data, threads=threads)
    parts = oracle.load_reads_and_positions(f, split_size)
    wall = time.perf_counter() - t0
    assert sum(len(p) for p in parts) == s.n_records, "oracle sample self-check failed"
    return {"value": round(data.size / wall / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"first {data.size / 1e6:.1f} MB compressed ({f.L / 1e6:.1f} MB uncompressed, {s.n_records} records) "
                      f"of the same synthetic generator: zlib inflate ({threads} threads) + per split FindBlockStart, "
                      f"FindRecordStart and the record chain @ {split_size >> 20} MiB (record offsets only, no "
                      f"column decode), {wall:.2f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size-gb", type=float, default=10.0, help="compressed GB per GPU")
    ap.add_argument("--split-mb", type=float, default=2.0)
    ap.add_argument("--tile-mb", type=float, default=64.0)
    ap.add_argument("--tiles", type=int, default=16,
                    help="distinct seeded tiles the synthetic file cycles through (1: one tile repeated)")
    ap.add_argument("--threads", type=int, default=0, help="host threads (generator, CPU baseline); 0 = the host share")
    ap.add_argument("--cpu-sample-mb", type=float, default=2000.0,
                    help="compressed MB of the same synthetic file timed on the CPU oracle (~10 s at 16 threads)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-windows", type=int, default=6,
                    help="windows of the pinned-host → results measurement (0 = skip it)")
    ap.add_argument("--e2e-steps", type=int, default=3)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EEDBA11)
    ap.add_argument("--workload", choices=["full-check", "load-reads"], default="full-check",
                    help="full-check: BASELINE metric (compute-splits + full-check); load-reads: configs[3] "
                         "(FindBlockStart → FindRecordStart → record chains → decoded columns)")
    ap.add_argument("--windows", type=int, default=1,
                    help="byte-range windows per GPU: streams a shard larger than HBM through one device "
                         "(two contexts: window w+1's host staging and PCIe copy overlap window w's kernels; "
                         "both inside the timed step)")
    ap.add_argument("--read-len", type=int, default=150, help="0 = long-read config (configs[4])")
    ap.add_argument("--level", type=int, default=6, help="zlib level of the synthetic BGZF blocks (0 = stored blocks, "
                                                         "as bgzip -l 0 / samtools view -u write)")
    ap.add_argument("--real", nargs="?", const=REAL_BAM, default=None,
                    help="tile a real BAM's data blocks to --size-gb behind its header block (default: the reference's "
                         "5k.bam) instead of the synthetic generator")
    ap.add_argument("--contigs", type=int, default=0,
                    help="check against N contig lengths (the file's 84, then N - 84 more: a scaffold-level reference, "
                         "so refIdx values up to N - 1 are in range); 0 = the file's own")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, the product path); gloo only to rehearse N ranks on one GPU (--device)")
    ap.add_argument("--device", type=int, default=None, help="GPU index (default LOCAL_RANK)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    threads, nproc = host_cores()
    if args.threads > 0:
        threads = args.threads
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
    from sbam import dist as sdist

    split_size = int(args.split_mb * (1 << 20))
    t = time.time()
    s = make_file(args, int(args.size_gb * 1e9 * world), threads)
    setup_s = time.time() - t
    if args.contigs > len(s.contig_lengths):  # many-contig reference: lengths past the 84 real ones
        extra = np.random.default_rng(args.seed).integers(1000, 1 << 28, args.contigs - len(s.contig_lengths))
        s.contig_lengths = np.concatenate([np.asarray(s.contig_lengths, np.int64), extra.astype(np.int64)])
    plans = sdist.plan_shards(s.size, split_size, world)  # rank-level plans (what all_gather sees)
    plan = plans[rank]
    W = args.windows
    if W == 0:  # as many windows as the shard's size, compression ratio and free HBM need (two contexts)
        W = sdist.auto_windows(plan.owned_hi - plan.lo, lambda lo, hi: s.slice(plan.lo + lo, plan.lo + hi),
                               sdist.device_free_bytes(local))
    W = max(1, W)

    def wplans_of(nw):
        return sdist.plan_shards(s.size, split_size, world * nw)[rank * nw:(rank + 1) * nw]

    shard = sdist.GpuShard(plan, s.slice, split_size, s.contig_lengths, device=local) if W == 1 else None
    log(f"[rank {rank}] synthetic file {s.size / 1e9:.2f} GB ({s.n_records} records), shard "
        f"[{plan.lo}, {plan.owned_hi}) splits {plan.split_first}+{plan.split_count} in {W} window(s), "
        f"workload {args.workload}, setup {time.time() - t:.1f}s, host threads {threads} of {nproc}")
    kernels = ("scan", "chain", "inflate", "inflate_decode", "inflate_resolve", "check_full", "check_pass0",
               "check_chains", "find_record", "records", "load_records")
    if args.workload == "load-reads":  # (the eager calls whose bitmap proves the splits' record chains)
        kernels += ("check_eager",)
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
        return r, ms, int(sh.f.uncompressed_size), int(sh.f.n_blocks)

    def merge(parts):
        res = sdist.ShardResult(np.sum([p[0].counts for p in parts], axis=0),
                                *(np.concatenate([getattr(p[0], a) for p in parts]) for a in
                                  ("first_block_pos", "first_offset", "nonempty", "n_records")))
        ms = {k: sum(p[1][k] for p in parts) for k in kernels}
        last.update(U=sum(p[2] for p in parts), nblocks=sum(p[3] for p in parts))
        return res, ms

    # --windows W: a shard larger than HBM streams through two contexts; each window's bytes are staged from
    # the synthetic generator into pinned host memory (16 copy threads) and copied to the device.
    pipe = None
    if W > 1:
        from concurrent.futures import ThreadPoolExecutor
        fill_pool = ThreadPoolExecutor(max_workers=threads)
        pinned = [None] * sdist.WindowPipe.NBUF

        def stage_synth(lo, hi, j):
            if j is None:  # a halo retry's private bytes (WindowPipe: never a shared staging slot)
                return s.slice(lo, hi)
            if pinned[j] is None or pinned[j].numel() < hi - lo:
                pinned[j] = torch.empty(int((hi - lo) * 1.05), dtype=torch.uint8, pin_memory=True)
            buf = pinned[j].numpy()[:hi - lo]
            n, k = hi - lo, threads
            step_b = -(-n // k)
            futs = [fill_pool.submit(s.slice, lo + a, lo + min(n, a + step_b), buf[a:min(n, a + step_b)])
                    for a in range(0, n, step_b)]
            for fu in futs:
                fu.result()
            return buf

        pipe = sdist.WindowPipe(wplans_of(W), stage_synth, split_size, s.contig_lengths, local, run_window,
                                prefetch=True)

    gathered = {}

    def step():
        res, ms = merge([run_window(shard)] if W == 1 else pipe.step())
        if world > 1 and args.workload == "full-check":
            gathered["all"] = sdist.gather_results(res, plans, device=cdev)
        return res, ms

    def sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        tt = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    res = None
    for _ in range(args.warmup):
        res, _ = step()
    # a streamed pipe runs on from the warm-up into the timed steps (steady state: every step loads W windows — its
    # windows 1..W-1 and the next step's window 0 — and the first timed step's window 0 was loaded during the
    # warm-up's last window); round 3 dropped that prefetch, so the first timed step loaded its window 0 in the
    # foreground (a step ~200 ms longer than the rest at 30 GB / 3 windows)
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
    elapsed = max_over_ranks(time.perf_counter() - t0)

    # --- size-independent parity properties of the last step (full sizes; fixtures cover exactness)
    counts = sdist.unpack_counts(res.counts)
    n_rec = int(res.n_records.sum())
    if args.workload == "load-reads":  # no checker pass in this workload: the record count is the property
        counts["n_success"] = n_rec
    ok_local = counts["n_success"] == n_rec
    if world > 1:
        v = torch.tensor([counts["n_success"], n_rec, int(not ok_local)], dtype=torch.int64, device=cdev)
        dist.all_reduce(v)
        tot_succ, tot_rec, n_bad = (int(x) for x in v.tolist())
    else:
        tot_succ, tot_rec, n_bad = counts["n_success"], n_rec, int(not ok_local)
    parity = {"records": tot_rec, "expected_records": s.n_records, "checker_true": tot_succ,
              "ok": bool(tot_rec == s.n_records and tot_succ == s.n_records and n_bad == 0)}
    # digests of the whole file's full-check Counts and split rows (first Pos, non-empty, records per split), whatever
    # the sharding: an N-rank run and a one-process run over the same file must print the same ones
    if args.workload == "full-check":
        import hashlib
        parts = gathered["all"] if world > 1 else [res]
        rows = np.concatenate([np.stack([p.first_block_pos, p.first_offset, p.nonempty, p.n_records]).T.ravel()
                               for p in parts]).astype(np.int64)
        parity["digest"] = {"counts": hashlib.sha1(parts[0].counts.astype(np.int64).tobytes()).hexdigest()[:16],
                            "splits": hashlib.sha1(rows.tobytes()).hexdigest()[:16], "n_splits": int(rows.size // 4)}
        # full-size exactness: the CPU oracle's digests of this same file (tests/golden/make_bench_digests.py)
        pin = pinned_digest(args, s)
        parity["digest_pinned"] = pin is not None
        if pin is not None:
            parity["digest_oracle"] = pin["digest"]
            parity["digest_source"] = "tests/golden/bench_digests.json: " + pin["made_by"]
            parity["ok"] = bool(parity["ok"] and parity["digest"] == pin["digest"])
    if not parity["ok"]:
        log(f"[rank {rank}] PARITY PROPERTY FAILED: {parity}")

    # --- roofline of the dominant kernel (this rank's shard; per launch).  Candidates are single kernels:
    # k_check_bits (full-check record-0 pass over the interior tiles: reads U, writes the U/8 PASS0 bitmap),
    # k_inflate_decode (reads the C payload; its token stream is an internal intermediate) and
    # k_inflate_resolve (writes U; tokens internal).
    U, nblocks = last["U"], last["nblocks"]
    if W == 1:  # the compressed payload bytes decode reads (block table of the shard, outside the timed region)
        comp_payload = int(shard.f.blocks()[1].astype(np.int64).sum())
    else:
        comp_payload = plan.owned_hi - plan.lo
    avg = {k: tot_ms[k] / args.steps for k in kernels}
    alg = {"check_pass0": U + U // 8, "inflate_decode": comp_payload, "inflate_resolve": U}
    names = {"check_pass0": "k_check_bits", "inflate_decode": "k_inflate_decode",
             "inflate_resolve": "k_inflate_resolve"}
    if args.workload == "load-reads":
        del alg["check_pass0"]
    dom = max(alg, key=lambda k: avg[k])
    # compute-splits' own checker (eager.Checker): not part of the step (the step's splits read the
    # full check's success bitmap), timed on the resident shard after the timed steps
    eager_ms = None
    if W == 1 and args.workload == "full-check" and shard is not None:
        em = []
        for _ in range(3):
            shard.f.check_eager_device(0, shard.f.uncompressed_size)
            em.append(shard.f.kernel_ms("check_eager_pass0"))
        eager_ms = float(np.median(em[1:]))
    # loadReads: the chain proof is skipped when the eager pass's list found every link (no false-positive PASS0 site
    # in the shard, as on the synthetic BAM); the same steps with the proof forced price a shard that has one
    proof = None
    if W == 1 and args.workload == "load-reads" and shard is not None:
        os.environ["SBAM_FORCE_PROOF"] = "1"
        try:
            sync()
            tp = time.perf_counter()
            pms = []
            for _ in range(max(2, args.steps // 2)):
                _, m = step()
                pms.append(m["records"])
            sync()
            pel = (time.perf_counter() - tp) / len(pms)
        finally:
            del os.environ["SBAM_FORCE_PROOF"]
        proof = {"value": round(s.size / pel / 1e9, 3), "ms_per_step": round(pel * 1e3, 3),
                 "records_ms": round(float(np.mean(pms)), 3), "steps": len(pms),
                 "how": "the same step with SBAM_FORCE_PROOF=1: k_chain_proof reads every record's hop although the "
                        "list pass found no missing link (what a shard with one false-positive PASS0 site costs)"}
    achieved = alg[dom] / (avg[dom] * 1e-3) / 1e9 if avg[dom] > 0 else 0.0
    traffic = (measured_traffic(names[dom], args) if (args.read_len == 150 and W == 1 and args.level == 6 and
                                                      not args.real) else None)

    # --- pinned host → results (SURVEY §8(d) "with H2D"): the same step with the shard's compressed bytes in
    # pinned host memory, streamed in `e2e_windows` windows through two contexts (window w+1's copy overlaps
    # window w's kernels; window 0's copy is not overlapped).
    retries = int(shard.retries if W == 1 else sum(c.retries for c in pipe.ctx if c))
    e2e = None
    if args.e2e_windows > 0 and W == 1 and args.workload == "full-check":
        if shard is not None:
            shard.close()
            shard = None
        torch.cuda.empty_cache()
        lo0, hi0 = plan.lo, min(s.size, plan.owned_hi + (64 << 20))
        host = torch.empty(hi0 - lo0, dtype=torch.uint8, pin_memory=True)
        hv = host.numpy()
        s.slice(lo0, hi0, hv)

        def stage_pinned(lo, hi, j):
            return hv[lo - lo0:hi - lo0] if lo >= lo0 and hi <= hi0 else s.slice(lo, hi)

        epipe = sdist.WindowPipe(wplans_of(args.e2e_windows), stage_pinned, split_size, s.contig_lengths, local,
                                 run_window, prefetch=True)
        merge(epipe.step())  # warm-up (allocations); the pipe runs on into the timed steps (steady state)
        sync()
        t1 = time.perf_counter()
        for _ in range(args.e2e_steps):
            eres, _ = merge(epipe.step())
        sync()
        e_el = max_over_ranks(time.perf_counter() - t1)
        e_ok = sdist.unpack_counts(eres.counts)["n_success"] == int(eres.n_records.sum())
        epipe.drop_prefetch()
        epipe.close()
        e2e = {"value": round(s.size * args.e2e_steps / e_el / 1e9, 3), "unit": "GB/s",
               "ms_per_step": round(e_el / args.e2e_steps * 1e3, 3), "windows": args.e2e_windows,
               "steps": args.e2e_steps, "parity_ok": bool(e_ok),
               "how": "compressed bytes in pinned host memory, streamed in windows through two contexts: window "
                      "w+1's H2D (sbam_load) overlaps window w's kernels, and a step's last window overlaps the next "
                      "step's window 0 (steady state: the pipe runs on from the warm-up step)"}
        del host

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.read_len == 150:
            try:
                base_fn = cpu_baseline if args.workload == "full-check" else cpu_baseline_load_reads
                cpu = base_fn(args, args.cpu_sample_mb, threads, split_size)
                cpu["host_nproc"] = nproc
            except Exception as e:  # reported, never substituted for the GPU number
                log(f"cpu baseline failed: {e!r}")
        try:
            cpk = copy_peak(dev)
        except Exception as e:
            log(f"copy peak failed: {e!r}")
            cpk = None
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
            "data": data_desc(args, s),
            "config": {"workload": ("%s %.0f GB %s BAM per GPU: " % (
                                   "Real-data" if args.real else "Synthetic", args.size_gb,
                                   "5k.bam-tiled" if args.real else
                                   ("Illumina-like" if args.read_len == 150 else "long-read" if args.read_len == 0
                                    else f"{args.read_len} bp") + ("" if args.level == 6 else f" zlib-{args.level}"))) +
                                   ("compute-splits @ %g MiB + full-check of every uncompressed offset" % args.split_mb
                                    if fc else "loadReads @ %g MiB splits: records decoded into device columns"
                                    % args.split_mb),
                       "file_gb": round(s.size / 1e9, 3), "uncompressed_gb_per_gpu": round(U / 1e9, 3),
                       "records": s.n_records, "blocks_per_gpu": nblocks, "split_mb": args.split_mb,
                       "windows_per_gpu": W, "parallelism": f"shard{world}",
                       "halo_retries": retries,
                       "tiles": min(args.tiles, s.copies), "setup_s": round(setup_s, 1),
                       **({"contigs": len(s.contig_lengths)} if args.contigs else {})},
            "uncompressed_gbps": round(U * world * args.steps / elapsed / 1e9, 3),
            "kernel_ms": {k: round(v, 3) for k, v in avg.items()},
            "roofline": {"bound": "hbm", "kernel": names[dom], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic["hbm_bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "algorithmic_bytes": alg[dom], "avg_launch_ms": round(avg[dom], 3)},
            "stage_rooflines": dict({k: {"achieved": round(alg[k] / (avg[k] * 1e-3) / 1e9, 2) if avg[k] > 0 else None,
                                         "algorithmic_bytes": alg[k], "avg_launch_ms": round(avg[k], 3)} for k in alg},
                                    **({"check_eager_pass0": {
                                        "achieved": round((U + U // 8) / (eager_ms * 1e-3) / 1e9, 2),
                                        "frac": round((U + U // 8) / (eager_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                        "algorithmic_bytes": U + U // 8, "avg_launch_ms": round(eager_ms, 3),
                                        "note": "compute-splits' eager checker (k_eager_wave + boundary tiles), timed "
                                                "after the steps; not in the step"}} if eager_ms else {})),
            "hbm_copy_peak": cpk,
            "e2e_h2d": e2e,
            **({"with_chain_proof": proof} if proof else {}),
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if shard is not None:
        shard.close()
    if pipe is not None:
        pipe.drop_prefetch()
        pipe.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

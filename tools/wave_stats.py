#!/usr/bin/env python3
"""Diagnostic (tools-only build, `make -C spark-bam_amd EXTRA=-DSBAM_WAVE_STATS BUILD=build_stats`): cycle
attribution inside k_inflate_wave and k_inflate_resolve (s_memtime per phase, summed over waves) on a synthetic BAM."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SBAM_LIB", os.path.join(ROOT, "spark-bam_amd", "build_stats", "libsbam.so"))
sys.path[:0] = [os.path.join(ROOT, "spark-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import sbam  # noqa: E402
import synth  # noqa: E402

size = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
s = synth.SynthBam.for_size(int(size * 1e9), tile_mb=min(64.0, size * 300))
f = sbam.BamFile(s.bytes(), inflate=False)
L = sbam.load_library()
fn = L.sbam_debug_wave_stats
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 40)()
f.reset(); f.run(contig_lengths=s.contig_lengths)
fn(buf, 1)
f.reset(); f.run(contig_lengths=s.contig_lengths)
fn(buf, 1)
v = list(buf)
names = ["header", "build", "stage", "phaseA", "phaseB", "build_dist", "rounds", "b_iters", "total", "headers",
         "hdr_cl_setup", "hdr_chain", "hdr_stage", "warmup"]
tot = v[8]
out = {n: v[i] for i, n in enumerate(names)}
out.update({f"{n}_pct": round(100.0 * v[i] / tot, 1) for i, n in list(enumerate(names[:6])) + [(13, "warmup")]})
out["blocks"] = int(f.n_blocks)
out["decode_ms"] = f.kernel_ms("inflate_decode")
out["fallbacks"] = f.inflate_fallbacks()
tok = {n: v[i] for i, n in ((14, "lanes"), (15, "lanes_phaseB"), (16, "lanes_gt64"), (17, "lanes_gt96"),
                              (18, "lanes_gt128"), (19, "rounds_any_phaseB"), (20, "rounds_any_gt96"),
                              (21, "rounds_any_gt64"), (22, "rounds_with_stop"), (23, "rounds_any_modeF"))}
out["tokens"] = tok
out["phaseC_cycles_per_round"] = {n: round(v[i] / max(v[6], 1)) for i, n in ((24, "prefix_scan"), (25, "run1"), (26, "dumpA"), (27, "dumpR"), (28, "tail"))}
out["b_iters_per_round"] = round(v[7] / max(v[6], 1), 3)
out["rounds_per_block"] = round(v[6] / out["blocks"], 3)
out["cycles_per_header"] = {n: round(v[i] / max(v[9], 1)) for i, n in ((0, "rest"), (10, "cl_setup"), (11, "chain"), (12, "stage"), (5, "build_dist"), (1, "build_lit"))}
out["cycles_per_round"] = {n: round(v[i] / max(v[6], 1)) for i, n in list(enumerate(names[2:6], 2)) + [(13, "warmup")]}
rsteps = max(v[38], 1)
rnames = ["positions_zero", "literals", "output_stores", "match_setup", "rounds", "token_wait"]
res = {n: round(v[32 + i] / rsteps) for i, n in enumerate(rnames)}
res["tail_and_rest"] = round((v[31] - sum(v[32:38])) / rsteps)
out["resolve_cycles_per_step"] = res
out["resolve_steps_per_block"] = round(v[38] / out["blocks"], 2)
out["resolve_rounds_per_step"] = round(v[39] / rsteps, 3)
out["resolve_cycles_per_block"] = round(v[31] / out["blocks"])
out["resolve_ms"] = f.kernel_ms("inflate_resolve")
out["resolve_copy_iters_per_step"] = {"wave": round(v[29] / rsteps, 2), "lane_sum": round(v[30] / rsteps, 2),
                                      "lane_efficiency": round(v[30] / max(64 * v[29], 1), 3)}
print(json.dumps(out))

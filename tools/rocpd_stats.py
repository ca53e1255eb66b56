#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db, or a kernel_trace.csv) as per-kernel stats:
calls, total / average / min / max device time.  Used to produce the profiles/ summaries that bench.py's
in-process HIP-event timings are checked against."""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur, lds, vgpr, agpr, sgpr, gx, wx in c.execute(
                "select name, duration, lds_size, vgpr_count, accum_vgpr_count, sgpr_count, grid_x, workgroup_x "
                "from kernels"):
            yield name, float(dur), (lds, vgpr, agpr, sgpr, gx, wx)
    else:
        for r in csv.DictReader(open(path)):
            yield (r["Kernel_Name"], float(r["End_Timestamp"]) - float(r["Start_Timestamp"]),
                   (r.get("LDS_Block_Size"), r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("SGPR_Count"),
                    r.get("Grid_Size"), r.get("Workgroup_Size")))


def main():
    acc = defaultdict(list)
    meta = {}
    for name, dur, m in rows(sys.argv[1]):
        short = name.split("(")[0].replace("void ", "")
        acc[short].append(dur)
        meta[short] = m
    tot_all = sum(sum(v) for v in acc.values())
    print("| kernel | calls | total ms | avg ms | min ms | max ms | % | lds, vgpr, agpr, sgpr, grid, wg |")
    print("|---|---|---|---|---|---|---|---|")
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        t = sum(v)
        print(f"| {k} | {len(v)} | {t / 1e6:.3f} | {t / len(v) / 1e6:.3f} | {min(v) / 1e6:.3f} | {max(v) / 1e6:.3f} "
              f"| {100 * t / tot_all:.1f} | {', '.join(str(x) for x in meta[k])} |")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes (one directory per pass) per kernel: counter totals, plus derived
per-wave / per-instruction ratios.  Usage: pmc_summary.py DIR [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    keys = sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    meta = {}
    for f in sorted(glob.glob(os.path.join(root, "*", "p_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if keys and not any(k in name for k in keys):
                continue
            acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[name] = {k: r.get(k) for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                                "SGPR_Count")}
    for name, c in acc.items():
        print(f"## {name}  {meta[name]}")
        for k in sorted(c):
            print(f"  {k:28s} {c[k]:.6g}")
        w = c.get("SQ_WAVES", 0)
        if w:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"):
                if k in c:
                    print(f"  {k + '/wave':28s} {c[k] / w:.6g}")
        if c.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if k in c:
                    print(f"  {k + '/WAVE_CYCLES':28s} {c[k] / c['SQ_WAVE_CYCLES']:.4f}")
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
            t = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            if t:
                print(f"  {'L2 hit rate':28s} {c['TCC_HIT_sum'] / t:.4f}")


if __name__ == "__main__":
    main()

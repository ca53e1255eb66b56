#!/usr/bin/env python3
"""Median-dispatch SQ counters per kernel for each build directory of scripts/gpu_pmc_ab.sh (one JSON line per
build and kernel)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, builds = sys.argv[1], sys.argv[2:]
    for b in builds:
        files = glob.glob(os.path.join(out, b, "**", "*counter_collection.csv"), recursive=True)
        per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
        for f in files:
            rows = defaultdict(lambda: defaultdict(float))
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"].split("(")[0]
                    rows[(k, r.get("Dispatch_Id", ""))][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, _), cs in rows.items():
                for c, v in cs.items():
                    per[k][c].append(v)
        for k in sorted(per):
            if not any(s in k for s in ("inflate_wave", "inflate_resolve")):
                continue
            med = {c: sorted(v)[len(v) // 2] for c, v in per[k].items()}
            print(json.dumps({"build": b, "kernel": k, **{c: round(v) for c, v in sorted(med.items())}}))


if __name__ == "__main__":
    main()

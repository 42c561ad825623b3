#!/usr/bin/env python3
"""Median per-call kernel times of the runs under gpurun_out/ab/<X>.<round>/ (tools/kernel_ab.sh)."""
import csv
import glob
import os
import statistics as st
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
pats = {"screen": "k_screen_x", "refine": "k_refine<2, 1>", "pair": "k_refine_pair", "fmt": "k_fmt_write"}
for d in sorted(glob.glob(os.path.join(base, "*.*/"))):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        continue
    rows = list(csv.DictReader(open(f[0])))
    out = []
    for name, pat in pats.items():
        ds = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                    for r in rows if pat in r["Kernel_Name"])
        ds = ds[len(ds) // 3:]  # drop the small warm-up calls
        if ds:
            out.append(f"{name} {st.median(ds):7.1f} us")
    print(os.path.basename(d.rstrip('/')), " | ".join(out))

#!/usr/bin/env python3
"""Per-dispatch means of rocprofv3 --pmc CSV output (run_counter_collection.csv) for the screen
kernels, grouped by run directory prefix: python tools/pmc_csv_summary.py gpurun_out/r9m ringpmc0 ringpmc12"""
import collections
import csv
import glob
import os
import sys

base = sys.argv[1]
for pre in sys.argv[2:]:
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(base, pre + "_*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_screen_x1" not in k:
                continue
            fam = "screen(W=%s, LDS %s, VGPR %s)" % (r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"])
            key = (f, r["Dispatch_Id"])
            vals[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[fam][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for fam in vals:
        ds = sorted(dur[fam].values())
        print(f"== {pre}: {fam}  dispatches {len(ds)}  median {ds[len(ds) // 2]:.1f} us")
        for c in sorted(vals[fam]):
            v = vals[fam][c]
            print(f"   {c:28s} {sum(v) / len(v):.4g}")

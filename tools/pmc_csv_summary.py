#!/usr/bin/env python3
"""Per-dispatch means of rocprofv3 --pmc CSV output (run_counter_collection.csv) for the screen
kernels, grouped by run directory prefix (<prefix>_<n> or <prefix><n>):
python tools/pmc_csv_summary.py gpurun_out/r9m ringpmc0 ringpmc12"""
import collections
import csv
import glob
import os
import re
import sys

base = sys.argv[1]
for pre in sys.argv[2:]:
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    runs = [d for d in glob.glob(os.path.join(base, pre + "*"))
            if os.path.isdir(d) and re.fullmatch(r"_?\d+", os.path.basename(d)[len(pre):])]
    files = [f for d in sorted(runs)
             for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)]
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            m = re.search(r"(k_screen_x1|k_refine_pair|k_refine)", k)
            if not m:
                continue
            fam = "%s(W=%s, LDS %s, VGPR %s)" % (m.group(1), r["Workgroup_Size"], r["LDS_Block_Size"],
                                               r["VGPR_Count"])
            key = (f, r["Dispatch_Id"])
            vals[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[fam][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for fam in vals:
        ds = sorted(dur[fam].values())
        print(f"== {pre}: {fam}  dispatches {len(ds)}  median {ds[len(ds) // 2]:.1f} us")
        for c in sorted(vals[fam]):
            v = vals[fam][c]
            print(f"   {c:28s} {sum(v) / len(v):.4g}")

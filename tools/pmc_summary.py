#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs per kernel family (screen / refine / other).

    python tools/pmc_summary.py gpurun_out/<tag>      (reads <tag>/pmc*/**/*counter_collection.csv)
"""
import collections
import csv
import glob
import sys


def family(name: str) -> str:
    for key in ("k_screen", "k_refine", "k_merge", "k_exact_topk", "k_exact", "k_fmt"):
        if key in name:
            return key
    return "other"


def main():
    root = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(f"{root}/pmc*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            tot[fam][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[fam].add((f, r.get("Dispatch_Id", "")))
    for fam in sorted(tot):
        v = tot[fam]
        print(f"{fam}: " + ", ".join(f"{k}={v[k]:.4g}" for k in sorted(v)))
        valu, mfma = v.get("SQ_INSTS_VALU", 0.0), v.get("SQ_INSTS_MFMA", 0.0)
        if valu and mfma:
            print(f"  VALU:MFMA instruction ratio {valu / mfma:.2f}")


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 --pmc output databases (rocpd sqlite): per kernel family, the mean of each
counter per dispatch (over the dispatches of the timed bench steps) and the mean duration.

    python tools/pmc_summary.py gpurun_out/r7j/pmc1 gpurun_out/r7j/pmc2 ...
"""
import collections
import glob
import re
import sqlite3
import sys


def family(name):
    m = re.search(r"(k_[a-z0-9_]+)", name)
    fam = m.group(1) if m else name[:40]
    t = re.search(r"k_screen_x1ILi(\d+)ELi(\d+)ELi4ELi2ELi(\d+)ELi(\d+)ELb\dELi(\d+)E", name) or \
        re.search(r"k_screen_x1ILi(\d+)ELi(\d+)ELi4ELi2ELi(\d+)ELi(\d+)()", name)
    if t:
        ring = f",RING{t.group(5)}" if t.group(5) else ""
        fam += f"<KT{t.group(1)},SUB{t.group(2)},CT{t.group(3)},MODE{t.group(4)}{ring}>"
    t = re.search(r"k_refine<(\d+), (\d+), (true|false)>", name) or re.search(r"k_refine_pairILi(\d+)", name)
    if t:
        fam += "<" + ",".join(t.groups()) + ">"
    return fam


def main(dirs):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for d in dirs:
        for db in glob.glob(f"{d}/**/*.db", recursive=True):
            c = sqlite3.connect(db)
            for disp, kname, cname, v, t in c.execute(
                    "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
                f = family(kname)
                vals[f][cname].append((db, disp, v))
                dur[f][(db, disp)] = t
    for f in sorted(vals):
        ds = list(dur[f].values())
        print(f"{f}: dispatches {len(ds)}, mean duration {sum(ds) / max(1, len(ds)) / 1e6:.3f} ms")
        for cname in sorted(vals[f]):
            per = collections.defaultdict(float)
            for db, disp, v in vals[f][cname]:
                per[(db, disp)] += v
            xs = list(per.values())
            print(f"    {cname:32s} {sum(xs) / len(xs):.4g}")


if __name__ == "__main__":
    main(sys.argv[1:])

#!/usr/bin/env python3
"""Merged kernel + memory-copy timeline (rocprofv3 csv) of the last T milliseconds.

    python tools/timeline.py gpurun_out/tl/prof [T_ms]
"""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    span = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
    ev = []
    kp = os.path.join(d, "run_kernel_trace.csv")
    mp = os.path.join(d, "run_memory_copy_trace.csv")
    for r in csv.DictReader(open(kp)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:60]))
    if os.path.exists(mp):
        for r in csv.DictReader(open(mp)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", r["Direction"]))
    ev.sort()
    tend = max(e for _, e, _, _ in ev)
    t0 = tend - span * 1e6
    for s, e, kind, name in ev:
        if e < t0:
            continue
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  {kind} {name}")


if __name__ == "__main__":
    main()

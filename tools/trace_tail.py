#!/usr/bin/env python3
"""Print the last N kernel dispatches of a rocprofv3 kernel trace as a timeline.

    python tools/trace_tail.py gpurun_out/r1d/prof/run_kernel_trace.csv [N]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    prev = None
    for r in rows[-n:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e6:10.3f} ms  gap {gap:8.1f} us  dur {(e - s) / 1e3:9.1f} us  "
              f"{r['Kernel_Name'][:70]}")
        prev = e


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summaries of rocprofv3 kernel + memory-copy traces for the copy-engine questions.

    python tools/copy_kind.py probe D  tests/native/copy_kind_probe.cpp's ops: blit kernel / SDMA
    python tools/copy_kind.py step D   per step of a bench run (between k_screen_x1 dispatches):
                                       every runtime kernel (__amd_rocclr_*) and SDMA copy
"""
import csv
import glob
import os
import sys


def _rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def _ev(d):
    ev = []
    for r in _rows(d, "kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"], r))
    mc = _rows(d, "memory_copy_trace.csv")
    if mc:
        print("# memory_copy_trace columns:", ", ".join(mc[0].keys()))
    for r in mc:
        nb = r.get("Bytes") or r.get("Size") or r.get("Copy_Bytes") or "?"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M",
                   f"SDMA {r.get('Direction', '?')} {nb}B", r))
    ev.sort(key=lambda e: e[0])
    return ev


def probe(d):
    ev = _ev(d)
    idx = -1
    per = {}
    for s, e, kind, name, _ in ev:
        if kind == "K" and "k_marker" in name:
            idx += 1
            continue
        if idx < 0:
            continue
        per.setdefault(idx, []).append(f"{'KERNEL ' + name.split('(')[0] if kind == 'K' else name}"
                                       f" {(e - s) / 1e3:.1f}us")
    # the probe prints "op kind bytes" for the second pass; ops are numbered from 0 over both
    # passes, markers precede every op
    for i in sorted(per):
        print(f"op {i}: " + "; ".join(per[i]))


def step(d):
    ev = _ev(d)
    # a step's events: from 0.5 ms before its screen dispatch (the query operands cross first)
    # to 0.5 ms before the next one's
    t_scr = [x[0] for x in ev if x[2] == "K" and "k_screen_x1" in x[3]]
    for a, t0 in enumerate(t_scr):
        t1 = t_scr[a + 1] - 500_000 if a + 1 < len(t_scr) else float("inf")
        lines = []
        nk = nm = 0
        tk = 0.0
        for s, e, kind, name, _ in ev:
            if s < t0 - 500_000 or s >= t1:
                continue
            if kind == "K" and name.startswith("__amd_rocclr"):
                nk += 1
                tk += (e - s) / 1e3
                lines.append(f"  {(s - t0) / 1e3:8.1f}us  {(e - s) / 1e3:7.1f}us  KERNEL {name.split('(')[0]}")
            elif kind == "M":
                nm += 1
                lines.append(f"  {(s - t0) / 1e3:8.1f}us  {(e - s) / 1e3:7.1f}us  {name}")
            elif kind == "K":
                lines.append(f"  {(s - t0) / 1e3:8.1f}us  {(e - s) / 1e3:7.1f}us  kernel {name[:50]}")
        print(f"== step at screen dispatch {a}: runtime kernels {nk} ({tk:.0f} us), SDMA copies {nm}")
        print("\n".join(lines))


if __name__ == "__main__":
    {"probe": probe, "step": step}[sys.argv[1]](sys.argv[2])

#!/usr/bin/env python3
"""Per-variant summary of plain kernel_ab.sh runs (AB_PROF=0): ms/step and the native step's
hipEvent timeline (bench.py's per_rank step_timeline_ms), averaged over the rounds."""
import collections
import glob
import json
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
acc = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(base, "*.log"))):
    name = os.path.basename(f).split(".")[0]
    lines = [ln for ln in open(f) if ln.startswith("{")]
    if lines:
        acc[name].append(json.loads(lines[-1]))
for name, runs in acc.items():
    ms = [r["ms_per_step"] for r in runs]
    tl = collections.defaultdict(list)
    for r in runs:
        for k, v in r["per_rank"][0].get("step_timeline_ms", {}).items():
            tl[k].append(v)
    ns = runs[-1].get("native_step", {})
    print(f"{name:8s} ms/step {' '.join(f'{m:.3f}' for m in ms)} | " +
          " ".join(f"{k} {sum(v) / len(v):.3f}" for k, v in tl.items()) +
          "")

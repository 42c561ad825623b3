#!/usr/bin/env python3
"""Bench sweep outside the headline shape:
N in {1e5, 1e6, 1e7} x A in {32, 128} x k in {16, mixed 1-64, 200}, one bench.py run per
config on one GPU (synthetic generate_input.py-distributed data, exact fp64 results).

    python tools/bench_sweep.py --out gpurun_out/sweep.jsonl [--q 16384] [--timeout 300]

Q per config is --q (default 16384: the N = 1e7 exact-path configs stay within minutes); each
line of the output is bench.py's JSON plus "sweep": {N, A, k}; a markdown table goes to stdout.
Configs that exceed --timeout are recorded as {"status": "timeout"}.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--q", type=int, default=16384)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--ns", default="100000,1000000,10000000")
    ap.add_argument("--attrs", default="32,128")
    ap.add_argument("--ks", default="16,1-64,200")
    ap.add_argument("--exact", action="store_true", help="bench.py --exact (fp64-only path)")
    ap.add_argument("--append", action="store_true", help="append to --out")
    a = ap.parse_args()
    rows = []
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "a" if a.append else "w") as f:
        for n in (int(x) for x in a.ns.split(",")):
            for attrs in (int(x) for x in a.attrs.split(",")):
                for ks in a.ks.split(","):
                    kmin, kmax = (int(x) for x in ks.split("-")) if "-" in ks else (int(ks),) * 2
                    big = n * attrs >= 10_000_000 * 32
                    steps, warm = (3, 1) if big else (10, 2)
                    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--n-data", str(n),
                           "--attrs", str(attrs), "--k", str(kmin), "--kmin", str(kmin),
                           "--kmax", str(kmax), "--q-per-gpu", str(a.q), "--steps", str(steps),
                           "--warmup", str(warm), "--no-busbw"] + (["--exact"] if a.exact else [])
                    t0 = time.time()
                    rec = {"sweep": {"N": n, "A": attrs, "k": ks, "exact": a.exact}}
                    try:
                        r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout,
                                           cwd=ROOT)
                        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
                        if r.returncode == 0 and line:
                            rec.update(json.loads(line[-1]))
                            rec["status"] = "ok"
                        else:
                            rec["status"] = f"rc={r.returncode}"
                            rec["stderr_tail"] = r.stderr[-600:]
                    except subprocess.TimeoutExpired:
                        rec["status"] = "timeout"
                    rec["wall_s"] = round(time.time() - t0, 1)
                    f.write(json.dumps(rec) + "\n")
                    f.flush()
                    rows.append(rec)
                    print(f"[sweep] N={n} A={attrs} k={ks}: {rec['status']} "
                          f"{rec.get('ms_per_step', '-')} ms/step ({rec['wall_s']} s)", flush=True)
    print("\n| N | A | k | ms/step | queries/s | status |\n|---|---|---|---|---|---|")
    for r in rows:
        s = r["sweep"]
        print(f"| {s['N']} | {s['A']} | {s['k']} | {r.get('ms_per_step', '-')} | "
              f"{r.get('value', '-')} | {r['status']} |")


if __name__ == "__main__":
    main()

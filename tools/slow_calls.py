#!/usr/bin/env python3
"""Name the host calls that blocked: stream every ``*hip_api_trace.csv`` (and ``*kernel_trace.csv``)
under a rocprofv3 output directory and print each HIP runtime call / kernel longer than a threshold,
with its thread, start time relative to the first record and duration, plus a per-function tally.

    rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d /tmp/wd -- python3 child.py
    python tools/slow_calls.py /tmp/wd 50 > gpurun_out/wd_slow_calls.txt

(Used for the watchdog rehearsal: which call on the healthy slot's path waited behind the hung
queue.)  The traces are read line by line, so multi-GB files cost no memory."""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def main() -> None:
    root = sys.argv[1]
    thr_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
    thr_ns = thr_ms * 1e6
    api = sorted(glob.glob(os.path.join(root, "**", "*hip_api_trace.csv"), recursive=True))
    ker = sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True))
    slow, tally, t_first = [], defaultdict(lambda: [0, 0, 0.0]), None
    for p in api:
        for r in rows(p):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            t_first = t0 if t_first is None else min(t_first, t0)
            fn = r["Function"]
            tl = tally[fn]
            tl[0] += 1
            if t1 - t0 > thr_ns:
                tl[1] += 1
                tl[2] = max(tl[2], (t1 - t0) / 1e6)
                slow.append((t0, t1, fn, r.get("Thread_Id", "?")))
    kslow = []
    for p in ker:
        for r in rows(p):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if t1 - t0 > thr_ns:
                kslow.append((t0, t1, r["Kernel_Name"][:90], r.get("Queue_Id", "?"), r.get("Thread_Id", "?")))
    t_first = t_first or 0
    print(f"# HIP runtime calls longer than {thr_ms} ms ({len(slow)}), start relative to the first call")
    print(f"{'start_s':>10} {'ms':>10}  thread      function")
    for t0, t1, fn, th in sorted(slow):
        print(f"{(t0 - t_first) / 1e9:10.3f} {(t1 - t0) / 1e6:10.2f}  {th:<10}  {fn}")
    print(f"\n# kernels longer than {thr_ms} ms ({len(kslow)})")
    for t0, t1, k, q, th in sorted(kslow):
        print(f"{(t0 - t_first) / 1e9:10.3f} {(t1 - t0) / 1e6:10.2f}  q{q:<4} thread {th:<10} {k}")
    print("\n# per function: calls, calls over the threshold, longest ms")
    for fn, (n, ns, mx) in sorted(tally.items(), key=lambda kv: -kv[1][2]):
        if ns:
            print(f"{fn:<40} {n:>10} {ns:>6} {mx:10.2f}")


if __name__ == "__main__":
    main()

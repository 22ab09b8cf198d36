#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 SQLite output (``-o run`` -> ``run_results.db``): dispatch
count, total / mean / max microseconds per kernel name, and the wall span of the dispatches.
Usage: ``python tools/rocpd_kernels.py <db> [--like sup_] [--top 30]``."""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--like", default="")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        n = re.sub(r"\(anonymous namespace\)::", "", str(n))
        n = re.sub(r"\((?!anonymous).*", "", n)
        if a.like and a.like not in n:
            continue
        d = (e - s) / 1000.0
        t = agg.setdefault(n, [0, 0.0, 0.0])
        t[0] += 1
        t[1] += d
        t[2] = max(t[2], d)
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':60s} {'n':>6s} {'total_us':>10s} {'mean_us':>8s} {'max_us':>8s}")
    for n, (k, s, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{n[:60]:60s} {k:6d} {s:10.1f} {s / k:8.2f} {mx:8.2f}")
    print(f"total {tot:.1f} us over {sum(v[0] for v in agg.values())} dispatches")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel SUMS of rocprofv3 --pmc counters over all dispatches (one counter group per run dir),
with time-weighted rates — for kernels launched many times at varying sizes (the CCH level
kernels: ~1000 dispatches per customization), where a mean per dispatch hides the big levels.

    python tools/pmc_sum.py gpurun_out/r5c/pmc 'level|pull|prune' > profiles/cch_pmc_r5c.md

Columns: dispatches, total device time (from the first group's trace), the summed counters, and
derived: wave-cycles waiting on any instruction (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES), issue share
(SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES), L2 hit rate (TCC_HIT / (TCC_HIT + TCC_MISS)), HBM traffic
(FETCH_SIZE + WRITE_SIZE, KB -> GB) and its rate over the kernel's device time, mean waves per
dispatch."""
from __future__ import annotations

import csv
import glob
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("rt::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:60]


def main() -> None:
    prefix, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    tot = defaultdict(lambda: defaultdict(float))
    ns = defaultdict(float)
    disp = defaultdict(set)
    for gi, f in enumerate(sorted(glob.glob(prefix + "*/*counter_collection.csv"))):
        seen = set()
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if not pat.search(k):
                    continue
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                key = (k, r["Dispatch_Id"])
                if gi == 0 and key not in seen:
                    seen.add(key)
                    ns[k] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                    disp[k].add(r["Dispatch_Id"])
    cols = sorted({c for k in tot for c in tot[k]})
    hdr = ["kernel", "dispatches", "device ms"] + cols + ["wait/wave-cyc", "issue/wave-cyc", "L2 hit %",
                                                          "HBM GB", "HBM GB/s", "waves/dispatch"]
    print("| " + " | ".join(hdr) + " |")
    print("|---" * len(hdr) + "|")
    for k in sorted(tot, key=lambda x: -ns[x]):
        t = tot[k]
        ms = ns[k] / 1e6
        wc = t.get("SQ_WAVE_CYCLES", 0.0)
        wait = t.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else float("nan")
        issue = t.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else float("nan")
        hm = t.get("TCC_HIT_sum", 0.0) + t.get("TCC_MISS_sum", 0.0)
        hit = 100 * t.get("TCC_HIT_sum", 0.0) / hm if hm else float("nan")
        gb = (t.get("FETCH_SIZE", 0.0) + t.get("WRITE_SIZE", 0.0)) / 1024 / 1024
        nd = max(1, len(disp[k]))
        row = [f"`{k}`", str(len(disp[k])), f"{ms:.2f}"] + [f"{t[c]:.4g}" if c in t else "" for c in cols]
        row += [f"{wait:.2f}", f"{issue:.3f}", f"{hit:.1f}", f"{gb:.2f}", f"{gb / (ms / 1e3):.0f}" if ms else "",
                f"{t.get('SQ_WAVES', 0.0) / nd:.0f}"]
        print("| " + " | ".join(row) + " |")


if __name__ == "__main__":
    main()

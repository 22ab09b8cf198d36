#!/usr/bin/env python3
"""Mean-per-dispatch PMC table from several single-group rocprofv3 --pmc runs of the same program.

    python tools/pmc_table.py gpurun_out/r3g/astar 'astar' > profiles/astar_pmc_r3.md

reads <prefix>1/ ... <prefix>N/ (*counter_collection.csv: one counter group per run, as gpurun
requires), keeps kernels whose name matches the regex, and prints one markdown row per kernel with
the mean of every counter over its dispatches plus derived ratios: VALU per MFMA instruction, LDS
bank-conflict cycles per LDS instruction, MFMA-busy share of the busy cycles, and L2<->HBM bytes
(FETCH_SIZE / WRITE_SIZE are in KB)."""
from __future__ import annotations

import csv
import glob
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("rt::", "")
    return name.replace("(anonymous namespace)::", "")[:70]


def main() -> None:
    prefix, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    vals = defaultdict(lambda: defaultdict(list))        # kernel -> counter -> per-dispatch values
    dur = defaultdict(list)
    for f in sorted(glob.glob(prefix + "*/*counter_collection.csv")):
        per = defaultdict(dict)
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if not pat.search(k):
                    continue
                d = r["Dispatch_Id"]
                per[(k, d)][r["Counter_Name"]] = float(r["Counter_Value"])
                per[(k, d)]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for (k, d), cs in per.items():
            for c, v in cs.items():
                if c == "_ns":
                    dur[k].append(v)
                else:
                    vals[k][c].append(v)
    cols = sorted({c for k in vals for c in vals[k]})
    print("| kernel | dispatches | mean us | " + " | ".join(cols) + " | VALU/MFMA | LDS conflict/inst | MFMA busy % | HBM MB |")
    print("|---" * (len(cols) + 7) + "|")
    for k in sorted(vals):
        m = {c: sum(v) / len(v) for c, v in vals[k].items()}
        n = max(len(v) for v in vals[k].values())
        us = sum(dur[k]) / len(dur[k]) / 1e3 if dur[k] else float("nan")
        valu_mfma = m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"] if m.get("SQ_INSTS_MFMA") else float("nan")
        conf = (m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"]) if m.get("SQ_INSTS_LDS") else float("nan")
        busy = (100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / m["SQ_BUSY_CYCLES"]) if m.get("SQ_BUSY_CYCLES") else float("nan")
        hbm = (m.get("FETCH_SIZE", 0) + m.get("WRITE_SIZE", 0)) / 1024
        print(f"| `{k}` | {n} | {us:.1f} | " + " | ".join(f"{m[c]:.4g}" if c in m else "" for c in cols)
              + f" | {valu_mfma:.2f} | {conf:.3f} | {busy:.1f} | {hbm:.1f} |")


if __name__ == "__main__":
    main()

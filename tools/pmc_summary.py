#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (bench/profile_pmc.sh output) per kernel as a markdown table:
MFMA busy % of SQ busy cycles, MFMA / VALU / LDS instructions per wave, LDS bank-conflict rate,
waves.  Usage: python tools/pmc_summary.py gpurun_out/pmc > profiles/pmc_summary_r1.md"""
from __future__ import annotations

import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("rt::", "")
    return name[:60]


FLOP_PER_MFMA = 32 * 32 * 16 * 2      # v_mfma_f32_32x32x16_bf16: every hand-written kernel here


def durations(root: str):
    """(tag, kernel) -> total ns from the kernel traces of the same counter runs."""
    out = defaultdict(float)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        d = os.path.basename(os.path.dirname(f))
        if not d.endswith("_g1"):
            continue
        tag = d.split("_")[0]
        with open(f) as fh:
            for r in csv.DictReader(fh):
                out[(tag, short(r["Kernel_Name"]))] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return out


def main() -> None:
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    dur = durations(root)
    acc = defaultdict(lambda: defaultdict(float))     # (tag, kernel) -> counter -> sum
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        tag = os.path.basename(os.path.dirname(f)).split("_")[0]
        with open(f) as fh:
            for r in csv.DictReader(fh):
                acc[(tag, short(r["Kernel_Name"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    print("| workload | kernel | waves | MFMA inst/wave | VALU inst/wave | LDS inst/wave | LDS bank conflicts | "
          "LDS-wait % of wave cycles | MFMA TFLOP/s (under PMC) |")
    print("|---|---|---|---|---|---|---|---|---|")
    for (tag, k), c in sorted(acc.items()):
        waves = c.get("SQ_WAVES", 0)
        if waves < 500 and "SQ_WAVE_CYCLES" not in c:
            continue

        def per_wave(n):
            return f"{c[n] / waves:.0f}" if waves and n in c else "–"
        wave_cyc = c.get("SQ_WAVE_CYCLES", 0)
        lds_wait = f"{100 * c.get('SQ_WAIT_INST_LDS', 0) / wave_cyc:.1f}" if wave_cyc else "–"
        conf = f"{c['SQ_LDS_BANK_CONFLICT']:.3g}" if "SQ_LDS_BANK_CONFLICT" in c else "–"
        ns = dur.get((tag, k), 0.0)
        lib = k.startswith("Cijk")                    # hipBLASLt: different MFMA shapes
        tf = (f"{c['SQ_INSTS_MFMA'] * FLOP_PER_MFMA / ns / 1e3:.0f}"
              if ns and c.get("SQ_INSTS_MFMA") and not lib else "–")
        print(f"| {tag} | `{k}` | {waves:.0f} | {per_wave('SQ_INSTS_MFMA')} | {per_wave('SQ_INSTS_VALU')} | "
              f"{per_wave('SQ_INSTS_LDS')} | {conf} | {lds_wait} | {tf} |")


if __name__ == "__main__":
    main()

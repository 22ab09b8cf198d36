#!/usr/bin/env python3
"""Scaling table from ``bench.py`` JSON lines run at several GPU counts (one line per N, e.g.
``for n in 1 2 4 8; do python bench.py --gpus $n; done > scale.jsonl``).

Prints a markdown table per config the line carries: the headline (config 2, inference sharding),
DP training at 64k and 1M rows per GPU over RCCL and over the one-shot all-reduce (config 3), the GCN
scorer replicated / row-partitioned (config 4) and the route optimizer (config 5), each with the
whole-job rate per N and the efficiency at the largest N against the smallest:
rate_N / (N / N0 * rate_N0).  All rates are whole-job rates; the headline and training are weak
scaling (fixed work per GPU), the GCN and route steps split a fixed 10k total over the ranks.
Usage: python tools/scaling_table.py scale.jsonl [more.jsonl ...]  (or stdin)."""
from __future__ import annotations

import json
import sys
from typing import Callable, Dict, List, Optional, Tuple


def _get(d: dict, path: str) -> Optional[float]:
    cur = d
    for k in path.split("."):
        if not isinstance(cur, dict) or k not in cur or cur[k] is None:
            return None
        cur = cur[k]
    return float(cur) if isinstance(cur, (int, float)) else None


ROWS: List[Tuple[str, str, str]] = [
    ("config 2: ETA preds/s (headline)", "value", "preds/s"),
    ("config 3: DP training, 64k rows/GPU, RCCL", "dp_training.samples_per_s", "samples/s"),
    ("config 3: DP training, 64k rows/GPU, one-shot", "dp_training_oneshot.samples_per_s", "samples/s"),
    ("config 3: DP training, 1M rows/GPU, RCCL", "dp_training_large_batch.samples_per_s", "samples/s"),
    ("config 4: GCN scorer, replicated", "gcn.replicate.routes_per_s", "routes/s"),
    ("config 4: GCN scorer, row-partitioned (RCCL)", "gcn.partition.routes_per_s", "routes/s"),
    ("config 4: GCN scorer, row-partitioned (one-shot)", "gcn.partition_oneshot.routes_per_s", "routes/s"),
    ("config 5: route optimizer", "route_optimizer.requests_per_s", "requests/s"),
]


def load(lines: List[str]) -> Dict[int, dict]:
    out: Dict[int, dict] = {}
    for ln in lines:
        ln = ln.strip()
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        if "n_gpus" in d and "value" in d:
            out[int(d["n_gpus"])] = d
    return out


def table(runs: Dict[int, dict], fmt: Callable[[float], str] = lambda v: f"{v:.4g}") -> str:
    ns = sorted(runs)
    if not ns:
        return "(no bench lines)\n"
    n0 = ns[0]
    head = "| config | unit | " + " | ".join(f"N={n}" for n in ns) + " | efficiency at N=" + str(ns[-1]) + " |\n"
    head += "|---|---|" + "---|" * len(ns) + "---|\n"
    body = ""
    for name, path, unit in ROWS:
        vals = [_get(runs[n], path) for n in ns]
        if all(v is None for v in vals):
            continue
        v0, vl = vals[0], vals[-1]
        eff = (f"{100.0 * vl / (v0 * ns[-1] / n0):.1f} %" if v0 and vl is not None and len(ns) > 1 else "-")
        body += f"| {name} | {unit} | " + " | ".join("-" if v is None else fmt(v) for v in vals) + f" | {eff} |\n"
    shared = [n for n in ns if runs[n].get("shared_gpu")]
    note = (f"\nN = {shared}: ranks SHARED one GPU (rehearsal) — not a whole-node number.\n" if shared else "")
    return head + body + note


def main(argv: List[str]) -> int:
    lines: List[str] = []
    if len(argv) > 1:
        for p in argv[1:]:
            with open(p) as f:
                lines.extend(f.readlines())
    else:
        lines = sys.stdin.readlines()
    sys.stdout.write(table(load(lines)))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))

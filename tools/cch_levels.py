#!/usr/bin/env python3
"""Work per elimination-tree level of the CCH customization (csrc/cch.hip): how many levels the
basic (by height) and perfect (by depth) phases have, and how their items are distributed — the
input for choosing which levels run in the one-workgroup persistent kernel and which get a full
grid launch.  Usage: ``python tools/cch_levels.py [nodes] [--json out]``."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def level_stats(n: int, seed: int = 0) -> dict:
    from routest_amd.data.graph import synth_road_graph
    import routest_amd._rt as rt
    g = synth_road_graph(n, seed=seed)
    c = rt.CCH(g.indptr, g.indices, g.lat, g.lon, 8)
    a = c.arrays()
    out = {"stats": {k: (int(v) if isinstance(v, (int, np.integer)) else v) for k, v in c.stats().items()}}
    k = np.diff(np.asarray(a["up_ptr"])).astype(np.int64)
    for name, lev, it in (("basic", np.asarray(a["height"]), k * (k + 1) // 2),
                          ("perfect", np.asarray(a["depth"]), k * (k - 1))):
        L = int(lev.max()) + 1
        items = np.bincount(lev, weights=it, minlength=L)
        sec = {"levels": L, "items": float(items.sum()),
               "pct_items": [float(x) for x in np.percentile(items, [10, 50, 90, 99])],
               "max_items": float(items.max()), "below": {}}
        for thr in (256, 1024, 4096, 16384, 65536, 262144):
            m = items < thr
            sec["below"][thr] = {"levels": int(m.sum()), "share_of_items": float(items[m].sum() / items.sum())}
        out[name] = sec
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("nodes", type=int, nargs="?", default=100_000)
    ap.add_argument("--json")
    a = ap.parse_args()
    r = level_stats(a.nodes)
    print(json.dumps(r, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(r, f, indent=1)

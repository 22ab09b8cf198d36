#!/usr/bin/env python3
"""Print the PCIe path from each visible GPU up to the root port (sysfs only, no GPU init):
link speed / width of every bridge, and how many GPUs sit below each bridge.  Tells whether the
host links of the node's GPUs are private x16 links or share a switch uplink (which would cap
whole-node host->device streaming)."""
import glob
import json
import os


def attr(p, n):
    try:
        return open(os.path.join(p, n)).read().strip()
    except OSError:
        return None


def main():
    gpus = []
    for d in glob.glob("/sys/bus/pci/devices/*"):
        cls = attr(d, "class") or ""
        ven = attr(d, "vendor") or ""
        if ven == "0x1002" and cls.startswith("0x0380") or (ven == "0x1002" and cls.startswith("0x0300")):
            gpus.append(os.path.realpath(d))
    out = {"gpus_in_sysfs": len(gpus), "paths": []}
    below = {}
    for g in gpus:
        p = g
        while True:
            p = os.path.dirname(p)
            if not os.path.basename(p).count(":"):
                break
            below.setdefault(p, set()).add(g)
    for g in sorted(gpus):
        chain = []
        p = g
        while os.path.basename(p).count(":"):
            chain.append({"bdf": os.path.basename(p), "speed": attr(p, "current_link_speed"),
                          "width": attr(p, "current_link_width"), "max_width": attr(p, "max_link_width"),
                          "numa": attr(p, "numa_node"), "gpus_below": len(below.get(p, {g}))})
            p = os.path.dirname(p)
        out["paths"].append(chain)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

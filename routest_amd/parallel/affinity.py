"""NUMA placement: pin a rank's host threads (and hence its first-touch pinned buffers) to the CPUs
local to its GPU's PCIe root.  Matters for the zero-copy serving path, where the fused kernel
streams request records out of pinned host memory over that GPU's own PCIe x16 link."""
from __future__ import annotations

import os
from typing import List, Optional


def _parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_numa_node(device_index: int) -> Optional[int]:
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        bdf = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read().strip())
        return node if node >= 0 else None
    except Exception:
        return None


def bind_to_gpu_numa(device_index: int) -> Optional[int]:
    """Restrict this process to the CPUs of the GPU's NUMA node; returns the node (or None)."""
    node = gpu_numa_node(device_index)
    if node is None:
        return None
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = set(_parse_cpulist(f.read())) & set(os.sched_getaffinity(0))
        if cpus:
            os.sched_setaffinity(0, cpus)
            return node
    except Exception:
        pass
    return None

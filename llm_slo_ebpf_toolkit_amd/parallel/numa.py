"""NUMA placement for one-process-per-GPU runs.

Each rank streams its window records host -> device over its own PCIe link (24 MiB per 1M-event
window at ~55 GB/s on MI355X). On a two-socket 8-GPU node half of the GPUs hang off each socket;
a rank whose pinned ring sits on the far socket's DRAM pulls every DMA across the inter-socket
fabric, so 4 ranks x 55 GB/s contend there and weak scaling sags. Binding the rank to the CPUs
local to its GPU before anything pinned is allocated keeps the ring (first-touch placement) and
the host threads on the GPU's socket.

REF has no equivalent (one Go agent per node, no device boundary).
"""

from __future__ import annotations

import os
from typing import Iterable, Optional, Set


def parse_cpulist(text: str) -> Set[int]:
    """``"0-3,8,10-11"`` -> {0, 1, 2, 3, 8, 10, 11} (Linux cpulist format)."""
    out: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.update(range(int(lo), int(hi) + 1))
        else:
            out.add(int(part))
    return out


def pci_bdf(domain: int, bus: int, device: int, function: int = 0) -> str:
    return f"{domain:04x}:{bus:02x}:{device:02x}.{function:x}"


def local_cpus_of_pci(bdf: str, sysfs: str = "/sys/bus/pci/devices") -> Optional[Set[int]]:
    """CPUs local to a PCI device, or None when sysfs does not say (VMs report numa_node -1)."""
    base = os.path.join(sysfs, bdf)
    try:
        with open(os.path.join(base, "numa_node")) as fh:
            if int(fh.read().strip()) < 0:
                return None
        with open(os.path.join(base, "local_cpulist")) as fh:
            cpus = parse_cpulist(fh.read())
    except (OSError, ValueError):
        return None
    return cpus or None


def choose_affinity(allowed: Iterable[int], local: Optional[Set[int]]) -> Optional[Set[int]]:
    """The rank's CPU set: allowed ∩ local, unless that is empty or changes nothing."""
    allowed = set(allowed)
    if not local:
        return None
    pick = allowed & local
    if not pick or pick == allowed:
        return None
    return pick


def bind_to_device_numa(device_index: int, sysfs: str = "/sys/bus/pci/devices") -> Optional[Set[int]]:
    """Pin this process to the CPUs local to GPU ``device_index``. Returns the new CPU set, or
    None when nothing changed (single socket, unknown topology, restricted cpuset, or
    ``MISLO_NUMA_BIND=0``). Call before allocating pinned host memory."""
    if os.environ.get("MISLO_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    import torch

    p = torch.cuda.get_device_properties(device_index)
    bdf = pci_bdf(int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    pick = choose_affinity(os.sched_getaffinity(0), local_cpus_of_pci(bdf, sysfs))
    if pick is None:
        return None
    try:
        os.sched_setaffinity(0, pick)
    except OSError:
        return None
    return pick


def visible_gpu_count(topology: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this process may use, WITHOUT initialising the HIP runtime (a process that forks or
    spawns GPU workers must not): the device-visibility env if set, else the KFD topology's GPU
    nodes (gpu_id != 0; readable without root)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    n = 0
    try:
        for node in os.listdir(topology):
            try:
                with open(os.path.join(topology, node, "gpu_id")) as fh:
                    n += int(fh.read().strip() or 0) != 0
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    return n

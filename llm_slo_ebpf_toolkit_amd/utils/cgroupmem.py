"""The memory a process's cgroup is charged, next to its RSS.

RSS counts every resident page a process maps, including pages the kernel never charges to the
process's memory cgroup and shared pages another process first touched. A pod's memory limit is
enforced on the cgroup's charge, so the charge is the number a memory budget is about:

* cgroup v2: ``memory.current`` and ``memory.stat`` (``anon``, ``file``, ``shmem``, ``kernel``)
  of the directory ``/proc/<pid>/cgroup``'s ``0::`` line names;
* cgroup v1: ``memory.usage_in_bytes`` and ``memory.stat`` (``rss``, ``cache``, ``shmem``,
  ``mapped_file``) of the ``memory`` controller's directory.

Inside a cgroup namespace the path a process sees may not exist under ``/sys/fs/cgroup``; the
controller's root directory is then the process's own cgroup (the namespace root).

The charge is per cgroup, not per process: ``delta()`` of two readings around a process's start
is that process's charge when nothing else in the cgroup changes meanwhile (the measuring tools
take it that way and say so).
"""

from __future__ import annotations

import os
from typing import Dict, Optional

ROOT = "/sys/fs/cgroup"
V2_KEYS = ("anon", "file", "shmem", "kernel", "sock", "file_mapped")
V1_KEYS = ("rss", "cache", "shmem", "mapped_file")


def _read_int(path: str) -> Optional[int]:
    try:
        with open(path) as f:
            return int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return None


def _stat(path: str, keys) -> Dict[str, int]:
    out = {}
    try:
        with open(path) as f:
            for ln in f:
                k, _, v = ln.partition(" ")
                if k in keys:
                    out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def cgroup_dir(pid: str = "self", root: str = ROOT) -> Optional[tuple]:
    """(version, directory) of ``pid``'s memory cgroup, or None without one."""
    try:
        with open(f"/proc/{pid}/cgroup") as f:
            lines = [ln.rstrip("\n").split(":", 2) for ln in f if ln.strip()]
    except OSError:
        return None
    for hid, ctrls, path in lines:  # v1 memory controller first: a hybrid host has both
        if "memory" in ctrls.split(","):
            for d in (os.path.join(root, "memory", path.lstrip("/")), os.path.join(root, "memory")):
                if os.path.exists(os.path.join(d, "memory.usage_in_bytes")):
                    return 1, d
    for hid, ctrls, path in lines:
        if hid == "0" and ctrls == "":
            for d in (os.path.join(root, path.lstrip("/")), root):
                if os.path.exists(os.path.join(d, "memory.current")):
                    return 2, d
    return None


def reading(pid: str = "self", root: str = ROOT) -> Optional[Dict[str, object]]:
    """{"version", "dir", "charged_bytes", "stat": {...}} of ``pid``'s memory cgroup."""
    cd = cgroup_dir(pid, root)
    if cd is None:
        return None
    ver, d = cd
    if ver == 2:
        cur, st = _read_int(os.path.join(d, "memory.current")), _stat(os.path.join(d, "memory.stat"), V2_KEYS)
    else:
        cur, st = _read_int(os.path.join(d, "memory.usage_in_bytes")), _stat(os.path.join(d, "memory.stat"), V1_KEYS)
    if cur is None:
        return None
    return {"version": ver, "dir": d, "charged_bytes": cur, "stat": st}


def delta(before: Optional[dict], after: Optional[dict]) -> Optional[Dict[str, float]]:
    """MB the cgroup's charge and each stat field grew between two readings."""
    if not before or not after or before["dir"] != after["dir"]:
        return None
    out = {"charged_mb": round((after["charged_bytes"] - before["charged_bytes"]) / 2**20, 1)}
    for k, v in after["stat"].items():
        out[f"{k}_mb"] = round((v - before["stat"].get(k, 0)) / 2**20, 1)
    return out

"""Facts about the GPU box that shape the unprivileged signal sources (printed as one JSON object).

* the process's cgroup v2 group: cpu.max (a CPU quota makes CFS throttling observable in
  cpu.stat without root), cpu.stat, cpu.pressure / memory.pressure, and whether the group (or a
  child) is writable by this user;
* node-wide PSI;
* the amdgpu sysfs files of the visible GPU (gpu_busy_percent, gpu_metrics) that a "foreign GPU
  load" signal reads.

    python tools/box_facts.py > gpurun_out/box_facts.json
"""

from __future__ import annotations

import glob
import json
import os
import sys


def read(path: str, limit: int = 4096):
    try:
        with open(path, "rb") as fh:
            b = fh.read(limit)
        try:
            return b.decode()
        except UnicodeDecodeError:
            return f"<{len(b)} binary bytes>"
    except OSError as e:
        return f"<{type(e).__name__}: {e.errno}>"


def main() -> int:
    out = {"uid": os.getuid(), "nproc_affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    cg = read("/proc/self/cgroup")
    out["proc_self_cgroup"] = cg
    rel = next((ln[3:].strip() for ln in cg.splitlines() if ln.startswith("0::")), None)
    out["cgroup_mounts"] = [ln for ln in read("/proc/self/mounts", 1 << 16).splitlines() if "cgroup" in ln]
    if rel is not None:
        base = os.path.join("/sys/fs/cgroup", rel.lstrip("/"))
        out["cgroup_dir"] = base
        for up in (base, os.path.dirname(base)):
            d = {}
            for f in ("cpu.max", "cpu.stat", "cpu.pressure", "memory.pressure", "memory.max", "cgroup.controllers",
                      "cgroup.subtree_control", "cpu.weight", "cpuset.cpus.effective"):
                d[f] = read(os.path.join(up, f))
            d["writable"] = os.access(up, os.W_OK)
            d["procs_writable"] = os.access(os.path.join(up, "cgroup.procs"), os.W_OK)
            out[f"cg:{up}"] = d
        try:
            child = os.path.join(base, "mislo-probe")
            os.mkdir(child)
            out["mkdir_child"] = "ok"
            out["child_cpu_max_writable"] = os.access(os.path.join(child, "cpu.max"), os.W_OK)
            os.rmdir(child)
        except OSError as e:
            out["mkdir_child"] = f"{type(e).__name__}: {e.errno}"
    for ln in cg.splitlines():   # cgroup v1 cpu / cpuacct hierarchies
        parts = ln.split(":", 2)
        if len(parts) == 3 and parts[0] != "0" and ("cpu" in parts[1].split(",") or "cpuacct" in parts[1].split(",")):
            for mnt in glob.glob("/sys/fs/cgroup/cpu*"):
                d = os.path.join(mnt, parts[2].lstrip("/"))
                out[f"v1:{d}"] = {f: read(os.path.join(d, f)) for f in ("cpu.cfs_quota_us", "cpu.cfs_period_us",
                                                                        "cpu.stat", "cpu.pressure", "cpuacct.usage")}
                out[f"v1:{d}"]["writable"] = os.access(d, os.W_OK)
    for f in ("cpu", "memory", "io"):
        out[f"psi_{f}"] = read(f"/proc/pressure/{f}")
    out["schedstat_self"] = read("/proc/self/schedstat")
    out["sched_features_autogroup"] = read("/proc/sys/kernel/sched_autogroup_enabled")
    drm = {}
    for card in sorted(glob.glob("/sys/class/drm/card*/device")):
        busy = os.path.join(card, "gpu_busy_percent")
        if not os.path.exists(busy):
            continue
        drm[card] = {"gpu_busy_percent": read(busy), "gpu_metrics": read(os.path.join(card, "gpu_metrics")),
                     "mem_busy_percent": read(os.path.join(card, "mem_busy_percent")),
                     "vram_used": read(os.path.join(card, "mem_info_vram_used"))}
    out["drm"] = drm
    out["kfd_nodes"] = sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*"))
    out["kfd_procs"] = read_dir("/sys/class/kfd/kfd/proc")
    json.dump(out, sys.stdout, indent=1)
    print()
    return 0


def read_dir(d: str):
    try:
        return sorted(os.listdir(d))[:16]
    except OSError as e:
        return f"<{type(e).__name__}>"


if __name__ == "__main__":
    sys.exit(main())

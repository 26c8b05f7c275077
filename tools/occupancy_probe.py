"""What KFD tells about each process's use of a GPU (/sys/class/kfd/kfd/proc/<pid>/...): lists the
per-process files, then samples every process's per-GPU ``cu_occupancy`` while a decode-like
victim runs alone and then next to a GEMM burner -- the data behind a foreign-GPU-load signal
that separates another process's work from the victim's own.

    python tools/occupancy_probe.py > gpurun_out/occupancy_probe.json
"""

from __future__ import annotations

import glob
import json
import os
import subprocess
import sys
import time

VICTIM = r"""
import sys, time, torch
w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
v = torch.randn(1, 4096, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
print("ready", flush=True)
end = time.time() + float(sys.argv[1])
while time.time() < end:
    h = v
    for _ in range(64):
        h = torch.nn.functional.silu(h @ w) * 0.01 + h
        h = h / (h.float().pow(2).mean().sqrt().to(h.dtype) + 1)
    torch.cuda.synchronize()
    time.sleep(0.005)
"""

BURNER = r"""
import sys, time, torch
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
print("ready", flush=True)
end = time.time() + float(sys.argv[1])
while time.time() < end:
    for _ in range(8):
        a = (a @ a).clamp_(-1, 1)
    torch.cuda.synchronize()
"""


def read(p: str) -> str:
    try:
        with open(p) as fh:
            return fh.read().strip()
    except OSError as e:
        return f"<{type(e).__name__} {e.errno}>"


def snapshot(pids=None):
    """cu_occupancy of every KFD process on the node (the entries are host pids: this box runs
    us in a pid namespace, so ``pids`` may not name them)."""
    out = {}
    for f in glob.glob("/sys/class/kfd/kfd/proc/*/stats_*/cu_occupancy"):
        parts = f.split("/")
        out[f"{parts[-3]}:{parts[-2]}"] = read(f)
    return out


def main() -> int:
    res = {"kfd_proc_entries": sorted(os.listdir("/sys/class/kfd/kfd/proc"))[:32]}
    v = subprocess.Popen([sys.executable, "-c", VICTIM, "12"], stdout=subprocess.PIPE, text=True)
    assert v.stdout.readline().startswith("ready")
    res["victim_files"] = {}
    for ent in sorted(os.listdir("/sys/class/kfd/kfd/proc"))[:6]:
        me = f"/sys/class/kfd/kfd/proc/{ent}"
        for root, dirs, files in os.walk(me):
            for f in files:
                p = os.path.join(root, f)
                res["victim_files"][p[len("/sys/class/kfd/kfd/proc/"):]] = read(p)[:120]
    res["status_nspid"] = [ln for ln in open("/proc/self/status") if ln.startswith(("NSpid", "Pid"))]
    samples = []
    b = None
    t0 = time.time()
    while time.time() - t0 < 9.0:
        if b is None and time.time() - t0 > 3.0:
            b = subprocess.Popen([sys.executable, "-c", BURNER, "8"], stdout=subprocess.PIPE, text=True)
            b.stdout.readline()
            res["burner_started_s"] = round(time.time() - t0, 3)
        pids = [v.pid] + ([b.pid] if b is not None else [])
        samples.append((round(time.time() - t0, 3), snapshot(pids)))
        time.sleep(0.02)
    res["victim_pid"] = v.pid
    res["burner_pid"] = b.pid if b is not None else None
    res["samples"] = samples
    for p in (v, b):
        if p is not None:
            p.kill()
            p.wait(10)
    json.dump(res, sys.stdout)
    print()
    return 0


if __name__ == "__main__":
    sys.exit(main())

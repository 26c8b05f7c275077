"""Is a HIP hardware queue's context save area charged to the process's memory cgroup?
(the agent's RSS is dominated by ~173 MB per queue on MI355X.)

For 0, 1, 2 and 3 streams (-1: the null stream only), a child process brings up the HIP runtime through ctypes (no torch),
creates that many streams (each with its own hardware queue: GPU_MAX_HW_QUEUES is set to the
stream count) and runs one memset on each, then holds still while the parent reads:

* the child's RSS and its split (the large equal-size anonymous mappings are the save areas,
  tools/agent_overhead.py rss_split);
* the growth of the cgroup's charge (utils/cgroupmem.py) from before the child started.

If the charge grows by the save areas, they count against a pod's memory limit; if it grows by
RSS minus the save areas, they do not (the kernel driver pins them outside the cgroup's charge).

    python tools/queue_mem_probe.py --out gpurun_out/queue_mem.json
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

CHILD = r"""
import ctypes, sys, time
n = int(sys.argv[1])
hip = ctypes.CDLL("libamdhip64.so")
assert hip.hipSetDevice(0) == 0
p = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)) == 0
if n < 0:  # the null stream only
    assert hip.hipMemsetAsync(p, 0, ctypes.c_size_t(1 << 20), None) == 0
for i in range(max(n, 0)):
    s = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
    assert hip.hipMemsetAsync(p, 0, ctypes.c_size_t(1 << 20), s) == 0
    assert hip.hipStreamSynchronize(s) == 0
assert hip.hipDeviceSynchronize() == 0
print("ready", flush=True)
time.sleep(float(sys.argv[2]))
"""


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--streams", default="0,1,2,3")
    ap.add_argument("--hold-s", type=float, default=6.0)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for the children (repeatable)")
    ap.add_argument("--out", default="gpurun_out/queue_mem.json")
    a = ap.parse_args()
    from agent_overhead import rss_split

    from llm_slo_ebpf_toolkit_amd.utils import cgroupmem

    rows = []
    for n in (int(x) for x in a.streams.split(",")):
        env = dict(os.environ, GPU_MAX_HW_QUEUES=str(max(1, n)))
        env.update(kv.split("=", 1) for kv in a.env)
        time.sleep(1.0)  # the previous child's pages are uncharged
        cg0 = cgroupmem.reading()
        ch = subprocess.Popen([sys.executable, "-c", CHILD, str(n), str(a.hold_s)], stdout=subprocess.PIPE, text=True,
                              env=env)
        try:
            line = ch.stdout.readline()
            if not line.startswith("ready"):
                raise RuntimeError(f"child with {n} streams failed: {line!r} rc={ch.wait(30)}")
            time.sleep(1.0)
            cg1 = cgroupmem.reading()
            split = rss_split(ch.pid)
        finally:
            ch.kill()
            ch.wait(30)
        r = {"streams": n, "rss_split_mb": split, "cgroup_charge_delta_mb": cgroupmem.delta(cg0, cg1),
             "cgroup": {"version": cg1["version"], "dir": cg1["dir"]} if cg1 else None}
        rows.append(r)
        print(json.dumps(r), flush=True)
    out = {"rows": rows, "env": a.env}
    if len(rows) >= 2 and all(r["cgroup_charge_delta_mb"] for r in rows):
        d_rss = rows[-1]["rss_split_mb"]["total_mb"] - rows[0]["rss_split_mb"]["total_mb"]
        d_q = rows[-1]["rss_split_mb"]["queue_save_areas_mb"] - rows[0]["rss_split_mb"]["queue_save_areas_mb"]
        d_cg = rows[-1]["cgroup_charge_delta_mb"]["charged_mb"] - rows[0]["cgroup_charge_delta_mb"]["charged_mb"]
        out["from_first_to_last"] = {"rss_mb": round(d_rss, 1), "save_areas_mb": round(d_q, 1),
                                     "cgroup_charge_mb": round(d_cg, 1),
                                     "save_areas_charged": bool(d_q > 0 and d_cg >= 0.5 * d_q)}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out.get("from_first_to_last")), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

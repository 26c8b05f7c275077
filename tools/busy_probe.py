"""How the amdgpu driver reports this GPU's activity, for a "foreign GPU load" signal.

Runs known duty cycles on the visible GPU and samples, on a side thread, the PCI device's
``gpu_busy_percent`` (every ~5 ms) and raw ``gpu_metrics`` snapshots (every ~50 ms). Writes the
time series as JSON; ``--analyze`` on that file finds the gpu_metrics words that move with the
load (an activity accumulator gives exact busy fractions over any interval).

    python tools/busy_probe.py --out gpurun_out/busy_probe.json
    python tools/busy_probe.py --analyze gpurun_out/busy_probe.json
"""

from __future__ import annotations

import argparse
import base64
import ctypes
import json
import os
import sys
import threading
import time


def pci_dir(device: int = 0) -> str:
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
        raise RuntimeError("hipDeviceGetPCIBusId failed")
    bdf = buf.value.decode().lower()
    return os.path.join("/sys/bus/pci/devices", bdf)


def sampler(d: str, stop: threading.Event, busy: list, metrics: list) -> None:
    fb = os.open(os.path.join(d, "gpu_busy_percent"), os.O_RDONLY)
    fm = os.open(os.path.join(d, "gpu_metrics"), os.O_RDONLY)
    k = 0
    while not stop.is_set():
        t0 = time.monotonic_ns()
        v = os.pread(fb, 16, 0)
        t1 = time.monotonic_ns()
        busy.append((t0, t1 - t0, int(v.strip() or b"-1")))
        if k % 10 == 0:
            t2 = time.monotonic_ns()
            m = os.pread(fm, 8192, 0)
            metrics.append((t2, time.monotonic_ns() - t2, base64.b64encode(m).decode()))
        k += 1
        time.sleep(0.005)


def run(out: str) -> None:
    import torch

    d = pci_dir(0)
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        (a @ b).sum().item()
    # one GEMM's time
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        c = a @ b
    torch.cuda.synchronize()
    gemm_ms = (time.perf_counter() - t) / 20 * 1e3
    stop = threading.Event()
    busy, metrics, phases = [], [], []
    th = threading.Thread(target=sampler, args=(d, stop, busy, metrics), daemon=True)
    th.start()

    def phase(name, seconds, on_ms, period_ms):
        t0 = time.monotonic_ns()
        end = time.monotonic() + seconds
        n_on = max(0, int(round(on_ms / gemm_ms)))
        while time.monotonic() < end:
            p0 = time.monotonic()
            for _ in range(n_on):
                c = a @ b  # noqa: F841
            torch.cuda.synchronize()
            rest = period_ms / 1e3 - (time.monotonic() - p0)
            if rest > 0:
                time.sleep(rest)
        phases.append((name, t0, time.monotonic_ns(), on_ms, period_ms))

    phase("idle", 1.5, 0, 100)
    phase("duty30", 2.0, 30, 100)
    phase("idle2", 1.0, 0, 100)
    phase("duty70", 2.0, 70, 100)
    phase("full", 1.5, 100, 100)
    phase("idle3", 1.5, 0, 100)
    stop.set()
    th.join()
    with open(out, "w") as f:
        json.dump({"pci": d, "gemm_ms": gemm_ms, "phases": phases, "busy": busy, "metrics": metrics}, f)
    print(json.dumps({"pci": d, "gemm_ms": gemm_ms, "busy_samples": len(busy), "metric_samples": len(metrics),
                      "read_us_busy_p50": sorted(x[1] for x in busy)[len(busy) // 2] / 1e3,
                      "read_us_metrics_p50": sorted(x[1] for x in metrics)[len(metrics) // 2] / 1e3}))


def analyze(path: str) -> None:
    import struct

    import numpy as np

    d = json.load(open(path))
    phases = d["phases"]
    busy = np.array([(t, v) for t, _, v in d["busy"]], dtype=np.int64)
    print("gemm_ms", d["gemm_ms"])
    for name, t0, t1, on, per in phases:
        m = (busy[:, 0] >= t0) & (busy[:, 0] < t1)
        v = busy[m, 1]
        print(f"{name:7s} expected {100 * on / per:5.1f}%  gpu_busy_percent mean {v.mean():6.1f} p10 {np.percentile(v, 10):5.1f} "
              f"p90 {np.percentile(v, 90):5.1f} n {m.sum()}")
    ms = [(t, base64.b64decode(b)) for t, _, b in d["metrics"]]
    raw = ms[0][1]
    size, fmt, content = struct.unpack_from("<HBB", raw, 0)
    print("gpu_metrics header: size", size, "format", fmt, "content", content, "bytes", len(raw))
    n32 = len(raw) // 4
    A = np.array([np.frombuffer(b[: n32 * 4], dtype="<u4") for _, b in ms], dtype=np.float64)
    T = np.array([t for t, _ in ms], dtype=np.float64)
    # expected busy fraction at each snapshot (the phase's duty)
    duty = np.zeros(len(T))
    for name, t0, t1, on, per in phases:
        duty[(T >= t0) & (T < t1)] = on / per
    dA = np.diff(A, axis=0)
    dT = np.diff(T) / 1e6
    dd = duty[1:]
    cands = []
    for j in range(n32):
        x = dA[:, j]
        if np.all(x == 0) or np.any(x < 0) and np.any(x > 0):
            continue
        if np.std(x) == 0:
            continue
        rate = x / dT
        c = np.corrcoef(rate, dd)[0, 1]
        if np.isfinite(c) and abs(c) > 0.6:
            cands.append((abs(c), j, c, float(np.mean(rate[dd == 0])) if np.any(dd == 0) else None,
                          float(np.mean(rate[dd >= 0.99])) if np.any(dd >= 0.99) else None))
    cands.sort(reverse=True)
    print("u32 words whose per-ms growth follows the duty cycle (corr, word, offset, idle rate/ms, full rate/ms):")
    for c, j, cc, idle, full in cands[:20]:
        print(f"  word {j:4d} off {4 * j:5d} corr {cc:+.3f} idle {idle} full {full}")
    # level fields (instantaneous activity) that follow the duty
    lev = []
    for j in range(n32):
        x = A[:, j]
        if np.std(x) == 0:
            continue
        c = np.corrcoef(x, duty)[0, 1]
        if np.isfinite(c) and abs(c) > 0.6:
            lev.append((abs(c), j, c, x[duty == 0].mean() if np.any(duty == 0) else None,
                        x[duty >= .99].mean() if np.any(duty >= .99) else None))
    lev.sort(reverse=True)
    print("u32 level words following the duty (corr, word, offset, idle mean, full mean):")
    for c, j, cc, idle, full in lev[:20]:
        print(f"  word {j:4d} off {4 * j:5d} corr {cc:+.3f} idle {idle} full {full}")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/busy_probe.json")
    ap.add_argument("--analyze", default="")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())

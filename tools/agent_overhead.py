"""Agent CPU and memory overhead measured on the shipped agent process.

Starts `agent --engine gpu --source replay` as its own process; the replay producer the agent
forks plays the kernel's role, writing RATE events/s through the probe model into the BPF
ring plus the user-space and span rings. After a warm-up this samples the AGENT process only
(the producer's CPU is the probes' in-kernel cost, reported separately): its CPU share of one
core over the measured interval, its own REF-formula gauge from /metrics
(llm_slo_agent_cpu_overhead_pct, REF pkg/safety/overhead_guard.go:77-107), RSS / USS / PSS,
windows and attributions done. Then SIGTERM, and a clean exit is required.

    python tools/agent_overhead.py --rate 1e6 --seconds 20 --out gpurun_out/agent_overhead.json
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scrape(port: int) -> dict:
    try:
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2).read().decode()
    except OSError:
        return {}
    out = {}
    for ln in body.splitlines():
        if ln and not ln.startswith("#"):
            k, _, v = ln.rpartition(" ")
            try:
                out[k] = float(v)
            except ValueError:
                pass
    return out


def _ready(port: int) -> bool:
    try:
        return urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=1).status == 200
    except OSError:
        return False


def _smaps_top(pid: int, top: int = 14) -> list:
    """[(mapping, rss MB, private MB)] largest first, from /proc/<pid>/smaps."""
    agg = {}
    name = "?"
    try:
        with open(f"/proc/{pid}/smaps") as f:
            for ln in f:
                parts = ln.split()
                if not parts:
                    continue
                if not parts[0].endswith(":") or "-" in parts[0]:
                    name = parts[5] if len(parts) > 5 else "[anon]"
                    if name.startswith("/dev/shm/") or name.startswith("/memfd:"):
                        name = name.replace("(anonymous namespace)::", "").split("(")[0]
                    continue
                if parts[0] in ("Rss:", "Private_Clean:", "Private_Dirty:"):
                    r = agg.setdefault(name, [0, 0])
                    kb = int(parts[1])
                    if parts[0] == "Rss:":
                        r[0] += kb
                    else:
                        r[1] += kb
    except OSError:
        return []
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]
    return [(k, round(v[0] / 1024, 1), round(v[1] / 1024, 1)) for k, v in rows]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=1e6, help="events/s the producer writes")
    ap.add_argument("--window-ms", type=int, default=1000)
    ap.add_argument("--seconds", type=float, default=20.0, help="measured interval")
    ap.add_argument("--warmup", type=float, default=5.0)
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--spans", type=int, default=16384)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import psutil

    port = _free_port()
    n_win = int(a.rate * a.window_ms / 1000)
    out_path = os.path.join("/tmp", f"agent_overhead_{os.getpid()}.jsonl")
    cmd = [sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--engine", "gpu", "--source", "replay",
           "--window-ms", str(a.window_ms), "--window-events", str(n_win), "--window-spans", str(a.spans),
           "--window-groups", str(a.groups), "--scenario", "full", "--output", "jsonl", "--output-path", out_path,
           "--metrics-bind", f"127.0.0.1:{port}"]
    t_start = time.time()
    # the agent as the DaemonSet starts it: the pod env has no GPU_MAX_HW_QUEUES, so the agent's own
    # cap (--gpu-hw-queues, default 1) applies; a box-wide value (4 on the GPU pool) would win over it
    # and map three more 173 MB queue save areas into the agent
    env = dict(os.environ)
    box_queues = env.pop("GPU_MAX_HW_QUEUES", None)
    agent = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    proc = psutil.Process(agent.pid)
    try:
        deadline = time.time() + 300
        while not _ready(port):
            if agent.poll() is not None or time.time() > deadline:
                raise RuntimeError(f"agent did not become ready (rc={agent.poll()}): {agent.stdout.read()[-2000:]}")
            time.sleep(0.5)
        t_ready = time.time()
        print(f"[agent_overhead] ready after {t_ready - t_start:.1f}s; warming {a.warmup}s", flush=True)
        time.sleep(a.warmup)
        kids = proc.children()
        c0, w0 = proc.cpu_times(), time.perf_counter()
        k0 = [k.cpu_times() for k in kids]
        m0 = _scrape(port)
        samples = []
        t_end = time.perf_counter() + a.seconds
        while time.perf_counter() < t_end:
            time.sleep(1.0)
            mi = proc.memory_info()
            samples.append(mi.rss)
            print(f"[agent_overhead] rss {mi.rss / 2**20:.1f} MB", flush=True)
        c1, w1 = proc.cpu_times(), time.perf_counter()
        k1 = [k.cpu_times() for k in kids]
        m1 = _scrape(port)
        full = proc.memory_full_info()
        smaps = _smaps_top(agent.pid)
        wall = w1 - w0
        agent_cpu = (c1.user + c1.system - c0.user - c0.system) / wall * 100.0
        prod_cpu = sum(b.user + b.system - x.user - x.system for x, b in zip(k0, k1)) / wall * 100.0
        win = m1.get("llm_slo_agent_gpu_windows_total", 0.0) - m0.get("llm_slo_agent_gpu_windows_total", 0.0)
        res = {
            "rate_events_per_s": a.rate,
            "window_ms": a.window_ms,
            "measured_s": round(wall, 2),
            "agent_cpu_pct_of_one_core": round(agent_cpu, 3),
            "box_gpu_max_hw_queues_removed_from_agent_env": box_queues,
            "agent_cpu_pct_gauge_ref_formula": m1.get("llm_slo_agent_cpu_overhead_pct"),
            "producer_cpu_pct_of_one_core": round(prod_cpu, 3),
            "agent_rss_mb": round(full.rss / 2**20, 1),
            "agent_rss_mb_max": round(max(samples) / 2**20, 1) if samples else None,
            "agent_uss_mb": round(full.uss / 2**20, 1),
            "agent_pss_mb": round(getattr(full, "pss", 0) / 2**20, 1),
            "windows_in_interval": win,
            "rss_by_mapping_mb": smaps,
            "metrics": {k: v for k, v in m1.items() if k.startswith("llm_slo_agent_")},
        }
    finally:
        if agent.poll() is None:
            agent.send_signal(signal.SIGTERM)
        try:
            rc = agent.wait(timeout=30)
        except subprocess.TimeoutExpired:
            agent.send_signal(signal.SIGUSR1)
            time.sleep(1)
            agent.kill()
            rc = agent.wait()
        log = agent.stdout.read()
    res["exit_code"] = rc
    res["attributions"] = sum(1 for _ in open(out_path)) if os.path.exists(out_path) else 0
    res["agent_log_tail"] = log[-1500:]
    if os.path.exists(out_path):
        os.remove(out_path)
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    return 0 if rc == 0 else 1


if __name__ == "__main__":
    sys.exit(main())

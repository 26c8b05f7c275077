"""Agent CPU and memory overhead measured on the shipped agent process.

Starts `agent --engine gpu --source replay` as its own process; the replay producer the agent
forks plays the kernel's role, writing RATE events/s through the probe model into the BPF
ring plus the user-space and span rings. After a warm-up this samples the AGENT process only
(the producer's CPU is the probes' in-kernel cost, reported separately): its CPU share of one
core over the measured interval, its own REF-formula gauge from /metrics
(llm_slo_agent_cpu_overhead_pct, REF pkg/safety/overhead_guard.go:77-107), RSS / USS / PSS,
windows and attributions done. Then SIGTERM, and a clean exit is required.

    python tools/agent_overhead.py --rate 1e6 --seconds 20 --out gpurun_out/agent_overhead.json

Shipped configuration (the default; ``--bare`` measures the agent with its built-in defaults): the
ConfigMap's toolkit.yaml (deploy/k8s/configmap.yaml: its 14-signal set, sampling limits, gpu block),
the shipped learned model, the ConfigMap's min confidence, the native schedstat sampler over a set of
watched workload processes and the KFD sampler (when /sys/class/kfd exists), and the OTLP span
receiver fed by a sender posting ``--span-rate`` spans/s. RSS is split into the HIP runtime's queue
save areas (the large equal-size anonymous mappings ROCr allocates per hardware queue for context
save/restore) and the rest. ``--csv`` appends the release gate's collector_overhead.csv row (REF
pkg/releasegate/gate.go:303-376 reads timestamp,node,collector_cpu_pct,collector_memory_mb,
events_per_second,dropped_events) from this measurement of the window agent.
"""

from __future__ import annotations

import argparse
import http.client
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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


def rss_split(pid: int, min_queue_area_mb: float = 64.0) -> dict:
    """RSS of the HIP runtime's per-queue context save areas vs everything else, from smaps: ROCr
    maps one anonymous area per hardware queue, all of one size (~173 MB on MI355X); they are
    the unnamed (anonymous) mappings of at least ``min_queue_area_mb`` (the agent's own large host
    buffers are pinned /dev/zero mappings or smaller)."""
    maps = []  # (name, size kB, rss kB)
    cur = None
    try:
        with open(f"/proc/{pid}/smaps") as f:
            for ln in f:
                parts = ln.split()
                if not parts:
                    continue
                if not parts[0].endswith(":") or "-" in parts[0]:
                    cur = [parts[5] if len(parts) > 5 else "", 0, 0]
                    maps.append(cur)
                elif parts[0] == "Size:" and cur is not None:
                    cur[1] = int(parts[1])
                elif parts[0] == "Rss:" and cur is not None:
                    cur[2] = int(parts[1])
    except OSError:
        return {}
    qa = [m for m in maps if not m[0] and m[1] >= min_queue_area_mb * 1024 and m[2] > 0]
    zero = sorted((m for m in maps if m[0] == "/dev/zero" and m[2] >= 1024), key=lambda m: -m[2])
    q_rss = sum(m[2] for m in qa)
    total = sum(m[2] for m in maps)
    shm = sum(m[2] for m in maps if m[0].startswith("/dev/shm/"))
    return {"total_mb": round(total / 1024, 1), "queue_save_areas_mb": round(q_rss / 1024, 1),
            "queue_save_areas": len(qa), "queue_save_area_size_mb": sorted({round(m[1] / 1024, 1) for m in qa}),
            "shared_rings_mb": round(shm / 1024, 1),
            # MAP_SHARED|MAP_ANONYMOUS mappings (ROCr's host allocations: pinned buffers, pools), >= 1 MB
            "dev_zero_maps_mb": [[round(m[1] / 1024, 1), round(m[2] / 1024, 1)] for m in zero],
            "rest_mb": round((total - q_rss - shm) / 1024, 1)}


def configmap_toolkit(path: str, out: str) -> dict:
    """The ConfigMap's toolkit.yaml written to ``out``; returns the ConfigMap's data block."""
    import yaml

    with open(path) as f:
        cm = yaml.safe_load(f)
    data = cm["data"]
    with open(out, "w") as f:
        f.write(data["toolkit.yaml"])
    return data


class SpanSender:
    """Posts OTLP/HTTP JSON request spans to the agent's receiver at a fixed rate (batches every
    100 ms), as the node's instrumented services would."""

    def __init__(self, port: int, rate: float, pids):
        import threading

        self.port, self.rate, self.pids = port, rate, list(pids)
        self.stop = threading.Event()
        self.sent = self.failed = 0
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        import random

        rng = random.Random(7)
        per = max(1, int(round(self.rate / 10)))
        conn = None
        i = 0
        while not self.stop.wait(0.1):
            now = time.time_ns()
            spans = []
            for _ in range(per):
                i += 1
                t0 = now - rng.randrange(50_000_000, 400_000_000)
                spans.append({"traceId": f"{i:032x}", "spanId": f"{i:016x}", "name": "chat.request", "kind": 2,
                              "startTimeUnixNano": str(t0), "endTimeUnixNano": str(now),
                              "attributes": [{"key": "llm.slo.ttft_ms",
                                              "value": {"doubleValue": rng.uniform(40, 900)}}]})
            pid = self.pids[i % len(self.pids)] if self.pids else 0
            body = {"resourceSpans": [{"resource": {"attributes": [
                {"key": "service.name", "value": {"stringValue": f"svc-{i % 8}"}},
                {"key": "process.pid", "value": {"intValue": str(pid)}}]},
                "scopeSpans": [{"scope": {"name": "overhead"}, "spans": spans}]}]}
            try:  # one keep-alive connection, as an OTLP/HTTP exporter holds
                if conn is None:
                    conn = http.client.HTTPConnection("127.0.0.1", self.port, timeout=2)
                conn.request("POST", "/v1/traces", body=json.dumps(body).encode(),
                             headers={"Content-Type": "application/json"})
                conn.getresponse().read()
                self.sent += len(spans)
            except (OSError, http.client.HTTPException):
                self.failed += 1
                if conn is not None:
                    conn.close()
                conn = None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=1e6, help="events/s the producer writes")
    ap.add_argument("--window-ms", type=int, default=1000)
    ap.add_argument("--seconds", type=float, default=20.0, help="measured interval")
    ap.add_argument("--warmup", type=float, default=5.0)
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--spans", type=int, default=16384)
    ap.add_argument("--out", default="")
    ap.add_argument("--engine", default="gpu", choices=("gpu", "cpu"))
    ap.add_argument("--bare", action="store_true", help="the agent's built-in defaults instead of the shipped config")
    ap.add_argument("--configmap", default=os.path.join(ROOT, "deploy", "k8s", "configmap.yaml"))
    ap.add_argument("--model-path", default=os.path.join(ROOT, "config", "models", "mislo-learned.safetensors"))
    ap.add_argument("--watched", type=int, default=8, help="workload processes the schedstat / KFD samplers watch")
    ap.add_argument("--span-rate", type=float, default=200.0, help="OTLP spans/s posted to the receiver")
    ap.add_argument("--csv", default="", help="append the release gate's collector_overhead.csv row here")
    ap.add_argument("--node", default=os.environ.get("NODE_NAME", "node-a"))
    ap.add_argument("--no-samplers", action="store_true", help="shipped config without the schedstat / KFD samplers")
    ap.add_argument("--no-otlp", action="store_true", help="shipped config without the OTLP receiver and its spans")
    ap.add_argument("--env-hw-queues", type=int, default=0, help="diagnostic: GPU_MAX_HW_QUEUES in the agent's env")
    a = ap.parse_args()
    import psutil

    port = _free_port()
    n_win = int(a.rate * a.window_ms / 1000)
    out_path = os.path.join("/tmp", f"agent_overhead_{os.getpid()}.jsonl")
    cmd = [sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--engine", a.engine, "--source", "replay",
           "--window-ms", str(a.window_ms), "--window-events", str(n_win), "--window-spans", str(a.spans),
           "--window-groups", str(a.groups), "--scenario", "full", "--output", "jsonl", "--output-path", out_path,
           "--metrics-bind", f"127.0.0.1:{port}"]
    shipped, watched, sender, rx = {}, [], None, 0
    if not a.bare:
        cfg_path = os.path.join("/tmp", f"agent_overhead_toolkit_{os.getpid()}.yaml")
        data = configmap_toolkit(a.configmap, cfg_path)
        rx = 0 if a.no_otlp else _free_port()
        # workload stand-ins the samplers watch (idle processes: the samplers' cost is per watched
        # process and interval, not per unit of the workload's activity)
        watched = [subprocess.Popen([sys.executable, "-c", "import time\nwhile True: time.sleep(1)"])
                   for _ in range(0 if a.no_samplers else max(0, a.watched))]
        pods = ",".join(f"{p.pid}:c0f14000-0000-4000-8000-{i:012d}" for i, p in enumerate(watched))
        kfd = "on" if os.path.isdir("/sys/class/kfd") and not a.no_samplers else "off"
        cmd += ["--config", cfg_path, "--model-path", a.model_path, "--min-confidence", data.get("MIN_CONFIDENCE", "0.6"),
                "--gpus", data.get("GPUS", "1"), "--kfd-sampler", kfd]
        if rx:
            cmd += ["--otlp-receiver-bind", f"127.0.0.1:{rx}", "--otlp-receiver-allow", "127.0.0.0/8"]
        if watched:
            cmd += ["--procfs-sampler", "--procfs-pods", pods, "--procfs-interval-ms", "100"]
        shipped = {"config": os.path.relpath(a.configmap, ROOT) + ":toolkit.yaml", "model": os.path.relpath(a.model_path, ROOT),
                   "min_confidence": data.get("MIN_CONFIDENCE"), "gpus": data.get("GPUS"), "kfd_sampler": kfd,
                   "schedstat_sampler_pids": len(watched), "otlp_span_rate": a.span_rate if rx else 0}
    t_start = time.time()
    # the agent as the DaemonSet starts it: the pod env has no GPU_MAX_HW_QUEUES, so the agent's own
    # cap (--gpu-hw-queues, default 1) applies; a box-wide value (4 on the GPU pool) would win over it
    # and map three more 173 MB queue save areas into the agent
    env = dict(os.environ)
    box_queues = env.pop("GPU_MAX_HW_QUEUES", None)
    if a.env_hw_queues:  # diagnostic: the cap in the agent's environment from the start
        env["GPU_MAX_HW_QUEUES"] = str(a.env_hw_queues)
    from llm_slo_ebpf_toolkit_amd.utils import cgroupmem

    cg0 = cgroupmem.reading()  # the cgroup's charge before the agent (and its producer) start
    agent = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    proc = psutil.Process(agent.pid)
    try:
        deadline = time.time() + 300
        while not _ready(port):
            if agent.poll() is not None or time.time() > deadline:
                raise RuntimeError(f"agent did not become ready (rc={agent.poll()}): {agent.stdout.read()[-2000:]}")
            time.sleep(0.5)
        t_ready = time.time()
        if rx and a.span_rate > 0:
            sender = SpanSender(rx, a.span_rate, [p.pid for p in watched])
            sender.t.start()
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
        cg1 = cgroupmem.reading()
        smaps = _smaps_top(agent.pid)
        split = rss_split(agent.pid)
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
            "rss_split_mb": split,
            # what the agent's start added to the cgroup's charge (agent + its replay producer + the
            # watched stand-ins; nothing else in the cgroup runs meanwhile): the number a pod memory
            # limit is enforced on, next to RSS
            "cgroup": {"version": cg1["version"], "dir": cg1["dir"]} if cg1 else None,
            "cgroup_charge_delta_mb": cgroupmem.delta(cg0, cg1),
            "shipped_config": shipped or None,
            "spans_posted": sender.sent if sender else 0,
            "dropped_events": sum(v for k, v in m1.items() if k.startswith("llm_slo_agent_dropped_events_total"))
                              - sum(v for k, v in m0.items() if k.startswith("llm_slo_agent_dropped_events_total")),
            "metrics": {k: v for k, v in m1.items() if k.startswith("llm_slo_agent_")},
        }
    finally:
        if sender is not None:
            sender.stop.set()
        for p in watched:
            p.kill()
            p.wait(5)
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
    if a.csv:
        import csv

        new = not os.path.exists(a.csv)
        with open(a.csv, "a", newline="") as fh:
            w = csv.writer(fh)
            if new:
                w.writerow(["timestamp", "node", "collector_cpu_pct", "collector_memory_mb", "events_per_second",
                            "dropped_events"])
            w.writerow([time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), a.node,
                        f"{res['agent_cpu_pct_of_one_core']:.4f}", f"{res['agent_rss_mb']:.1f}",
                        f"{res['windows_in_interval'] * n_win / max(res['measured_s'], 1e-9):.1f}",
                        int(res.get("dropped_events") or 0)])
    return 0 if rc == 0 else 1


if __name__ == "__main__":
    sys.exit(main())

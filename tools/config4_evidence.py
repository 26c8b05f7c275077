"""Config-4 evidence harness (BASELINE.json config 4: "8xMI355X TP inference under RCCL-latency +
CPU-steal injection; node-wide histograms via RCCL all-reduce over xGMI").

One node, N GPUs (default: every GPU the amdgpu driver exposes):

* workload: the tensor-parallel Llama server (demo/tp_server.py), one rank per GPU over RCCL, each
  rank pinned to its own two CPUs and loading the rocprofiler tool (GPU queue delay, HBM, RCCL
  collective time into the agent's user ring); rank 0 serves /chat and exports the spans;
* agent: ``--engine gpu --gpus N`` -- one window worker per GPU, group sharding, the packet
  all-reduce and incident all-gather over RCCL -- with the shipped learned 2-fault model and the
  unprivileged sampler on every rank's process;
* faults:
  - ``gpu_interconnect``: an xGMI hog (tools/xgmi_hog.py) streams large peer-to-peer copies over
    every GPU pair, so the TP all-reduces queue behind it on the links -- a real fault;
  - ``cpu_throttle``: CPU burners pinned to the ranks' CPUs (real run-queue delay) plus the
    ``cpu_steal_pct`` records a hypervisor's steal would produce, injected with
    ``faultinject --emit-ring`` (bare metal has no steal to measure);
  - ``compound``: both (the 2-fault case);
* out: per phase top-1 of the server's incident group, accuracy, compound partial / coverage,
  detection delay, TTFT, and the agent's node-wide window counters (all-reduced over RCCL).

    python tools/config4_evidence.py --out gpurun_out/config4 [--gpus 8] [--preset 7b]

With one GPU the harness still runs (TP 1, no collectives): the interconnect phase then has no
fault to inject and is skipped.
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from config2_evidence import Tailer, free_port, pct, wait_http  # noqa: E402
from config3_evidence import (GPU_SIGNALS, MODEL, TOOL, Client, load_cuts, scrape_counters, scrape_overhead, score,  # noqa: E402
                              slo_from_warmup)

POD_UID = "c0f14000-0000-4000-8000-000000000004"
BURN = "import os, sys\nos.sched_setaffinity(0, {int(sys.argv[1])})\nwhile True:\n    pass\n"
EXPECT = {"baseline": set(), "fault_interconnect": {"gpu_interconnect"}, "recovery_1": set(),
          "fault_cpu": {"cpu_throttle"}, "recovery_2": set(),
          "fault_compound": {"gpu_interconnect", "cpu_throttle"}, "recovery_3": set()}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/config4")
    ap.add_argument("--gpus", type=int, default=0, help="TP ranks = agent workers (0 = every visible GPU)")
    ap.add_argument("--preset", default="7b")
    ap.add_argument("--phase-s", type=float, default=15.0)
    ap.add_argument("--window-ms", type=int, default=1000)
    ap.add_argument("--recover-s", type=float, default=8.0)
    ap.add_argument("--burners-per-cpu", type=int, default=2,
                    help="busy loops per rank CPU: 2 slows the server ~3x; 4 starves it to a request every few s")
    ap.add_argument("--steal-pct", type=float, default=9.0, help="injected cpu_steal_pct (REF's cpu_throttle level)")
    ap.add_argument("--ttft-slo-ms", type=float, default=0.0,
                    help="the agent's TTFT SLO; 0 = calibrated from the healthy warmup (slo_from_warmup)")
    ap.add_argument("--clients", type=int, default=3,
                    help="closed-loop clients: a server slowed by a fault keeps completing requests in every "
                         "1 s window (one client left windows without a request, so without an incident)")
    ap.add_argument("--max-tokens", type=int, default=8,
                    help="tokens per completion: short chat turns, so a CPU-starved 7B server still completes "
                         "a request in most 1 s windows (16 tokens took > 1 s per request under the fault)")
    ap.add_argument("--model-path", default=MODEL)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from llm_slo_ebpf_toolkit_amd.collector import bpf, procfs
    from llm_slo_ebpf_toolkit_amd.parallel.numa import visible_gpu_count

    n = a.gpus or max(1, visible_gpu_count())
    cpus = sorted(os.sched_getaffinity(0))
    rank_cpus = [cpus[(2 * r) % len(cpus):(2 * r) % len(cpus) + 2] for r in range(n)]
    rest = cpus[2 * n:] or cpus
    prefix = f"/mislo-cfg4-{os.getpid()}"
    names = bpf.RingNames.of(prefix)
    rings = bpf.create_rings(names, 1 << 26, 1 << 20, 1 << 14)  # noqa: F841 - kept alive for the children
    rx, mport, hport, master = free_port(), free_port(), free_port(), free_port()
    attr_path = os.path.join(a.out, "attributions.jsonl")
    if os.path.exists(attr_path):
        os.remove(attr_path)
    log = open(os.path.join(a.out, "run.log"), "w")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)

    def pinned(cset):
        return lambda: os.sched_setaffinity(0, set(cset))

    ranks = []
    for r in range(n):
        renv = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(master), OMP_NUM_THREADS="2", POD_UID=POD_UID, POD_NAME="llm-tp-config4",
                    OTEL_EXPORTER_OTLP_TRACES_ENDPOINT=f"http://127.0.0.1:{rx}/v1/traces")
        if os.path.exists(TOOL):
            renv.update(ROCP_TOOL_LIBRARIES=TOOL, MISLO_RING=names.user, MISLO_POD_ID="1", MISLO_QUEUE_FLOOR_NS="200000")
        ranks.append(subprocess.Popen([sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.demo.tp_server", "--preset",
                                       a.preset, "--bind", f"127.0.0.1:{hport}"], cwd=ROOT, env=renv, stdout=log,
                                      stderr=subprocess.STDOUT, preexec_fn=pinned(rank_cpus[r])))
    observable = ["runqueue_delay_ms", "cpu_steal_pct"] + (["mem_reclaim_latency_ms"] if procfs.psi_available() else [])
    observable += [s for s in GPU_SIGNALS if s != "xgmi_link_latency_us"] if os.path.exists(TOOL) else []

    def start_agent(slo_ms):
        return subprocess.Popen(
            [sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--engine", "gpu", "--gpus", str(n),
             "--source", "shm", "--ring-name", prefix, "--otlp-receiver-bind", f"127.0.0.1:{rx}",
             "--metrics-bind", f"127.0.0.1:{mport}", "--window-ms", str(a.window_ms), "--window-events", "262144",
             "--window-spans", "4096", "--window-groups", "8", "--model-path", a.model_path, "--min-confidence", "0.3",
             "--halo-ms", "1500", "--ttft-slo-ms", str(slo_ms), "--procfs-sampler",
             "--procfs-pods", ",".join(f"{p.pid}:{POD_UID}" for p in ranks), "--procfs-interval-ms", "100",
             "--model-signals", ",".join(observable), "--output", "jsonl", "--output-path", attr_path,
             "--decision-log", os.path.join(a.out, "decisions.jsonl")],
            cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT, preexec_fn=pinned(rest))

    agent = None
    slo = a.ttft_slo_ms
    stop, tstop = threading.Event(), threading.Event()
    rows: list = []
    cur = {"phase": "warmup"}
    clients, burners, hogs, injectors = [], [], [], []
    tailer = Tailer(attr_path, tstop)
    phases, counters, overhead = [], {}, {}
    try:
        wait_http(f"http://127.0.0.1:{hport}/healthz", ranks[0], 600)
        clients = [Client(hport, i, lambda: cur["phase"], stop, rows, 0.05, max_tokens=a.max_tokens) for i in range(a.clients)]
        for c in clients:
            c.start()
        t_w = time.time()
        while time.time() - t_w < 180 and sum(r["phase"] == "warmup" for r in rows) < 24:
            time.sleep(0.2)
        if slo <= 0:  # the service's SLO from its own healthy latency, before the agent watches it
            slo = slo_from_warmup([r["ttft_ms"] for r in rows if r["phase"] == "warmup" and r["ttft_ms"] is not None])
        print(f"[config4] TTFT SLO {slo:.1f} ms", flush=True)
        agent = start_agent(slo)
        wait_http(f"http://127.0.0.1:{mport}/readyz", agent, 300)
        tailer.start()
        time.sleep(3.0)  # a few windows of the agent on the healthy server
        print(f"[config4] ready: TP {n}, rank pids {[p.pid for p in ranks]}", flush=True)
        plan = [("baseline", a.phase_s), ("fault_interconnect", a.phase_s), ("recovery_1", a.recover_s),
                ("fault_cpu", a.phase_s), ("recovery_2", a.recover_s), ("fault_compound", a.phase_s),
                ("recovery_3", a.recover_s)]
        for name, dur in plan:
            exp = EXPECT[name]
            if "gpu_interconnect" in exp and n < 2:
                print(f"[config4] {name}: skipped (one GPU: no links to load)", flush=True)
                continue
            t0 = time.time_ns()
            cur["phase"] = name
            m0 = scrape_counters(mport)
            if "gpu_interconnect" in exp:
                hogs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "xgmi_hog.py"), "--gpus", str(n),
                                          "--seconds", str(dur)], cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT,
                                         preexec_fn=pinned(rest))]
            if "cpu_throttle" in exp:
                burners = [subprocess.Popen([sys.executable, "-c", BURN, str(c)], cwd=ROOT, env=env,
                                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                           for cs in rank_cpus for c in cs for _ in range(a.burners_per_cpu)]
                injectors = [subprocess.Popen(
                    [sys.executable, "-m", "llm_slo_ebpf_toolkit_amd.cli.faultinject", "--emit-ring", prefix, "--signal",
                     "cpu_steal_pct", "--value", str(a.steal_pct), "--pid", str(p.pid), "--pod-uid", POD_UID,
                     "--agent", f"http://127.0.0.1:{mport}", "--rate", "10", "--duration", str(dur)],
                    cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT, preexec_fn=pinned(rest)) for p in ranks]
            time.sleep(dur)
            for p in injectors + hogs:
                try:
                    p.wait(60)
                except subprocess.TimeoutExpired:
                    p.kill()
            for b in burners:
                b.kill()
                b.wait(10)
            burners, hogs, injectors = [], [], []
            t1 = time.time_ns()
            phases.append((name, t0, t1))
            m1 = scrape_counters(mport)
            counters[name] = {k: v - m0.get(k, 0.0) for k, v in m1.items() if v - m0.get(k, 0.0)}
            ph = [r["ttft_ms"] for r in rows if r["phase"] == name and r["ttft_ms"] is not None]
            print(f"[config4] {name}: {len(ph)} requests, TTFT p50 {pct(ph, .5)} ms p95 {pct(ph, .95)} ms", flush=True)
        time.sleep(3.0)
        overhead = scrape_overhead(mport)
    finally:
        stop.set()
        for p in burners + hogs + injectors:
            if p.poll() is None:
                p.kill()
        for c in clients:
            c.join(60)
        for p in [ranks[0]] + ([agent] if agent is not None else []):
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
                try:
                    p.wait(120)
                except subprocess.TimeoutExpired:
                    p.kill()
        for p in ranks[1:]:
            try:
                p.wait(60)
            except subprocess.TimeoutExpired:
                p.kill()
        tstop.set()
        if tailer.is_alive():
            tailer.join(10)
        log.close()
    res = score(phases, tailer.rows, float(a.window_ms), service="llm-tp", expect=EXPECT,
                cuts=load_cuts(os.path.join(a.out, "decisions.jsonl")))
    res["ttft_ms"] = {nm: {"n": len(v), "p50": pct(v, .5), "p95": pct(v, .95)}
                      for nm, _t0, _t1 in phases for v in [[r["ttft_ms"] for r in rows if r["phase"] == nm]]}
    res["agent_overhead_metrics"] = overhead
    res["agent_counters_by_phase"] = counters
    res["setup"] = {"tp_ranks": n, "preset": a.preset, "model": os.path.relpath(a.model_path, ROOT),
                    "ttft_slo_ms": slo, "clients": a.clients, "max_tokens": a.max_tokens, "window_ms": a.window_ms,
                    "slo_source": "given" if a.ttft_slo_ms > 0 else "1.5 x healthy warmup TTFT p95",
                    "observable_signals": observable, "rank_cpus": rank_cpus, "burners_per_cpu": a.burners_per_cpu,
                    "interconnect_fault": "tools/xgmi_hog.py peer copies over every GPU pair",
                    "cpu_fault": "pinned burners (measured run-queue delay) + injected cpu_steal_pct records"}
    res["exit"] = {"agent": agent.returncode if agent is not None else None, "ranks": [p.returncode for p in ranks]}
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

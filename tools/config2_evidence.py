"""Config-2 evidence on one MI355X (REF demo/llama-cpp/k8s/deployment.yaml:29-63 +
scripts/chaos/run_fault_matrix.sh:46-94; VERDICT r1 "do this" #7).

On one GPU, in one run:

* the LLM workload: the demo RAG service with the Llama backend (models/llama.py, bf16) and the
  rocprofiler-sdk tool (libmislo_rocprof.so) loaded into it. The tool's GPU signals go to the
  agent's user-space ring; the service's request spans go over OTLP/HTTP to the agent;
* the agent: ``--engine gpu`` on the same GPU, joining the tool's signals with the spans;
* a baseline phase, then a fault phase. In the fault phase a GPU burner process (back-to-back
  large GEMMs on the same GPU) contends with the LLM, then the fault is lifted;
* out: per-phase TTFT (p50 / p95, from the service's own responses) and the agent's
  IncidentAttributions for the service, with the fault phase's predicted domain and evidence,
  and the measured detection delay: the burner's first GEMM on the GPU (fault onset) -> the
  arrival of the first gpu_contention attribution of the service in the agent's output.

    python tools/config2_evidence.py --out gpurun_out/config2     # 7B preset, TTFT SLO 800 ms
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TOOL = os.path.join(ROOT, "llm_slo_ebpf_toolkit_amd", "probes", "rocprof", "libmislo_rocprof.so")
POD_UID = "c0nf1g2-0000-4000-8000-000000000001"

BURNER = r"""
import sys, time, torch
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
end = time.time() + float(sys.argv[1])
(a @ b).sum().item()  # first GEMM done: the contention starts now
print("burner on", time.time_ns(), flush=True)
while time.time() < end:
    for _ in range(8):
        a = (a @ b).clamp_(-1, 1)
    torch.cuda.synchronize()
print("burner off", flush=True)
"""


class Tailer(threading.Thread):
    """Reads the agent's attribution JSONL as it grows: (arrival wall-clock ns, row)."""

    def __init__(self, path: str, stop: threading.Event):
        super().__init__(daemon=True)
        self.path, self.stop, self.rows = path, stop, []

    def run(self):
        buf, pos = "", 0
        while True:
            try:
                with open(self.path) as fh:
                    fh.seek(pos)
                    data = fh.read()
                    pos = fh.tell()
            except OSError:
                data = ""
            now = time.time_ns()
            buf += data
            *lines, buf = buf.split("\n")
            for ln in lines:
                if ln.strip():
                    try:
                        self.rows.append((now, json.loads(ln)))
                    except ValueError:
                        pass
            if self.stop.is_set() and not data:
                return
            time.sleep(0.1)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def wait_http(url: str, proc, timeout: float) -> None:
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"{url}: process exited with {proc.returncode}")
        try:
            if urllib.request.urlopen(url, timeout=1).status == 200:
                return
        except OSError:
            pass
        time.sleep(0.5)
    raise RuntimeError(f"{url} not ready after {timeout}s")


def chat(port: int, i: int, phase: str, prompt_words: int = 16, max_tokens: int = 16) -> dict:
    words = " ".join(f"token{(i * 7 + k) % 997}" for k in range(max(0, prompt_words - 8)))
    body = json.dumps({"prompt": f"why did the {phase} request {i} slow down on the gpu {words}".strip(),
                       "profile": "chat_short", "max_tokens": max_tokens, "request_id": f"{phase}-{i}"}).encode()
    req = urllib.request.Request(f"http://127.0.0.1:{port}/chat", data=body, method="POST",
                                 headers={"Content-Type": "application/json"})
    t = time.time_ns()
    out = json.loads(urllib.request.urlopen(req, timeout=120).read())
    return {"phase": phase, "t_ns": t, "ttft_ms": out["ttft_ms"], "trace_id": out["trace_id"]}


def scrape(port: int) -> dict:
    """The agent's /metrics counters this run reads: GPU-signal events by status, join outcomes."""
    out = {}
    try:
        text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    except OSError:
        return out
    for ln in text.splitlines():
        if ln.startswith(("llm_ebpf_probe_events_total{", "llm_slo_agent_correlation_pairs_total{",
                          "llm_ebpf_gpu_queue_delay_ms_")):
            key, val = ln.rsplit(" ", 1)
            if "llm_ebpf_probe_events_total" in key and not any(s in key for s in ("gpu_", "hbm_", "xgmi_", "rccl_")):
                continue
            out[key] = float(val)
    return out


def delta(a: dict, b: dict) -> dict:
    return {k: b[k] - a.get(k, 0.0) for k in b if b[k] - a.get(k, 0.0)}


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))] if xs else None


MODEL = os.path.join(ROOT, "config", "models", "mislo-learned.safetensors")
GPU_SIGNALS = ("gpu_queue_delay_ms", "hbm_pressure_pct", "xgmi_link_latency_us", "rccl_collective_ms")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/config2")
    ap.add_argument("--preset", default="7b", help="Llama preset of the workload (BASELINE config 2: 7B)")
    ap.add_argument("--ttft-slo-ms", type=float, default=800.0, help="the agent's TTFT SLO (BASELINE config 2: 800 ms)")
    ap.add_argument("--phase-s", type=float, default=48.0, help="seconds of the baseline and fault phases")
    ap.add_argument("--recover-s", type=float, default=16.0)
    ap.add_argument("--burners", type=int, default=3,
                    help="GEMM burner processes on the GPU in the fault phase (4 left 2 requests in 24 s, "
                         "profiles/r4_config2_first)")
    ap.add_argument("--prompt-words", type=int, default=256, help="prompt length (prefill tokens)")
    ap.add_argument("--max-tokens", type=int, default=1, help="tokens per request: TTFT is the SLO; under the "
                                                              "fault each decoded token costs ~1 s more, one token "
                                                              "keeps requests completing in every 1 s window")
    ap.add_argument("--clients", type=int, default=3, help="concurrent closed-loop clients")
    ap.add_argument("--gap-s", type=float, default=0.05, help="client think time between requests")
    ap.add_argument("--halo-ms", type=int, default=3000,
                    help="agent halo: a contended request's span arrives ~1-2 s after its start (its TTFT plus "
                         "the exporter's batch delay), and its records are joined around that start")
    ap.add_argument("--window-ms", type=int, default=1000,
                    help="agent window (1 s: with 1-token requests from 3 clients every window holds a completed "
                         "request under the fault; 2 s windows put the first attribution ~3.6 s after the onset)")
    ap.add_argument("--model-path", default=MODEL, help="the agent's model ('' = the bayes_gpu expert table)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from config3_evidence import load_cuts, score  # noqa: E402 - tools/ sibling (imports this module at load)
    from llm_slo_ebpf_toolkit_amd.collector import bpf

    prefix = f"/mislo-cfg2-{os.getpid()}"
    names = bpf.RingNames.of(prefix)
    rings = bpf.create_rings(names, 1 << 24, 1 << 18, 1 << 14)  # noqa: F841 - kept alive for the children
    rx, mport, hport = free_port(), free_port(), free_port()
    attr_path = os.path.join(a.out, "attributions.jsonl")
    if os.path.exists(attr_path):
        os.remove(attr_path)
    log = open(os.path.join(a.out, "run.log"), "w")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)
    model_args = ["--model-path", a.model_path, "--model-signals", ",".join(GPU_SIGNALS)] if a.model_path else \
        ["--model", "bayes_gpu"]
    agent = subprocess.Popen(
        [sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--engine", "gpu", "--source", "shm",
         "--ring-name", prefix, "--otlp-receiver-bind", f"127.0.0.1:{rx}", "--metrics-bind", f"127.0.0.1:{mport}",
         "--window-ms", str(a.window_ms), "--window-events", "262144", "--window-spans", "4096", "--window-groups", "8",
         *model_args, "--min-confidence", "0.3", "--halo-ms", str(a.halo_ms), "--ttft-slo-ms", str(a.ttft_slo_ms),
         "--output", "jsonl", "--output-path", attr_path,
         "--decision-log", os.path.join(a.out, "decisions.jsonl")], cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT)
    llm_env = dict(env, ROCP_TOOL_LIBRARIES=TOOL, MISLO_RING=names.user, MISLO_POD_ID="1", MISLO_ROCPROF_VERBOSE="1",
                   OTEL_EXPORTER_OTLP_TRACES_ENDPOINT=f"http://127.0.0.1:{rx}/v1/traces",
                   POD_UID=POD_UID, POD_NAME="llm-server-config2")
    llm = subprocess.Popen([sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.demo.rag_service", "--backend", "llama",
                            "--llama-preset", a.preset, "--bind", f"127.0.0.1:{hport}", "--metrics-bind", ""],
                           cwd=ROOT, env=llm_env, stdout=log, stderr=subprocess.STDOUT)
    burners = []
    rows = []
    counters = {}
    onset_ns = None
    phases = []
    tstop = threading.Event()
    tailer = Tailer(attr_path, tstop)
    try:
        wait_http(f"http://127.0.0.1:{mport}/readyz", agent, 180)
        wait_http(f"http://127.0.0.1:{hport}/healthz", llm, 300)
        print("[config2] agent and llm ready", flush=True)
        tailer.start()
        for i in range(4):  # warm the model (first-request compilation / allocation)
            chat(hport, i, "warmup", a.prompt_words, a.max_tokens)
        plan = [("baseline", a.phase_s, False), ("fault_gpu_contention", a.phase_s, True),
                ("recovery", a.recover_s, False)]
        for phase, dur, fault in plan:
            if fault:
                burners = [subprocess.Popen([sys.executable, "-c", BURNER, "600"], cwd=ROOT, env=env,
                                            stdout=subprocess.PIPE, stderr=log, text=True) for _ in range(a.burners)]
                ons = []
                for b in burners:
                    ln = b.stdout.readline()  # "burner on <ns>" once its first GEMM finished
                    ons.append(int(ln.split()[-1]) if ln.startswith("burner on") else time.time_ns())
                onset_ns = min(ons)
            t0 = time.time_ns()
            m0 = scrape(mport)

            def client(c, phase=phase, t0=t0, dur=dur):
                i = 0
                while time.time_ns() - t0 < dur * 1e9:
                    try:
                        rows.append(chat(hport, 1000 * c + i, phase, a.prompt_words, a.max_tokens))
                    except (OSError, ValueError, KeyError):
                        time.sleep(0.2)
                    i += 1
                    time.sleep(a.gap_s)

            cl = [threading.Thread(target=client, args=(c,), daemon=True) for c in range(a.clients)]
            for t in cl:
                t.start()
            for t in cl:
                t.join(dur + 120)
            for b in burners:
                b.send_signal(signal.SIGTERM)
                b.wait(30)
            burners = []
            t1 = time.time_ns()
            phases.append((phase, t0, t1))
            rs = [r["ttft_ms"] for r in rows if r["phase"] == phase]
            print(f"[config2] {phase}: {len(rs)} requests, TTFT p50 {pct(rs, .5):.1f} ms p95 {pct(rs, .95):.1f} ms",
                  flush=True)
            counters[phase] = delta(m0, scrape(mport))
        time.sleep(3 * a.window_ms / 1000.0)  # the last windows' attributions
    finally:
        for p in burners + [llm]:
            if p is not None and p.poll() is None:
                p.send_signal(signal.SIGTERM)
                try:
                    p.wait(30)
                except subprocess.TimeoutExpired:
                    p.kill()
        if agent.poll() is None:
            agent.send_signal(signal.SIGTERM)
            try:
                agent.wait(60)
            except subprocess.TimeoutExpired:
                agent.kill()
        tstop.set()
        if tailer.is_alive():
            tailer.join(10)
        log.close()
    with open(os.path.join(a.out, "ttft.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    expect = {"baseline": set(), "fault_gpu_contention": {"gpu_contention"}, "recovery": set()}
    res = score(phases, tailer.rows, a.window_ms, service="rag-service", expect=expect,
                cuts=load_cuts(os.path.join(a.out, "decisions.jsonl")))
    fault = res["phases"].get("fault_gpu_contention", {})
    # detection delay: the burners' first GEMM (fault onset) -> arrival of the service's first
    # gpu_contention attribution
    hits = [arr for arr, x in tailer.rows if x.get("service") == "rag-service"
            and x.get("predicted_fault_domain") == "gpu_contention" and onset_ns is not None
            and int(x["incident_id"].split("-")[1]) > onset_ns]
    res["detection"] = {"onset_ns": onset_ns, "first_attribution_arrival_ns": min(hits) if hits else None,
                        "detection_delay_s": round((min(hits) - onset_ns) / 1e9, 3) if hits else None}
    res["ttft_ms"] = {p: {"n": len(v), "p50": pct(v, .5), "p95": pct(v, .95),
                          "slo_breach_fraction": round(sum(x > a.ttft_slo_ms for x in v) / max(1, len(v)), 4)}
                      for p, _t0, _t1 in phases for v in [[r["ttft_ms"] for r in rows if r["phase"] == p]]}
    res["gpu_contention_windows"] = f"{fault.get('top1', {}).get('gpu_contention', 0)}/{fault.get('windows', 0)}"
    res["evidence_samples"] = [{"domain": x["predicted_fault_domain"], "confidence": round(x["confidence"], 3),
                                "evidence": x["evidence"]} for _arr, x in tailer.rows
                               if x.get("service") == "rag-service" and x.get("predicted_fault_domain") != "unknown"][:4]
    res["agent_counters_by_phase"] = counters
    res["setup"] = {"preset": a.preset, "ttft_slo_ms": a.ttft_slo_ms, "burners": a.burners,
                    "prompt_words": a.prompt_words, "max_tokens": a.max_tokens, "clients": a.clients,
                    "window_ms": a.window_ms, "halo_ms": a.halo_ms, "phase_s": a.phase_s, "recover_s": a.recover_s,
                    "model": os.path.relpath(a.model_path, ROOT) if a.model_path else "bayes_gpu",
                    "observable_signals": list(GPU_SIGNALS) if a.model_path else "all",
                    "fault": f"{a.burners} processes of back-to-back 8192^3 bf16 GEMMs on the service's GPU"}
    res["exit"] = {"agent": agent.returncode, "llm": llm.returncode}
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

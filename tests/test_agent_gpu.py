"""The agent daemon's GPU window loop end to end (REF cmd/agent/main.go:269-633 run loop):
a forked replay producer writes the BPF ring (probe model), the user-space GPU-signal ring and
the span ring; the agent cuts windows, the native engine attributes them, and the agent emits
one attribution per incident group per window, then exits cleanly (engine closed, producer
reaped) -- run as a child process, as an operator would start it."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_agent_replay_windows_and_clean_exit(tmp_path):
    out = tmp_path / "attr.jsonl"
    n_win, groups = 3, 32
    cmd = [sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--engine", "gpu", "--source", "replay",
           "--count", str(n_win), "--window-ms", "300", "--window-events", "65536", "--window-spans", "2048",
           "--window-groups", str(groups), "--output", "jsonl", "--output-path", str(out), "--metrics-bind", "",
           "--scenario", "full", "--emit-min-burn", "0"]  # every scored group (no SLO-impact gate)
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-2000:]
    rows = [json.loads(x) for x in out.read_text().splitlines() if x.strip()]
    # windows are cut on the agent's clock, not the producer's: a window that caught only the
    # producer's first slices may hold no request of some group (no incident to attribute)
    per_win = {}
    for r in rows:
        per_win.setdefault(r["incident_id"].rsplit("-", 1)[0], []).append(r["service"])
    assert len(per_win) == n_win and all(len(s) == len(set(s)) <= groups for s in per_win.values())
    assert sum(len(s) == groups for s in per_win.values()) >= n_win - 1, {k: len(v) for k, v in per_win.items()}
    doms = {r["predicted_fault_domain"] for r in rows}
    assert len(doms) >= 3  # the replay's full scenario spans several fault domains
    assert all(0.0 <= r["confidence"] <= 1.0 for r in rows)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rag_service_spans_through_agent_to_attribution(tmp_path):
    """REF's request path end to end on the GPU engine: the demo RAG service exports its spans
    over OTLP/HTTP to the agent's receiver (span ring); slow DNS lookups on the same requests
    reach the (emulated) BPF ring through the probes' record path (ProbeSim: definitions,
    trace ids, epochs published by the agent); the agent joins them on the device and emits an
    IncidentAttribution for the service naming network_dns, with the measured DNS latency as
    evidence and the TTFT burn rate from the service's own spans."""
    import time
    import urllib.request

    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector import bpf, otlp
    from llm_slo_ebpf_toolkit_amd.collector import records as R
    from llm_slo_ebpf_toolkit_amd.demo.rag_service import RagService, StubBackend
    from llm_slo_ebpf_toolkit_amd.runtime import load

    prefix = f"/mislo-e2e-{os.getpid()}"
    names = bpf.RingNames.of(prefix)
    ring, user, spans = bpf.create_rings(names, 1 << 22, 1 << 12, 1 << 12)
    rx_port, m_port = _free_port(), _free_port()
    out = tmp_path / "attr.jsonl"
    cmd = [sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--engine", "gpu", "--source", "shm",
           "--ring-name", prefix, "--otlp-receiver-bind", f"127.0.0.1:{rx_port}",
           "--metrics-bind", f"127.0.0.1:{m_port}", "--count", "12", "--window-ms", "400", "--window-events", "65536",
           "--window-spans", "1024", "--window-groups", "8", "--model", "bayes", "--output", "jsonl",
           "--output-path", str(out),
           # the stub's requests take tens of ms (the plan's DNS / network / vector-DB sleeps): an
           # SLO they breach, so the service burns its budget and the agent attributes the incident
           "--ttft-slo-ms", "5"]
    agent = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        deadline = time.time() + 90
        while True:
            try:
                if urllib.request.urlopen(f"http://127.0.0.1:{m_port}/readyz", timeout=1).status == 200:
                    break
            except OSError:
                pass
            assert agent.poll() is None and time.time() < deadline, agent.stdout.read()[-2000:]
            time.sleep(0.2)
        uid = "0f1e2d3c-4b5a-6978-8796-a5b4c3d2e1f0"  # the agent's first pod uid -> pod id 1
        svc = RagService(StubBackend(), otlp_endpoint=f"http://127.0.0.1:{rx_port}/v1/traces",
                         resource={"k8s.pod.uid": uid})
        sim = load().ProbeSim(ring, R.milli_shift_table(), 1 << 16)
        for i in range(8):
            o = svc.chat({"prompt": f"incident {i}", "profile": "chat_short", "max_tokens": 2})
            svc.spans.flush()
            ev = np.zeros(4, dtype=R.EVENT)
            ev["ts_ns"] = time.time_ns() - np.arange(4) * 1_000_000
            ev["signal_type"] = 1              # dns_latency (ns)
            ev["value"] = 180_000_000          # 180 ms lookups
            ev["pid"] = os.getpid()
            ev["pod_id"] = 1
            ev["trace_h"] = otlp.trace_hash(o["trace_id"])
            assert sim.submit(ev) == 4
            time.sleep(0.1)
        rc = agent.wait(timeout=60)
        log = agent.stdout.read()
    finally:
        if agent.poll() is None:
            agent.kill()
            agent.wait()
    assert rc == 0, log[-2000:]
    rows = [json.loads(x) for x in out.read_text().splitlines() if x.strip()]
    mine = [r for r in rows if r["service"] == "rag-service"]
    assert mine, rows[:3]
    dns = [r for r in mine if r["predicted_fault_domain"] == "network_dns"]
    assert dns, [(r["predicted_fault_domain"], r["confidence"]) for r in mine]
    ev = {e["signal"]: e["value"] for e in dns[0]["evidence"]}
    assert any(abs(float(v) - 180.0) < 1.0 for v in ev.values() if not isinstance(v, str)), ev

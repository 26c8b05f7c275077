"""Demo RAG service over real HTTP (stub backend): retrieval plan, DNS correlation,
streaming NDJSON, Prometheus metrics incl. the errors / burn-rate series cdgate queries."""

import json
import urllib.request

import pytest

from llm_slo_ebpf_toolkit_amd.demo import rag_service as rs
from llm_slo_ebpf_toolkit_amd.export.prometheus import parse_exposition


@pytest.fixture
def service(http_recorder):
    traces = http_recorder()
    svc = rs.RagService(rs.StubBackend(), otlp_endpoint=traces.url + "/v1/traces")
    svc.spans.max_batch = 3
    httpd, metrics = svc.serve("127.0.0.1:0", "127.0.0.1:0")
    yield svc, f"http://127.0.0.1:{httpd.server_address[1]}", f"http://127.0.0.1:{metrics.port}", traces
    httpd.shutdown()
    metrics.stop()


def post(url, body):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    return urllib.request.urlopen(req, timeout=30)


def test_plan_is_deterministic_and_profile_shaped():
    a, b = rs.plan_for("chat_short", "hi there", 42), rs.plan_for("chat_short", "hi there", 42)
    assert a == b and 2 <= a.dns_ms < 6 and 10 <= a.vectordb_ms < 30
    c = rs.plan_for("context_long", "hi there", 42)
    assert 70 <= c.vectordb_ms < 150


def test_chat_roundtrip_metrics_and_traces(service):
    svc, api, metrics, traces = service
    out = json.load(post(api + "/chat", {"prompt": "why is ttft high", "profile": "chat_short", "max_tokens": 5,
                                         "request_id": "r1"}))
    assert out["tokens"][:4] == ["why", "is", "ttft", "high"] and len(out["tokens"]) == 5
    assert out["correlation"]["tier"] == "trace_id_exact" and out["correlation"]["confidence"] == 1.0
    assert out["attributes"]["llm.ebpf.dns.latency_ms"] > 0
    m = parse_exposition(urllib.request.urlopen(metrics + "/metrics").read().decode())
    assert m['llm_slo_requests_total{status="ok",profile="chat_short"}'] == 1
    assert m['llm_slo_correlation_total{tier="trace_id_exact",enriched="true"}'] == 1
    assert m["llm_slo_ttft_ms_count"] == 1 and m["llm_slo_burn_rate"] == 0
    svc.spans.flush()
    spans = [s for r in traces.requests for s in json.loads(r["body"])["resourceSpans"][0]["scopeSpans"][0]["spans"]]
    # exported as an OTel SDK ends them: the retrieval, then the first-token record (the TTFT SLI
    # when the first token is out, llm.slo.ttft_early), then the generation and the request
    assert [s["name"] for s in spans] == ["chat.retrieval", "chat.first_token", "chat.generation", "chat.request"]
    assert len({s["traceId"] for s in spans}) == 1
    ft = {a["key"]: a["value"] for a in spans[1]["attributes"]}
    assert ft["llm.slo.ttft_early"] == {"boolValue": True} and ft["llm.slo.ttft_ms"]["doubleValue"] > 0


def test_streaming_and_errors(service):
    svc, api, metrics, _ = service
    lines = [json.loads(x) for x in post(api + "/chat", {"prompt": "stream me", "max_tokens": 3, "stream": True})
             .read().decode().splitlines() if x.strip()]
    assert [d.get("token") for d in lines[:3]] == ["stream", "me", lines[2]["token"]]
    assert lines[-1]["done"] is True
    with pytest.raises(urllib.error.HTTPError):
        post(api + "/chat", {"prompt": "  "})

    class Boom(rs.StubBackend):
        def generate(self, *a, **k):
            raise RuntimeError("backend down")

    svc.backend = Boom()
    with pytest.raises(urllib.error.HTTPError):
        post(api + "/chat", {"prompt": "x", "max_tokens": 1})
    m = parse_exposition(urllib.request.urlopen(metrics + "/metrics").read().decode())
    assert m['llm_slo_errors_total{profile="rag_medium"}'] == 1 and m["llm_slo_burn_rate"] > 0


def test_burn_rate_window():
    b = rs.BurnRate(0.99, window_s=10)
    for i in range(99):
        b.observe(True, now=i * 0.01)
    assert b.observe(False, now=1.0) == pytest.approx(1.0)
    assert b.observe(True, now=100.0) == 0.0  # old events aged out


def test_span_exporter_flushes_on_its_schedule():
    """A partial batch goes out after max_delay_s (spans must reach the agent's windows promptly)."""
    import http.server
    import threading
    import time

    got = []

    class H(http.server.BaseHTTPRequestHandler):
        def do_POST(self):  # noqa: N802
            got.append(json.loads(self.rfile.read(int(self.headers["Content-Length"]))))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = http.server.HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        ex = rs.SpanExporter(f"http://127.0.0.1:{srv.server_port}/v1/traces", max_batch=64, max_delay_s=0.05)
        ex.add([rs.SpanExporter.span("0af7651916cd43dd8448eb211c80319c", "b7ad6b7169203331", "", "chat.request",
                                     1, 2, {})])
        deadline = time.time() + 5
        while not got and time.time() < deadline:
            time.sleep(0.02)
        assert got and got[0]["resourceSpans"][0]["scopeSpans"][0]["spans"][0]["name"] == "chat.request"
    finally:
        srv.shutdown()


def test_gpu_trace_tag_is_a_noop_without_the_tool():
    tag = rs.GpuTraceTag()
    assert not tag.active
    tag.set("0af7651916cd43dd8448eb211c80319c")  # must not raise

"""Exporters against local HTTP servers (REF pkg/webhook, pkg/otel, pkg/cdgate tests) and
the Prometheus registry / metrics server."""

import json
import urllib.request

import pytest

from llm_slo_ebpf_toolkit_amd.contracts.types import Evidence, IncidentAttribution, ProbeEventV1, SLOEvent, SLOImpact
from llm_slo_ebpf_toolkit_amd.export import cdgate, otel, prometheus, webhook


def attribution(conf=0.9, burn=2.0):
    return IncidentAttribution(incident_id="inc-1", timestamp=1_700_000_000_123_000_000, cluster="prod",
                               namespace="default", service="chat", predicted_fault_domain="network_dns",
                               confidence=conf, evidence=[Evidence("llm.ebpf.dns.latency_ms", 220.0, "ebpf")],
                               slo_impact=SLOImpact("ttft_ms", burn, 5))


def test_webhook_generic_and_hmac(http_recorder):
    srv = http_recorder([(200, "ok")])
    webhook.WebhookExporter(srv.url, secret="s3cr3t").send(attribution())
    req = srv.requests[0]
    body = json.loads(req["body"])
    assert body["predicted_fault_domain"] == "network_dns"
    sig = req["headers"]["X-Webhook-Signature"]
    assert sig.startswith("sha256=") and webhook.verify_hmac(req["body"], "s3cr3t", sig)
    assert not webhook.verify_hmac(req["body"], "other", sig)


def test_webhook_retries_5xx_then_succeeds(http_recorder):
    srv = http_recorder([(500, "x"), (503, "x"), (200, "ok")])
    sleeps = []
    webhook.WebhookExporter(srv.url, sleep=sleeps.append).send(attribution())
    assert len(srv.requests) == 3 and sleeps == [1.0, 2.0]


def test_webhook_fails_after_max_retries(http_recorder):
    srv = http_recorder([(500, "x")] * 5)
    with pytest.raises(Exception):
        webhook.WebhookExporter(srv.url, sleep=lambda s: None).send(attribution())
    assert len(srv.requests) == 3


def test_webhook_no_retry_on_4xx(http_recorder):
    srv = http_recorder([(400, "bad")])
    with pytest.raises(webhook.NonRetryableError):
        webhook.WebhookExporter(srv.url, sleep=lambda s: None).send(attribution())
    assert len(srv.requests) == 1


def test_pagerduty_and_opsgenie_payloads():
    pd = json.loads(webhook.pagerduty_payload(attribution(0.9)))
    assert pd["event_action"] == "trigger" and pd["payload"]["severity"] == "critical"
    assert json.loads(webhook.pagerduty_payload(attribution(0.5)))["payload"]["severity"] == "warning"
    assert pd["payload"]["custom_details"]["evidence"] == "llm.ebpf.dns.latency_ms=220"
    og = json.loads(webhook.opsgenie_payload(attribution(0.9, 2.0)))
    assert og["priority"] == "P2" and og["alias"] == "inc-1"
    assert json.loads(webhook.opsgenie_payload(attribution(0.5, 2.0)))["priority"] == "P3"
    assert json.loads(webhook.opsgenie_payload(attribution(0.5, 3.0)))["priority"] == "P1"
    with pytest.raises(ValueError):
        webhook.parse_format("carrier-pigeon")


def slo_ev(status="breach"):
    return SLOEvent(event_id="e1", timestamp=1_700_000_000_000_000_000, cluster="c", namespace="n", workload="w",
                    service="s", request_id="r", sli_name="ttft_ms", sli_value=1200.0, unit="ms", status=status)


def test_otlp_slo_batch(http_recorder):
    srv = http_recorder()
    exp = otel.OTLPLogExporter(srv.url + "/v1/logs")
    exp.export_slo_batch([slo_ev("breach"), slo_ev("warning"), slo_ev("ok")])
    body = json.loads(srv.requests[0]["body"])
    recs = body["resourceLogs"][0]["scopeLogs"][0]["logRecords"]
    assert [r["severityText"] for r in recs] == ["ERROR", "WARN", "INFO"]
    res = body["resourceLogs"][0]["resource"]["attributes"]
    assert {"key": "service.name", "value": {"stringValue": "llm-slo-ebpf-toolkit"}} in res


def test_otlp_probe_batching_and_non2xx(http_recorder):
    srv = http_recorder([(200, "{}"), (500, "{}")])
    exp = otel.OTLPLogExporter(srv.url, max_batch=3, max_age_s=60)
    pe = ProbeEventV1(ts_unix_nano=5, signal="dns_latency_ms", node="n", namespace="ns", pod="p", container="c",
                      pid=1, tid=1, value=3.0, unit="ms", status="ok")
    for _ in range(3):
        exp.add_probe(pe)  # third add flushes one POST with 3 records
    assert len(srv.requests) == 1
    assert len(json.loads(srv.requests[0]["body"])["resourceLogs"][0]["scopeLogs"][0]["logRecords"]) == 3
    with pytest.raises(ConnectionError):
        exp.export_probe_batch([pe])


class MockQuerier:
    def __init__(self, vals, fail=None):
        self.vals, self.fail = vals, fail

    def query(self, q):
        if self.fail and self.fail in q:
            raise RuntimeError("boom")
        for k, v in self.vals.items():
            if k in q:
                return v
        return 0.0


def test_cdgate_pass_and_violations():
    t = cdgate.Thresholds()
    r = cdgate.evaluate_slo_gate(MockQuerier({"ttft": 500, "errors": 0.01, "burn": 1.0}), t)
    assert r.passed and not r.violations
    r = cdgate.evaluate_slo_gate(MockQuerier({"ttft": 900, "errors": 0.5, "burn": 1.0}), t)
    assert not r.passed and {v.metric for v in r.violations} == {"ttft_p95_ms", "error_rate"}
    r = cdgate.evaluate_slo_gate(MockQuerier({}, fail="ttft"), t)
    assert not r.passed and "failed" in r.error


def test_cdgate_http_querier(http_recorder):
    ok = json.dumps({"status": "success", "data": {"resultType": "vector",
                                                     "result": [{"metric": {}, "value": [1, "412.5"]}]}})
    empty = json.dumps({"status": "success", "data": {"resultType": "vector", "result": []}})
    srv = http_recorder([(200, ok), (200, empty), (500, "err")])
    q = cdgate.HTTPQuerier(srv.url, 2.0)
    assert q.query("up") == 412.5
    assert "/api/v1/query" in srv.requests[0]["path"]
    with pytest.raises(Exception):
        q.query("up")
    with pytest.raises(Exception):
        q.query("up")


def test_cdgate_default_queries():
    qs = cdgate.default_queries()
    assert set(qs) == {"ttft_p95_ms", "error_rate", "burn_rate"}
    assert "llm_slo_ttft_ms_bucket" in qs["ttft_p95_ms"]


def test_prometheus_registry_exposition_roundtrip():
    r = prometheus.Registry()
    c = r.counter("x_total", "x", ("reason",))
    c.inc(2, "a")
    g = r.gauge("y", "y")
    g.set(3.5)
    h = r.histogram("z_ms", "z", (1, 2, 5), ("node",))
    for v in (0.5, 1.0, 1.5, 7.0):
        h.observe(v, "n1")
    h.add_counts([1, 0, 0, 1], 9.0, "n1")
    text = r.exposition()
    parsed = prometheus.parse_exposition(text)
    assert parsed['x_total{reason="a"}'] == 2 and parsed["y"] == 3.5
    assert parsed['z_ms_bucket{node="n1",le="1"}'] == 3
    assert parsed['z_ms_bucket{node="n1",le="+Inf"}'] == 6
    assert parsed['z_ms_count{node="n1"}'] == 6 and parsed['z_ms_sum{node="n1"}'] == pytest.approx(19.0)
    assert "# TYPE z_ms histogram" in text


def test_metrics_server_endpoints():
    r = prometheus.Registry()
    r.gauge("llm_slo_agent_up", "up").set(1)
    state = {"ready": False}
    srv = prometheus.MetricsServer(r, "127.0.0.1:0", ready=lambda: state["ready"]).start()
    try:
        base = f"http://127.0.0.1:{srv.port}"
        assert "llm_slo_agent_up 1" in urllib.request.urlopen(base + "/metrics").read().decode()
        assert urllib.request.urlopen(base + "/healthz").status == 200
        with pytest.raises(urllib.error.HTTPError):
            urllib.request.urlopen(base + "/readyz")
        state["ready"] = True
        assert urllib.request.urlopen(base + "/readyz").status == 200
    finally:
        srv.stop()

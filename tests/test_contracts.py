"""Contracts, validator and config (REF pkg/schema/validator_test.go, pkg/toolkitcfg/config_test.go)."""

import json
import os

import pytest

from llm_slo_ebpf_toolkit_amd.contracts import config as toolkitcfg
from llm_slo_ebpf_toolkit_amd.contracts import schemas, validator
from llm_slo_ebpf_toolkit_amd.contracts.types import ConnTuple, Evidence, FaultHypothesis, IncidentAttribution, \
    ProbeEventV1, SLOEvent, SLOImpact

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def slo_event(**kw):
    d = dict(event_id="evt-1", timestamp=1_700_000_000_000_000_000, cluster="local", namespace="default",
             workload="gateway", service="chat", request_id="req-1", sli_name="ttft_ms", sli_value=220.0, unit="ms",
             status="ok", trace_id="trace-1")
    d.update(kw)
    return SLOEvent(**d)


def test_slo_event_schema_accepts_and_rejects():
    validator.validate("slo-event", slo_event())
    with pytest.raises(validator.ValidationError):
        validator.validate("slo-event", slo_event(sli_name="made_up"))
    with pytest.raises(validator.ValidationError):
        validator.validate("slo-event", slo_event(status="error"))  # SLO status is ok|warning|breach
    bad = slo_event().to_dict()
    bad["extra"] = 1  # additionalProperties: false
    with pytest.raises(validator.ValidationError):
        validator.validate("slo-event", bad)


def test_incident_schema():
    inc = IncidentAttribution(incident_id="inc-1", timestamp=1, cluster="c", namespace="n", service="s",
                              predicted_fault_domain="provider_throttle", confidence=0.9,
                              evidence=[Evidence("llm.ebpf.tcp.retransmits", 7, "ebpf")],
                              slo_impact=SLOImpact("ttft_ms", 2.0, 5),
                              fault_hypotheses=[FaultHypothesis("provider_throttle", 0.8, ["syscall_latency_ms"])])
    validator.validate("incident-attribution", inc)
    d = inc.to_dict()
    d["confidence"] = 1.5
    assert not validator.compiled("incident-attribution").is_valid(d)
    d = inc.to_dict()
    d["slo_impact"]["window_minutes"] = 0
    assert not validator.compiled("incident-attribution").is_valid(d)
    d = inc.to_dict()
    d["evidence"][0]["source"] = "telepathy"
    assert not validator.compiled("incident-attribution").is_valid(d)
    # GPU domains are an additive extension of the v1 enum
    d = inc.to_dict()
    d["predicted_fault_domain"] = "gpu_contention"
    assert validator.compiled("incident-attribution").is_valid(d)


def test_probe_event_schema():
    ev = ProbeEventV1(ts_unix_nano=1, signal="dns_latency_ms", node="n", namespace="ns", pod="p", container="c",
                      pid=1, tid=1, value=3.0, unit="ms", status="error",
                      conn_tuple=ConnTuple("10.0.0.1", "10.0.0.2", 1, 53, "udp"))
    validator.validate("probe-event", ev)
    d = ev.to_dict()
    d["conn_tuple"]["dst_port"] = 70000
    assert not validator.compiled("probe-event").is_valid(d)
    d = ev.to_dict()
    d["status"] = "breach"  # probe status is ok|warning|error
    assert not validator.compiled("probe-event").is_valid(d)
    d = ev.to_dict()
    d["pid"] = -1
    assert not validator.compiled("probe-event").is_valid(d)


def test_toolkit_config_schema_rejects_unknown_section_and_signal():
    good = toolkitcfg.default().to_dict()
    validator.validate("toolkit-config", good)
    bad = dict(good)
    bad["unexpected_section"] = {"x": 1}
    errs = validator.compiled("toolkit-config").errors(bad)
    assert errs and any("unexpected_section" in e for e in errs)
    bad = dict(good)
    bad["signal_set"] = ["dns_latency_ms", "not_a_signal"]
    errs = validator.compiled("toolkit-config").errors(bad)
    assert errs and any("signal_set" in e for e in errs)


def test_schema_files_match_programmatic_contracts():
    for name, rel in schemas.EXPORT_PATHS.items():
        with open(os.path.join(ROOT, rel)) as fh:
            assert json.load(fh) == schemas.get(name), rel


def test_validator_compiles_once():
    a = validator.compiled("slo-event")
    assert validator.compiled("slo-event") is a


def test_config_load(tmp_path):
    p = tmp_path / "toolkit.yaml"
    p.write_text("""
apiVersion: toolkit.llm-slo.dev/v1alpha1
kind: ToolkitConfig
signal_set: [dns_latency_ms, tcp_retransmits_total]
sampling: {events_per_second_limit: 500, burst_limit: 1000}
correlation: {window_ms: 1500}
otlp: {endpoint: "http://localhost:4317"}
safety: {max_overhead_pct: 4}
webhook: {enabled: true, url: "https://hooks.example.dev/incident", secret: s, format: opsgenie, timeout_ms: 2500}
cdgate: {enabled: true, prometheus_url: "http://prometheus.monitoring:9090", ttft_p95_ms: 900, error_rate: 0.07,
         burn_rate: 2.5, fail_open: false}
""")
    cfg = toolkitcfg.load(str(p))
    assert cfg.sampling.events_per_second_limit == 500 and cfg.safety.max_overhead_pct == 4
    assert len(cfg.signal_set) == 2
    assert cfg.webhook.enabled and cfg.webhook.format == "opsgenie" and cfg.webhook.timeout_ms == 2500
    assert cfg.cdgate.enabled and cfg.cdgate.prometheus_url == "http://prometheus.monitoring:9090"
    assert cfg.cdgate.fail_open is False


def test_config_defaults_for_extensions(tmp_path):
    p = tmp_path / "toolkit.yaml"
    p.write_text("""
signal_set: [dns_latency_ms]
sampling: {events_per_second_limit: 10, burst_limit: 20}
correlation: {window_ms: 200}
otlp: {endpoint: "http://otel-collector:4317"}
safety: {max_overhead_pct: 3}
""")
    cfg = toolkitcfg.load(str(p))
    assert cfg.webhook.format == "generic" and cfg.webhook.timeout_ms == 5000
    assert cfg.cdgate.prometheus_url == "http://prometheus:9090"
    assert (cfg.cdgate.ttft_p95_ms, cfg.cdgate.error_rate, cfg.cdgate.burn_rate, cfg.cdgate.fail_open) == \
        (800, 0.05, 2.0, True)
    assert len(toolkitcfg.default().signal_set) == 9


def test_repo_config_is_valid():
    cfg = toolkitcfg.load(os.path.join(ROOT, "config", "toolkit.yaml"))
    assert cfg.gpu.window_ms > 0


def test_resolve_config_path():
    assert toolkitcfg.resolve_config_path(["--x", "1", "--config", "a.yaml"], "d") == "a.yaml"
    assert toolkitcfg.resolve_config_path(["--config=b.yaml"], "d") == "b.yaml"
    assert toolkitcfg.resolve_config_path([], "d") == "d"

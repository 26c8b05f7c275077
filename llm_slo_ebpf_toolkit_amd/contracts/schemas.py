"""Contract definitions (JSON Schema draft 2020-12), built programmatically.

The four REF contracts are reproduced field-for-field (closed objects, same
required sets, same enums and bounds):

* SLO event v1            -- REF docs/contracts/v1/slo-event.schema.json:1-53
* incident attribution v1 -- REF docs/contracts/v1/incident-attribution.schema.json:1-96
* probe event v1alpha1    -- REF docs/contracts/v1alpha1/probe-event.schema.json:1-109
* toolkit config v1alpha1 -- REF config/toolkit.schema.json:1-197

Additive NEW extensions (REF's v1 policy allows additive change only,
docs/contracts/v1/README.md:9-12): the two GPU fault domains in the attribution
domain enum, the four GPU signals in the config ``signal_set`` enum, and an optional
``gpu`` config block. Schemas are exported to JSON files with
``schemavalidate --export DIR`` rather than checked in twice.
"""

from __future__ import annotations

import copy
import json
import os
from typing import Any, Dict, Iterable, List, Optional

from ..signals import catalog

DRAFT = "https://json-schema.org/draft/2020-12/schema"
BASE_ID = "https://llm-slo-ebpf-toolkit.dev"


def _s(**kw) -> Dict[str, Any]:
    out: Dict[str, Any] = {"type": "string"}
    out.update(kw)
    return out


def _num(lo: Optional[float] = None, hi: Optional[float] = None, **kw) -> Dict[str, Any]:
    out: Dict[str, Any] = {"type": "number"}
    if lo is not None:
        out["minimum"] = lo
    if hi is not None:
        out["maximum"] = hi
    out.update(kw)
    return out


def _int(lo: Optional[int] = None, hi: Optional[int] = None, **kw) -> Dict[str, Any]:
    out: Dict[str, Any] = {"type": "integer"}
    if lo is not None:
        out["minimum"] = lo
    if hi is not None:
        out["maximum"] = hi
    out.update(kw)
    return out


def _bool(**kw) -> Dict[str, Any]:
    out: Dict[str, Any] = {"type": "boolean"}
    out.update(kw)
    return out


def _enum(values: Iterable[str], **kw) -> Dict[str, Any]:
    return _s(enum=list(values), **kw)


def _arr(items: Dict[str, Any], **kw) -> Dict[str, Any]:
    out: Dict[str, Any] = {"type": "array", "items": items}
    out.update(kw)
    return out


def _obj(props: Dict[str, Any], required: Iterable[str] = (), **kw) -> Dict[str, Any]:
    out: Dict[str, Any] = {"type": "object", "additionalProperties": False}
    req = list(required)
    if req:
        out["required"] = req
    out["properties"] = props
    out.update(kw)
    return out


def _doc(rel_id: str, title: str, body: Dict[str, Any]) -> Dict[str, Any]:
    doc = {"$schema": DRAFT, "$id": f"{BASE_ID}/{rel_id}", "title": title}
    doc.update(body)
    return doc


SLI_NAMES = ("ttft_ms", "request_latency_ms", "token_throughput_tps", "error_rate",
             "retrieval_latency_ms", "provider_error_rate")
SLO_STATUSES = ("ok", "warning", "breach")
PROBE_STATUSES = ("ok", "warning", "error")
EVIDENCE_SOURCES = ("ebpf", "otel", "kubernetes", "application")
WEBHOOK_FORMATS = ("generic", "pagerduty", "opsgenie")


def slo_event_schema() -> Dict[str, Any]:
    props = {
        "event_id": _s(), "timestamp": _s(format="date-time"), "cluster": _s(),
        "namespace": _s(), "workload": _s(), "service": _s(), "request_id": _s(),
        "trace_id": _s(), "sli_name": _enum(SLI_NAMES), "sli_value": _num(), "unit": _s(),
        "status": _enum(SLO_STATUSES),
        "labels": {"type": "object", "additionalProperties": _s()},
    }
    req = ["event_id", "timestamp", "cluster", "namespace", "workload", "service",
           "request_id", "sli_name", "sli_value", "unit", "status"]
    return _doc("contracts/v1/slo-event.schema.json", "SloEventV1", _obj(props, req))


def incident_attribution_schema() -> Dict[str, Any]:
    evidence = _obj({"signal": _s(), "value": {"type": ["string", "number", "boolean"]},
                     "source": _enum(EVIDENCE_SOURCES)}, ["signal", "value", "source"])
    impact = _obj({"sli": _s(), "burn_rate": _num(), "window_minutes": _int(1)},
                  ["sli", "burn_rate", "window_minutes"])
    hypothesis = _obj({"domain": _s(), "posterior": _num(0, 1), "evidence": _arr(_s())},
                      ["domain", "posterior", "evidence"])
    props = {
        "incident_id": _s(), "timestamp": _s(format="date-time"), "cluster": _s(),
        "namespace": _s(), "service": _s(),
        "predicted_fault_domain": _enum(catalog.ALL_DOMAINS),
        "confidence": _num(0, 1), "evidence": _arr(evidence), "slo_impact": impact,
        "trace_ids": _arr(_s()), "request_ids": _arr(_s()),
        "fault_hypotheses": _arr(hypothesis),
    }
    req = ["incident_id", "timestamp", "cluster", "service", "predicted_fault_domain",
           "confidence", "evidence", "slo_impact"]
    return _doc("contracts/v1/incident-attribution.schema.json", "IncidentAttributionV1",
                _obj(props, req))


def probe_event_schema() -> Dict[str, Any]:
    port = _int(0, 65535)
    conn = _obj({"src_ip": _s(), "dst_ip": _s(), "src_port": port, "dst_port": port,
                 "protocol": _s()}, ["src_ip", "dst_ip", "src_port", "dst_port", "protocol"])
    props = {
        "ts_unix_nano": _int(0), "signal": _s(), "node": _s(), "namespace": _s(),
        "pod": _s(), "container": _s(), "pid": _int(0), "tid": _int(0),
        "conn_tuple": conn, "value": _num(), "unit": _s(), "status": _enum(PROBE_STATUSES),
        "trace_id": _s(), "span_id": _s(), "errno": _int(), "confidence": _num(0, 1),
        # NEW additive: which GPU the event is attributed to (GPU signals only).
        "gpu_id": _int(0),
    }
    req = ["ts_unix_nano", "signal", "node", "namespace", "pod", "container", "pid", "tid",
           "value", "unit", "status"]
    return _doc("contracts/v1alpha1/probe-event.schema.json", "ProbeEventV1", _obj(props, req))


def toolkit_config_schema() -> Dict[str, Any]:
    sig_enum = [s.name for s in catalog.SIGNALS if s.in_config_enum]
    props = {
        "apiVersion": _s(default="toolkit.llm-slo.dev/v1alpha1"),
        "kind": _s(default="ToolkitConfig"),
        "signal_set": {"type": "array", "minItems": 1, "items": _enum(sig_enum),
                       "default": list(catalog.DEFAULT_CONFIG_SIGNALS)},
        "sampling": _obj({"events_per_second_limit": _int(1, default=10000),
                          "burst_limit": _int(1, default=20000)},
                         ["events_per_second_limit", "burst_limit"]),
        "correlation": _obj({"window_ms": _int(1, default=2000)}, ["window_ms"]),
        "otlp": _obj({"endpoint": _s(minLength=1, default="http://otel-collector:4317")},
                     ["endpoint"]),
        "safety": _obj({"max_overhead_pct": _num(0, default=5)}, ["max_overhead_pct"]),
        "webhook": _obj({"enabled": _bool(default=False), "url": _s(default=""),
                         "secret": _s(default=""), "format": _enum(WEBHOOK_FORMATS, default="generic"),
                         "timeout_ms": _int(1, default=5000)},
                        ["enabled", "url", "secret", "format", "timeout_ms"]),
        "cdgate": _obj({"enabled": _bool(default=False),
                        "prometheus_url": _s(minLength=1, default="http://prometheus:9090"),
                        "ttft_p95_ms": _num(0, default=800), "error_rate": _num(0, 1, default=0.05),
                        "burn_rate": _num(0, default=2.0), "fail_open": _bool(default=True)},
                       ["enabled", "prometheus_url", "ttft_p95_ms", "error_rate", "burn_rate",
                        "fail_open"]),
        # NEW additive block: GPU engine knobs.
        "gpu": _obj({"enabled": _bool(default=True), "window_ms": _int(1, default=1000),
                     "max_events_per_window": _int(1, default=1 << 20),
                     "world_size": _int(0, default=1),  # 0 = every GPU visible to the agent
                     "attribution_model": _enum(("bayes", "bayes_gpu", "bayes_learned", "lda", "rule"),
                                                default="bayes")}),
    }
    req = ["signal_set", "sampling", "correlation", "otlp", "safety"]
    return _doc("config/v1alpha1/toolkit.schema.json", "ToolkitConfigV1Alpha1", _obj(props, req))


_BUILDERS = {
    "slo-event": slo_event_schema,
    "incident-attribution": incident_attribution_schema,
    "probe-event": probe_event_schema,
    "toolkit-config": toolkit_config_schema,
}

EXPORT_PATHS = {
    "slo-event": os.path.join("docs", "contracts", "v1", "slo-event.schema.json"),
    "incident-attribution": os.path.join("docs", "contracts", "v1", "incident-attribution.schema.json"),
    "probe-event": os.path.join("docs", "contracts", "v1alpha1", "probe-event.schema.json"),
    "toolkit-config": os.path.join("config", "toolkit.schema.json"),
}


def get(name: str) -> Dict[str, Any]:
    return copy.deepcopy(_BUILDERS[name]())


def names() -> List[str]:
    return list(_BUILDERS)


def export_all(root: str) -> List[str]:
    written = []
    for name, rel in EXPORT_PATHS.items():
        path = os.path.join(root, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w", encoding="utf-8") as fh:
            json.dump(get(name), fh, indent=2)
            fh.write("\n")
        written.append(path)
    return written

"""FaultSample (benchmark/attribution input) and the rule-based label mapper.

REF pkg/attribution/mapper.go:11-98 and io.go:12-39.
"""

from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List

from ..contracts import semconv
from ..contracts.types import Evidence, IncidentAttribution, SLOImpact
from ..utils.timeutil import format_rfc3339_ns, parse_rfc3339_ns

LABEL_TO_DOMAIN = {
    "dns_latency": "network_dns",
    "egress_drop": "network_egress",
    "cpu_throttle": "cpu_throttle",
    "memory_pressure": "memory_pressure",
    "network_partition": "network_egress",
    "provider_throttle": "provider_throttle",
    "provider_error": "provider_error",
    "retrieval_slowdown": "retrieval_backend",
    # NEW (MI355X) fault labels
    "gpu_contention": "gpu_contention",
    "gpu_compute_contention": "gpu_contention",
    "hbm_pressure": "gpu_contention",
    "cpu_contention": "cpu_throttle",
    "rccl_latency": "gpu_interconnect",
    "xgmi_degraded": "gpu_interconnect",
}


def map_fault_label(label: str) -> str:
    """REF MapFaultLabel (mapper.go:29-50); unmapped labels -> "unknown"."""
    return LABEL_TO_DOMAIN.get(label, "unknown")


@dataclass
class FaultSample:
    incident_id: str = ""
    timestamp: int = 0
    cluster: str = ""
    namespace: str = ""
    service: str = ""
    fault_label: str = ""
    expected_domain: str = ""
    expected_domains: List[str] = field(default_factory=list)
    signals: Dict[str, float] = field(default_factory=dict)
    confidence: float = 0.0
    burn_rate: float = 0.0
    window_minutes: int = 0
    request_id: str = ""
    trace_id: str = ""

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "FaultSample":
        return cls(
            incident_id=d.get("incident_id", ""), timestamp=parse_rfc3339_ns(d.get("timestamp")),
            cluster=d.get("cluster", ""), namespace=d.get("namespace", ""),
            service=d.get("service", ""), fault_label=d.get("fault_label", ""),
            expected_domain=d.get("expected_domain", "") or "",
            expected_domains=list(d.get("expected_domains") or []),
            signals={k: float(v) for k, v in (d.get("signals") or {}).items()},
            confidence=float(d.get("confidence", 0.0)), burn_rate=float(d.get("burn_rate", 0.0)),
            window_minutes=int(d.get("window_minutes", 0)), request_id=d.get("request_id", ""),
            trace_id=d.get("trace_id", ""))

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {
            "incident_id": self.incident_id, "timestamp": format_rfc3339_ns(self.timestamp),
            "cluster": self.cluster, "namespace": self.namespace, "service": self.service,
            "fault_label": self.fault_label,
        }
        if self.expected_domain:
            out["expected_domain"] = self.expected_domain
        if self.expected_domains:
            out["expected_domains"] = list(self.expected_domains)
        if self.signals:
            out["signals"] = dict(self.signals)
        out.update({"confidence": self.confidence, "burn_rate": self.burn_rate,
                    "window_minutes": self.window_minutes, "request_id": self.request_id,
                    "trace_id": self.trace_id})
        return out

    def actual_domain(self) -> str:
        return self.expected_domain or map_fault_label(self.fault_label)

    def expected_set(self) -> List[str]:
        return list(self.expected_domains) if self.expected_domains else [self.actual_domain()]


def build_attribution(sample: FaultSample) -> IncidentAttribution:
    """REF BuildAttribution (mapper.go:53-98), including the hard-coded DNS 180.0 evidence."""
    domain = map_fault_label(sample.fault_label)
    evidence = [
        Evidence("fault_label", sample.fault_label, "application"),
        Evidence("mapped_domain", domain, "ebpf"),
        Evidence(semconv.ATTR_CORRELATION_CONF, sample.confidence, "otel"),
    ]
    if sample.fault_label == "dns_latency":
        evidence.append(Evidence(semconv.ATTR_DNS_LATENCY_MS, 180.0, "ebpf"))
    return IncidentAttribution(
        incident_id=sample.incident_id, timestamp=sample.timestamp, cluster=sample.cluster,
        namespace=sample.namespace, service=sample.service, predicted_fault_domain=domain,
        confidence=sample.confidence, evidence=evidence,
        slo_impact=SLOImpact("ttft_ms", sample.burn_rate, sample.window_minutes),
        trace_ids=[sample.trace_id], request_ids=[sample.request_id])


def load_samples_jsonl(path: str) -> List[FaultSample]:
    out: List[FaultSample] = []
    with open(path, "r", encoding="utf-8") as fh:
        for line in fh:
            line = line.strip()
            if not line:
                continue
            try:
                out.append(FaultSample.from_dict(json.loads(line)))
            except ValueError as exc:
                raise ValueError(f"parse sample: {exc}") from exc
    if not out:
        raise ValueError(f"no samples loaded from {path}")
    return out


def write_samples_jsonl(path: str, samples: List[FaultSample]) -> None:
    with open(path, "w", encoding="utf-8") as fh:
        for s in samples:
            fh.write(json.dumps(s.to_dict(), separators=(",", ":")) + "\n")

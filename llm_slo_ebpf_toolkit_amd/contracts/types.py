"""Typed contract objects with Go-compatible JSON encoding.

Mirrors REF pkg/schema/types.go:6-86 (SLOEvent, Evidence, SLOImpact, FaultHypothesis,
IncidentAttribution, ConnTuple, ProbeEventV1), including ``omitempty`` behaviour so
the emitted JSON validates against the same contracts. Timestamps are int Unix ns.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

from ..utils.timeutil import format_rfc3339_ns, parse_rfc3339_ns

EvidenceValue = Union[str, float, int, bool]


@dataclass
class SLOEvent:
    event_id: str
    timestamp: int
    cluster: str
    namespace: str
    workload: str
    service: str
    request_id: str
    sli_name: str
    sli_value: float
    unit: str
    status: str
    trace_id: str = ""
    labels: Dict[str, str] = field(default_factory=dict)

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {
            "event_id": self.event_id, "timestamp": format_rfc3339_ns(self.timestamp),
            "cluster": self.cluster, "namespace": self.namespace, "workload": self.workload,
            "service": self.service, "request_id": self.request_id,
        }
        if self.trace_id:
            out["trace_id"] = self.trace_id
        out.update({"sli_name": self.sli_name, "sli_value": self.sli_value, "unit": self.unit,
                    "status": self.status})
        if self.labels:
            out["labels"] = dict(self.labels)
        return out

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "SLOEvent":
        return cls(event_id=d.get("event_id", ""), timestamp=parse_rfc3339_ns(d.get("timestamp")),
                   cluster=d.get("cluster", ""), namespace=d.get("namespace", ""),
                   workload=d.get("workload", ""), service=d.get("service", ""),
                   request_id=d.get("request_id", ""), sli_name=d.get("sli_name", ""),
                   sli_value=float(d.get("sli_value", 0.0)), unit=d.get("unit", ""),
                   status=d.get("status", ""), trace_id=d.get("trace_id", ""),
                   labels=dict(d.get("labels") or {}))


@dataclass
class Evidence:
    signal: str
    value: EvidenceValue
    source: str

    def to_dict(self) -> Dict[str, Any]:
        return {"signal": self.signal, "value": self.value, "source": self.source}


@dataclass
class SLOImpact:
    sli: str
    burn_rate: float
    window_minutes: int

    def to_dict(self) -> Dict[str, Any]:
        return {"sli": self.sli, "burn_rate": self.burn_rate, "window_minutes": self.window_minutes}


@dataclass
class FaultHypothesis:
    domain: str
    posterior: float
    evidence: List[str] = field(default_factory=list)

    def to_dict(self) -> Dict[str, Any]:
        return {"domain": self.domain, "posterior": self.posterior, "evidence": list(self.evidence)}


@dataclass
class IncidentAttribution:
    incident_id: str
    timestamp: int
    cluster: str
    service: str
    predicted_fault_domain: str
    confidence: float
    evidence: List[Evidence]
    slo_impact: SLOImpact
    namespace: str = ""
    trace_ids: List[str] = field(default_factory=list)
    request_ids: List[str] = field(default_factory=list)
    fault_hypotheses: List[FaultHypothesis] = field(default_factory=list)

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {"incident_id": self.incident_id,
                               "timestamp": format_rfc3339_ns(self.timestamp),
                               "cluster": self.cluster}
        if self.namespace:
            out["namespace"] = self.namespace
        out.update({
            "service": self.service, "predicted_fault_domain": self.predicted_fault_domain,
            "confidence": self.confidence, "evidence": [e.to_dict() for e in self.evidence],
            "slo_impact": self.slo_impact.to_dict(),
        })
        if self.trace_ids:
            out["trace_ids"] = list(self.trace_ids)
        if self.request_ids:
            out["request_ids"] = list(self.request_ids)
        if self.fault_hypotheses:
            out["fault_hypotheses"] = [h.to_dict() for h in self.fault_hypotheses]
        return out

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "IncidentAttribution":
        imp = d.get("slo_impact") or {}
        return cls(
            incident_id=d.get("incident_id", ""), timestamp=parse_rfc3339_ns(d.get("timestamp")),
            cluster=d.get("cluster", ""), service=d.get("service", ""),
            predicted_fault_domain=d.get("predicted_fault_domain", ""),
            confidence=float(d.get("confidence", 0.0)),
            evidence=[Evidence(e["signal"], e["value"], e["source"]) for e in d.get("evidence") or []],
            slo_impact=SLOImpact(imp.get("sli", ""), float(imp.get("burn_rate", 0.0)),
                                 int(imp.get("window_minutes", 0))),
            namespace=d.get("namespace", ""), trace_ids=list(d.get("trace_ids") or []),
            request_ids=list(d.get("request_ids") or []),
            fault_hypotheses=[FaultHypothesis(h["domain"], float(h["posterior"]), list(h.get("evidence") or []))
                              for h in d.get("fault_hypotheses") or []])


@dataclass
class ConnTuple:
    src_ip: str
    dst_ip: str
    src_port: int
    dst_port: int
    protocol: str

    def to_dict(self) -> Dict[str, Any]:
        return {"src_ip": self.src_ip, "dst_ip": self.dst_ip, "src_port": self.src_port,
                "dst_port": self.dst_port, "protocol": self.protocol}

    def key(self) -> str:
        """Canonical string form used as the correlation conn-tuple key."""
        return f"{self.protocol}:{self.src_ip}:{self.src_port}->{self.dst_ip}:{self.dst_port}"


@dataclass
class ProbeEventV1:
    ts_unix_nano: int
    signal: str
    node: str
    namespace: str
    pod: str
    container: str
    pid: int
    tid: int
    value: float
    unit: str
    status: str
    conn_tuple: Optional[ConnTuple] = None
    trace_id: str = ""
    span_id: str = ""
    errno: Optional[int] = None
    confidence: Optional[float] = None
    gpu_id: Optional[int] = None

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {
            "ts_unix_nano": self.ts_unix_nano, "signal": self.signal, "node": self.node,
            "namespace": self.namespace, "pod": self.pod, "container": self.container,
            "pid": self.pid, "tid": self.tid,
        }
        if self.conn_tuple is not None:
            out["conn_tuple"] = self.conn_tuple.to_dict()
        out.update({"value": self.value, "unit": self.unit, "status": self.status})
        if self.trace_id:
            out["trace_id"] = self.trace_id
        if self.span_id:
            out["span_id"] = self.span_id
        if self.errno is not None:
            out["errno"] = self.errno
        if self.confidence is not None:
            out["confidence"] = self.confidence
        if self.gpu_id is not None:
            out["gpu_id"] = self.gpu_id
        return out

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ProbeEventV1":
        ct = d.get("conn_tuple")
        return cls(
            ts_unix_nano=int(d.get("ts_unix_nano", 0)), signal=d.get("signal", ""),
            node=d.get("node", ""), namespace=d.get("namespace", ""), pod=d.get("pod", ""),
            container=d.get("container", ""), pid=int(d.get("pid", 0)), tid=int(d.get("tid", 0)),
            value=float(d.get("value", 0.0)), unit=d.get("unit", ""), status=d.get("status", ""),
            conn_tuple=ConnTuple(**ct) if ct else None, trace_id=d.get("trace_id", ""),
            span_id=d.get("span_id", ""), errno=d.get("errno"), confidence=d.get("confidence"),
            gpu_id=d.get("gpu_id"))

"""RawSample -> SLO events, and the deterministic synthetic scenario generator.

* ``RawSample`` / ``normalize_sample`` -- REF pkg/collector/pipeline.go:11-84: four SLO
  events per sample with thresholds ttft 500/1000, latency 700/1500, tps inverse 30/10,
  error 0.02/0.05 (``>=`` breach first; inverse ``<=``).
* ``SCENARIO_SEQUENCE`` / ``build_synthetic_sample`` -- REF pkg/collector/synthetic.go:17-132.
"""

from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Any, Dict, List

from ..contracts.types import SLOEvent
from ..utils.timeutil import SECOND, format_rfc3339_ns, parse_rfc3339_ns


@dataclass
class RawSample:
    timestamp: int = 0
    cluster: str = ""
    namespace: str = ""
    workload: str = ""
    service: str = ""
    node: str = ""
    request_id: str = ""
    trace_id: str = ""
    ttft_ms: float = 0.0
    request_latency_ms: float = 0.0
    token_throughput_tps: float = 0.0
    error_rate: float = 0.0
    fault_label: str = ""

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {"timestamp": format_rfc3339_ns(self.timestamp), "cluster": self.cluster,
                               "namespace": self.namespace, "workload": self.workload,
                               "service": self.service}
        if self.node:
            out["node"] = self.node
        out.update({"request_id": self.request_id, "trace_id": self.trace_id, "ttft_ms": self.ttft_ms,
                    "request_latency_ms": self.request_latency_ms,
                    "token_throughput_tps": self.token_throughput_tps, "error_rate": self.error_rate})
        if self.fault_label:
            out["fault_label"] = self.fault_label
        return out

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RawSample":
        return cls(timestamp=parse_rfc3339_ns(d.get("timestamp")), cluster=d.get("cluster", ""),
                   namespace=d.get("namespace", ""), workload=d.get("workload", ""),
                   service=d.get("service", ""), node=d.get("node", "") or "",
                   request_id=d.get("request_id", ""), trace_id=d.get("trace_id", ""),
                   ttft_ms=float(d.get("ttft_ms", 0.0)),
                   request_latency_ms=float(d.get("request_latency_ms", 0.0)),
                   token_throughput_tps=float(d.get("token_throughput_tps", 0.0)),
                   error_rate=float(d.get("error_rate", 0.0)), fault_label=d.get("fault_label", "") or "")


def threshold_status(value: float, warning: float, breach: float) -> str:
    if value >= breach:
        return "breach"
    if value >= warning:
        return "warning"
    return "ok"


def inverse_threshold_status(value: float, warning: float, breach: float) -> str:
    if value <= breach:
        return "breach"
    if value <= warning:
        return "warning"
    return "ok"


def _event(sample: RawSample, sli: str, value: float, unit: str, status: str) -> SLOEvent:
    labels = {"source": "synthetic"}
    if sample.node:
        labels["node"] = sample.node
    if sample.fault_label:
        labels["fault_label"] = sample.fault_label
    return SLOEvent(event_id=f"{sample.request_id}-{sli}", timestamp=sample.timestamp,
                    cluster=sample.cluster, namespace=sample.namespace, workload=sample.workload,
                    service=sample.service, request_id=sample.request_id, sli_name=sli,
                    sli_value=value, unit=unit, status=status, trace_id=sample.trace_id, labels=labels)


def normalize_sample(s: RawSample) -> List[SLOEvent]:
    return [
        _event(s, "ttft_ms", s.ttft_ms, "ms", threshold_status(s.ttft_ms, 500, 1000)),
        _event(s, "request_latency_ms", s.request_latency_ms, "ms",
               threshold_status(s.request_latency_ms, 700, 1500)),
        _event(s, "token_throughput_tps", s.token_throughput_tps, "tps",
               inverse_threshold_status(s.token_throughput_tps, 30, 10)),
        _event(s, "error_rate", s.error_rate, "ratio", threshold_status(s.error_rate, 0.02, 0.05)),
    ]


SCENARIO_SEQUENCE: Dict[str, List[str]] = {
    "baseline": ["baseline"],
    "provider_throttle": ["provider_throttle"],
    "dns_latency": ["dns_latency"],
    "cpu_throttle": ["cpu_throttle"],
    "memory_pressure": ["memory_pressure"],
    "network_partition": ["network_partition"],
    "mixed": ["provider_throttle", "dns_latency", "cpu_throttle", "memory_pressure", "network_partition"],
    "mixed_multi": ["mixed_multi"],
    # NEW (MI355X) scenarios
    "gpu_contention": ["gpu_contention"],
    "rccl_latency": ["rccl_latency"],
}

SUPPORTED_SYNTHETIC_SCENARIOS = list(SCENARIO_SEQUENCE)

# (ttft, latency, tps, error_rate) per fault label (REF synthetic.go:80-132)
SLI_PROFILE: Dict[str, tuple] = {
    "provider_throttle": (980, 2100, 7, 0.14),
    "dns_latency": (820, 1600, 18, 0.03),
    "cpu_throttle": (700, 1350, 11, 0.05),
    "memory_pressure": (650, 1250, 13, 0.04),
    "network_partition": (1200, 3500, 3, 0.25),
    "mixed_multi": (1450, 4200, 2, 0.31),
    "gpu_contention": (900, 1900, 9, 0.02),
    "rccl_latency": (1100, 2600, 6, 0.03),
    # NEW (REF has no SLI profile for them): a provider failing requests costs errors more than
    # time; a slow vector store delays the first token by the retrieval stall
    "provider_error": (620, 1300, 20, 0.22),
    "retrieval_slowdown": (1050, 1500, 24, 0.01),
}
BASE_SLI = (340, 720, 36, 0.005)


@dataclass
class SampleMeta:
    cluster: str = "local"
    namespace: str = "default"
    workload: str = "gateway"
    service: str = "chat"
    node: str = "unknown-node"


def build_synthetic_sample(scenario: str, idx: int, timestamp: int, meta: SampleMeta) -> RawSample:
    labels = SCENARIO_SEQUENCE.get(scenario)
    if labels is None:
        raise ValueError(f'unsupported scenario "{scenario}"')
    label = labels[idx % len(labels)]
    ttft, lat, tps, err = SLI_PROFILE.get(label, BASE_SLI)
    return RawSample(timestamp=timestamp, cluster=meta.cluster, namespace=meta.namespace,
                     workload=meta.workload, service=meta.service, node=meta.node,
                     request_id=f"collector-req-{idx + 1:04d}", trace_id=f"collector-trace-{idx + 1:04d}",
                     ttft_ms=float(ttft), request_latency_ms=float(lat), token_throughput_tps=float(tps),
                     error_rate=float(err), fault_label=label)


def generate_synthetic_samples(scenario: str, count: int, start_ns: int, meta: SampleMeta) -> List[RawSample]:
    if count < 1:
        raise ValueError("count must be >= 1")
    return [build_synthetic_sample(scenario, i, start_ns + i * SECOND, meta) for i in range(count)]


def read_raw_samples(lines) -> List[RawSample]:
    out = []
    for line in lines:
        line = line.strip()
        if line:
            out.append(RawSample.from_dict(json.loads(line)))
    return out

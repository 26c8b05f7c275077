"""Span <-> signal correlation tiers (CPU reference; the GPU join kernel must agree bit-exactly).

Semantics follow REF pkg/correlation/dns.go:50-113 exactly:

* outer window (default 2 s) first; a zero timestamp on either side never matches;
* tier precedence: trace_id exact (1.0) > pod+pid within 100 ms (0.9) >
  pod+conn-tuple within 250 ms (0.8) > service+node within 500 ms (0.65);
* every window test is ``abs(dt) <= window`` on integer nanoseconds;
* empty strings / non-positive pid never satisfy an equality tier.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Tuple

from ..contracts import semconv
from ..utils.timeutil import MS, SECOND, format_rfc3339_ns, parse_rfc3339_ns

DEFAULT_WINDOW_NS = 2 * SECOND
DEFAULT_ENRICHMENT_THRESHOLD = 0.7

TIER_TRACE = "trace_id_exact"
TIER_POD_PID = "pod_pid_100ms"
TIER_POD_CONN = "pod_conn_250ms"
TIER_SVC_NODE = "service_node_500ms"

# (name, confidence, window_ns); index+1 is the tier id used by the GPU kernels.
TIERS: Tuple[Tuple[str, float, int], ...] = (
    (TIER_TRACE, 1.0, 0),            # bounded by the outer window only
    (TIER_POD_PID, 0.9, 100 * MS),
    (TIER_POD_CONN, 0.8, 250 * MS),
    (TIER_SVC_NODE, 0.65, 500 * MS),
)
TIER_CONF = {name: conf for name, conf, _ in TIERS}
TIER_ID = {name: i + 1 for i, (name, _, _) in enumerate(TIERS)}


@dataclass
class SpanRef:
    trace_id: str = ""
    service: str = ""
    node: str = ""
    pod: str = ""
    pid: int = 0
    conn_tuple: str = ""
    timestamp: int = 0  # Unix ns, 0 = zero time

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "SpanRef":
        return cls(trace_id=d.get("trace_id", "") or "", service=d.get("service", "") or "",
                   node=d.get("node", "") or "", pod=d.get("pod", "") or "",
                   pid=int(d.get("pid", 0) or 0), conn_tuple=d.get("conn_tuple", "") or "",
                   timestamp=parse_rfc3339_ns(d.get("timestamp")))

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {}
        for k in ("trace_id", "service", "node", "pod"):
            if getattr(self, k):
                out[k] = getattr(self, k)
        if self.pid:
            out["pid"] = self.pid
        if self.conn_tuple:
            out["conn_tuple"] = self.conn_tuple
        out["timestamp"] = format_rfc3339_ns(self.timestamp)
        return out


@dataclass
class SignalRef:
    signal: str = ""
    trace_id: str = ""
    service: str = ""
    node: str = ""
    pod: str = ""
    pid: int = 0
    conn_tuple: str = ""
    timestamp: int = 0
    value: float = 0.0

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "SignalRef":
        return cls(signal=d.get("signal", "") or "", trace_id=d.get("trace_id", "") or "",
                   service=d.get("service", "") or "", node=d.get("node", "") or "",
                   pod=d.get("pod", "") or "", pid=int(d.get("pid", 0) or 0),
                   conn_tuple=d.get("conn_tuple", "") or "",
                   timestamp=parse_rfc3339_ns(d.get("timestamp")), value=float(d.get("value", 0.0)))

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {"signal": self.signal}
        for k in ("trace_id", "service", "node", "pod"):
            if getattr(self, k):
                out[k] = getattr(self, k)
        if self.pid:
            out["pid"] = self.pid
        if self.conn_tuple:
            out["conn_tuple"] = self.conn_tuple
        out["timestamp"] = format_rfc3339_ns(self.timestamp)
        out["value"] = self.value
        return out


@dataclass
class Decision:
    matched: bool = False
    confidence: float = 0.0
    tier: str = ""


def within_window(a_ns: int, b_ns: int, window_ns: int) -> bool:
    if a_ns == 0 or b_ns == 0:
        return False
    return abs(a_ns - b_ns) <= window_ns


def match(span: SpanRef, signal: SignalRef, window_ns: int = DEFAULT_WINDOW_NS) -> Decision:
    if window_ns <= 0:
        window_ns = DEFAULT_WINDOW_NS
    if not within_window(span.timestamp, signal.timestamp, window_ns):
        return Decision()
    if span.trace_id and span.trace_id == signal.trace_id:
        return Decision(True, 1.0, TIER_TRACE)
    if (span.pod and span.pod == signal.pod and span.pid > 0 and span.pid == signal.pid
            and within_window(span.timestamp, signal.timestamp, 100 * MS)):
        return Decision(True, 0.9, TIER_POD_PID)
    if (span.pod and span.pod == signal.pod and span.conn_tuple and span.conn_tuple == signal.conn_tuple
            and within_window(span.timestamp, signal.timestamp, 250 * MS)):
        return Decision(True, 0.8, TIER_POD_CONN)
    if (span.service and span.service == signal.service and span.node and span.node == signal.node
            and within_window(span.timestamp, signal.timestamp, 500 * MS)):
        return Decision(True, 0.65, TIER_SVC_NODE)
    return Decision()


def enrich_dns(base: Optional[Dict[str, float]], span: SpanRef, signal: SignalRef,
               window_ns: int = DEFAULT_WINDOW_NS,
               threshold: float = DEFAULT_ENRICHMENT_THRESHOLD) -> Tuple[Dict[str, float], Decision]:
    """REF EnrichDNS (dns.go:79-105): only dns_latency_ms signals at conf >= threshold enrich."""
    base = {} if base is None else base
    if threshold <= 0:
        threshold = DEFAULT_ENRICHMENT_THRESHOLD
    decision = match(span, signal, window_ns)
    if not decision.matched or decision.confidence < threshold:
        return base, decision
    if signal.signal != "dns_latency_ms":
        return base, Decision()
    out = dict(base)
    out[semconv.ATTR_DNS_LATENCY_MS] = signal.value
    out[semconv.ATTR_CORRELATION_CONF] = decision.confidence
    return out, decision

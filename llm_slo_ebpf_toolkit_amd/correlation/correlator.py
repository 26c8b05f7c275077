"""Multi-signal span enrichment (CPU oracle of the GPU join kernel ``ops.join``).

REF pkg/otel/processor/ebpfcorrelator/correlator.go:50-194 and processor.go:29-58:

* per span, every supported signal is matched (``match``); unsupported types,
  unmatched and low-confidence pairs are counted in ``DebugStats``;
* candidates are stable-sorted by (confidence desc, |dt| asc) and capped at the join
  fanout (3); the surplus is ``fanout_dropped``;
* each kept candidate max-merges its value into the span attribute for its signal
  (an existing base attribute participates in the max); the span gets
  ``llm.ebpf.correlation_confidence`` = max candidate confidence;
* ``decompose_retrieval`` sums dns+connect+tls into
  ``llm.ebpf.retrieval.kernel_attributed_ms`` when positive.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from ..contracts import semconv
from .match import (DEFAULT_ENRICHMENT_THRESHOLD, Decision, SignalRef, SpanRef, match)
from ..utils.timeutil import MS


@dataclass
class DebugStats:
    unmatched: int = 0
    low_confidence: int = 0
    fanout_dropped: int = 0
    unsupported_type: int = 0

    def merge(self, other: "DebugStats") -> "DebugStats":
        return DebugStats(self.unmatched + other.unmatched, self.low_confidence + other.low_confidence,
                          self.fanout_dropped + other.fanout_dropped,
                          self.unsupported_type + other.unsupported_type)

    def as_tuple(self):
        return (self.unmatched, self.low_confidence, self.fanout_dropped, self.unsupported_type)


@dataclass
class Candidate:
    signal: SignalRef
    decision: Decision


@dataclass
class EnrichmentResult:
    attributes: Dict[str, float]
    candidates: List[Candidate]
    debug: DebugStats


@dataclass
class SpanRecord:
    trace_id: str = ""
    span_id: str = ""
    service: str = ""
    node: str = ""
    pod: str = ""
    pid: int = 0
    conn_tuple: str = ""
    timestamp: int = 0
    attributes: Dict[str, float] = field(default_factory=dict)

    def ref(self) -> SpanRef:
        return SpanRef(self.trace_id, self.service, self.node, self.pod, self.pid,
                       self.conn_tuple, self.timestamp)


@dataclass
class ProcessedBatch:
    spans: List[SpanRecord]
    debug: DebugStats


@dataclass
class Correlator:
    window_ms: int = 2000
    enrichment_threshold: float = DEFAULT_ENRICHMENT_THRESHOLD
    max_join_fanout: int = 3

    def enrich_attributes(self, base: Optional[Dict[str, float]], span: SpanRef,
                          signals: Sequence[SignalRef]) -> EnrichmentResult:
        base = {} if base is None else base
        window_ns = self.window_ms * MS
        threshold = self.enrichment_threshold if self.enrichment_threshold > 0 else DEFAULT_ENRICHMENT_THRESHOLD
        fanout = self.max_join_fanout if self.max_join_fanout > 0 else 3

        debug = DebugStats()
        cands: List[Candidate] = []
        for sig in signals:
            _, supported = semconv.signal_attr_key(sig.signal)
            if not supported:
                debug.unsupported_type += 1
                continue
            dec = match(span, sig, window_ns)
            if not dec.matched:
                debug.unmatched += 1
                continue
            if dec.confidence < threshold:
                debug.low_confidence += 1
                continue
            cands.append(Candidate(sig, dec))

        # Stable sort: confidence desc, then |dt| asc; ties keep input order.
        cands.sort(key=lambda c: (-c.decision.confidence, abs(span.timestamp - c.signal.timestamp)))
        if len(cands) > fanout:
            debug.fanout_dropped = len(cands) - fanout
            cands = cands[:fanout]

        out = dict(base)
        max_conf = 0.0
        for c in cands:
            attr, _ = semconv.signal_attr_key(c.signal.signal)
            if attr not in out or c.signal.value > out[attr]:
                out[attr] = c.signal.value
            if c.decision.confidence > max_conf:
                max_conf = c.decision.confidence
        if max_conf > 0:
            out[semconv.ATTR_CORRELATION_CONF] = max_conf
        return EnrichmentResult(out, cands, debug)

    def enrich_dns_attributes(self, base: Optional[Dict[str, float]], span: SpanRef,
                              signal: SignalRef):
        res = self.enrich_attributes(base, span, [signal])
        if not res.candidates:
            return (res.attributes or {}), Decision()
        return res.attributes, res.candidates[0].decision

    def process_batch(self, spans: Sequence[SpanRecord], signals: Sequence[SignalRef]) -> ProcessedBatch:
        out: List[SpanRecord] = []
        debug = DebugStats()
        for item in spans:
            res = self.enrich_attributes(item.attributes, item.ref(), signals)
            decompose_retrieval(res.attributes)
            rec = SpanRecord(item.trace_id, item.span_id, item.service, item.node, item.pod, item.pid,
                             item.conn_tuple, item.timestamp, res.attributes)
            out.append(rec)
            debug = debug.merge(res.debug)
        return ProcessedBatch(out, debug)


def decompose_retrieval(attrs: Dict[str, float]) -> float:
    total = 0.0
    for key in semconv.RETRIEVAL_COMPONENTS:
        if key in attrs:
            total += attrs[key]
    if total > 0:
        attrs[semconv.ATTR_RETRIEVAL_KERNEL_MS] = total
    return total

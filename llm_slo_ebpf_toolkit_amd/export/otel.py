"""OTLP/HTTP JSON logs exporters for SLO events and probe events.

Payload shape and attribute names follow REF pkg/otel/slo_event_exporter.go:79-203 and
probe_event_exporter.go:79-160 (resourceLogs -> scopeLogs -> logRecords, service.name
resource attribute, severity breach/error -> ERROR, warning -> WARN, else INFO,
doubleValue for numeric attributes, ``label.<k>`` for SLO labels, conn-tuple attrs as
net.*). REF POSTs one request per event from the agent (cmd/agent/main.go:103-127);
here exporters batch (size- and age-bounded) and the agent flushes per window.
"""

from __future__ import annotations

import json
import threading
import time
import urllib.error
import urllib.request
from typing import Any, Dict, List, Optional, Sequence

from ..contracts.types import ProbeEventV1, SLOEvent


def _s(key: str, value: str) -> Dict[str, Any]:
    return {"key": key, "value": {"stringValue": value}}


def _d(key: str, value: float) -> Dict[str, Any]:
    return {"key": key, "value": {"doubleValue": float(value)}}


def severity_from_status(status: str) -> str:
    if status in ("breach", "error"):
        return "ERROR"
    if status == "warning":
        return "WARN"
    return "INFO"


def slo_log_record(ev: SLOEvent, now_ns: Optional[int] = None) -> Dict[str, Any]:
    now = str(now_ns if now_ns is not None else time.time_ns())
    ts = str(ev.timestamp) if ev.timestamp else now
    attrs = [_s("event.id", ev.event_id), _s("cluster", ev.cluster), _s("namespace", ev.namespace),
             _s("workload", ev.workload), _s("service", ev.service), _s("request.id", ev.request_id),
             _s("trace.id", ev.trace_id), _s("sli.name", ev.sli_name), _d("sli.value", ev.sli_value),
             _s("sli.unit", ev.unit), _s("sli.status", ev.status)]
    attrs += [_s("label." + k, v) for k, v in ev.labels.items()]
    return {"timeUnixNano": ts, "observedTimeUnixNano": now, "severityText": severity_from_status(ev.status),
            "body": {"stringValue": f"sli={ev.sli_name} value={ev.sli_value:.6f} status={ev.status} service={ev.service}"},
            "attributes": attrs}


def probe_log_record(ev: ProbeEventV1, now_ns: Optional[int] = None) -> Dict[str, Any]:
    now = str(now_ns if now_ns is not None else time.time_ns())
    ts = str(ev.ts_unix_nano) if ev.ts_unix_nano > 0 else now
    attrs = [_s("signal", ev.signal), _s("node", ev.node), _s("namespace", ev.namespace), _s("pod", ev.pod),
             _s("container", ev.container), _d("pid", ev.pid), _d("tid", ev.tid), _d("value", ev.value),
             _s("unit", ev.unit), _s("status", ev.status)]
    if ev.trace_id:
        attrs.append(_s("trace.id", ev.trace_id))
    if ev.span_id:
        attrs.append(_s("span.id", ev.span_id))
    if ev.conn_tuple is not None:
        c = ev.conn_tuple
        attrs += [_s("net.src.ip", c.src_ip), _s("net.dst.ip", c.dst_ip), _d("net.src.port", c.src_port),
                  _d("net.dst.port", c.dst_port), _s("net.transport", c.protocol)]
    if ev.errno is not None:
        attrs.append(_d("errno", ev.errno))
    if ev.confidence is not None:
        attrs.append(_d("correlation.confidence", ev.confidence))
    if ev.gpu_id is not None:
        attrs.append(_d("gpu.id", ev.gpu_id))
    return {"timeUnixNano": ts, "observedTimeUnixNano": now, "severityText": severity_from_status(ev.status),
            "body": {"stringValue": f"signal={ev.signal} value={ev.value:.6f} status={ev.status} pod={ev.pod}"},
            "attributes": attrs}


def logs_payload(service_name: str, scope_name: str, records: List[Dict[str, Any]]) -> Dict[str, Any]:
    return {"resourceLogs": [{"resource": {"attributes": [_s("service.name", service_name)]},
                              "scopeLogs": [{"scope": {"name": scope_name}, "logRecords": records}]}]}


class OTLPLogExporter:
    """Batched OTLP/HTTP JSON exporter. ``export_*_batch`` posts immediately (REF
    ExportBatch); ``add_*`` buffers and posts when ``max_batch`` or ``max_age_s`` is hit."""

    def __init__(self, endpoint: str, service_name: str = "llm-slo-ebpf-toolkit",
                 scope_name: str = "llm-slo-ebpf-toolkit/agent", timeout_s: float = 5.0, max_batch: int = 512,
                 max_age_s: float = 1.0):
        self.endpoint = endpoint
        self.service_name = service_name or "llm-slo-ebpf-toolkit"
        self.scope_name = scope_name or "llm-slo-ebpf-toolkit/collector"
        self.timeout_s = timeout_s if timeout_s > 0 else 5.0
        self.max_batch = max_batch
        self.max_age_s = max_age_s
        self._buf: List[Dict[str, Any]] = []
        self._oldest = 0.0
        self._lock = threading.Lock()
        self.posts = 0
        self.errors = 0

    def _post(self, records: List[Dict[str, Any]]) -> None:
        if not records:
            return
        if not self.endpoint:
            raise ValueError("otlp endpoint is required")
        body = json.dumps(logs_payload(self.service_name, self.scope_name, records)).encode()
        req = urllib.request.Request(self.endpoint, data=body, method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout_s) as resp:
                status = resp.status
        except urllib.error.HTTPError as exc:
            status = exc.code
        except (urllib.error.URLError, OSError) as exc:
            self.errors += 1
            raise ConnectionError(f"send otlp payload: {exc}") from exc
        self.posts += 1
        if status < 200 or status >= 300:
            self.errors += 1
            raise ConnectionError(f"otlp endpoint returned status {status}")

    def export_slo_batch(self, events: Sequence[SLOEvent]) -> None:
        self._post([slo_log_record(e) for e in events])

    def export_probe_batch(self, events: Sequence[ProbeEventV1]) -> None:
        self._post([probe_log_record(e) for e in events])

    def _add(self, rec: Dict[str, Any]) -> None:
        flush = None
        with self._lock:
            if not self._buf:
                self._oldest = time.monotonic()
            self._buf.append(rec)
            if len(self._buf) >= self.max_batch or time.monotonic() - self._oldest >= self.max_age_s:
                flush, self._buf = self._buf, []
        if flush:
            self._post(flush)

    def add_slo(self, ev: SLOEvent) -> None:
        self._add(slo_log_record(ev))

    def add_probe(self, ev: ProbeEventV1) -> None:
        self._add(probe_log_record(ev))

    def flush(self) -> None:
        with self._lock:
            buf, self._buf = self._buf, []
        self._post(buf)

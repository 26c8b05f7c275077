"""Incident webhooks: generic JSON, PagerDuty Events v2, Opsgenie; HMAC-SHA256 signing.

REF pkg/webhook/exporter.go:18-140, pagerduty.go:29-61, opsgenie.go:24-58:
``X-Webhook-Signature: sha256=<hex>`` over the exact body, up to ``max_retry`` (3)
attempts with 1 s, 2 s backoff, 5xx retried, 4xx not retried; PagerDuty severity
critical if confidence >= 0.8; Opsgenie priority P3 -> P2 (conf >= 0.8) -> P1 (burn >= 3).
"""

from __future__ import annotations

import hashlib
import hmac
import json
import time
import urllib.error
import urllib.request
from typing import Callable, Optional, Tuple

from ..contracts.types import IncidentAttribution
from ..utils.timeutil import SECOND

FORMAT_GENERIC = "generic"
FORMAT_PAGERDUTY = "pagerduty"
FORMAT_OPSGENIE = "opsgenie"
FORMATS = (FORMAT_GENERIC, FORMAT_PAGERDUTY, FORMAT_OPSGENIE)


class NonRetryableError(RuntimeError):
    pass


def compute_hmac(payload: bytes, secret: str) -> str:
    return "sha256=" + hmac.new(secret.encode(), payload, hashlib.sha256).hexdigest()


def verify_hmac(payload: bytes, secret: str, signature: str) -> bool:
    return hmac.compare_digest(compute_hmac(payload, secret).encode(), signature.encode())


def _go_v(v) -> str:
    """Go %v formatting of an evidence value (floats without trailing .0 noise)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return repr(v) if not v.is_integer() else str(int(v))
    return str(v)


def _evidence_str(attr: IncidentAttribution) -> str:
    return "; ".join(f"{e.signal}={_go_v(e.value)}" for e in attr.evidence)


def pagerduty_payload(attr: IncidentAttribution) -> bytes:
    import time as _t

    severity = "critical" if attr.confidence >= 0.8 else "warning"
    secs, ns = divmod(attr.timestamp, SECOND)
    ts = _t.strftime("%Y-%m-%dT%H:%M:%S", _t.gmtime(secs)) + f".{ns // 1_000_000:03d}+0000"
    body = {"routing_key": "", "event_action": "trigger", "payload": {
        "summary": f"[{attr.service}] {attr.predicted_fault_domain} fault detected (confidence={attr.confidence:.2f})",
        "source": f"{attr.cluster}/{attr.service}", "severity": severity, "timestamp": ts,
        "component": attr.service, "group": attr.cluster,
        "custom_details": {"incident_id": attr.incident_id, "fault_domain": attr.predicted_fault_domain,
                           "confidence": f"{attr.confidence:.4f}", "evidence": _evidence_str(attr),
                           "burn_rate": f"{attr.slo_impact.burn_rate:.2f}"}}}
    return json.dumps(body).encode()


def opsgenie_payload(attr: IncidentAttribution) -> bytes:
    priority = "P3"
    if attr.confidence >= 0.8:
        priority = "P2"
    if attr.slo_impact.burn_rate >= 3.0:
        priority = "P1"
    body = {"message": f"[{attr.service}] {attr.predicted_fault_domain} fault detected", "alias": attr.incident_id,
            "description": (f"Fault domain: {attr.predicted_fault_domain}\nConfidence: {attr.confidence:.4f}\n"
                            f"Burn rate: {attr.slo_impact.burn_rate:.2f}\nEvidence: {_evidence_str(attr)}"),
            "priority": priority, "source": "llm-slo-ebpf-toolkit",
            "tags": ["llm-slo", attr.predicted_fault_domain, attr.cluster],
            "details": {"incident_id": attr.incident_id, "cluster": attr.cluster, "service": attr.service,
                        "fault_domain": attr.predicted_fault_domain, "confidence": f"{attr.confidence:.4f}",
                        "burn_rate": f"{attr.slo_impact.burn_rate:.2f}"},
            "entity": f"{attr.cluster}/{attr.service}"}
    return json.dumps(body).encode()


def parse_format(raw: str) -> str:
    f = (raw or "").strip().lower()
    if f in ("", FORMAT_GENERIC):
        return FORMAT_GENERIC
    if f in FORMATS:
        return f
    raise ValueError(f'unsupported format "{raw}"')


class WebhookExporter:
    def __init__(self, url: str, secret: str = "", fmt: str = FORMAT_GENERIC, timeout_ms: int = 5000,
                 max_retry: int = 3, sleep: Callable[[float], None] = time.sleep):
        self.url = url
        self.secret = secret
        self.format = fmt or FORMAT_GENERIC
        self.timeout_s = (timeout_ms if timeout_ms > 0 else 5000) / 1000.0
        self.max_retry = max_retry
        self._sleep = sleep

    def build_payload(self, attr: IncidentAttribution) -> Tuple[bytes, str]:
        if self.format == FORMAT_PAGERDUTY:
            return pagerduty_payload(attr), "application/json"
        if self.format == FORMAT_OPSGENIE:
            return opsgenie_payload(attr), "application/json"
        return json.dumps(attr.to_dict()).encode(), "application/json"

    def _post(self, payload: bytes, ctype: str) -> None:
        headers = {"Content-Type": ctype, "User-Agent": "llm-slo-ebpf-toolkit/webhook"}
        if self.secret:
            headers["X-Webhook-Signature"] = compute_hmac(payload, self.secret)
        req = urllib.request.Request(self.url, data=payload, method="POST", headers=headers)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout_s) as resp:
                resp.read()
                status = resp.status
        except urllib.error.HTTPError as exc:
            status = exc.code
        except (urllib.error.URLError, OSError) as exc:
            raise ConnectionError(f"http post: {exc}") from exc
        if status >= 500:
            raise ConnectionError(f"server error: HTTP {status}")
        if status >= 400:
            raise NonRetryableError(f"client error: HTTP {status}")

    def send(self, attr: IncidentAttribution) -> None:
        payload, ctype = self.build_payload(attr)
        last: Optional[Exception] = None
        for attempt in range(self.max_retry):
            if attempt > 0:
                self._sleep(float(1 << (attempt - 1)))
            try:
                self._post(payload, ctype)
                return
            except NonRetryableError:
                raise
            except ConnectionError as exc:
                last = exc
        raise ConnectionError(f"webhook delivery failed after {self.max_retry} attempts: {last}")


class AsyncWebhook:
    """Webhook delivery off the caller's thread: a bounded queue and one sender thread.

    REF's agent posts inside its tick (cmd/agent/main.go:567-585), so one hung endpoint -- 5 s
    timeout x 3 attempts plus 1 s + 2 s backoff (exporter.go:63-85) -- stalls the tick by ~18 s per
    attribution. The window agent's clock must not wait on a pager: ``send`` only enqueues; a full
    queue drops the attribution and calls ``on_drop`` (the agent counts it as
    ``llm_slo_agent_dropped_events_total{reason="emit"}``, as REF counts a failed delivery), and so
    does a delivery that fails after the exporter's retries."""

    def __init__(self, exporter: WebhookExporter, maxsize: int = 256,
                 on_drop: Optional[Callable[[str], None]] = None, log: Optional[Callable[[str], None]] = None):
        import queue
        import threading

        self.exporter = exporter
        self.q: "queue.Queue" = queue.Queue(maxsize=max(1, int(maxsize)))
        self.on_drop = on_drop or (lambda reason: None)
        self.log = log or (lambda msg: None)
        self.sent = self.failed = self.dropped = 0
        self._t = threading.Thread(target=self._run, name="mislo-webhook", daemon=True)
        self._t.start()

    def send(self, attr: IncidentAttribution) -> bool:
        import queue

        try:
            self.q.put_nowait(attr)
            return True
        except queue.Full:
            self.dropped += 1
            self.on_drop("queue_full")
            return False

    def _run(self) -> None:
        while True:
            attr = self.q.get()
            if attr is None:
                return
            try:
                self.exporter.send(attr)
                self.sent += 1
            except Exception as exc:  # noqa: BLE001 - a delivery failure never reaches the caller
                self.failed += 1
                self.on_drop("failed")
                self.log(f"webhook send failed: {exc}")
            finally:
                self.q.task_done()

    def pending(self) -> int:
        return self.q.unfinished_tasks

    def close(self, timeout: float = 5.0) -> None:
        """Stop after the queued deliveries (at most ``timeout`` s; the thread is a daemon)."""
        deadline = time.monotonic() + timeout
        while True:
            try:
                self.q.put(None, timeout=max(0.0, deadline - time.monotonic()))
                break
            except Exception:  # noqa: BLE001 - queue full past the deadline
                break
        self._t.join(max(0.0, deadline - time.monotonic()))

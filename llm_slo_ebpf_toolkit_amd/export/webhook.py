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

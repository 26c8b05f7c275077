"""CD gate: PromQL instant queries for TTFT p95 / error rate / burn rate vs thresholds.

REF pkg/cdgate/gate.go:15-175: violation iff actual > threshold; any query error fails
the gate (fail-open is applied by the CLI, cmd/sloctl/cdgate.go:91-95). NEW: the agent
now actually emits ``llm_slo_errors_total``, ``llm_slo_requests_total`` and
``llm_slo_burn_rate`` (REF queries them but nothing in REF produces them).
"""

from __future__ import annotations

import json
import time
import urllib.error
import urllib.parse
import urllib.request
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Protocol

from ..utils.timeutil import format_rfc3339_ns

METRIC_TTFT_P95 = "ttft_p95_ms"
METRIC_ERROR_RATE = "error_rate"
METRIC_BURN_RATE = "burn_rate"


def default_queries() -> Dict[str, str]:
    return {
        METRIC_TTFT_P95: "histogram_quantile(0.95, sum(rate(llm_slo_ttft_ms_bucket[5m])) by (le))",
        METRIC_ERROR_RATE: "sum(rate(llm_slo_errors_total[5m])) / sum(rate(llm_slo_requests_total[5m]))",
        METRIC_BURN_RATE: "llm_slo_burn_rate",
    }


@dataclass
class Thresholds:
    ttft_p95_ms: float = 800.0
    error_rate: float = 0.05
    burn_rate: float = 2.0


@dataclass
class Violation:
    metric: str
    threshold: float
    actual: float


@dataclass
class Result:
    passed: bool = True
    violations: List[Violation] = field(default_factory=list)
    timestamp: int = 0
    error: str = ""

    def to_dict(self) -> Dict[str, object]:
        out: Dict[str, object] = {"pass": self.passed,
                                  "violations": [v.__dict__ for v in self.violations] or None,
                                  "timestamp": format_rfc3339_ns(self.timestamp)}
        if self.error:
            out["error"] = self.error
        return out


class Querier(Protocol):
    def query(self, q: str) -> float: ...


class HTTPQuerier:
    def __init__(self, base_url: str, timeout_s: float = 10.0):
        self.base_url = base_url
        self.timeout_s = timeout_s

    def query(self, q: str) -> float:
        u = urllib.parse.urlsplit(self.base_url)
        url = urllib.parse.urlunsplit((u.scheme, u.netloc, "/api/v1/query", urllib.parse.urlencode({"query": q}), ""))
        try:
            with urllib.request.urlopen(url, timeout=self.timeout_s) as resp:
                body = resp.read()
                status = resp.status
        except urllib.error.HTTPError as exc:
            raise ConnectionError(f"prometheus returned HTTP {exc.code}: {exc.read().decode(errors='replace')}")
        except (urllib.error.URLError, OSError) as exc:
            raise ConnectionError(f"prometheus query: {exc}") from exc
        if status != 200:
            raise ConnectionError(f"prometheus returned HTTP {status}")
        pr = json.loads(body)
        if pr.get("status") != "success":
            raise ValueError(f"prometheus query status: {pr.get('status')}")
        res = (pr.get("data") or {}).get("result") or []
        if not res:
            raise ValueError(f"prometheus query returned no results for: {q}")
        val = res[0].get("value", [None, None])[1]
        if not isinstance(val, str):
            raise ValueError("unexpected value type in prometheus result")
        return float(val)


def evaluate_slo_gate(querier: Querier, t: Thresholds) -> Result:
    res = Result(passed=True, timestamp=time.time_ns())
    qs = default_queries()
    for metric, thr in ((METRIC_TTFT_P95, t.ttft_p95_ms), (METRIC_ERROR_RATE, t.error_rate),
                        (METRIC_BURN_RATE, t.burn_rate)):
        try:
            val = querier.query(qs[metric])
        except Exception as exc:  # noqa: BLE001 - any query failure fails the gate
            res.error = f"query {metric} failed: {exc}"
            res.passed = False
            return res
        if val > thr:
            res.passed = False
            res.violations.append(Violation(metric, thr, val))
    return res

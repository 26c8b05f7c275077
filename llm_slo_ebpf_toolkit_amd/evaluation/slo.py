"""SLO math: TTFT, tokens/s, retrieval breakdown and percentile aggregation.

REF pkg/slo/calculator.go:11-157 (linear-interpolated quantiles on the sorted copy,
negative values clamped to 0 before aggregation, TTFT truncated to whole ms like Go's
``Duration.Milliseconds``).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Sequence

from ..utils.timeutil import MS, SECOND


@dataclass
class Timing:
    request_start: int = 0
    first_token_at: int = 0
    last_token_at: int = 0
    token_count: int = 0


@dataclass
class RetrievalBreakdown:
    vectordb_ms: float = 0.0
    network_ms: float = 0.0
    dns_ms: float = 0.0


@dataclass
class Snapshot:
    ttft_ms: float
    tokens_per_s: float
    retrieval: RetrievalBreakdown


@dataclass
class Percentiles:
    ttft_p50: float = 0.0
    ttft_p95: float = 0.0
    ttft_p99: float = 0.0
    tokens_per_s_p50: float = 0.0
    tokens_per_s_p95: float = 0.0
    retrieval_p95_ms: float = 0.0


def ttft_ms(request_start: int, first_token_at: int) -> float:
    if request_start == 0 or first_token_at == 0:
        raise ValueError("requestStart and firstTokenAt are required")
    if first_token_at < request_start:
        raise ValueError("firstTokenAt must be after requestStart")
    return float((first_token_at - request_start) // MS)


def tokens_per_second(first_token_at: int, last_token_at: int, token_count: int) -> float:
    if first_token_at == 0 or last_token_at == 0:
        raise ValueError("firstTokenAt and lastTokenAt are required")
    if token_count < 1:
        raise ValueError("tokenCount must be >= 1")
    if last_token_at < first_token_at:
        raise ValueError("lastTokenAt must be after firstTokenAt")
    window = (last_token_at - first_token_at) / SECOND
    if window == 0:
        return float(token_count)
    return token_count / window


def calculate(t: Timing, retrieval: RetrievalBreakdown) -> Snapshot:
    return Snapshot(ttft_ms(t.request_start, t.first_token_at),
                    tokens_per_second(t.first_token_at, t.last_token_at, t.token_count), retrieval)


def _nn(v: float) -> float:
    return v if v > 0 else 0.0


def total_retrieval_ms(b: RetrievalBreakdown) -> float:
    return _nn(b.vectordb_ms) + _nn(b.network_ms) + _nn(b.dns_ms)


def quantile(values: Sequence[float], q: float) -> float:
    """Linear interpolation between closest ranks (REF calculator.go:121-149, gate.go:737-760)."""
    if not values:
        return 0.0
    q = min(max(q, 0.0), 1.0)
    s = sorted(values)
    if len(s) == 1:
        return s[0]
    pos = q * (len(s) - 1)
    lo, hi = math.floor(pos), math.ceil(pos)
    if lo == hi:
        return s[lo]
    frac = pos - lo
    return s[lo] * (1 - frac) + s[hi] * frac


def aggregate(items: Sequence[Snapshot]) -> Percentiles:
    if not items:
        return Percentiles()
    ttft = [_nn(i.ttft_ms) for i in items]
    tps = [_nn(i.tokens_per_s) for i in items]
    ret = [total_retrieval_ms(i.retrieval) for i in items]
    return Percentiles(quantile(ttft, .5), quantile(ttft, .95), quantile(ttft, .99), quantile(tps, .5),
                       quantile(tps, .95), quantile(ret, .95))


def mean(values: Sequence[float]) -> float:
    return sum(values) / len(values) if values else 0.0


def stddev(values: Sequence[float]) -> float:
    if len(values) <= 1:
        return 0.0
    m = mean(values)
    return math.sqrt(sum((v - m) ** 2 for v in values) / (len(values) - 1))


def cv_pct(values: Sequence[float]) -> float:
    m = mean(values)
    return 0.0 if m == 0 else stddev(values) / m * 100


def histogram_quantile(q: float, edges: Sequence[float], cumulative_counts: Sequence[float]) -> float:
    """Prometheus ``histogram_quantile`` over cumulative ``le`` buckets (last edge +Inf).
    Used to read p95s out of the GPU-built histograms exactly as PromQL would."""
    if not cumulative_counts or cumulative_counts[-1] <= 0:
        return float("nan")
    total = cumulative_counts[-1]
    rank = q * total
    prev_edge, prev_cnt = 0.0, 0.0
    for e, c in zip(edges, cumulative_counts):
        if c >= rank:
            if math.isinf(e):
                return prev_edge
            if c == prev_cnt:
                return e
            return prev_edge + (e - prev_edge) * (rank - prev_cnt) / (c - prev_cnt)
        prev_edge, prev_cnt = e, c
    return prev_edge

"""SLO math: TTFT, tokens/s, retrieval breakdown and percentile aggregation.

REF pkg/slo/calculator.go:11-157 (linear-interpolated quantiles on the sorted copy,
negative values clamped to 0 before aggregation, TTFT truncated to whole ms like Go's
``Duration.Milliseconds``).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

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


class BurnRateForecaster:
    """Forecasts an SLO's burn rate over the next ``horizon`` windows and scores its forecasts.

    burn = (breaching requests / requests) / (1 - target), the multiwindow burn-rate of SRE
    alerting. ``alert(key)`` is the burn over the last ``short`` windows (the short alerting
    window). The forecast at window t is the burn over the shortest trailing run of windows
    holding at least ``min_requests`` requests (the current rate, on enough requests to be
    stable: an ongoing fault is expected to persist); it is scored once ``horizon`` more
    windows have been seen, against the burn realised over them. ``error()`` is the mean
    absolute error of the scored forecasts relative to the realised burn (REF reports this
    metric as the hard-coded 0.07, pkg/benchmark/harness.go:103; here it is measured). Keyed
    per SLO owner (service / incident group)."""

    def __init__(self, target: float = 0.99, horizon: int = 300, short: int = 30, floor: float = 0.05,
                 min_requests: float = 1000.0):
        if not 0.0 < target < 1.0 or horizon < 1 or short < 1:
            raise ValueError("target in (0, 1), horizon and short >= 1")
        self.budget = 1.0 - target
        self.horizon, self.short, self.floor = int(horizon), int(short), float(floor)
        self.min_requests = float(min_requests)
        self._hist: dict = {}     # key -> list of (n, breach) per window
        self._pending: dict = {}  # key -> list of (window index, forecast)
        self.scored: List[float] = []

    def burn(self, n: float, breach: float) -> float:
        return (breach / n) / self.budget if n > 0 else 0.0

    def observe(self, key, n: float, breach: float, forecast: bool = True) -> float:
        """Adds one window's request and breach counts; returns the forecast made at it (and
        keeps it for scoring unless ``forecast`` is False)."""
        h = self._hist.setdefault(key, [])
        h.append((float(n), float(breach)))
        t = len(h) - 1
        pend = self._pending.setdefault(key, [])
        while pend and pend[0][0] + self.horizon <= t:  # matured: windows (t0, t0 + horizon]
            t0, f = pend.pop(0)
            seg = h[t0 + 1:t0 + 1 + self.horizon]
            real = self.burn(sum(x[0] for x in seg), sum(x[1] for x in seg))
            self.scored.append(abs(f - real) / max(real, self.floor))
        n_acc = b_acc = 0.0
        for x in reversed(h[-self.short:]):
            n_acc += x[0]
            b_acc += x[1]
            if n_acc >= self.min_requests:
                break
        f = self.burn(n_acc, b_acc)
        if forecast:
            pend.append((t, f))
        # keep what the short window and the oldest pending forecast still need
        keep = max(self.short, t - pend[0][0] + 1 if pend else 0)
        if len(h) > 4 * keep + 64:
            drop = len(h) - keep
            del h[:drop]
            self._pending[key] = [(t0 - drop, f0) for t0, f0 in pend]
        return f

    def current(self, key, windows: int = 3, min_requests: float = 20.0) -> float:
        """The burn now: over the shortest trailing run of at most ``windows`` windows holding at
        least ``min_requests`` requests (all of them if fewer). The agent's emission gate -- a
        fast-burn alert: the forecast (``observe``) keeps a fault's breaches for up to ``short``
        windows after the service recovered, which would page "unknown" through the recovery."""
        n_acc = b_acc = 0.0
        for x in reversed(self._hist.get(key, [])[-int(windows):]):
            n_acc += x[0]
            b_acc += x[1]
            if n_acc >= min_requests:
                break
        return self.burn(n_acc, b_acc)

    def alert(self, key) -> float:
        recent = self._hist.get(key, [])[-self.short:]
        return self.burn(sum(x[0] for x in recent), sum(x[1] for x in recent))

    def error(self) -> Optional[float]:
        return float(sum(self.scored) / len(self.scored)) if self.scored else None

    def state(self) -> dict:
        """JSON-able state (agent checkpoint): per-key window history and pending forecasts."""
        return {"hist": {str(k): v for k, v in self._hist.items()},
                "pending": {str(k): v for k, v in self._pending.items()},
                "scored": self.scored[-10000:]}

    def restore(self, st: dict) -> None:
        self._hist = {k: [tuple(x) for x in v] for k, v in (st.get("hist") or {}).items()}
        self._pending = {k: [tuple(x) for x in v] for k, v in (st.get("pending") or {}).items()}
        self.scored = [float(x) for x in st.get("scored") or []]


def simulate_burn_prediction_error(burn_rates: Sequence[float], target: float = 0.99, horizon: int = 300,
                                   short: int = 30, requests_per_window: float = 50.0, seed: int = 42) -> float:
    """Burn-rate forecast error over synthetic fault episodes, one per incident sample.

    Each episode is a request stream in 1 s windows: a baseline breach rate, a fault onset that
    ramps over 5-30 windows to the sample's nominal burn rate and then persists, with Poisson
    request counts and binomial breaches. From the window its short-window alert burn first
    exceeds 1 (detection) on, the forecaster (``BurnRateForecaster``) forecasts at every window
    for ``horizon`` windows, as an agent re-forecasting each window does; each forecast is scored
    against the burn realised over the ``horizon`` windows after it."""
    import numpy as np

    rng = np.random.default_rng(seed)
    budget = 1.0 - target
    errs = []
    for i, b in enumerate(burn_rates):
        b = float(b) if b and b > 0 else 2.0
        fc = BurnRateForecaster(target, horizon, short)
        p_base, p_fault = 0.1 * budget, min(1.0, b * budget)
        ramp = int(rng.integers(5, 31))
        lead = short + int(rng.integers(0, 60))
        T = lead + ramp + 4 * horizon
        detected = None
        for t in range(T):
            x = min(1.0, max(0.0, (t - lead) / ramp))
            p = p_base + (p_fault - p_base) * x
            n = int(rng.poisson(requests_per_window))
            br = int(rng.binomial(n, p)) if n else 0
            if detected is None and t >= lead and fc.alert(i) > 1.0:
                detected = t
            fc.observe(i, n, br, forecast=detected is not None and t < detected + horizon)
            if detected is not None and t >= detected + 2 * horizon:
                break
        e = fc.error()
        if e is not None:
            errs.append(e)
    return float(np.mean(errs)) if errs else float("nan")

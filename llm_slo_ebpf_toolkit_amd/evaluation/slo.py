"""SLO math: TTFT, tokens/s, retrieval breakdown and percentile aggregation.

REF pkg/slo/calculator.go:11-157 (linear-interpolated quantiles on the sorted copy,
negative values clamped to 0 before aggregation, TTFT truncated to whole ms like Go's
``Duration.Milliseconds``).
"""

from __future__ import annotations

import math
from collections import deque
from dataclasses import dataclass
from typing import Deque, List, Optional, Sequence, Tuple

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


def _binom_ll(n: float, b: float) -> float:
    """Maximised binomial log-likelihood of b breaches in n requests (rate b / n)."""
    if n <= 0 or b <= 0 or b >= n:
        return 0.0
    p = b / n
    return b * math.log(p) + (n - b) * math.log1p(-p)


def _binom_ll_np(n, b):
    """``_binom_ll`` over arrays (the logs only where 0 < b < n: no floating-point state to switch)."""
    import numpy as np

    ok = (b > 0) & (b < n)
    out = np.zeros(np.shape(n), dtype=np.float64)
    if ok.any():
        nn, bb = n[ok], b[ok]
        p = bb / nn
        out[ok] = bb * np.log(p) + (nn - bb) * np.log1p(-p)
    return out


class BurnRateForecaster:
    """Forecasts an SLO's burn rate over the next ``horizon`` windows and scores its forecasts.

    burn = (breaching requests / requests) / (1 - target), the multiwindow burn-rate of SRE
    alerting. ``alert(key)`` is the burn over the last ``short`` windows (the short alerting
    window). Two forecasts (``method``):

    * ``"segment"`` (default): the burn over the latest **homogeneous segment** of the window
      history, i.e. the windows since the breach rate last changed. Change points come from
      binary segmentation with the binomial likelihood ratio: a split of the segment into an
      older and a newer run is accepted when its log-likelihood ratio exceeds ``change_llr``.
      The search covers at most ``long`` windows, and the newest run always holds at least
      ``segment_min_requests`` requests. A persistent fault's rate is thus estimated from every
      window since its onset rather than the last ~20. Those 20 windows' sampling noise
      (~1/sqrt(breaches in the run)) is what dominates a persistence forecast's error. The
      search runs only when the newest run departs from the current segment (binomial z-test,
      ``|z| >= 2``), so a steady key costs O(1) per window.
    * ``"persistence"``: the burn over the shortest trailing run of windows holding at least
      ``min_requests`` requests (the round-5 forecaster).

    Each forecast is scored once ``horizon`` more windows have been seen, against the burn
    realised over them. ``error()`` is the mean absolute error of the scored forecasts relative
    to the realised burn. REF reports this metric as the hard-coded 0.07
    (pkg/benchmark/harness.go:103); here it is measured. Keyed per SLO owner (service /
    incident group).

    On the benchgen episodes the segment forecast is at the data's floor: an estimator told where
    each fault's plateau starts scores no better (tools/burn_floor.py, profiles/r6_burn/)."""

    def __init__(self, target: float = 0.99, horizon: int = 300, short: int = 30, floor: float = 0.05,
                 min_requests: float = 1000.0, method: str = "segment", change_llr: float = 8.0,
                 long: Optional[int] = None, segment_min_requests: Optional[float] = None):
        if not 0.0 < target < 1.0 or horizon < 1 or short < 1:
            raise ValueError("target in (0, 1), horizon and short >= 1")
        if method not in ("segment", "persistence"):
            raise ValueError("method is 'segment' or 'persistence'")
        self.budget = 1.0 - target
        self.horizon, self.short, self.floor = int(horizon), int(short), float(floor)
        self.min_requests = float(min_requests)
        self.method, self.change_llr = method, float(change_llr)
        self.long = int(long) if long is not None else 2 * int(horizon)
        # the newest run of a segment holds at least this many requests: half the persistence
        # run, so a change is followed sooner (the best of 250 / 500 / 1000 on the episodes)
        self.seg_min = float(segment_min_requests) if segment_min_requests is not None else 0.5 * self.min_requests
        # per key: prefix sums of requests / breaches over the kept windows ([0] = 0; window i of
        # the kept history is cum[i + 1] - cum[i]): every trailing or forecast-horizon sum is one
        # subtraction (the agent observes every incident group every window)
        self._cum: dict = {}      # key -> [cum_n list, cum_b list]
        self._seg: dict = {}      # key -> start of the current segment (index into the kept history)
        self._pending: dict = {}  # key -> deque of (window index, forecast)
        self.scored: Deque[float] = deque(maxlen=10000)  # the latest scored errors (checkpoint state)
        self._err_sum, self._err_n = 0.0, 0                 # every scored error (error())

    def burn(self, n: float, breach: float) -> float:
        return (breach / n) / self.budget if n > 0 else 0.0

    def _trailing(self, cn: List[float], cb: List[float], windows: int, min_requests: float) -> float:
        """Burn over the shortest trailing run of at most ``windows`` windows holding at least
        ``min_requests`` requests (all of them if fewer)."""
        t = len(cn) - 1  # windows kept
        jmax = min(int(windows), t)
        if jmax <= 0:
            return 0.0
        if cn[t] - cn[t - jmax] < min_requests:
            j = jmax
        else:  # the smallest j with the last j windows' requests >= min_requests
            lo, hi = 1, jmax
            while lo < hi:
                mid = (lo + hi) >> 1
                if cn[t] - cn[t - mid] >= min_requests:
                    hi = mid
                else:
                    lo = mid + 1
            j = lo
        return self.burn(cn[t] - cn[t - j], cb[t] - cb[t - j])

    def observe(self, key, n: float, breach: float, forecast: bool = True, late: float = 0.0) -> float:
        """Adds one window's request and breach counts; returns the forecast made at it (and
        keeps it for scoring unless ``forecast`` is False). ``late``: breaching requests reported
        in this window whose SLO deadline passed in an earlier one (collector/otlp.py SPAN_LATE);
        they are credited to the previous window, where the breach happened."""
        c = self._cum.get(key)
        if c is None:
            c = self._cum[key] = [[0.0], [0.0]]
        cn, cb = c
        if late:
            if len(cn) > 1:
                cn[-1] += float(late)
                cb[-1] += float(late)
            else:
                n, breach = float(n) + float(late), float(breach) + float(late)
        cn.append(cn[-1] + float(n))
        cb.append(cb[-1] + float(breach))
        t = len(cn) - 2  # this window's index in the kept history
        pend = self._pending.get(key)
        if pend is None:
            pend = self._pending[key] = deque()
        while pend and pend[0][0] + self.horizon <= t:  # matured: windows (t0, t0 + horizon]
            t0, f = pend.popleft()
            a, b = t0 + 1, t0 + 1 + self.horizon
            real = self.burn(cn[b] - cn[a], cb[b] - cb[a])
            err = abs(f - real) / max(real, self.floor)
            self.scored.append(err)
            self._err_sum += err
            self._err_n += 1
        if self.method == "segment":
            f = self._segment(key, cn, cb)
        else:
            f = self._trailing(cn, cb, self.short, self.min_requests)
        if forecast:
            pend.append((t, f))
        # keep what the short window, the segment search and the oldest pending forecast need
        keep = max(self.short, self.long if self.method == "segment" else 0, t - pend[0][0] + 1 if pend else 0)
        if len(cn) - 1 > 2 * keep + 64:
            drop = len(cn) - 1 - keep
            base_n, base_b = cn[drop], cb[drop]
            c[0] = [x - base_n for x in cn[drop:]]
            c[1] = [x - base_b for x in cb[drop:]]
            self._pending[key] = deque((t0 - drop, f0) for t0, f0 in pend)
            if key in self._seg:
                self._seg[key] = max(0, self._seg[key] - drop)
        return f

    def _segment(self, key, cn: List[float], cb: List[float]) -> float:
        """Burn over the current homogeneous segment (class docstring)."""
        t = len(cn) - 1
        if t <= 0:
            return 0.0
        jmax = min(self.short, t)
        j = jmax  # the newest run: the shortest trailing run holding seg_min requests
        if cn[t] - cn[t - jmax] >= self.seg_min:
            lo_j, hi_j = 1, jmax
            while lo_j < hi_j:
                mid = (lo_j + hi_j) >> 1
                if cn[t] - cn[t - mid] >= self.seg_min:
                    hi_j = mid
                else:
                    lo_j = mid + 1
            j = lo_j
        lo = max(self._seg.get(key, 0), t - self.long, 0)
        if t - lo > j:  # is the newest run still at the segment's rate?
            n_new, b_new = cn[t] - cn[t - j], cb[t] - cb[t - j]
            n_old, b_old = cn[t - j] - cn[lo], cb[t - j] - cb[lo]
            n_all = n_new + n_old
            if n_new > 0 and n_old > 0:
                p = (b_new + b_old) / n_all
                p = min(max(p, 0.5 / n_all), 1.0 - 0.5 / n_all)
                z = abs(b_new / n_new - b_old / n_old) / math.sqrt(p * (1.0 - p) * (1.0 / n_new + 1.0 / n_old))
                if z >= 2.0:
                    lo = self._split(cn, cb, max(t - self.long, 0), t, j)
        else:
            lo = max(min(lo, t - j), 0)
        self._seg[key] = lo
        return self.burn(cn[t] - cn[lo], cb[t] - cb[lo])

    def _split(self, cn: List[float], cb: List[float], lo: int, t: int, j: int) -> int:
        """Binary segmentation of windows [lo, t): the start of the newest homogeneous segment
        (at least ``j`` windows long). Every candidate split of a pass at once (numpy)."""
        import numpy as np

        CN = np.asarray(cn[lo:t + 1], dtype=np.float64)
        CB = np.asarray(cb[lo:t + 1], dtype=np.float64)
        base, L, s0 = lo, t - lo, 0
        while L - s0 > j:
            n_all, b_all = CN[L] - CN[s0], CB[L] - CB[s0]
            nl, bl = CN[s0 + 1:L - j + 1] - CN[s0], CB[s0 + 1:L - j + 1] - CB[s0]
            m = len(nl)  # both sides of every split in one pass
            ll = _binom_ll_np(np.concatenate([nl, n_all - nl]), np.concatenate([bl, b_all - bl]))
            llr = ll[:m] + ll[m:] - _binom_ll(n_all, b_all)
            k = int(np.argmax(llr))
            if not llr[k] > self.change_llr:
                break
            s0 += 1 + k
        return base + s0

    def current(self, key, windows: int = 3, min_requests: float = 20.0) -> float:
        """The burn now: over the shortest trailing run of at most ``windows`` windows holding at
        least ``min_requests`` requests (all of them if fewer). The agent's emission gate -- a
        fast-burn alert: the forecast (``observe``) keeps a fault's breaches for up to ``short``
        windows after the service recovered, which would page "unknown" through the recovery."""
        c = self._cum.get(key)
        return self._trailing(c[0], c[1], windows, min_requests) if c is not None else 0.0

    def alert(self, key) -> float:
        c = self._cum.get(key)
        if c is None:
            return 0.0
        cn, cb = c
        j = min(self.short, len(cn) - 1)
        return self.burn(cn[-1] - cn[-1 - j], cb[-1] - cb[-1 - j])

    def error(self) -> Optional[float]:
        return float(self._err_sum / self._err_n) if self._err_n else None

    def history(self, key) -> List[Tuple[float, float]]:
        """The kept per-window (requests, breaches) of ``key``."""
        c = self._cum.get(key)
        if c is None:
            return []
        cn, cb = c
        return [(cn[i + 1] - cn[i], cb[i + 1] - cb[i]) for i in range(len(cn) - 1)]

    def state(self) -> dict:
        """JSON-able state (agent checkpoint): per-key window history and pending forecasts."""
        return {"hist": {str(k): self.history(k) for k in self._cum},
                "pending": {str(k): list(v) for k, v in self._pending.items()},
                "scored": list(self.scored), "err": [self._err_sum, self._err_n]}

    def restore(self, st: dict) -> None:
        self._cum = {}
        self._seg = {}
        for k, v in (st.get("hist") or {}).items():
            cn, cb = [0.0], [0.0]
            for n, b in v:
                cn.append(cn[-1] + float(n))
                cb.append(cb[-1] + float(b))
            self._cum[k] = [cn, cb]
        self._pending = {k: deque(tuple(x) for x in v) for k, v in (st.get("pending") or {}).items()}
        self.scored = deque((float(x) for x in st.get("scored") or []), maxlen=10000)
        err = st.get("err")
        if err:
            self._err_sum, self._err_n = float(err[0]), int(err[1])
        else:
            self._err_sum, self._err_n = float(sum(self.scored)), len(self.scored)


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

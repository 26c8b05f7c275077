"""Prometheus registry + text exposition + /metrics /healthz /readyz server.

The agent metric surface keeps REF's names, types and label sets (cmd/agent/main.go:
137-326): llm_slo_agent_heartbeat, _up, _cpu_overhead_pct, _event_kind,
_capability_mode, _signal_enabled, _dropped_events_total{reason},
llm_ebpf_hello_syscalls_total, llm_ebpf_dns_latency_ms (buckets 1..800),
llm_ebpf_probe_events_total{signal,status}. NEW: every signal's GPU-built histogram is
exposed as llm_ebpf_<signal>_hist with the catalogue buckets (``le`` semantics preserved:
the kernel bins by ``value <= edge`` and the exporter cumulates), plus window/engine
metrics. Histograms accept whole bucket vectors (``add_counts``) so a window's
node-wide (RCCL-reduced) histogram is merged with one call instead of one observe() per
event.
"""

from __future__ import annotations

import math
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, Iterable, List, Optional, Sequence, Tuple


def _fmt(v: float) -> str:
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if math.isnan(v):
        return "NaN"
    if float(v).is_integer() and abs(v) < 1e15:
        return str(int(v))
    return repr(float(v))


def _esc(s: str) -> str:
    return s.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _labels(names: Sequence[str], values: Sequence[str], extra: Optional[Tuple[str, str]] = None) -> str:
    pairs = [f'{n}="{_esc(v)}"' for n, v in zip(names, values)]
    if extra:
        pairs.append(f'{extra[0]}="{_esc(extra[1])}"')
    return "{" + ",".join(pairs) + "}" if pairs else ""


class _Metric:
    kind = "untyped"

    def __init__(self, name: str, help_: str, labelnames: Sequence[str] = ()):
        self.name, self.help, self.labelnames = name, help_, tuple(labelnames)
        self._lock = threading.Lock()


class Counter(_Metric):
    kind = "counter"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._v: Dict[Tuple[str, ...], float] = {}

    def inc(self, amount: float = 1.0, *labels: str) -> None:
        if amount < 0:
            raise ValueError("counters only go up")
        with self._lock:
            self._v[labels] = self._v.get(labels, 0.0) + amount

    def labels(self, *labels: str) -> "_Bound":
        return _Bound(self, labels)

    def value(self, *labels: str) -> float:
        return self._v.get(labels, 0.0)

    def samples(self) -> Iterable[str]:
        for lv, v in sorted(self._v.items()):
            yield f"{self.name}{_labels(self.labelnames, lv)} {_fmt(v)}"


class Gauge(Counter):
    kind = "gauge"

    def set(self, value: float, *labels: str) -> None:
        with self._lock:
            self._v[labels] = float(value)

    def inc(self, amount: float = 1.0, *labels: str) -> None:
        with self._lock:
            self._v[labels] = self._v.get(labels, 0.0) + amount


class _Bound:
    def __init__(self, metric, labels):
        self.m, self.l = metric, labels

    def inc(self, amount: float = 1.0):
        self.m.inc(amount, *self.l)

    def set(self, value: float):
        self.m.set(value, *self.l)

    def observe(self, value: float):
        self.m.observe(value, *self.l)


class Histogram(_Metric):
    kind = "histogram"

    def __init__(self, name: str, help_: str, buckets: Sequence[float], labelnames: Sequence[str] = ()):
        super().__init__(name, help_, labelnames)
        b = [float(x) for x in buckets if not math.isinf(x)]
        self.buckets = sorted(b) + [math.inf]
        self._c: Dict[Tuple[str, ...], List[float]] = {}
        self._sum: Dict[Tuple[str, ...], float] = {}

    def observe(self, value: float, *labels: str) -> None:
        with self._lock:
            c = self._c.setdefault(labels, [0.0] * len(self.buckets))
            for i, e in enumerate(self.buckets):
                if value <= e:
                    c[i] += 1
                    break
            self._sum[labels] = self._sum.get(labels, 0.0) + value

    def add_counts(self, counts: Sequence[float], total_sum: float = 0.0, *labels: str) -> None:
        """Merge per-bucket (non-cumulative) counts aligned with ``buckets``."""
        if len(counts) != len(self.buckets):
            raise ValueError(f"{self.name}: expected {len(self.buckets)} bucket counts, got {len(counts)}")
        with self._lock:
            c = self._c.setdefault(labels, [0.0] * len(self.buckets))
            for i, v in enumerate(counts):
                c[i] += float(v)
            self._sum[labels] = self._sum.get(labels, 0.0) + total_sum

    def labels(self, *labels: str) -> _Bound:
        return _Bound(self, labels)

    def cumulative(self, *labels: str) -> List[float]:
        c = self._c.get(labels, [0.0] * len(self.buckets))
        out, run = [], 0.0
        for v in c:
            run += v
            out.append(run)
        return out

    def samples(self) -> Iterable[str]:
        for lv in sorted(self._c):
            cum = self.cumulative(*lv)
            for e, v in zip(self.buckets, cum):
                yield f"{self.name}_bucket{_labels(self.labelnames, lv, ('le', _fmt(e)))} {_fmt(v)}"
            yield f"{self.name}_sum{_labels(self.labelnames, lv)} {_fmt(self._sum.get(lv, 0.0))}"
            yield f"{self.name}_count{_labels(self.labelnames, lv)} {_fmt(cum[-1])}"


class Registry:
    def __init__(self):
        self._m: Dict[str, _Metric] = {}
        self._lock = threading.Lock()

    def register(self, m: _Metric) -> _Metric:
        with self._lock:
            if m.name in self._m:
                raise ValueError(f"duplicate metric {m.name}")
            self._m[m.name] = m
        return m

    def counter(self, name, help_, labelnames=()):
        return self.register(Counter(name, help_, labelnames))

    def gauge(self, name, help_, labelnames=()):
        return self.register(Gauge(name, help_, labelnames))

    def histogram(self, name, help_, buckets, labelnames=()):
        return self.register(Histogram(name, help_, buckets, labelnames))

    def get(self, name: str) -> _Metric:
        return self._m[name]

    def exposition(self) -> str:
        lines: List[str] = []
        with self._lock:
            metrics = list(self._m.values())
        for m in metrics:
            lines.append(f"# HELP {m.name} {m.help}")
            lines.append(f"# TYPE {m.name} {m.kind}")
            lines.extend(m.samples())
        return "\n".join(lines) + "\n"


def parse_exposition(text: str) -> Dict[str, float]:
    """Tiny parser for tests / evidence capture: 'name{labels}' -> value."""
    out = {}
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        key, _, val = line.rpartition(" ")
        out[key] = float(val.replace("+Inf", "inf"))
    return out


class MetricsServer:
    """/metrics, /healthz ("ok"), /readyz ("ready") -- REF cmd/agent/main.go:304-326."""

    def __init__(self, registry: Registry, bind: str = ":2112", ready=lambda: True, debug=None):
        """``debug``: name -> callable returning a JSON-able object, served as /debug/<name>
        (the agent's pod-uid -> pod-id table, for fault injectors and operators)."""
        import json

        host, _, port = bind.rpartition(":")
        self.registry = registry
        self.ready = ready
        reg = registry
        is_ready = ready
        routes = dict(debug or {})

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def do_GET(self):
                if self.path.startswith("/metrics"):
                    body = reg.exposition().encode()
                    ctype = "text/plain; version=0.0.4; charset=utf-8"
                    code = 200
                elif self.path.startswith("/healthz"):
                    body, ctype, code = b"ok", "text/plain", 200
                elif self.path.startswith("/readyz"):
                    ok = is_ready()
                    body, ctype, code = (b"ready", "text/plain", 200) if ok else (b"not ready", "text/plain", 503)
                elif self.path.startswith("/debug/") and self.path[7:].split("?")[0] in routes:
                    body = json.dumps(routes[self.path[7:].split("?")[0]]()).encode()
                    ctype, code = "application/json", 200
                else:
                    body, ctype, code = b"not found", "text/plain", 404
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.httpd = ThreadingHTTPServer((host or "0.0.0.0", int(port)), H)
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def start(self) -> "MetricsServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

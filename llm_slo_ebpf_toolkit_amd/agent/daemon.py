"""Node agent: REF cmd/agent/main.go (per-tick synthetic emit loop, Prometheus surface,
overhead guard with cost-ordered shedding, per-second rate limiter, hello tracer,
stdout/jsonl/OTLP outputs, Bayes + webhook) re-built around the MI355X window engine.

Two engines share one process, one Prometheus registry and one set of outputs:

* ``synthetic`` (REF parity, ``emit_one``): every tick builds a RawSample for the
  scenario, emits the 4 SLO events and the enabled probe events (schema-validated,
  rate-limited), attributes the sample with naive Bayes when a webhook is configured, and
  evaluates the overhead guard, shedding the highest-cost signal when over budget
  (REF cmd/agent/main.go:515-604).
* ``gpu`` (``run_windows``): records from probe producers (native shared-memory rings
  fed by the BPF loader / the rocprofiler-sdk tool library, or the seeded replay
  generator) are cut into windows and pushed through ``WindowPipeline`` on this node's
  MI355X: K1 decode -> K2 LDS join -> K3 MFMA posterior (+ RCCL packet all-reduce when
  several GPUs share the node). Per window the agent folds the kernel histograms into the
  Prometheus histograms (no per-event Python work), and emits one IncidentAttribution per
  incident group whose top posterior clears ``min_confidence``, over the same outputs and
  webhook. Everything per-event stays on the device; the host does O(groups) work.
"""

from __future__ import annotations

import os
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Iterator, List, Optional, Sequence

import numpy as np

from ..collector.pipeline import SampleMeta, build_synthetic_sample, normalize_sample
from ..collector.probes import HelloEvent, HelloTracer
from ..contracts import config as toolkitcfg
from ..contracts import validator
from ..contracts.types import Evidence, FaultHypothesis, IncidentAttribution, ProbeEventV1, SLOImpact
from ..export.otel import OTLPLogExporter
from ..export.prometheus import MetricsServer
from ..export.webhook import WebhookExporter
from ..models.bayes import NaiveBayes
from ..models.sample import FaultSample
from ..safety import OverheadGuard, RateLimiter
from ..signals import catalog
from ..signals.generator import Generator
from ..signals.metadata import Metadata, ProcMetadataEnricher, StaticMetadataEnricher
from ..utils.timeutil import now_ns
from .metrics import AgentMetrics


# ---------------------------------------------------------------------------------------
# outputs
# ---------------------------------------------------------------------------------------

class OutputWriters:
    """stdout | jsonl | otlp sinks for SLO events, probe events and attributions
    (REF cmd/agent/main.go:68-135). Thread-safe; OTLP is batched instead of one POST per
    event (``otlp_batch`` records or 1 s, whichever first)."""

    def __init__(self, mode: str, path: str = "", endpoint: str = "", timeout_ms: int = 5000,
                 otlp_batch: int = 256, stream=None):
        self.mode = mode
        self._lock = threading.Lock()
        self._fh = None
        self._own = False
        self._otlp: Optional[OTLPLogExporter] = None
        if mode == "stdout":
            self._fh = stream or sys.stdout
        elif mode == "jsonl":
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._fh = open(path, "w", encoding="utf-8")
            self._own = True
        elif mode == "otlp":
            self._otlp = OTLPLogExporter(endpoint, "llm-slo-ebpf-toolkit", "llm-slo-ebpf-toolkit/agent",
                                         timeout_ms / 1000.0, max_batch=max(1, otlp_batch))
        else:
            raise ValueError(f'unsupported output mode "{mode}"')

    def _write(self, d) -> None:
        import json

        line = json.dumps(d, separators=(",", ":")) + "\n"
        with self._lock:
            self._fh.write(line)

    def emit_slo(self, ev) -> None:
        if self._otlp is not None:
            self._otlp.add_slo(ev)
        else:
            self._write(ev.to_dict())

    def emit_probe(self, ev: ProbeEventV1) -> None:
        if self._otlp is not None:
            self._otlp.add_probe(ev)
        else:
            self._write(ev.to_dict())

    def emit_attribution(self, attr: IncidentAttribution) -> None:
        if self._otlp is not None:
            return  # attributions travel via webhook / JSONL; the OTLP plane carries events
        self._write(attr.to_dict())

    def flush(self) -> None:
        if self._otlp is not None:
            self._otlp.flush()
        elif self._fh is not None:
            with self._lock:
                self._fh.flush()

    def close(self) -> None:
        try:
            self.flush()
        finally:
            if self._own and self._fh is not None:
                self._fh.close()


# ---------------------------------------------------------------------------------------
# options
# ---------------------------------------------------------------------------------------

@dataclass
class AgentOptions:
    cluster: str = "local"
    namespace: str = "default"
    workload: str = "llm-slo-agent"
    service: str = "agent"
    node: str = "unknown-node"
    pod: str = "llm-slo-agent"
    container: str = "agent"
    scenario: str = "baseline"
    count: int = 0
    interval_ms: int = 1000
    event_kind: str = "probe"
    output: str = "stdout"
    output_path: str = "artifacts/agent/events.jsonl"
    otlp_endpoint: str = "http://otel-collector.observability.svc.cluster.local:4318/v1/logs"
    otlp_timeout_ms: int = 5000
    otlp_batch: int = 256
    webhook_url: str = ""
    webhook_secret: str = ""
    webhook_format: str = "generic"
    webhook_timeout_ms: int = 5000
    capability_mode: str = "auto"
    disable_signals: List[str] = field(default_factory=list)
    disable_overhead_guard: bool = False
    config: str = os.path.join("config", "toolkit.yaml")
    enable_hello_tracer: bool = False
    hello_target_comm: List[str] = field(default_factory=lambda: ["rag-service", "llama-server"])
    enable_real_probe_metrics: bool = True
    metrics_bind: str = ":2112"
    # GPU window engine (additive)
    engine: str = "synthetic"            # synthetic | gpu
    source: str = "replay"               # replay | ring
    ring_name: str = "/mislo-agent"
    window_ms: int = 1000
    window_events: int = 1 << 20
    window_spans: int = 16384
    window_groups: int = 64
    device: int = 0
    model: str = "bayes"
    min_confidence: float = 0.5
    wire: int = 16


def choose_enabled_signals(config_signals: Sequence[str], disabled: Sequence[str],
                           supported: Sequence[str]) -> List[str]:
    """REF chooseEnabledSignals (cmd/agent/main.go:649-691)."""
    dis, sup = set(disabled), set(supported)
    if config_signals:
        sel = [s for s in config_signals if s in sup and s not in dis]
        if sel:
            return sel
    return [s for s in supported if s not in dis]


class Agent:
    def __init__(self, opts: AgentOptions, out_stream=None):
        self.o = opts
        if opts.event_kind not in ("slo", "probe", "both"):
            raise ValueError(f'invalid event-kind "{opts.event_kind}" (expected slo|probe|both)')
        if opts.interval_ms <= 0:
            raise ValueError("interval-ms must be > 0")
        self.cfg = toolkitcfg.default()
        if opts.config:
            try:
                self.cfg = toolkitcfg.load(opts.config)
            except Exception as exc:  # noqa: BLE001 - REF: log and use defaults
                print(f"config load warning ({opts.config}): {exc}; using defaults", file=sys.stderr)
        self.mode = catalog.parse_capability_mode(opts.capability_mode)
        self.supported = catalog.supported_signals_for_mode(self.mode)
        enabled = choose_enabled_signals(self.cfg.signal_set, opts.disable_signals, self.supported)
        base = Metadata(node=opts.node, namespace=opts.namespace, pod=opts.pod, container=opts.container,
                        service=opts.service, workload=opts.workload, pid=os.getpid(), tid=os.getpid())
        self.enricher = ProcMetadataEnricher(StaticMetadataEnricher(base))
        self.generator = Generator(self.mode, enabled, self.enricher)
        self.writers = OutputWriters(opts.output, opts.output_path, opts.otlp_endpoint, opts.otlp_timeout_ms,
                                     opts.otlp_batch, out_stream)
        wh_url, wh_secret, wh_fmt, wh_to = opts.webhook_url, opts.webhook_secret, opts.webhook_format, \
            opts.webhook_timeout_ms
        if not wh_url and self.cfg.webhook.enabled and self.cfg.webhook.url:
            wh_url, wh_secret = self.cfg.webhook.url, self.cfg.webhook.secret
            wh_fmt = self.cfg.webhook.format or wh_fmt
            wh_to = self.cfg.webhook.timeout_ms if self.cfg.webhook.timeout_ms > 0 else wh_to
        self.webhook = WebhookExporter(wh_url, wh_secret, wh_fmt, wh_to) if wh_url else None
        self.bayes = NaiveBayes.ref() if self.webhook is not None else None
        self.metrics = AgentMetrics(opts.event_kind, self.mode, self.supported, self.generator.enabled_signals())
        self.server: Optional[MetricsServer] = None
        self.limiter = RateLimiter(self.cfg.sampling.events_per_second_limit)
        self.guard = None if opts.disable_overhead_guard or not sys.platform.startswith("linux") else \
            OverheadGuard(self.cfg.safety.max_overhead_pct)
        self.stop_event = threading.Event()
        self.meta = SampleMeta(cluster=opts.cluster, namespace=opts.namespace, workload=opts.workload,
                               service=opts.service, node=opts.node)
        self._slo_schema = validator.compiled("slo-event")
        self._probe_schema = validator.compiled("probe-event")
        self.ready = False
        self.windows_done = 0
        self.attributions_emitted = 0

    # ---- lifecycle ------------------------------------------------------------------------
    def start_server(self) -> Optional[MetricsServer]:
        if self.o.metrics_bind:
            self.server = MetricsServer(self.metrics.registry, self.o.metrics_bind, ready=lambda: self.ready).start()
        return self.server

    def close(self) -> None:
        self.stop_event.set()
        try:
            self.writers.close()
        finally:
            if self.server is not None:
                self.server.stop()

    def includes_slo(self) -> bool:
        return self.o.event_kind in ("slo", "both")

    def includes_probe(self) -> bool:
        return self.o.event_kind in ("probe", "both")

    # ---- hello tracer -------------------------------------------------------------------
    def _on_hello(self, ev: HelloEvent) -> None:
        self.metrics.inc_hello(self.o.node, self.o.pod, ev.comm, ev.count)
        if not self.includes_probe():
            return
        pe = ProbeEventV1(ts_unix_nano=ev.timestamp, signal=catalog.HELLO_SIGNAL, node=self.o.node,
                          namespace=self.o.namespace, pod=self.o.pod, container=self.o.container, pid=os.getpid(),
                          tid=os.getpid(), value=float(ev.count), unit="count", status="ok")
        if not self.limiter.allow(ev.timestamp):
            self.metrics.inc_dropped("rate_limit")
            return
        if not self._probe_schema.is_valid(pe.to_dict()):
            self.metrics.inc_dropped("schema")
            return
        try:
            self.writers.emit_probe(pe)
        except Exception:  # noqa: BLE001
            self.metrics.inc_dropped("emit")

    def start_hello_tracer(self) -> Optional[threading.Thread]:
        if not self.o.enable_hello_tracer:
            return None
        tracer = HelloTracer(self.o.hello_target_comm, 2.0)
        t = threading.Thread(target=tracer.start, args=(self.stop_event, self._on_hello), daemon=True)
        t.start()
        return t

    # ---- synthetic engine (REF parity) ---------------------------------------------------
    def emit_one(self, idx: int, t_ns: int) -> None:
        sample = build_synthetic_sample(self.o.scenario, idx, t_ns, self.meta)
        if self.includes_slo():
            for ev in normalize_sample(sample):
                errs = self._slo_schema.errors(ev.to_dict())
                if errs:
                    self.metrics.inc_dropped("schema")
                    raise validator.ValidationError(errs)
                try:
                    self.writers.emit_slo(ev)
                except Exception:
                    self.metrics.inc_dropped("emit")
                    raise
        pmeta = Metadata(node=self.o.node, namespace=self.o.namespace, pod=self.o.pod, container=self.o.container,
                         service=self.o.service, workload=self.o.workload, pid=os.getpid(), tid=os.getpid(),
                         trace_id=sample.trace_id)
        for ev in self.generator.generate(sample, pmeta):
            self.metrics.observe_probe_event(ev, self.o.enable_real_probe_metrics)
            if not self.includes_probe():
                continue
            if not self.limiter.allow(t_ns):
                self.metrics.inc_dropped("rate_limit")
                continue
            if not self._probe_schema.is_valid(ev.to_dict()):
                self.metrics.inc_dropped("schema")
                continue
            try:
                self.writers.emit_probe(ev)
            except Exception:  # noqa: BLE001
                self.metrics.inc_dropped("emit")
        if self.webhook is not None:
            fs = FaultSample(incident_id=f"agent-{sample.trace_id}-{idx}", timestamp=t_ns, cluster=self.o.cluster,
                             namespace=self.o.namespace, service=self.o.service, fault_label=sample.fault_label,
                             confidence=0.9, burn_rate=2.0, window_minutes=5, request_id=sample.request_id,
                             trace_id=sample.trace_id)
            try:
                self.webhook.send(self.bayes.attribute_sample(fs))
            except Exception as exc:  # noqa: BLE001
                print(f"webhook send failed: {exc}", file=sys.stderr)
        self._guard_tick()
        self.metrics.set_heartbeat(t_ns / 1e9)

    def _guard_tick(self) -> None:
        if self.guard is None:
            return
        try:
            pct, exceeded = self.guard.evaluate()
        except Exception as exc:  # noqa: BLE001
            print(f"overhead guard warning: {exc}", file=sys.stderr)
            return
        self.metrics.set_cpu_overhead(pct)
        if exceeded:
            sig = self.generator.disable_highest_cost()
            if sig:
                print(f"overhead budget exceeded: disabled signal {sig}", file=sys.stderr)
                self.metrics.set_enabled_signals(self.supported, self.generator.enabled_signals())

    def run_synthetic(self) -> int:
        self.ready = True
        if self.o.count > 0:
            for idx in range(self.o.count):
                self.emit_one(idx, now_ns())
            self.writers.flush()
            return 0
        idx = 0
        period = self.o.interval_ms / 1000.0
        nxt = time.monotonic()
        while not self.stop_event.is_set():
            self.emit_one(idx, now_ns())
            idx += 1
            nxt += period
            self.stop_event.wait(max(0.0, nxt - time.monotonic()))
        self.writers.flush()
        return 0

    # ---- GPU window engine ----------------------------------------------------------------
    def _window_source(self) -> Iterator:
        """Yields (StagedWindow, group_names, t0_ns) per window."""
        o = self.o
        if o.source == "replay":
            from ..pipeline.replay import ReplayConfig, ReplayGenerator

            gen = ReplayGenerator(ReplayConfig(scenario=o.scenario if o.scenario != "baseline" else "full",
                                               events_per_window=o.window_events, spans_per_window=o.window_spans,
                                               n_services=o.window_groups, window_ms=o.window_ms))
            # The replay producer stands in for the BPF / rocprofiler producers, which run
            # outside the agent and write records in the wire format: pre-generate and
            # pre-stage a few windows and cycle them, so the agent's overhead guard
            # measures the agent, not the synthetic trace generator.
            import torch

            from ..collector.records import ConnInterner, native_encoder
            from ..pipeline.window import stage_window

            it, enc = ConnInterner(), native_encoder()
            pool = []
            for _ in range(4):
                w = gen.next_window()
                pool.append(stage_window(torch, w.events, w.spans, min(w.n_groups, o.window_groups), None,
                                         o.window_groups, None, wire=o.wire, interner=it, encoder=enc))
            names = [f"svc-{g + 1}" for g in range(o.window_groups)]
            i = 0
            while True:
                yield pool[i % len(pool)], names, now_ns()
                i += 1
        elif o.source == "ring":
            import torch

            from ..pipeline.window import stage_window

            from ..collector.records import ConnInterner, native_encoder

            # ring records are 64-byte EVENTs; the native encoder converts each window to the
            # configured wire format (one encoder per stream keeps ids consistent)
            it, enc = ConnInterner(), native_encoder()
            src = RingSource(o.ring_name, o.window_events, o.window_spans)
            for ev, sp, n_groups, names, t0 in src.windows(o.window_ms, self.stop_event, o.window_groups):
                yield stage_window(torch, ev, sp, n_groups, None, o.window_groups, None, wire=o.wire, interner=it,
                                   encoder=enc), names, t0
        else:
            raise ValueError(f"unknown window source {o.source!r}")

    def _attributions(self, G: int, names: Sequence[str], post: np.ndarray, pred: np.ndarray,
                      bits: np.ndarray, t_ns: int, model) -> List[IncidentAttribution]:
        out = []
        D = model.weights.shape[1]
        for g in range(G):
            ranked = model.ranked(post[g, :D], bits[g, :D])
            if not ranked or ranked[0].posterior < self.o.min_confidence:
                continue
            top = ranked[0]
            out.append(IncidentAttribution(
                incident_id=f"gpu-{t_ns}-{g:03d}", timestamp=t_ns, cluster=self.o.cluster,
                namespace=self.o.namespace, service=names[g] if g < len(names) else f"group-{g}",
                predicted_fault_domain=top.domain, confidence=float(top.posterior),
                evidence=[Evidence(catalog.BY_NAME[s].semconv or s, "elevated", "ebpf") for s in top.evidence] or
                [Evidence("llm.ebpf.correlation_confidence", float(top.posterior), "ebpf")],
                slo_impact=SLOImpact("ttft_ms", 2.0, 5),
                fault_hypotheses=[FaultHypothesis(p.domain, p.posterior, p.evidence) for p in ranked
                                  if p.posterior >= 0.01]))
        return out

    def run_windows(self, max_windows: int = 0, process_group=None) -> int:
        """GPU engine main loop (one process per MI355X; ``process_group`` = RCCL node group)."""
        import torch

        from ..pipeline.window import WindowPipeline

        o = self.o
        torch.cuda.set_device(o.device)
        pipe = WindowPipeline(o.window_events, o.window_spans, o.window_groups, o.device, process_group,
                              model=o.model, learn=False)
        source = self._window_source()
        first = next(source)  # producer warm-up happens before the guard's first sample
        if self.guard is not None:
            self.guard.evaluate()
        self.ready = True
        period = o.window_ms / 1000.0
        nxt = time.monotonic()
        import itertools

        for w, names, t0 in itertools.chain([first], source):
            if self.stop_event.is_set():
                break
            t_start = time.perf_counter()
            pipe.submit(w, with_labels=False)
            pipe.drain()
            e = pipe.eng
            pk = pipe.last_packet()
            lat_ms = 1e3 * (time.perf_counter() - t_start)
            self.metrics.observe_window(pk["hist"], pk["status"], pk["dbg"], w.n_events, lat_ms, o.node, o.pod,
                                        o.namespace)
            G = w.n_groups
            post = e.post[:G].cpu().numpy()
            pred = e.pred[:G].cpu().numpy()
            bits = e.evbits[:G].cpu().numpy().view(np.uint32)
            for attr in self._attributions(G, names, post, pred, bits, t0 or now_ns(), pipe.model):
                self.metrics.observe_attribution(attr.predicted_fault_domain)
                self.writers.emit_attribution(attr)
                self.attributions_emitted += 1
                if self.webhook is not None:
                    try:
                        self.webhook.send(attr)
                    except Exception as exc:  # noqa: BLE001
                        self.metrics.inc_dropped("emit")
                        print(f"webhook send failed: {exc}", file=sys.stderr)
            self._guard_tick()
            self.metrics.set_heartbeat()
            self.windows_done += 1
            if max_windows and self.windows_done >= max_windows:
                break
            nxt += period
            if o.source == "replay":
                self.stop_event.wait(max(0.0, nxt - time.monotonic()))
        self.writers.flush()
        return 0


class RingSource:
    """Windows cut from the native shared-memory rings that probe producers write into
    (``/<name>-events`` 64-byte EVENT records, ``/<name>-spans`` SPAN records).

    The C ABI (runtime/csrc/ring.h) lets the BPF ring-buffer reader and the
    rocprofiler-sdk tool library (``tools/rocprof_tool``) push without Python; the agent
    drains whatever arrived each window (O(1) per window, two segments at most)."""

    def __init__(self, name: str, max_events: int, max_spans: int):
        from ..collector import records
        from ..runtime import load

        rt = load()
        cap_e = 1 << max(1, (max_events * 4 - 1).bit_length())
        cap_s = 1 << max(1, (max_spans * 4 - 1).bit_length())
        self.events = rt.HostRing(cap_e, 64, name + "-events")
        self.spans = rt.HostRing(cap_s, 64, name + "-spans")
        self.max_events, self.max_spans = max_events, max_spans
        self._ev_dtype, self._sp_dtype = records.EVENT, records.SPAN

    @staticmethod
    def _drain(ring, limit: int, dtype) -> np.ndarray:
        segs = ring.peek(limit)
        view = ring.records_view()
        parts = []
        n = 0
        for _pos, idx, cnt in segs:
            parts.append(np.frombuffer(view[idx * 64:(idx + cnt) * 64].tobytes(), dtype=dtype))
            n += cnt
        ring.release(n)
        return np.concatenate(parts) if parts else np.zeros(0, dtype=dtype)

    def windows(self, window_ms: int, stop: threading.Event, n_groups: int) -> Iterator:
        period = window_ms / 1000.0
        nxt = time.monotonic() + period
        while not stop.is_set():
            stop.wait(max(0.0, nxt - time.monotonic()))
            nxt += period
            ev = self._drain(self.events, self.max_events, self._ev_dtype)
            sp = self._drain(self.spans, self.max_spans, self._sp_dtype)
            yield ev, sp, n_groups, [f"group-{g}" for g in range(n_groups)], now_ns()


def run_forever(agent: Agent, fn: Callable[[], int]) -> int:
    import signal as _signal

    def _stop(*_):
        agent.stop_event.set()

    for s in (_signal.SIGINT, _signal.SIGTERM):
        try:
            _signal.signal(s, _stop)
        except ValueError:  # not main thread
            pass
    try:
        return fn()
    finally:
        agent.close()

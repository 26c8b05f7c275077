"""Node agent: REF cmd/agent/main.go (per-tick synthetic emit loop, Prometheus surface,
overhead guard with cost-ordered shedding, per-second rate limiter, hello tracer,
stdout/jsonl/OTLP outputs, Bayes + webhook) re-built around the MI355X window engine.

Two engines share one process, one Prometheus registry and one set of outputs:

* ``synthetic`` (REF parity, ``emit_one``): every tick builds a RawSample for the
  scenario, emits the 4 SLO events and the enabled probe events (schema-validated,
  rate-limited), attributes the sample with naive Bayes when a webhook is configured, and
  evaluates the overhead guard, shedding the highest-cost signal when over budget
  (REF cmd/agent/main.go:515-604).
* ``gpu`` (``run_windows``): the probes' BPF ring buffer (pinned ``mislo_events``; or the
  shared-memory emulation), the rocprofiler-sdk tool's / services' user-space event ring and
  the span ring are cut into windows (epoch published into ``mislo_cfg`` at each cut) and
  assembled natively into the native window engine's pinned blocks on this node's MI355X:
  K1 decode -> K2 LDS join -> K3 MFMA posterior (+ RCCL packet all-reduce when several GPUs
  share the node). Per window the agent folds the kernel histograms into the Prometheus
  histograms and emits one IncidentAttribution per incident group whose top posterior clears
  ``min_confidence``, over the same outputs and webhook. No per-event Python work and no
  PyTorch in the process; the host does O(groups) work per window.
"""

from __future__ import annotations

import collections
import json
import math
import os
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from ..collector.pipeline import SampleMeta, build_synthetic_sample, normalize_sample
from ..collector.probes import HelloEvent, HelloTracer
from ..contracts import config as toolkitcfg
from ..contracts import validator
from ..contracts.types import Evidence, FaultHypothesis, IncidentAttribution, ProbeEventV1, SLOImpact
from ..export.otel import OTLPLogExporter
from ..export.prometheus import MetricsServer
from ..export.webhook import AsyncWebhook, WebhookExporter
from ..models.bayes import NaiveBayes
from ..models.sample import FaultSample
from ..safety import OverheadGuard, RateLimiter
from ..signals import catalog
from ..signals.generator import Generator
from ..signals.metadata import Interner, Metadata, ProcMetadataEnricher, StaticMetadataEnricher
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
    webhook_queue: int = 256             # attributions waiting for delivery; more are dropped (reason "emit")
    emit_min_burn: float = 1.0           # attribute a group only while its SLO burns at least this (x budget rate;
                                         # <= 0: every scored group, REF's emit-per-tick)
    emit_min_requests: float = 8.0       # the gate's burn "now": the last windows (at most 3) holding this many
                                         # requests -- one busy window with no breach ends a page
    emit_recovered_requests: int = -1    # a window completing at least this many requests, none breaching in it,
                                         # is recovered: not attributed (0 = off; -1 = 4 per second of window,
                                         # at least 2)
    emit_wait_ms: int = 250              # after a cut, wait up to this long for the window's results (0 = emit
                                         # window k at cut k+1)
    decision_log: str = ""               # JSONL of every scored group per window, emitted or not, and why
                                         # ("" = off; the evidence harnesses' per-window audit trail)
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
    source: str = "replay"               # bpf | shm | replay
    ring_name: str = "/mislo-agent"
    pin_dir: str = "/sys/fs/bpf/mislo"
    probe_objs: str = ""  # --source bpf: compiled probes to load + attach (empty: loaded externally)
    window_ms: int = 1000
    window_events: int = 1 << 20
    window_spans: int = 16384
    window_groups: int = 64
    device: int = 0
    model: str = "bayes"
    min_confidence: float = 0.5
    ttft_slo_ms: float = 800.0           # per-incident SLO: a span breaches when its TTFT exceeds this
    slo_target: float = 0.99             # TTFT SLO objective (burn rate = breach fraction / (1 - target))
    otlp_receiver_bind: str = ""         # OTLP/HTTP /v1/traces receiver feeding the span ring ("" = off)
    halo_ms: float = 2000.0              # carry records this close to a window's end into the next window
    state_dir: str = ""                  # agent state checkpoint directory ("" = none; resumed on start)
    checkpoint_every: int = 60           # windows between checkpoints
    gpus: int = 1                        # window workers (one per GPU); 0 = every GPU visible to the agent
    split_rings: bool = True             # gpus > 1: one ring set per worker, producers route by owner
    model_path: str = ""                 # trained model file (attributor --train); overrides --model
    otlp_receiver_allow: str = ""        # CIDRs allowed to export spans to the receiver ("" = any)
    otlp_forwarders: str = ""            # CIDRs of trusted span forwarders (no pod-address check)
    procfs_sampler: bool = False         # runqueue_delay_ms from /proc schedstat (no BPF needed)
    procfs_pods: str = ""                # pid:pod-uid,... to watch ("" = the node's kubepods cgroups)
    procfs_interval_ms: int = 100
    procfs_cpu_psi: bool = False         # cpu_steal_pct also from the pod group's cpu.pressure (pod-private cgroups)
    # gpu_queue_delay_ms from the KFD driver's per-process occupancy / eviction files (runtime/csrc/
    # gpusampler.h): "auto" = when /sys/class/kfd exists and pod processes are watched (bpf source or
    # the procfs sampler); needs the host pid namespace (hostPID) to match KFD's pids to pods
    kfd_sampler: str = "auto"
    kfd_proc: str = "/sys/class/kfd/kfd/proc"
    model_signals: str = ""              # signals the node's sources produce (others marginalised; "" = all)
    # application evidence (models/bayes.py AppEvidence): a group's retrieval time beyond the
    # kernel-attributed share at least this long is elevated (<= 0: off)
    retrieval_residual_ms: float = 100.0
    # per-launch HIP uprobes (hipLaunchKernel & co.): off -- ~39,000 hits/s on an LLM decode loop
    # (profiles/r6_uprobe/); the KFD sampler's activity decision does without them
    hip_launch_uprobes: bool = False
    pair_prior: float = 0.0              # 2-fault prior mass added to a table model without pairs (0 = none)
    explicit_flags: Tuple[str, ...] = ()  # flags given on the command line (they win over the config's gpu: block)


# the config file's gpu: block -> the agent option it sets (flag name, option field)
GPU_CONFIG_FLAGS = (("window_ms", "window-ms", "window_ms"),
                    ("max_events_per_window", "window-events", "window_events"),
                    ("world_size", "gpus", "gpus"),
                    ("attribution_model", "model", "model"))


def apply_gpu_config(opts: "AgentOptions", gpu) -> "AgentOptions":
    """The toolkit config's ``gpu:`` block (window_ms, max_events_per_window, world_size,
    attribution_model, enabled) as the window engine's settings; a flag given on the command line
    wins, with a warning when it disagrees (REF: CLI overrides config, cmd/agent/main.go:426-440).
    ``enabled: false`` runs REF's tick loop (engine synthetic) unless --engine was given. A learned
    ``attribution_model`` needs --model-path, so with none the config's model is not taken."""
    from dataclasses import replace

    given = set(opts.explicit_flags)
    upd = {}
    for key, flag, field_ in GPU_CONFIG_FLAGS:
        v = getattr(gpu, key)
        if key == "attribution_model" and (opts.model_path or v not in ("bayes", "bayes_gpu")):
            continue
        if flag in given:
            if v != getattr(opts, field_):
                print(f"config gpu.{key}={v!r} overridden by --{flag}={getattr(opts, field_)!r}", file=sys.stderr)
            continue
        upd[field_] = type(getattr(opts, field_))(v)
    if not gpu.enabled:
        if "engine" in given:
            if opts.engine in ("gpu", "cpu"):
                print(f"config gpu.enabled=false overridden by --engine={opts.engine}", file=sys.stderr)
        else:
            upd["engine"] = "synthetic"
    return replace(opts, **upd) if upd else opts


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
                opts = self.o = apply_gpu_config(opts, self.cfg.gpu)
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
        # deliveries leave on their own thread: the window clock never waits on the endpoint
        self.webhook_q = AsyncWebhook(self.webhook, maxsize=opts.webhook_queue,
                                      on_drop=lambda reason: self.metrics.inc_dropped("emit"),
                                      log=lambda m: print(m, file=sys.stderr)) if self.webhook is not None else None
        self.decisions = None
        if opts.decision_log:
            os.makedirs(os.path.dirname(os.path.abspath(opts.decision_log)), exist_ok=True)
            self.decisions = open(opts.decision_log, "a", buffering=1)  # line-buffered: tailed while it runs
        self.server: Optional[MetricsServer] = None
        self.limiter = RateLimiter(self.cfg.sampling.events_per_second_limit)
        # the window engine evaluates the guard every window: REF's formula over a 30 s horizon
        self.guard = None if opts.disable_overhead_guard or not sys.platform.startswith("linux") else \
            OverheadGuard(self.cfg.safety.max_overhead_pct, horizon_s=30.0 if opts.engine in ("gpu", "cpu") else 0.0)
        self.stop_event = threading.Event()
        self.meta = SampleMeta(cluster=opts.cluster, namespace=opts.namespace, workload=opts.workload,
                               service=opts.service, node=opts.node)
        self._slo_schema = validator.compiled("slo-event")
        self._probe_schema = validator.compiled("probe-event")
        self.ready = False
        self.windows_done = 0
        self.pod_ids = Interner()  # pod uid -> pod id (cgroup map and OTLP spans)
        # per-group SLO burn forecast over the next 5 minutes of windows, scored as it matures
        from ..evaluation.slo import BurnRateForecaster

        self.burn = BurnRateForecaster(opts.slo_target, horizon=max(1, int(round(300_000 / max(opts.window_ms, 1)))),
                                       short=max(1, int(round(30_000 / max(opts.window_ms, 1)))))
        self.receiver = None
        self.attributions_emitted = 0
        # cut -> emission time of every window (ms): the agent's own share of detection delay
        self.emit_lag_ms: "collections.deque" = collections.deque(maxlen=4096)
        self.cut_skew_ms: "collections.deque" = collections.deque(maxlen=4096)

    # ---- lifecycle ------------------------------------------------------------------------
    def start_server(self) -> Optional[MetricsServer]:
        if self.o.metrics_bind:
            pods = lambda: {n: i for i, n in enumerate(self.pod_ids.names()) if n}  # noqa: E731
            self.server = MetricsServer(self.metrics.registry, self.o.metrics_bind, ready=lambda: self.ready,
                                        debug={"pods": pods}).start()
        return self.server

    def close(self) -> None:
        self.stop_event.set()
        try:
            self.writers.close()
            if self.webhook_q is not None:
                self.webhook_q.close()
            if self.decisions is not None:
                self.decisions.close()
                self.decisions = None
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
            try:  # a failed attribution is logged and counted; it never ends the tick loop
                self.webhook_q.send(self.bayes.attribute_sample(fs))
            except Exception as exc:  # noqa: BLE001
                print(f"attribution for the webhook failed: {exc}", file=sys.stderr)
                self.metrics.inc_dropped("emit")
        self._guard_tick()
        self.metrics.set_heartbeat(t_ns / 1e9)

    def _guard_tick(self) -> None:
        self.metrics.set_rss()
        if self.guard is None:
            return
        try:
            pct, exceeded = self.guard.evaluate()
        except Exception as exc:  # noqa: BLE001
            print(f"overhead guard warning: {exc}", file=sys.stderr)
            return
        self.metrics.set_cpu_overhead(pct)
        if exceeded:
            ladder = getattr(self, "ladder", None)
            if ladder is not None:  # window engine: floors -> sampler -> GPU producers -> probes
                what = ladder.step()
                if what:
                    print(f"overhead budget exceeded: shed {what}", file=sys.stderr)
                    gone = ladder.disabled()
                    self.metrics.set_enabled_signals(
                        self.supported, [x for x in self.generator.enabled_signals() if x not in gone])
                return
            pm = getattr(self, "probe_manager", None)
            sig = pm.shed_next() if pm is not None else None  # really detach a kernel probe
            if pm is not None and sig:
                self.generator.disable(sig)
            else:
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

    # ---- window engine (GPU, or the CPU oracle engine) ---------------------------------------
    def _open_source(self, world: int = 1):
        """Rings + maps for the configured source. ``bpf``: the probes' pinned maps (root);
        ``shm``: emulated rings another process produces into (tests, CI); ``replay``: a forked
        replay producer writing seeded fault-replay windows at window_events per window_ms
        (stands in for the kernel probes and the rocprofiler tool: its CPU is not the agent's).
        ``world`` > 1: split rings, one (kernel, user-space, span) ring set per worker, every
        producer routing each record to its owner's set (collector/bpf.py ShardRouter).
        Returns (maps, [(ring, user ring, span ring)] per worker, pod metadata or None)."""
        from ..collector import bpf
        from ..runtime import load

        o = self.o
        rt = load()
        sets_names = [bpf.RingNames.of(o.ring_name, r) for r in range(max(1, world))]
        if o.source == "bpf":
            if o.probe_objs:  # load + attach the compiled probes; their shared maps get pinned
                from ..collector.loader import BpfProbeLoader, probe_specs
                from ..collector.probes import ProbeManager

                self.probe_manager = ProbeManager(self.mode, self.generator.enabled_signals())
                self.bpf_loader = BpfProbeLoader(o.probe_objs, o.pin_dir, launch_uprobes=o.hip_launch_uprobes)
                for spec in probe_specs(self.bpf_loader, self.generator.enabled_signals()):
                    self.probe_manager.register(spec)
                attached = self.probe_manager.attach_all()
                print(f"attached probes for {len(attached)} signals from {o.probe_objs}", file=sys.stderr)
                try:
                    self.bpf_loader.load_flush()
                except Exception as exc:  # noqa: BLE001 - reported below through flush_fd < 0
                    print(f"WARNING: flush program not loaded: {exc}", file=sys.stderr)
            maps = bpf.BpfMaps(o.pin_dir)
            if maps.flush_fd < 0:
                print(f"WARNING: no flush program pinned at {o.pin_dir}/progs/mislo_flush: partial per-CPU "
                      f"batches of quiet CPUs reach the ring only with that CPU's next events", file=sys.stderr)
            self.metrics.flush_loaded.set(1 if maps.flush_fd >= 0 else 0)
            sets = []
            for r, names in enumerate(sets_names):
                ring = maps.ring if r == 0 else rt.Ringbuf.open_pinned(os.path.join(o.pin_dir, f"mislo_events{r}"))
                sets.append((ring, rt.HostRing(1 << 20, 16, names.user),   # the rocprofiler tool pushes USER16
                             rt.HostRing(1 << 18, 64, names.spans)))       # OTLP receiver / services
            return maps, sets, None
        if o.source == "shm":
            sets = [(rt.Ringbuf.attach_shm(n.ring), rt.HostRing(0, 64, n.user, True), rt.HostRing(0, 64, n.spans, True))
                    for n in sets_names]
            return bpf.EmulatedMaps(sets[0][0], [s[0] for s in sets[1:]]), sets, None
        if o.source == "replay":
            kw = dict(scenario=o.scenario if o.scenario not in ("baseline",) else "full",
                      events_per_window=o.window_events, spans_per_window=o.window_spans,
                      n_services=o.window_groups)
            # rings sized by rate: a window's space is freed as soon as its
            # chain is collected (worker.collect), so each ring holds one window plus a quarter
            # for late collection -- the kernel records at <= 24 B per event (18.6 measured), the
            # GPU-signal records (~1/4 of a window's events) and the spans; the shared pages count
            # in the agent's RSS once registered for DMA
            w = max(1, world)
            ev = o.window_events // w
            sets = [tuple(bpf.create_rings(n, 5 * 24 * ev // 4 + (1 << 20), 5 * ev // 16 + 1024,
                                           5 * o.window_spans // (4 * w) + 1024)) for n in sets_names]
            self._producer = bpf.start_replay_producer(sets_names[0], kw, o.window_events * 1000.0 / o.window_ms,
                                                       o.window_ms, max_windows=0,
                                                       shard_names=sets_names if w > 1 else None)
            return bpf.EmulatedMaps(sets[0][0], [s[0] for s in sets[1:]]), sets, bpf.pod_metadata(kw)
        raise ValueError(f"unknown window source {o.source!r} (bpf | shm | replay)")

    def _shard_table(self, world: int):
        """The shared-memory pod id -> shard table the rocprofiler tool in the workloads routes its
        records by (MISLO_SHARD_TABLE; 2^20 pod ids, one byte each; pods it does not list: 0)."""
        from ..collector import bpf

        path = "/dev/shm" + bpf.RingNames.shard_table(self.o.ring_name)
        try:
            with open(path, "wb") as fh:
                fh.truncate(1 << 20)
            os.chmod(path, 0o644)
            self._shard_table_path = path
            return np.memmap(path, dtype=np.uint8, mode="r+", shape=(1 << 20,))
        except OSError as exc:
            print(f"shard table {path}: {exc}; the GPU tool's records stay on ring 0", file=sys.stderr)
            return None

    def _load_model(self):
        """(host model, PosteriorModel image, metadata): the file ``--model-path`` names (written by
        ``attributor --train``), else the built-in expert tables."""
        from ..ops.engine import model_bytes

        from ..models.bayes import marginalize, with_pairs

        o = self.o
        if o.model_path:
            from ..models.train import load_model

            m, image, meta = load_model(o.model_path)
        elif o.model in ("bayes", "bayes_gpu", ""):
            m = NaiveBayes.gpu() if o.model == "bayes_gpu" else NaiveBayes.ref()
            image, meta = model_bytes(m), {"name": m.name}
        else:
            raise ValueError(f"--model {o.model} is learned: give --model-path (a file `attributor --train` wrote)")
        T = float(meta.get("temperature", 1.0))
        if o.retrieval_residual_ms > 0:  # spans' retrieval breakdowns as application evidence
            from ..models.bayes import AppEvidence

            m.app = AppEvidence.expert(o.retrieval_residual_ms, temperature=T)
        if o.pair_prior > 0 and m.pairs is None:
            m = with_pairs(m, o.pair_prior, T)
            meta = dict(meta, pair_rho=o.pair_prior)
        if o.model_signals:
            # signals no source on this node produces are summed out of the likelihood: their
            # absence says nothing about the domains they would indicate
            obs = [x.strip() for x in o.model_signals.split(",") if x.strip()]
            m = marginalize(m, obs, T)
            meta = dict(meta, observable_signals=obs)
        if o.pair_prior > 0 or o.model_signals:
            image = model_bytes(m)
        return m, image, meta

    def n_gpus(self) -> int:
        """Window workers: --gpus, or every GPU visible to the agent (--gpus 0; counted without
        initialising HIP, which the controller never does)."""
        if self.o.gpus > 0:
            return int(self.o.gpus)
        if self.o.engine == "cpu":
            return 1
        from ..parallel.numa import visible_gpu_count

        return max(1, visible_gpu_count())

    # ---- agent state (checkpoint / resume) ----------------------------------------------------
    def _state_path(self) -> str:
        if not self.o.state_dir:
            return ""
        safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in self.o.node)
        return os.path.join(self.o.state_dir, f"agent-{safe}.state.json")

    def save_state(self, path: str) -> None:
        """What the agent has learned at run time: the window counter, every incident group's
        burn-rate history and pending forecasts (the SLO-impact forecaster), the pod-uid -> pod-id
        interning (ids the probes' cgroup map and the engine's pod table carry) and the model in
        use. Written to a temporary file and renamed."""
        import json

        st = {"format": "mislo-agent-state/2", "node": self.o.node, "windows": self.windows_done,
              "model": getattr(self, "model_meta", {}).get("name", ""),
              "burn": self.burn.state(), "pods": self.pod_ids.names()}
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = f"{path}.tmp.{os.getpid()}"
        try:
            with open(tmp, "w", encoding="utf-8") as fh:
                json.dump(st, fh)
            os.replace(tmp, path)
        except OSError as exc:
            print(f"state checkpoint {path} failed: {exc}", file=sys.stderr)

    def load_state(self, path: str) -> bool:
        import json

        try:
            with open(path, encoding="utf-8") as fh:
                st = json.load(fh)
            if st.get("format") != "mislo-agent-state/2":
                raise ValueError("unknown state format")
            self.windows_done = int(st.get("windows", 0))
            self.burn.restore(st.get("burn", {}))
            for name in st.get("pods", [])[1:]:
                self.pod_ids.id(name)
        except (OSError, ValueError, KeyError, TypeError) as exc:
            print(f"state {path} not usable ({exc}); starting fresh", file=sys.stderr)
            return False
        print(f"resumed agent state from {path} ({self.windows_done} windows)", file=sys.stderr)
        return True

    def _scan_pods(self, maps) -> None:
        """kubepods cgroups -> the probes' cgroup -> pod id map (pod ids from the interner the
        OTLP receiver maps ``k8s.pod.uid`` through, so spans and kernel records agree)."""
        from ..collector import bpf

        for cg, (pid, _uid) in bpf.discover_pods(interner=self.pod_ids).items():
            try:
                maps.set_pod(cg, pid)
            except OSError as exc:
                print(f"pod map update failed: {exc}", file=sys.stderr)
                return

    def _attributions(self, G: int, names: Sequence[str], res: dict, t_ns: int, model) -> List[IncidentAttribution]:
        """One IncidentAttribution per incident group with SLO impact whose top posterior clears
        min_confidence. Evidence carries the group's measured signal values (mean over joined
        kernel signals); SLO impact comes from the group's spans (TTFT SLO breach fraction over the
        error budget = burn rate, forecast over the next 5 minutes from the recent windows), not
        from constants.

        Emission is gated on SLO impact: a group is attributed only while its SLO burns its error
        budget at least ``emit_min_burn`` times the sustainable rate NOW (the burn over the shortest
        run of the last <= 3 windows holding ``emit_min_requests`` requests, >= 1 by default: a
        fast-burn alert), so "unknown" never
        leaves at zero burn, one slow request among a few does not page, and a recovered service
        stops paging although its 5-minute forecast still carries the fault. The attribution's
        SLO impact quotes the forecast burn. Every scored group still counts in
        ``llm_slo_agent_incidents_scored_total{domain, emitted}``; a healthy node emits nothing (REF
        posts every tick, cmd/agent/main.go:567-585 -- with a webhook configured that pages on
        every healthy window)."""
        out = []
        D = model.weights.shape[1]
        post, bits, feat = res["post"], res["evbits"].view(np.uint32), res["feat"]
        sli = res.get("sli")
        forecast, now_burn = {}, {}
        if sli is not None:
            late = res.get("late")
            for g in range(min(G, sli.shape[0])):
                key = names[g] if g < len(names) else f"group-{g}"
                lb = float(late[g, 0]) if late is not None and g < late.shape[0] else 0.0
                forecast[g] = self.burn.observe(key, float(sli[g, 0]), float(sli[g, 1]), late=lb)
                now_burn[g] = self.burn.current(key, windows=3, min_requests=self.o.emit_min_requests)
            err = self.burn.error()
            if err is not None:
                self.metrics.burn_err.set(err)
        # the SLO-impact window is the forecast horizon the burn rate is quoted over (5 minutes)
        impact_min = max(1, int(round(self.burn.horizon * self.o.window_ms / 60000.0)))
        reqs = sli[:, 0].tolist() if sli is not None else []
        feat_l = np.asarray(feat, dtype=np.float64).tolist()  # Python rows: one conversion per window
        log = self.decisions
        # every group's top hypothesis at once (the live domains' argmax: ranked()'s stable sort puts
        # the first of equal posteriors first); the full ranking is built only for groups that emit
        # (or for the decision log) -- it was ~15 us a group, the epilogue's largest share
        live = np.isfinite(np.asarray(model.bias, dtype=np.float64)[:D])
        pl = np.where(live[None, :], np.asarray(post, dtype=np.float64)[:G, :D], -np.inf)
        top_d = pl.argmax(axis=1).tolist() if G else []
        top_p = pl.max(axis=1).tolist() if G else []
        any_live = bool(live.any())
        late_l = res["late"][:, 0].tolist() if res.get("late") is not None else []
        rec_n = int(self.o.emit_recovered_requests)
        if rec_n < 0:  # 4 requests per 1 s window (the first recovery windows of config 3), at least 2
            rec_n = max(2, int(round(4 * self.o.window_ms / 1000.0)))
        for g in range(G):
            if g < len(reqs) and reqs[g] == 0 and not (g < len(late_l) and late_l[g]):
                continue  # no request of this group in the window: no incident to attribute
            burn = forecast.get(g, 0.0)  # forecast burn over the SLO window (measured counts)
            # (1 - 1e-9: the budget 1 - target is not exact in binary, a burn of exactly 1 lands a hair under)
            cur = now_burn.get(g, 0.0)
            confident = any_live and top_p[g] >= self.o.min_confidence
            # recovered: the window itself completed enough requests and none breached in it (a breach
            # whose deadline passed in an earlier window is that window's, SPAN_LATE); the pooled burn
            # still holds the fault's windows, but the service no longer burns
            recovered = (sli is not None and rec_n > 0 and self.o.emit_min_burn > 0 and g < sli.shape[0]
                         and sli[g, 0] >= rec_n and sli[g, 1] == 0)
            burning = (sli is None or self.o.emit_min_burn <= 0
                       or (cur > 0 and cur >= self.o.emit_min_burn * (1.0 - 1e-9)))
            emit = confident and burning and not recovered
            ranked = model.ranked(post[g, :D], bits[g, :D]) if (emit or log is not None) else None
            if log is not None:
                log.write(json.dumps({
                    "t_ns": int(t_ns), "group": g, "service": names[g] if g < len(names) else f"group-{g}",
                    "requests": float(sli[g, 0]) if sli is not None and g < sli.shape[0] else None,
                    "breaches": float(sli[g, 1]) if sli is not None and g < sli.shape[0] else None,
                    "burn_now": round(cur, 4), "burn_forecast": round(burn, 4),
                    "top": [[p.domain, round(float(p.posterior), 4)] for p in ranked[:3]],
                    "late": late_l[g] if g < len(late_l) else 0, "emitted": emit,
                    "why": "emitted" if emit else ("low_confidence" if not confident else
                                                   ("no_burn" if not burning else "recovered"))}) + "\n")
            if not confident:
                continue
            self.metrics.observe_incident(catalog.ALL_DOMAINS[top_d[g]], emit)
            if not emit:
                continue
            top = ranked[0]
            ev = []
            for sname in top.evidence:
                if sname == catalog.APP_RETRIEVAL_SIGNAL:  # application evidence (AppEvidence)
                    ev.extend(self._retrieval_evidence(res, g))
                    continue
                spec = catalog.BY_NAME[sname]
                v = feat_l[g][spec.slot]
                ev.append(Evidence(spec.semconv or sname, round(v, 3) if math.isfinite(v) else "elevated", "ebpf"))
            if not ev:
                ev = [Evidence("llm.ebpf.correlation_confidence", float(top.posterior), "ebpf")]
            out.append(IncidentAttribution(
                incident_id=f"gpu-{t_ns}-{g:03d}", timestamp=t_ns, cluster=self.o.cluster,
                namespace=self.o.namespace, service=names[g] if g < len(names) else f"group-{g}",
                predicted_fault_domain=top.domain, confidence=float(top.posterior), evidence=ev,
                slo_impact=SLOImpact("ttft_ms", round(burn, 4), impact_min),
                fault_hypotheses=[FaultHypothesis(p.domain, p.posterior, p.evidence) for p in ranked
                                  if p.posterior >= 0.01]))
        return out

    @staticmethod
    def _retrieval_evidence(res: dict, g: int) -> List[Evidence]:
        """The application evidence of group g: its retrieval time beyond the kernel-attributed share
        (source "application", REF incident-attribution.schema.json:41-56) and that share itself,
        REF's llm.ebpf.retrieval.kernel_attributed_ms (DecomposeRetrieval, source "ebpf")."""
        from ..contracts import semconv
        from ..models.bayes import AppEvidence

        app, feat = res.get("app"), res["feat"]
        if app is None:
            return [Evidence(catalog.APP_RETRIEVAL_SEMCONV, "elevated", "application")]
        resid = float(AppEvidence.residual(app[g:g + 1], feat[g:g + 1])[0])
        f = np.asarray(feat[g], dtype=np.float64)
        kern = float(sum(f[s] for s in (0, 3, 5) if math.isfinite(f[s])))
        return [Evidence(catalog.APP_RETRIEVAL_SEMCONV, round(max(resid, 0.0), 3), "application"),
                Evidence(semconv.ATTR_RETRIEVAL_KERNEL_MS, round(kern, 3), "ebpf")]

    def _emit_window(self, prevs: List[dict], t_ns: int, G: int, names, ring, model) -> None:
        """One finished window, as every worker's part of it in rank order (worker.PrevJoiner):
        worker 0's carries the node-wide packet (RCCL all-reduce) and every worker's incidents
        (all-gather); each worker its own ring accounting."""
        from ..pipeline.window import RING_FIELDS, unpack_packet
        from .worker import merge_results

        if not prevs or "packet" not in prevs[0]:
            return
        head = prevs[0]
        pk = unpack_packet(head["packet"])
        rings = [dict(zip(RING_FIELDS, (int(x) for x in p["ring"]))) for p in prevs]
        events = sum(r["events"] for r in rings)
        rs = dict(rings[0])
        rs["first_busy"] = max(r["first_busy"] for r in rings)
        self.metrics.observe_window(pk["hist"], pk["status"], pk["dbg"], events, max(p["latency_ms"] for p in prevs),
                                    self.o.node, self.o.pod, self.o.namespace, value_sums_milli=pk["misc"][2:18])
        self.metrics.set_ring(ring.stats() if ring is not None else {}, rs, max(p["host_us"] for p in prevs))
        res = merge_results(head["results"], G)
        self.last_results = res
        attrs = self._attributions(G, names, res, t_ns, model)
        for attr in attrs:
            self.metrics.observe_attribution(attr.predicted_fault_domain)
            self.writers.emit_attribution(attr)
            self.attributions_emitted += 1
            if self.webhook_q is not None:
                self.webhook_q.send(attr)  # enqueued; delivered on the webhook thread
        if attrs:
            self.writers.flush()  # a window's incidents leave with the window (detection delay)
        self.emit_lag_ms.append(1e-6 * (time.time_ns() - t_ns))

    def _start_fresh(self, pool, maps, sets, split: bool) -> None:
        """Spawned workers start at the rings' current positions: what the producers wrote while
        the workers started (seconds) is skipped. Those records would be a backlog the windows
        never work off in shared-ring mode, and once more than 3 cuts old their 2-bit epoch tags
        decode against the wrong bases (timestamps off by whole windows). The interning maps are
        reset first, so every id is defined again after the start point."""
        if hasattr(maps, "reset_definitions"):
            try:
                maps.reset_definitions(len(pool.workers) if split else 1)
            except OSError as exc:
                print(f"id redefinition at the workers' start failed: {exc}", file=sys.stderr)
        maps.flush_cpus()
        pos = [(int(rs[0].producer_pos) if rs[0] is not None else 0, int(rs[1].head) if rs[1] is not None else 0,
                int(rs[2].head) if rs[2] is not None else 0) for rs in sets]
        skipped = sum(p[0] - int(rs[0].consumer_pos) for p, rs in zip(pos, sets) if rs[0] is not None)
        pool.start_at(pos[:len(pool.workers)] if split else pos[0])
        if skipped > 0:
            print(f"window workers start at the rings' current positions ({skipped} kernel-ring bytes written "
                  f"while they started are skipped)", file=sys.stderr)

    def _restart_workers(self, exc, rings, sets, maps, G: int):
        """A worker died or stopped answering: its communicator is broken for every worker. Stop
        them all and start fresh processes for the surviving GPUs -- a new communicator (RCCL id,
        or a new gloo port for the CPU engine), world N - 1, the services re-sharded over them
        (split rings: the producers' routing follows at once; the lost worker's ring set is left
        behind). The new workers resume from the ring positions already released, so the windows
        that were in flight are read again. Returns (pool, split)."""
        from dataclasses import replace

        from .worker import WorkerPool, groups_of

        old = self.pool
        dead = set(old.dead_ranks())
        if exc.rank is not None:
            dead.add(int(exc.rank))
        old.close(timeout=2.0)
        survivors = [s for s in self.specs if s.rank not in dead]
        print(f"window worker(s) {sorted(dead)} lost ({str(exc).splitlines()[0]}); restarting on "
              f"{len(survivors)} worker(s)", file=sys.stderr)
        if not survivors:
            raise exc
        N = len(survivors)
        split = bool(self.specs[0].split) and N > 1
        port = self.specs[0].master[1]
        if self.o.engine == "cpu" and N > 1:
            import socket

            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
            sk.close()
        xchg = self.specs[0].xchg_cap if N > 1 else 0
        specs = [replace(s, rank=r, world=N, group_cap=max(1, groups_of(0, N, G)), xchg_cap=xchg,
                         import_cap=(N - 1) * xchg, master=(s.master[0], port), split=split)
                 for r, s in enumerate(survivors)]
        if self.router is not None:  # producers route to the surviving workers' ring sets
            pods, sh = self.router.resize(N if split else 1)
            if hasattr(maps, "set_shards") and len(pods):
                maps.set_shards(pods, sh)

        if self.pod_table:  # every new worker starts with the pods' services known so far
            keys = np.array(sorted(self.pod_table), dtype=np.uint32)
            specs = [replace(s, pods=(keys, np.array([self.pod_table[k] for k in keys.tolist()], dtype=np.uint32)))
                     for s in specs]
        self.pool = WorkerPool(specs, rings, in_process=False)
        self.specs = specs
        # the new workers' context / trace tables start empty: the interning maps are reset (the
        # replay producer re-interns and re-routes) and the workers start at the rings' current
        # positions -- the windows in flight when the worker died are lost, not re-read with ids
        # the new workers never saw defined
        self._start_fresh(self.pool, maps, sets, split)
        self.metrics.worker_restarts.inc()
        self.metrics.workers.set(N)
        return self.pool, split

    def run_windows(self, max_windows: int = 0) -> int:
        """Window engine main loop. This process is the controller: every window_ms it cuts
        the node's rings (publishes epoch k into mislo_cfg -- the only writer -- then snapshots
        the producer positions) and hands the cut to the window workers, one per GPU
        (agent/worker.py; in this process when the node uses one). Each worker DMAs the window
        straight from the rings into its GPU, decodes it, keeps the services it owns (group
        sharding) and joins / scores them; the RCCL all-reduce and all-gather leave the
        node-wide packet and incident list on worker 0. Window k-1's results, complete by the
        time window k is staged, become metrics and attributions while window k computes."""
        from ..collector import bpf
        from ..collector.records import EpochClock
        from ..ops.engine import app_model_bytes
        from ..pipeline.window import Cut
        from ..safety import TreeCPUSampler
        from .worker import PrevJoiner, WorkerError, WorkerPool, WorkerSpec, groups_of

        o = self.o
        N = self.n_gpus()
        split = N > 1 and o.split_rings
        # a replay producer forks here, before any GPU work
        maps, sets, pods = self._open_source(N if split else 1)
        ring, user, spans = sets[0]
        router = None
        if split:  # producers route every record to its owner's ring set
            router = bpf.ShardRouter(N, self._shard_table(N))
            if pods is not None:
                router.set_pods(*pods)
        self.router = router
        # pod id -> svc|node as the workers know it (fresh workers after a restart start from it)
        self.pod_table = {}
        if pods is not None:
            self.pod_table.update(zip(np.asarray(pods[0]).tolist(), np.asarray(pods[1]).tolist()))
        node_id = bpf.stable_node_id(o.node)
        maps.init(node_id)
        model, image, self.model_meta = self._load_model()
        self.model = model
        G = o.window_groups
        # rows: events plus the definitions ahead of them and the pad slots of batches a
        # definition or a cut flushed part-full
        budget = o.window_events + o.window_events // 2
        # joins reach across the window cut (halo: the rows of the earlier windows it spans stay
        # resident on the device) and, on a multi-GPU node, across GPUs (trace-tagged rows
        # exchanged over RCCL, bounded per peer)
        xchg = min(65536, budget) if N > 1 else 0
        icap = (N - 1) * xchg
        halo_windows = int(min(3, max(1, math.ceil(o.halo_ms / max(o.window_ms, 1)) + 1)))
        port = 0
        if o.engine == "cpu" and N > 1:
            import socket

            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
            sk.close()
        specs = [WorkerSpec(rank=r, world=N, device=r if o.engine == "gpu" and N > 1 else o.device, engine=o.engine,
                            source="bpf" if o.source == "bpf" else "shm", ring_name=o.ring_name, pin_dir=o.pin_dir,
                            user_rec=int(user.rec_size), sig_cap=budget, span_cap=o.window_spans,
                            group_cap=max(1, groups_of(0, N, G)), user_cap=max(1024, o.window_events // 4),
                            window_ms=float(o.window_ms), ttft_slo_ms=o.ttft_slo_ms, halo_ms=o.halo_ms,
                            import_cap=icap, xchg_cap=xchg, model_image=np.asarray(image, np.uint8).tobytes(),
                            pods=pods, master=("127.0.0.1", port), halo_windows=halo_windows, split=split,
                            app_image=app_model_bytes(model).tobytes() if model.app is not None else b"")
                 for r in range(N)]
        state = self._state_path()
        if state and os.path.exists(state):
            self.load_state(state)
        pool = WorkerPool(specs, (ring, user, spans), in_process=N == 1)
        self.pool = pool
        self.specs = specs
        if N > 1:  # spawned workers: the records written while they started are skipped
            self._start_fresh(pool, maps, sets, split)
        self.metrics.workers.set(N)
        print(f"window engine: {o.engine} x {N} worker(s){' on split rings' if split else ''}, model "
              f"{self.model_meta.get('name')}"
              f"{' T=%.3g' % self.model_meta['temperature'] if 'temperature' in self.model_meta else ''}",
              file=sys.stderr)
        if o.source == "bpf":
            self._scan_pods(maps)
        names = [f"svc-{g + 1}" for g in range(G)]
        receiver = None
        mapper = None
        if o.otlp_receiver_bind and spans is not None:
            from ..collector.otlp import GroupTable, OtlpSpanReceiver, SpanMapper

            groups = GroupTable(G)
            names = groups.names  # incident groups are the services the receiver has seen
            pod_ips = None
            if o.source == "bpf":  # a span naming a node's pod must come from that pod's address
                from ..collector import procfs as _procfs

                ipcache = {"t": -1e9, "m": {}}

                def pod_ips():
                    if time.monotonic() - ipcache["t"] > 10.0:
                        ipcache["m"] = _procfs.pod_addresses(_procfs.pod_processes())
                        ipcache["t"] = time.monotonic()
                    return ipcache["m"]
            mapper = SpanMapper(groups, self.pod_ids.id, node_id, pod_ips=pod_ips, forwarders=o.otlp_forwarders)
            mapper.slo_ms = float(o.ttft_slo_ms)
            if router is not None:  # each span to the ring of the worker owning its incident group
                def push_spans(recs):
                    sh = router.span_shard(recs)
                    return sum(int(sets[r][2].push(part)) for r, part in router.split(recs, sh) if len(part))
            else:
                push_spans = spans.push
            receiver = OtlpSpanReceiver(o.otlp_receiver_bind, mapper, push_spans, allow=o.otlp_receiver_allow).start()
            self.receiver = receiver
        sampler = None
        from ..collector import kfd, procfs

        static = procfs.parse_pod_list(o.procfs_pods)
        cache = {"t": 0.0, "m": {}}
        tlock = threading.Lock()

        def targets():
            if static:
                return {pid: self.pod_ids.id(uid) for pid, uid in static.items()}
            with tlock:
                if time.monotonic() - cache["t"] > 10.0:  # pod churn: re-walk the cgroups every 10 s
                    cache["m"] = {pid: self.pod_ids.id(uid) for pid, uid in procfs.pod_processes().items()}
                    cache["t"] = time.monotonic()
                return cache["m"]

        def shard_targets(r):
            def f():
                t = targets()
                owner = router.pod_shard(np.array(list(t.values()), dtype=np.int64)) if t else []
                return {pid: pod for (pid, pod), s in zip(t.items(), owner) if int(s) == r}
            return f

        if o.procfs_sampler:
            # native: a C++ thread reads schedstat / cgroup / PSI and pushes into the user ring
            if router is None:
                sampler = procfs.NativeSampler(user, targets, node_id=node_id, cpu_psi=o.procfs_cpu_psi,
                                               refresh_s=10.0 if not static else 3600.0)
            else:  # split rings: one sampler per worker, over the pods its services own
                sampler = procfs.MultiSampler([procfs.NativeSampler(sets[r][1], shard_targets(r), node_id=node_id,
                                                                    cpu_psi=o.procfs_cpu_psi, refresh_s=10.0)
                                               for r in range(N)])
            sampler.start(o.procfs_interval_ms / 1000.0)
            self.procfs = sampler
        use_kfd = o.kfd_sampler == "on" or (o.kfd_sampler == "auto" and kfd.available(o.kfd_proc)
                                             and (o.procfs_sampler or o.source == "bpf"))
        if use_kfd:
            loader = getattr(self, "bpf_loader", None)
            bpf_gpu = loader is not None and "gpu_kfd" in loader.available()
            finder = kfd.hip_map_finder(lambda: loader.is_loaded("gpu_kfd")) if bpf_gpu else None
            kfds = [kfd.KfdSampler(user if router is None else sets[r][1],
                                   targets if router is None else shard_targets(r), node_id=node_id,
                                   kfd_proc=o.kfd_proc, refresh_s=10.0 if not static else 3600.0, hip_map=finder,
                                   evictions=not bpf_gpu)  # the probe's kprobes report evictions
                    for r in range(1 if router is None else N)]
            for k in kfds:
                k.start()
            self.kfd = kfds
        # the ladder's sampler stage sheds the procfs signals only: the KFD samplers emit
        # gpu_queue_delay_ms into the user rings and obey their drop mask -- the GPU stage, one
        # signal at a time -- so the procfs stage never pauses them
        from ..safety import ShedLadder

        self.ladder = ShedLadder(catalog.DISABLE_ORDER, maps=maps, sampler=sampler, user_ring=[x[1] for x in sets],
                                 probe_manager=getattr(self, "probe_manager", None), generator=self.generator)
        if self.guard is not None:
            self.guard.source = TreeCPUSampler(lambda: [os.getpid()] + self.pool.pids())
            self.guard.evaluate()
        clock = EpochClock()
        self.ready = True
        period = o.window_ms / 1000.0
        nxt = time.monotonic() + period
        cut_t = {}
        joiner = PrevJoiner(N)
        windows = 0
        try:
            while not self.stop_event.is_set():
                self.stop_event.wait(max(0.0, nxt - time.monotonic()))
                if self.stop_event.is_set():
                    break
                now = time.monotonic()
                self.cut_skew_ms.append(1e3 * (now - nxt))  # how late the cut is on its schedule
                nxt += period
                if now > nxt:
                    # a stall of more than a period (a worker restart, a paused process): the missed
                    # cuts are not made up back to back -- windows of a fraction of a period each --
                    # the schedule restarts from now
                    missed = int((now - nxt) // period) + 1
                    nxt += missed * period
                    self.metrics.windows_skipped.inc(missed)
                t = time.time_ns()
                maps.cfg_set(bpf.CFG_EPOCH, clock.publish(t))  # epoch first, then the ring snapshots
                maps.flush_cpus()  # every CPU's staged batches onto the rings before the snapshots
                self.metrics.flush_errors.set(float(getattr(maps, "flush_errors", 0)))
                bases = clock.bases()
                cuts = [Cut(kernel=rs[0].producer_pos, user=rs[1].head, spans=rs[2].head, bases=bases, t_ns=t)
                        for rs in sets]
                if mapper is not None:  # spans after this cut: a deadline before it is an earlier window's
                    mapper.late_before_ns = t
                    self.metrics.set_otlp(self.receiver, mapper)
                upd = mapper.take_pod_updates() if mapper is not None else None
                if upd is not None and len(upd[0]):
                    self.pod_table.update(zip(np.asarray(upd[0]).tolist(), np.asarray(upd[1]).tolist()))
                if upd is not None and router is not None:  # later records of these pods go to their owners' rings
                    router.set_pods(*upd)
                    if hasattr(maps, "set_shards"):
                        maps.set_shards(upd[0], router.pod_shard(upd[0]))
                try:
                    replies = pool.window(cuts if split else cuts[0], G, upd, timeout=max(30.0, 20 * period))
                except WorkerError as exc:
                    pool, split = self._restart_workers(exc, (ring, user, spans), sets, maps, G)
                    cut_t.clear()  # the lost windows' records are read again by the new workers
                    joiner.reset(len(self.specs))
                    continue
                cut_t[replies[0]["k"]] = t
                for parts in joiner.add(replies):
                    self._emit_window(parts, cut_t.pop(parts[0]["k"], t), G, names, ring, model)
                if o.emit_wait_ms > 0:
                    # window k leaves as soon as every worker's chain is done (~ms after the cut),
                    # not with the next cut: one window period less detection delay
                    wait = min(o.emit_wait_ms / 1000.0, max(0.0, nxt - time.monotonic() - 0.01))
                    try:
                        got = pool.collect(wait)
                    except WorkerError as exc:
                        pool, split = self._restart_workers(exc, (ring, user, spans), sets, maps, G)
                        cut_t.clear()
                        joiner.reset(len(self.specs))
                        continue
                    for parts in joiner.add(got):
                        self._emit_window(parts, cut_t.pop(parts[0]["k"], t), G, names, ring, model)
                if self.windows_done and self.windows_done % 64 == 0 and o.source == "bpf":
                    self._scan_pods(maps)  # pod churn
                    if getattr(self, "bpf_loader", None) is not None:
                        self.bpf_loader.rescan_uprobes(background=True)  # libssl / librccl / libamdhip64 of new workloads
                self.windows_done += 1
                windows += 1
                if state and o.checkpoint_every > 0 and self.windows_done % o.checkpoint_every == 0:
                    self.save_state(state)
                self._guard_tick()
                self.metrics.set_heartbeat()
                if max_windows and windows >= max_windows:
                    break
                if maps.ctx_ids_used() > (7 << 20) and hasattr(maps, "reset_ctx_ids"):
                    maps.reset_ctx_ids()  # kernel context ids run low: redefine from scratch
            pool = self.pool
            final = pool.stop()
            for parts in joiner.add(final or []):
                self._emit_window(parts, cut_t.pop(parts[0]["k"], time.time_ns()), G, names, ring, model)
            self.last_summary = final[0].get("summary") if final else None
            if state:
                self.save_state(state)
        finally:
            # workers unregister the rings from their GPUs and free device memory while the
            # ring mappings still exist (interpreter teardown order is arbitrary)
            self.pool.close()
            if sampler is not None:
                sampler.stop()
            for k in getattr(self, "kfd", None) or []:
                k.stop()
            if receiver is not None:
                receiver.stop()
            if getattr(self, "probe_manager", None) is not None:
                self.probe_manager.detach_all()
            if getattr(self, "_producer", None) is not None:
                self._producer.terminate()
                self._producer.join(5)
                if self._producer.is_alive():
                    self._producer.kill()
                    self._producer.join(5)
        self.writers.flush()
        return 0


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

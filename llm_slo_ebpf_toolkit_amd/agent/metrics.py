"""Agent Prometheus surface: every REF metric name/type/label set (REF cmd/agent/main.go:137-302,
SURVEY §2.8) plus the GPU window engine's metrics (additive, ``llm_slo_agent_gpu_*``).

GPU histograms arrive as per-window bucket counts from the decode kernel (LDS-privatised,
RCCL all-reduced across GPUs); ``observe_window_hist`` folds them into Prometheus
histograms without re-observing events. The kernel's buckets are ``le`` buckets
(v in (edge[b-1], edge[b]]) over the catalogue edges, of which REF's DNS edges
{1..800} are a prefix, so the REF-named DNS histogram keeps exact ``le`` semantics.
"""

from __future__ import annotations

import os
import time
from typing import Iterable, Sequence

import numpy as np

from ..contracts.types import ProbeEventV1
from ..export.prometheus import Registry
from ..signals import catalog

EVENT_KINDS = ("slo", "probe", "both")
DROP_REASONS = ("rate_limit", "schema", "emit", "xchg_cap", "import_cap")


def _nz(v: str, fallback: str) -> str:
    v = (v or "").strip()
    return v if v else fallback


class AgentMetrics:
    def __init__(self, event_kind: str, capability_mode: str, supported: Sequence[str], enabled: Sequence[str]):
        r = self.registry = Registry()
        self.heartbeat = r.gauge("llm_slo_agent_heartbeat", "Unix timestamp of latest emitted sample.")
        self.up = r.gauge("llm_slo_agent_up", "Agent process liveness.")
        self.cpu = r.gauge("llm_slo_agent_cpu_overhead_pct", "Estimated agent CPU overhead percentage.")
        self.kind = r.gauge("llm_slo_agent_event_kind", "Selected event-kind mode (one-hot gauge).", ("kind",))
        self.mode = r.gauge("llm_slo_agent_capability_mode", "Detected capability mode (one-hot gauge).", ("mode",))
        self.sig_enabled = r.gauge("llm_slo_agent_signal_enabled", "Signal enablement toggle by signal name.",
                                   ("signal",))
        self.dropped = r.counter("llm_slo_agent_dropped_events_total", "Dropped probe events by reason.", ("reason",))
        self.hello = r.counter("llm_ebpf_hello_syscalls_total", "Hello tracer syscall events by comm.",
                               ("node", "pod", "comm"))
        self.dns = r.histogram("llm_ebpf_dns_latency_ms", "DNS latency observed from probe events.",
                               catalog.REF_DNS_BUCKETS, ("node", "pod", "namespace"))
        self.probe_events = r.counter("llm_ebpf_probe_events_total", "Probe events observed by signal and status.",
                                      ("signal", "status"))
        # ---- GPU window engine (additive) ----
        self.win_events = r.counter("llm_slo_agent_gpu_window_events_total", "Events processed by the GPU engine.")
        self.win_total = r.counter("llm_slo_agent_gpu_windows_total", "Windows processed by the GPU engine.")
        self.win_latency = r.histogram("llm_slo_agent_gpu_window_latency_ms",
                                       "Ring drain to attribution latency per window.",
                                       (0.5, 1, 2, 5, 10, 20, 50, 100, 200, 500, 1000))
        self.attr = r.counter("llm_slo_agent_attributions_total", "Incident attributions by predicted domain.",
                              ("domain",))
        self.scored = r.counter("llm_slo_agent_incidents_scored_total",
                                "Incident groups scored per window by top domain, and whether an attribution was "
                                "emitted (only groups with SLO impact are).", ("domain", "emitted"))
        self.corr = r.counter("llm_slo_agent_correlation_pairs_total",
                              "Span/signal correlation outcomes (REF DebugStats) from the join kernel.", ("outcome",))
        self.ring_dropped = r.gauge("llm_slo_agent_ring_dropped_events", "Events dropped by full producer rings.")
        self.ring_defs = r.counter("llm_slo_agent_ring_definitions_total",
                                   "Context / trace id definition records consumed from the BPF ring.")
        self.ring_busy = r.counter("llm_slo_agent_ring_busy_stops_total",
                                   "Windows whose ring consumption stopped at a record still being written.")
        self.ring_backlog = r.gauge("llm_slo_agent_ring_backlog_bytes", "Unconsumed bytes in the BPF ring buffer.")
        self.flush_loaded = r.gauge("llm_slo_agent_flush_program_loaded",
                                    "1 when the cut's per-CPU flush program (mislo_flush) is pinned and run.")
        self.flush_errors = r.gauge("llm_slo_agent_flush_errors",
                                    "Per-CPU flush runs that failed (other than offline CPUs), since start.")
        self.host_us = r.gauge("llm_slo_agent_window_host_us", "Host time to assemble the last window (us).")
        self.windows_skipped = r.counter("llm_slo_agent_windows_skipped_total",
                                         "Window cuts skipped after the loop stalled for more than a window period.")
        self.workers = r.gauge("llm_slo_agent_window_workers", "Window workers (GPUs) the agent is running.")
        self.worker_restarts = r.counter("llm_slo_agent_worker_restarts_total",
                                         "Worker pool restarts after a worker died (the survivors' GPUs go on).")
        self.rss = r.gauge("llm_slo_agent_memory_rss_bytes", "Agent process resident set size (bytes).")
        self.otlp = r.gauge("llm_slo_agent_otlp_spans", "OTLP receiver span records since start by outcome: accepted "
                            "into the span ring, dropped (ring full), rejected (malformed export), conflict (a pod "
                            "bound to another service), spoofed (a pod named from another pod's address), "
                            "first_token_late (a first-token record after its request span, which counted it).",
                            ("outcome",))
        self.cg_mem = r.gauge("llm_slo_agent_memory_cgroup_bytes",
                              "Memory charged to the agent's cgroup (v2 memory.current, v1 usage_in_bytes): what a "
                              "pod memory limit is enforced on, next to RSS.")
        self.burn_err = r.gauge("llm_slo_agent_burn_rate_prediction_error",
                                "Mean relative error of the scored SLO burn-rate forecasts.")
        # GPU signals' value distributions (the window histograms the decode kernel builds)
        self.gpu_hist = {s.slot: r.histogram(f"llm_ebpf_{s.name}", f"{s.name} values observed from GPU signal records.",
                                             s.buckets)
                         for s in catalog.SIGNALS if s.gpu and s.buckets}
        self.up.set(1)
        for k in EVENT_KINDS:
            self.kind.set(1 if k == event_kind else 0, k)
        for m in catalog.CAPABILITY_MODES:
            self.mode.set(1 if m == capability_mode else 0, m)
        for reason in DROP_REASONS:
            self.dropped.inc(0, reason)
        self.set_enabled_signals(supported, enabled)

    def set_heartbeat(self, ts_s: float = 0.0) -> None:
        self.heartbeat.set(float(int(ts_s or time.time())))

    def set_cpu_overhead(self, pct: float) -> None:
        self.cpu.set(max(0.0, pct))

    def set_rss(self) -> None:
        try:
            with open("/proc/self/statm") as f:
                self.rss.set(float(int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")))
        except (OSError, ValueError, IndexError):
            pass
        from ..utils import cgroupmem

        cg = cgroupmem.reading()
        if cg is not None:
            self.cg_mem.set(float(cg["charged_bytes"]))

    def set_enabled_signals(self, supported: Iterable[str], enabled: Iterable[str]) -> None:
        en = set(enabled)
        for s in supported:
            self.sig_enabled.set(1 if s in en else 0, s)

    def observe_probe_event(self, ev: ProbeEventV1, real_probe_metrics: bool = True) -> None:
        self.probe_events.inc(1, ev.signal, ev.status)
        if real_probe_metrics and ev.signal == "dns_latency_ms":
            self.dns.observe(ev.value, _nz(ev.node, "unknown-node"), _nz(ev.pod, "unknown-pod"),
                             _nz(ev.namespace, "default"))

    def inc_dropped(self, reason: str) -> None:
        self.dropped.inc(1, reason)

    def inc_hello(self, node: str, pod: str, comm: str, count: int) -> None:
        if count:
            self.hello.inc(float(count), _nz(node, "unknown-node"), _nz(pod, "unknown-pod"), _nz(comm, "unknown"))

    # ---- GPU window outputs -------------------------------------------------------------
    def observe_window(self, hist: np.ndarray, status: np.ndarray, dbg, n_events: int, latency_ms: float,
                       node: str, pod: str, namespace: str, value_sums_milli=None) -> None:
        """hist [16 slots x 16 buckets], status [16 x 3], value sums (1/1000 unit) per slot from the
        window packet."""
        self.win_total.inc()
        self.win_events.inc(float(n_events))
        self.win_latency.observe(latency_ms)
        dns = catalog.BY_NAME["dns_latency_ms"].slot
        h = np.asarray(hist[dns], dtype=np.float64)
        nref = len(catalog.REF_DNS_BUCKETS)
        ref_counts = list(h[:nref]) + [float(h[nref:].sum())]  # buckets above 800 -> +Inf
        self.dns.add_counts(ref_counts, 0.0, _nz(node, "unknown-node"), _nz(pod, "unknown-pod"),
                            _nz(namespace, "default"))
        for slot, hm in self.gpu_hist.items():
            row = np.asarray(hist[slot], dtype=np.float64)
            nb = len(hm.buckets)
            if row[: nb + 1].sum():
                total = float(value_sums_milli[slot]) * 1e-3 if value_sums_milli is not None else 0.0
                hm.add_counts(list(row[:nb - 1]) + [float(row[nb - 1:].sum())], total)
        names = ("ok", "warning", "error")
        for s in catalog.SIGNALS:
            row = status[s.slot]
            for k in range(3):
                if row[k]:
                    self.probe_events.inc(float(row[k]), s.name, names[k])
        cand, low, overlap, dropped, enriched = (int(x) for x in list(dbg)[:5])
        d = list(dbg)
        if len(d) > 6:  # the multi-GPU exchange's losses (mislo_packet.h kDbgXchgDropped / kDbgImportDropped)
            if d[5]:
                self.dropped.inc(float(d[5]), "xchg_cap")
            if d[6]:
                self.dropped.inc(float(d[6]), "import_cap")
        self.corr.inc(float(cand), "candidate")
        self.corr.inc(float(max(0, low - overlap)), "low_confidence")
        self.corr.inc(float(dropped), "fanout_dropped")
        self.corr.inc(float(enriched), "span_enriched")

    def set_ring(self, ring_stats: dict, ring_state: dict, host_us: float) -> None:
        """Per-window ring accounting (counted on the device): id definitions applied, windows
        that met a record still being written, backlog, drops (the emulated ring counts failed
        reservations; the kernel's are invisible to user space), host time per window."""
        self.ring_defs.inc(float(ring_state.get("def_ctx", 0) + ring_state.get("def_trace", 0)))
        if ring_state.get("first_busy", -1) >= 0:
            self.ring_busy.inc()
        if ring_stats:
            self.ring_backlog.set(float(ring_stats.get("producer_pos", 0) - ring_stats.get("consumer_pos", 0)))
            self.ring_dropped.set(float(ring_stats.get("dropped", 0)))
        self.host_us.set(float(host_us))

    def set_otlp(self, receiver, mapper) -> None:
        """The OTLP receiver's and span mapper's running counts (collector/otlp.py)."""
        for outcome, v in (("accepted", getattr(receiver, "accepted", 0)), ("dropped", getattr(receiver, "dropped", 0)),
                           ("rejected", getattr(receiver, "rejected", 0)), ("conflict", getattr(mapper, "conflicts", 0)),
                           ("spoofed", getattr(mapper, "spoofed", 0)),
                           ("first_token_late", getattr(mapper, "early_dropped", 0))):
            self.otlp.set(float(v), outcome)

    def observe_attribution(self, domain: str) -> None:
        self.attr.inc(1, domain)

    def observe_incident(self, domain: str, emitted: bool) -> None:
        self.scored.inc(1, domain, "true" if emitted else "false")

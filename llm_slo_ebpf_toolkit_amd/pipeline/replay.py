"""Seeded fault-replay world: time-ordered probe events + spans + labelled incident groups.

This is the synthetic trace generator behind the benchmark and the GPU tests (the
"fault-replay scenarios" of BASELINE.json). Unlike REF's replay (pkg/faultreplay/
generator.go:20-116), whose samples carry no signals at all, every incident here is
observable only through correlated kernel/GPU events:

* a shard (one GPU / one node-agent) has ``n_nodes x pods_per_node`` pods spread over
  ``n_services`` services; each (service, window) is one incident group whose label is
  drawn from the scenario (REF label sets; "baseline" = no fault -> domain "unknown");
* spans are requests on a pod's serving pid / connection, with a random trace id;
* request-context events (dns/connect/tls/syscall/tcp) carry the request's pid, conn
  tuple and usually its trace id, a few ms around the span (tiers 1-3);
  background events (sched/mm/blk/GPU) land on the pod's pids with no trace (tier 2);
* event values follow REF's per-fault signal profiles (pkg/signals/generator.go:244-289,
  extended with GPU faults) with lognormal jitter (continuous) or Poisson (counts).

Records use the 64-byte EVENT/SPAN layouts (collector/records.py), raw values in each
signal's kernel unit, so the GPU decode path is exercised exactly as in production.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..collector import records
from ..models.sample import map_fault_label
from ..signals import catalog
from ..signals.generator import BASE_PROFILE, FAULT_OVERRIDES, FAULT_ERRNO

SCENARIOS: Dict[str, List[Tuple[str, ...]]] = {
    "baseline": [()],
    # the same fault-free node under another name: the agent's replay source reads its REF-default
    # --scenario "baseline" as "full" (a replay with nothing to attribute is no demo)
    "healthy": [()],
    "dns_latency": [("dns_latency",)],
    "cpu_throttle": [("cpu_throttle",)],
    "memory_pressure": [("memory_pressure",)],
    "provider_throttle": [("provider_throttle",)],
    "network_partition": [("network_partition",)],
    "gpu_contention": [("gpu_contention",)],
    "rccl_latency": [("rccl_latency",)],
    # REF faultreplay "mixed" label set (generator.go:16)
    "mixed": [("provider_throttle",), ("dns_latency",), ("cpu_throttle",), ("memory_pressure",),
              ("network_partition",)],
    # REF faultreplay mixed_multi pairs (generator.go:61-66)
    "mixed_multi": [("provider_throttle", "dns_latency"), ("cpu_throttle", "memory_pressure"),
                    ("network_partition", "dns_latency"), ("provider_throttle", "network_partition")],
    # NEW: every single fault incl. the MI355X GPU faults (config 5: all fault domains)
    "full": [("provider_throttle",), ("dns_latency",), ("cpu_throttle",), ("memory_pressure",),
             ("network_partition",), ("gpu_contention",), ("rccl_latency",), ("provider_error",),
             ("retrieval_slowdown",)],
    # the two REF domains REF's own generator cannot produce (mapper.go:43-46)
    "provider_error": [("provider_error",)],
    "retrieval_slowdown": [("retrieval_slowdown",)],
    # NEW: the live-node shapes of the CPU and GPU contention domains (signals/generator.py
    # cpu_contention, gpu_compute_contention) next to REF's, alone and with a network fault
    "live": [("cpu_contention",), ("gpu_compute_contention",), ("cpu_throttle",), ("gpu_contention",),
             ("cpu_contention", "network_partition"), ("gpu_compute_contention", "network_partition"),
             ("network_partition",), ("dns_latency",)],
}

COUNT_SIGNALS = {"tcp_retransmits_total", "connect_errors_total", "tls_handshake_fail_total"}
# Level gauges of a shared resource (a GPU's HBM in use): every reader sees nearly the same value,
# bounded by 100 %, not a per-event latency with a heavy tail
GAUGE_SIGMA = {"hbm_pressure_pct": 0.03}
CTX_SIGNALS = {"dns_latency_ms": .22, "connect_latency_ms": .2, "connect_errors_total": .06,
               "tls_handshake_ms": .18, "tls_handshake_fail_total": .05, "syscall_latency_ms": .17,
               "tcp_retransmits_total": .12}
BG_SIGNALS = {"runqueue_delay_ms": .13, "cpu_steal_pct": .09, "cfs_throttled_ms": .09,
              "mem_reclaim_latency_ms": .09, "disk_io_latency_ms": .09, "syscall_latency_ms": .08,
              "gpu_queue_delay_ms": .09, "hbm_pressure_pct": .07, "xgmi_link_latency_us": .07,
              "rccl_collective_ms": .07, "dns_latency_ms": .03, "tcp_retransmits_total": .04,
              "connect_latency_ms": .03, "tls_handshake_ms": .03}

UNSUPPORTED_TYPE = 99


@dataclass
class ReplayConfig:
    scenario: str = "full"
    n_nodes: int = 4
    pods_per_node: int = 64
    n_services: int = 64
    events_per_window: int = 1 << 20
    spans_per_window: int = 16384
    window_ms: int = 1000
    p_fault: float = 0.7
    ctx_frac: float = 0.35
    ctx_trace_prob: float = 0.8
    ctx_jitter_ms: float = 40.0
    jitter_sigma: float = 0.3
    unsupported_frac: float = 0.002
    seed: int = 42
    shard: int = 0
    start_ns: int = 1_760_000_000 * 1_000_000_000
    # windows a drawn fault assignment persists (faults last minutes in REF's incident-lab
    # phases, test/incident-lab/scenarios/*.yaml): with a halo, a window joins the previous
    # window's boundary rows, which must carry the same faults
    fault_hold: int = 1
    # symptom variability: each of a fault's elevated symptoms shows in an incident with this
    # probability (at least one always does). 1.0 = every symptom of REF's profile, every time
    # (REF's generator.go:244-289). REF's expert columns say real incidents are not that clean
    # (P(connect elevated | network_dns) = .50, bayesian.go:67-190): a model trained only on
    # complete profiles learns that a DNS fault always slows connects and then misses the DNS
    # incident whose connects stayed fast (REF row mf-51).
    symptom_keep: float = 1.0

    @property
    def n_pods(self) -> int:
        return self.n_nodes * self.pods_per_node


@dataclass
class ReplayWindow:
    index: int
    t0_ns: int
    events: np.ndarray           # EVENT[N]
    spans: np.ndarray            # SPAN[S]
    group_labels: np.ndarray     # int32[G] primary domain index
    group_faults: List[Tuple[str, ...]]
    group_domains: List[List[str]]
    n_groups: int

    @property
    def n_events(self) -> int:
        return int(self.events.shape[0])

    @property
    def n_spans(self) -> int:
        return int(self.spans.shape[0])


# Round 3 coupled cpu_throttle to GPU queue delay here (a CPU-starved launcher's dispatches
# queued behind its own burst read as GPU delay: profiles/r3_config3_*). The rocprofiler tool no
# longer counts waits behind the process's own queue, only waits above 10 ms and GPU time other
# processes hold (tests/test_rocprof_tool.py), none of which a CPU fault produces -- and with the
# coupling, a GPU-only node read real GPU contention as a CPU fault (profiles/r4_config2_first).
GPU_SERVED_COUPLING: Dict[str, Dict[str, float]] = {}


def _symptoms(lab: str, rng: Optional[np.random.Generator], keep: float) -> Dict[str, float]:
    """A fault's overrides in one incident: every elevated symptom with probability ``keep``
    (at least one of them), the sub-threshold ones always."""
    over = dict(FAULT_OVERRIDES.get(lab, {}))
    over.update(GPU_SERVED_COUPLING.get(lab, {}))
    if rng is None or keep >= 1.0:
        return over
    elev = [k for k, v in over.items() if v >= catalog.BY_NAME[k].elevated]
    if not elev:
        return over
    kept = [k for k in elev if rng.random() < keep]
    if not kept:
        kept = [elev[int(rng.integers(len(elev)))]]
    return {k: v for k, v in over.items() if k in kept or k not in elev}


def _profile(labels: Sequence[str], rng: Optional[np.random.Generator] = None, keep: float = 1.0) -> Dict[str, float]:
    prof = dict(BASE_PROFILE)
    for lab in labels:
        over = _symptoms(lab, rng, keep)
        for k, v in over.items():
            # multi-fault: the more severe symptom wins (latency up / tps down are both "up" here)
            prof[k] = max(prof[k], v) if k in prof else v
    return prof


def _sli(labels: Sequence[str]):
    from ..collector.pipeline import BASE_SLI, SLI_PROFILE

    if not labels:
        return BASE_SLI
    if len(labels) > 1:
        return SLI_PROFILE.get("mixed_multi", BASE_SLI)
    return SLI_PROFILE.get(labels[0], BASE_SLI)


def expected_domains(labels: Sequence[str]) -> List[str]:
    out: List[str] = []
    for lab in labels:
        d = map_fault_label(lab)
        if d != "unknown" and d not in out:
            out.append(d)
    return out or ["unknown"]


class ReplayGenerator:
    def __init__(self, cfg: ReplayConfig):
        if cfg.scenario not in SCENARIOS:
            raise ValueError(f"unsupported scenario {cfg.scenario!r}")
        self.cfg = cfg
        self.rng = np.random.default_rng([cfg.seed, cfg.shard])
        P = cfg.n_pods
        self.pod_ids = np.arange(1, P + 1, dtype=np.uint32) + np.uint32(cfg.shard * P)
        self.pod_node = (np.arange(P) // cfg.pods_per_node + 1 + cfg.shard * cfg.n_nodes).astype(np.uint16)
        self.pod_svc_idx = (np.arange(P) % cfg.n_services).astype(np.int64)
        self.pod_svc = (self.pod_svc_idx + 1).astype(np.uint16)
        self.pod_pid = (10_000 + np.arange(P) * 8).astype(np.uint32)
        ports = self.rng.integers(20_000, 60_000, size=P)
        self.pod_conn = records.conn_hash_np(ports.astype(np.uint16), np.full(P, 443, np.uint16),
                                             (0x0A000000 + np.arange(P)).astype(np.uint32))
        self.pod_sport = ports.astype(np.uint16)
        self.slot_of = {s.name: s.slot for s in catalog.SIGNALS}
        self.window = 0

    # ---------------------------------------------------------------------------------
    def _labels(self) -> List[Tuple[str, ...]]:
        cfg = self.cfg
        choices = SCENARIOS[cfg.scenario]
        out: List[Tuple[str, ...]] = []
        for _ in range(cfg.n_services):
            if choices != [()] and self.rng.random() < cfg.p_fault:
                out.append(choices[int(self.rng.integers(len(choices)))])
            else:
                out.append(())
        return out

    def _values(self, sig_names: np.ndarray, grp: np.ndarray, profiles: List[Dict[str, float]]) -> np.ndarray:
        """Physical values (signal unit) for events of signal ``sig_names`` in groups ``grp``."""
        n = sig_names.shape[0]
        out = np.zeros(n, dtype=np.float64)
        G = len(profiles)
        for name in np.unique(sig_names):
            m = sig_names == name
            prof = np.array([profiles[g][name] for g in range(G)], dtype=np.float64)[grp[m]]
            if name in COUNT_SIGNALS:
                out[m] = self.rng.poisson(prof)
            elif name in GAUGE_SIGMA:
                out[m] = np.minimum(100.0, prof * np.exp(self.rng.normal(0.0, GAUGE_SIGMA[name], size=int(m.sum()))))
            else:
                out[m] = prof * np.exp(self.rng.normal(0.0, self.cfg.jitter_sigma, size=int(m.sum())))
        return out

    def next_window(self) -> ReplayWindow:
        cfg = self.cfg
        rng = self.rng
        w = self.window
        self.window += 1
        W = cfg.window_ms * 1_000_000
        t0 = cfg.start_ns + w * W
        if w % max(1, cfg.fault_hold) == 0 or getattr(self, "_faults", None) is None:
            self._faults = self._labels()
        faults = self._faults
        if w % max(1, cfg.fault_hold) == 0 or getattr(self, "_profiles", None) is None:
            # drawn with the assignment: a held fault keeps its symptoms across windows
            self._profiles = [_profile(f, self.rng, cfg.symptom_keep) for f in faults]
        profiles = self._profiles
        G = cfg.n_services
        P = cfg.n_pods

        # --- spans ---
        S = cfg.spans_per_window
        sp = np.zeros(S, dtype=records.SPAN)
        sp_pod = rng.integers(0, P, size=S)
        sp_ts = np.sort(t0 + rng.integers(0, W, size=S))
        sp["ts_ns"] = sp_ts
        sp["trace_h"] = rng.integers(1, np.iinfo(np.int64).max, size=S, dtype=np.int64).astype(np.uint64)
        sp["conn_h"] = self.pod_conn[sp_pod]
        sp["pid"] = self.pod_pid[sp_pod]
        sp["pod_id"] = self.pod_ids[sp_pod]
        sp["node_id"] = self.pod_node[sp_pod]
        sp["svc_id"] = self.pod_svc[sp_pod]
        sp["group_id"] = self.pod_svc_idx[sp_pod].astype(np.uint32)
        sp["span_h"] = rng.integers(1, np.iinfo(np.int64).max, size=S, dtype=np.int64).astype(np.uint64)
        # request SLIs from REF's per-fault SLI profiles (pkg/collector/synthetic.go:80-132), jittered
        grp_sp = self.pod_svc_idx[sp_pod]
        ttft = np.array([_sli(faults[g])[0] for g in range(G)], dtype=np.float64)[grp_sp]
        lat = np.array([_sli(faults[g])[1] for g in range(G)], dtype=np.float64)[grp_sp]
        jit = np.exp(self.rng.normal(0.0, 0.25, size=S))
        sp["ttft_ms"] = (ttft * jit).astype(np.float32)
        sp["latency_ms"] = (lat * jit).astype(np.float32)

        # --- events ---
        N = cfg.events_per_window
        n_ctx = int(N * cfg.ctx_frac)
        n_uns = int(N * cfg.unsupported_frac)
        n_bg = N - n_ctx - n_uns
        ev = np.zeros(N, dtype=records.EVENT)

        ctx_names = np.array(list(CTX_SIGNALS))
        ctx_w = np.array(list(CTX_SIGNALS.values()))
        bg_names = np.array(list(BG_SIGNALS))
        bg_w = np.array(list(BG_SIGNALS.values()))

        # request-context events, attached to spans
        j = rng.integers(0, S, size=n_ctx)
        pod_c = sp_pod[j]
        names_c = ctx_names[rng.choice(len(ctx_names), size=n_ctx, p=ctx_w / ctx_w.sum())]
        jit = rng.uniform(-cfg.ctx_jitter_ms, cfg.ctx_jitter_ms, size=n_ctx) * 1e6
        ts_c = sp_ts[j] + jit.astype(np.int64)
        has_tr = rng.random(n_ctx) < cfg.ctx_trace_prob
        # background events
        pod_b = rng.integers(0, P, size=n_bg)
        names_b = bg_names[rng.choice(len(bg_names), size=n_bg, p=bg_w / bg_w.sum())]
        ts_b = t0 + rng.integers(0, W, size=n_bg)

        names = np.concatenate([names_c, names_b])
        pods = np.concatenate([pod_c, pod_b])
        grp = self.pod_svc_idx[pods]
        vals = self._values(names, grp, profiles)

        sl = slice(0, n_ctx + n_bg)
        ev_main = ev[sl]
        ev_main["ts_ns"] = np.concatenate([ts_c, ts_b])
        stype = np.zeros(n_ctx + n_bg, dtype=np.uint16)
        scale = np.zeros(n_ctx + n_bg, dtype=np.float64)
        for spec in catalog.SIGNALS:
            m = names == spec.name
            stype[m] = spec.kernel_type
            scale[m] = spec.decode_scale
        ev_main["signal_type"] = stype
        ev_main["value"] = np.round(vals / scale).astype(np.uint64)
        ev_main["trace_h"] = np.concatenate([np.where(has_tr, sp["trace_h"][j], 0).astype(np.uint64),
                                             np.zeros(n_bg, dtype=np.uint64)])
        other_pid = self.pod_pid[pod_b] + rng.integers(1, 8, size=n_bg).astype(np.uint32)
        main_pid = rng.random(n_bg) < 0.6
        ev_main["pid"] = np.concatenate([self.pod_pid[pod_c], np.where(main_pid, self.pod_pid[pod_b], other_pid)])
        ev_main["tid"] = ev_main["pid"]
        ev_main["pod_id"] = self.pod_ids[pods]
        ev_main["node_id"] = self.pod_node[pods]
        ev_main["svc_id"] = self.pod_svc[pods]
        net_bg = np.isin(names_b, list(CTX_SIGNALS)) & (rng.random(n_bg) < 0.5)
        conn = np.concatenate([self.pod_conn[pod_c], np.where(net_bg, self.pod_conn[pod_b], 0).astype(np.uint64)])
        ev_main["conn_h"] = conn
        has_conn = conn != 0
        ev_main["src_port"] = np.where(has_conn, self.pod_sport[pods], 0)
        ev_main["dst_port"] = np.where(has_conn, 443, 0)
        ev_main["dst_ip"] = np.where(has_conn, (0x0A000000 + (pods % 65536)).astype(np.uint32), 0)
        errno = np.zeros(n_ctx + n_bg, dtype=np.int32)
        for g, f in enumerate(faults):
            e = max((FAULT_ERRNO.get(x, 0) for x in f), default=0)
            if e:
                errno[(grp == g) & np.isin(names, ["connect_latency_ms", "connect_errors_total"])] = e
        ev_main["errno"] = errno
        gpu = np.isin(names, list(catalog.GPU_SIGNALS))
        ev_main["flags"] = np.where(gpu, records.FLAG_HAS_GPU | (pods % 8), 0).astype(np.uint16) | records.FLAG_SYNTHETIC
        ev[sl] = ev_main
        # unsupported / unknown-type noise (exercises the unsupported_type path)
        if n_uns:
            u = ev[n_ctx + n_bg:]
            up = rng.integers(0, P, size=n_uns)
            u["ts_ns"] = t0 + rng.integers(0, W, size=n_uns)
            u["signal_type"] = UNSUPPORTED_TYPE
            u["value"] = 1
            u["pid"] = self.pod_pid[up]
            u["pod_id"] = self.pod_ids[up]
            u["node_id"] = self.pod_node[up]
            u["svc_id"] = self.pod_svc[up]
            ev[n_ctx + n_bg:] = u
        # arrival order = time order (ring producers emit monotonically per CPU; the window
        # is merged by timestamp)
        ev = ev[np.argsort(ev["ts_ns"], kind="stable")]

        labels = np.array([catalog.DOMAIN_INDEX[expected_domains(f)[0]] for f in faults], dtype=np.int32)
        return ReplayWindow(w, t0, ev, sp, labels, faults, [expected_domains(f) for f in faults], G)


def window_fault_samples(win: ReplayWindow, features: np.ndarray, cluster: str = "local",
                         namespace: str = "default"):
    """Turn a window's incident features [G,16] into REF FaultSamples (for CPU attribution
    and the artefact bundle)."""
    from ..models.sample import FaultSample

    out = []
    for g in range(win.n_groups):
        sig = {catalog.SIGNAL_NAMES[s]: float(features[g, s]) for s in range(catalog.N_SLOTS)
               if not np.isnan(features[g, s])}
        faults = win.group_faults[g]
        doms = win.group_domains[g]
        out.append(FaultSample(
            incident_id=f"replay-w{win.index:05d}-g{g:03d}", timestamp=win.t0_ns, cluster=cluster,
            namespace=namespace, service=f"svc-{g + 1}", fault_label="+".join(faults) if faults else "baseline",
            expected_domain=doms[0], expected_domains=list(doms) if len(doms) > 1 else [],
            signals=sig, confidence=0.9, burn_rate=2.0, window_minutes=5,
            request_id=f"replay-req-{win.index:05d}-{g:03d}", trace_id=f"replay-trace-{win.index:05d}-{g:03d}"))
    return out

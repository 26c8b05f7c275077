"""Signal catalogue: the single source of truth for every signal and fault domain.

Everything that needs per-signal facts (decoder scale tables, status thresholds,
Bayes "elevated" thresholds, semconv keys, shed order, histogram buckets, the
16-slot feature layout used by the GPU kernels) derives from the tables here.

Reference parity (REF = ogulcanaydogan/llm-slo-ebpf-toolkit):
  * signal names / core set / BCC set / shed order: pkg/signals/constants.go:5-82
  * kernel type ids 1..9:                       pkg/collector/ringbuf.go:29-39
  * status warn/error thresholds:               pkg/signals/generator.go:203-232
  * Bayes elevated thresholds:                  pkg/attribution/bayesian.go:194-207
  * semconv attribute keys:                     pkg/semconv/llm_ebpf.go:3-27
  * likelihood table 12x8 + domain order:       pkg/attribution/bayesian.go:23-34,67-190
  * DNS histogram buckets:                      cmd/agent/main.go:190-194

NEW additions (additive, MI355X-specific): four GPU signals fed by the
rocprofiler-sdk tool library and the amdgpu/KFD + HIP/RCCL probes, and two GPU
fault domains. The feature layout is exactly 16 slots so the posterior/statistics
MFMA kernels run with K = 16 and no padding.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

INF = float("inf")

# --------------------------------------------------------------------------------------
# Signals
# --------------------------------------------------------------------------------------


@dataclass(frozen=True)
class SignalSpec:
    name: str
    slot: int                      # feature slot 0..15 (GPU kernel layout)
    unit: str                      # unit after decode
    kernel_type: int               # record signal_type id (0 = none)
    decode_scale: float            # raw record value * scale -> unit
    warn: float                    # status "warning" cutoff (>=)
    error: float                   # status "error" cutoff (>=)
    elevated: float                # Bayes evidence threshold (>=)
    semconv: str                   # span attribute key
    shed_rank: int                 # 1 = shed first under overhead pressure
    in_config_enum: bool           # allowed in toolkit config signal_set
    gpu: bool = False
    buckets: Tuple[float, ...] = field(default_factory=tuple)


_MS_BUCKETS = (1, 2, 5, 10, 20, 40, 80, 120, 200, 400, 800, 1600, 3200, 6400, INF)
_COUNT_BUCKETS = (0, 1, 2, 3, 5, 8, 13, 21, 34, 55, 89, 144, 233, 377, INF)
_PCT_BUCKETS = (0.5, 1, 2, 4, 8, 16, 25, 40, 50, 60, 70, 80, 90, 95, INF)
_US_BUCKETS = (1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, 2000, 5000, 10000, 20000, INF)

# The REF DNS histogram buckets (cmd/agent/main.go:190-194) are a prefix of _MS_BUCKETS,
# so the Prometheus `le` series for llm_ebpf_dns_latency_ms keep REF's edges.
REF_DNS_BUCKETS = (1, 2, 5, 10, 20, 40, 80, 120, 200, 400, 800)

SIGNALS: Tuple[SignalSpec, ...] = (
    SignalSpec("dns_latency_ms", 0, "ms", 1, 1e-6, 40, 120, 40, "llm.ebpf.dns.latency_ms", 10, True, buckets=_MS_BUCKETS),
    SignalSpec("tcp_retransmits_total", 1, "count", 2, 1.0, 2, 5, 2, "llm.ebpf.tcp.retransmits", 11, True, buckets=_COUNT_BUCKETS),
    SignalSpec("runqueue_delay_ms", 2, "ms", 3, 1e-6, 10, 25, 10, "llm.ebpf.sched.runqueue_delay_ms", 5, True, buckets=_MS_BUCKETS),
    SignalSpec("connect_latency_ms", 3, "ms", 4, 1e-6, 80, 180, 80, "llm.ebpf.net.connect_latency_ms", 7, True, buckets=_MS_BUCKETS),
    SignalSpec("connect_errors_total", 4, "count", 10, 1.0, 1, 3, 1, "llm.ebpf.net.connect_errors_total", 13, False, buckets=_COUNT_BUCKETS),
    SignalSpec("tls_handshake_ms", 5, "ms", 5, 1e-6, 60, 160, 60, "llm.ebpf.tls.handshake_ms", 3, True, buckets=_MS_BUCKETS),
    SignalSpec("tls_handshake_fail_total", 6, "count", 11, 1.0, 1, 3, 1, "llm.ebpf.tls.handshake_fail_total", 14, False, buckets=_COUNT_BUCKETS),
    SignalSpec("cpu_steal_pct", 7, "pct", 6, 1e-3, 2, 8, 2, "llm.ebpf.cpu.steal_pct", 9, True, buckets=_PCT_BUCKETS),
    # in the config enum (NEW, additive: REF's enum omits it although its generator and Bayes
    # table use it; cfs_throttle.bpf.c and the procfs sampler produce it here)
    SignalSpec("cfs_throttled_ms", 8, "ms", 12, 1e-6, 40, 120, 40, "llm.ebpf.cpu.cfs_throttled_ms", 12, True, buckets=_MS_BUCKETS),
    SignalSpec("mem_reclaim_latency_ms", 9, "ms", 7, 1e-6, 5, 20, 5, "llm.ebpf.mm.reclaim_latency_ms", 8, True, buckets=_MS_BUCKETS),
    SignalSpec("disk_io_latency_ms", 10, "ms", 8, 1e-6, 10, 50, 10, "llm.ebpf.blk.io_latency_ms", 6, True, buckets=_MS_BUCKETS),
    SignalSpec("syscall_latency_ms", 11, "ms", 9, 1e-6, 50, 200, 50, "llm.ebpf.syscall.latency_ms", 4, True, buckets=_MS_BUCKETS),
    # --- GPU signals (NEW, MI355X) ---
    # queue delay: a healthy MI355X starts a kernel well under 1 ms after enqueue (config-2
    # baseline: no record above the tool's 0.2 ms floor); under contention the mean sits at
    # ~5 ms with 85 % of records >= 2 ms (profiles/r2_config2_gpu_contention) -> elevated at 2 ms
    SignalSpec("gpu_queue_delay_ms", 12, "ms", 13, 1e-6, 2, 10, 2, "llm.ebpf.gpu.queue_delay_ms", 1, True, gpu=True, buckets=_MS_BUCKETS),
    SignalSpec("hbm_pressure_pct", 13, "pct", 14, 1e-3, 85, 95, 85, "llm.ebpf.gpu.hbm_pressure_pct", 15, True, gpu=True, buckets=_PCT_BUCKETS),
    SignalSpec("xgmi_link_latency_us", 14, "us", 15, 1e-3, 10, 50, 10, "llm.ebpf.gpu.xgmi_link_latency_us", 16, True, gpu=True, buckets=_US_BUCKETS),
    SignalSpec("rccl_collective_ms", 15, "ms", 16, 1e-6, 5, 20, 5, "llm.ebpf.gpu.rccl_collective_ms", 2, True, gpu=True, buckets=_MS_BUCKETS),
)

N_SLOTS = 16
assert len(SIGNALS) == N_SLOTS and [s.slot for s in SIGNALS] == list(range(N_SLOTS))

BY_NAME: Dict[str, SignalSpec] = {s.name: s for s in SIGNALS}
BY_TYPE: Dict[int, SignalSpec] = {s.kernel_type: s for s in SIGNALS if s.kernel_type}
SIGNAL_NAMES: Tuple[str, ...] = tuple(s.name for s in SIGNALS)

HELLO_SIGNAL = "hello_sys_enter_write_total"
HELLO_TYPE = 100

# REF constants.go:28-41 (order preserved)
CORE_SIGNALS: Tuple[str, ...] = SIGNAL_NAMES[:12]
# REF constants.go:42-45
BCC_SIGNALS: Tuple[str, ...] = ("dns_latency_ms", "tcp_retransmits_total")
GPU_SIGNALS: Tuple[str, ...] = SIGNAL_NAMES[12:]
# REF constants.go:63-72
REQUIRED_MINIMUM: Tuple[str, ...] = (
    "dns_latency_ms", "tcp_retransmits_total", "runqueue_delay_ms",
    "connect_latency_ms", "tls_handshake_ms", "cpu_steal_pct",
)
# REF config default signal_set (pkg/toolkitcfg/config.go:68-78)
DEFAULT_CONFIG_SIGNALS: Tuple[str, ...] = (
    "dns_latency_ms", "tcp_retransmits_total", "runqueue_delay_ms", "connect_latency_ms",
    "tls_handshake_ms", "cpu_steal_pct", "mem_reclaim_latency_ms", "disk_io_latency_ms",
    "syscall_latency_ms",
)
# What the shipped DaemonSet / Helm chart enable: REF's nine, CFS throttling (REF's cpu_throttle
# profile signal) and the four GPU signals (deploy/k8s/configmap.yaml, charts/llm-slo-agent).
DEPLOY_SIGNALS: Tuple[str, ...] = DEFAULT_CONFIG_SIGNALS + ("cfs_throttled_ms",) + GPU_SIGNALS
# The REF 12-signal shed order (constants.go:46-59). NEW inserts the GPU probes by cost:
# per-dispatch uprobes first, polled counters last.
REF_DISABLE_ORDER: Tuple[str, ...] = (
    "tls_handshake_ms", "syscall_latency_ms", "runqueue_delay_ms", "disk_io_latency_ms",
    "connect_latency_ms", "mem_reclaim_latency_ms", "cpu_steal_pct", "dns_latency_ms",
    "tcp_retransmits_total", "cfs_throttled_ms", "connect_errors_total",
    "tls_handshake_fail_total",
)
DISABLE_ORDER: Tuple[str, ...] = tuple(s.name for s in sorted(SIGNALS, key=lambda s: s.shed_rank))
assert [n for n in DISABLE_ORDER if n in REF_DISABLE_ORDER] == list(REF_DISABLE_ORDER)


def status_for(signal: str, value: float) -> str:
    """Probe status (REF generator.go:203-232, `threshold` at :234-242): >= error -> error."""
    spec = BY_NAME.get(signal)
    if spec is None:
        return "ok"
    if value >= spec.error:
        return "error"
    if value >= spec.warn:
        return "warning"
    return "ok"


def signal_from_type(kernel_type: int) -> Tuple[str, str]:
    """REF ringbuf.go:199-225 mapping; NEW ids extend it. Unknown -> ("unknown","unknown")."""
    if kernel_type == HELLO_TYPE:
        return HELLO_SIGNAL, "count"
    spec = BY_TYPE.get(kernel_type)
    if spec is None:
        return "unknown", "unknown"
    return spec.name, spec.unit


# --------------------------------------------------------------------------------------
# Capability modes (REF pkg/signals/constants.go:19-25, mode.go:9-29)
# --------------------------------------------------------------------------------------

MODE_CORE_FULL = "core_full"
MODE_BCC_DEGRADED = "bcc_degraded"
MODE_REPLAY = "replay"          # NEW: record-format replay (no kernel probes)
MODE_GPU = "gpu"                # NEW: core + GPU signals (rocprofiler-sdk / KFD)
CAPABILITY_MODES = (MODE_CORE_FULL, MODE_BCC_DEGRADED, MODE_REPLAY, MODE_GPU)


def supported_signals_for_mode(mode: str) -> List[str]:
    if mode == MODE_BCC_DEGRADED:
        return list(BCC_SIGNALS)
    if mode in (MODE_GPU, MODE_REPLAY):
        return list(SIGNAL_NAMES)
    return list(CORE_SIGNALS)


def detect_capability_mode(btf_path: str = "/sys/kernel/btf/vmlinux", kfd_path: str = "/dev/kfd") -> str:
    import os
    import sys

    if not sys.platform.startswith("linux"):
        return MODE_BCC_DEGRADED
    if not os.path.exists(btf_path):
        return MODE_BCC_DEGRADED
    if os.path.exists(kfd_path):
        return MODE_GPU
    return MODE_CORE_FULL


def parse_capability_mode(value: str) -> str:
    if value in CAPABILITY_MODES:
        return value
    return detect_capability_mode()


# --------------------------------------------------------------------------------------
# Fault domains and the likelihood table
# --------------------------------------------------------------------------------------

REF_DOMAINS: Tuple[str, ...] = (
    "network_dns", "network_egress", "cpu_throttle", "memory_pressure",
    "provider_throttle", "provider_error", "retrieval_backend", "unknown",
)
GPU_DOMAINS: Tuple[str, ...] = ("gpu_contention", "gpu_interconnect")
ALL_DOMAINS: Tuple[str, ...] = REF_DOMAINS + GPU_DOMAINS
DOMAIN_INDEX: Dict[str, int] = {d: i for i, d in enumerate(ALL_DOMAINS)}

# P(signal elevated | domain), rows = signals of REF (bayesian.go:67-190), columns = REF_DOMAINS.
_REF_LIKELIHOODS: Dict[str, Tuple[float, ...]] = {
    #                          dns   egr   cpu   mem   pthr  perr  retr  unk
    "dns_latency_ms":         (.95, .70, .10, .10, .10, .10, .15, .10),
    "tcp_retransmits_total":  (.15, .90, .10, .10, .10, .15, .10, .10),
    "runqueue_delay_ms":      (.10, .10, .90, .60, .10, .10, .10, .10),
    "connect_latency_ms":     (.50, .85, .10, .10, .75, .40, .30, .10),
    "tls_handshake_ms":       (.10, .30, .10, .10, .80, .50, .20, .10),
    "cpu_steal_pct":          (.10, .10, .90, .20, .10, .10, .10, .10),
    "cfs_throttled_ms":       (.10, .10, .85, .75, .10, .10, .10, .10),
    "mem_reclaim_latency_ms": (.05, .05, .15, .95, .05, .05, .05, .05),
    "disk_io_latency_ms":     (.05, .05, .10, .85, .05, .05, .30, .05),
    "syscall_latency_ms":     (.10, .20, .15, .10, .90, .60, .40, .10),
    "connect_errors_total":   (.10, .80, .05, .05, .60, .85, .15, .10),
    "tls_handshake_fail_total": (.05, .70, .05, .05, .30, .60, .10, .05),
}


def ref_likelihoods() -> Dict[str, Dict[str, float]]:
    """REF DefaultLikelihoods(): signal -> domain -> P(elevated|domain)."""
    return {s: dict(zip(REF_DOMAINS, row)) for s, row in _REF_LIKELIHOODS.items()}


# Extended table for the 16-signal x 10-domain NEW model (used as the initial point of
# the learned model; REF rows/columns are unchanged).
_GPU_ROWS: Dict[str, Tuple[float, ...]] = {
    #                          dns   egr   cpu   mem   pthr  perr  retr  unk   gcont gxgmi
    "gpu_queue_delay_ms":     (.05, .05, .20, .10, .10, .05, .05, .05, .90, .30),
    "hbm_pressure_pct":       (.05, .05, .05, .30, .05, .05, .05, .05, .80, .10),
    "xgmi_link_latency_us":   (.05, .10, .05, .05, .05, .05, .05, .05, .20, .90),
    "rccl_collective_ms":     (.05, .20, .15, .05, .05, .05, .05, .05, .40, .90),
}
_GPU_COLS_FOR_REF_ROWS = {  # P(REF signal elevated | gpu domain)
    "runqueue_delay_ms": (.20, .10), "cpu_steal_pct": (.10, .10),
    "cfs_throttled_ms": (.10, .05), "syscall_latency_ms": (.20, .10),
}


# Application evidence (NEW, additive; ops/csrc/mislo_launch.h AppModel, models/bayes.py
# AppEvidence): the incident group's retrieval time the kernel signals do not account for -- the
# application's llm.slo.retrieval.{vectordb,network,dns}_ms (REF demo/rag-service/main.go:393-397)
# minus REF's kernel-attributed share, dns + connect + TLS (DecomposeRetrieval,
# pkg/otel/processor/ebpfcorrelator/correlator.go:179-194). REF's table has no row for it; this is
# its expert row. A retrieval backend stall (vector DB, search index) is the one fault that lives
# there alone; a starved or network-slowed service inflates its own measured retrieval time too
# (CPU / memory / network 0.30-0.35), and a provider or GPU fault does not touch retrieval.
APP_RETRIEVAL_SIGNAL = "retrieval_residual_ms"
APP_RETRIEVAL_SEMCONV = "llm.slo.retrieval.residual_ms"
APP_RETRIEVAL_THRESHOLD_MS = 100.0
APP_RETRIEVAL_LIKELIHOOD: Dict[str, float] = {
    "network_dns": .30, "network_egress": .30, "cpu_throttle": .35, "memory_pressure": .30,
    "provider_throttle": .10, "provider_error": .10, "retrieval_backend": .90, "unknown": .05,
    "gpu_contention": .10, "gpu_interconnect": .05,
}


def extended_likelihood_matrix() -> List[List[float]]:
    """16 x 10 matrix [slot][domain] of P(elevated | domain)."""
    rows: List[List[float]] = []
    for spec in SIGNALS:
        if spec.name in _REF_LIKELIHOODS:
            gpu_cols = _GPU_COLS_FOR_REF_ROWS.get(spec.name, (.05, .05))
            rows.append(list(_REF_LIKELIHOODS[spec.name]) + list(gpu_cols))
        else:
            rows.append(list(_GPU_ROWS[spec.name]))
    return rows


def feature_vector(signals: Dict[str, float], missing: float = float("nan")) -> List[float]:
    """Map a {signal: value} dict to the 16-slot feature layout."""
    out = [missing] * N_SLOTS
    for name, value in signals.items():
        spec = BY_NAME.get(name)
        if spec is not None:
            out[spec.slot] = float(value)
    return out


def bucket_edges() -> List[List[float]]:
    return [list(s.buckets) for s in SIGNALS]


def names(seq: Optional[Sequence[int]] = None) -> List[str]:
    if seq is None:
        return list(SIGNAL_NAMES)
    return [SIGNAL_NAMES[i] for i in seq]

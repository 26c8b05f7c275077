"""Span-attribute semantic conventions (``llm.ebpf.*`` / ``llm.slo.*``).

Key strings are the REF contract (pkg/semconv/llm_ebpf.go:3-27); the per-signal keys
are derived from the signal catalogue so the two can never drift. Four GPU keys are
NEW additive attributes.
"""

from ..signals import catalog as _cat

ATTR_DNS_LATENCY_MS = "llm.ebpf.dns.latency_ms"
ATTR_TCP_RETRANSMITS = "llm.ebpf.tcp.retransmits"
ATTR_RUNQUEUE_DELAY_MS = "llm.ebpf.sched.runqueue_delay_ms"
ATTR_CPU_STEAL_PCT = "llm.ebpf.cpu.steal_pct"
ATTR_CONNECT_LATENCY_MS = "llm.ebpf.net.connect_latency_ms"
ATTR_TLS_HANDSHAKE_MS = "llm.ebpf.tls.handshake_ms"
ATTR_CORRELATION_CONF = "llm.ebpf.correlation_confidence"
ATTR_SLO_TTFT_MS = "llm.slo.ttft_ms"
# true on a record exported when the first token is out (the SLI, ahead of the request span)
ATTR_SLO_TTFT_EARLY = "llm.slo.ttft_early"
ATTR_SLO_TOKENS_PER_SEC = "llm.slo.tokens_per_sec"
ATTR_RETRIEVAL_VECTORDB = "llm.slo.retrieval.vectordb_ms"
ATTR_RETRIEVAL_NETWORK_MS = "llm.slo.retrieval.network_ms"
ATTR_RETRIEVAL_DNS_MS = "llm.slo.retrieval.dns_ms"
ATTR_CFS_THROTTLED_MS = "llm.ebpf.cpu.cfs_throttled_ms"
ATTR_RETRIEVAL_KERNEL_MS = "llm.ebpf.retrieval.kernel_attributed_ms"
ATTR_RETRY_STORM = "llm.ebpf.tcp.retry_storm"
ATTR_MEM_RECLAIM_LATENCY_MS = "llm.ebpf.mm.reclaim_latency_ms"
ATTR_DISK_IO_LATENCY_MS = "llm.ebpf.blk.io_latency_ms"
ATTR_SYSCALL_LATENCY_MS = "llm.ebpf.syscall.latency_ms"
ATTR_CONNECT_ERRORS = "llm.ebpf.net.connect_errors_total"
ATTR_TLS_HANDSHAKE_FAILS = "llm.ebpf.tls.handshake_fail_total"
# NEW (MI355X)
ATTR_GPU_QUEUE_DELAY_MS = "llm.ebpf.gpu.queue_delay_ms"
ATTR_HBM_PRESSURE_PCT = "llm.ebpf.gpu.hbm_pressure_pct"
ATTR_XGMI_LINK_LATENCY_US = "llm.ebpf.gpu.xgmi_link_latency_us"
ATTR_RCCL_COLLECTIVE_MS = "llm.ebpf.gpu.rccl_collective_ms"

SIGNAL_ATTR = {s.name: s.semconv for s in _cat.SIGNALS}
ATTR_SIGNAL = {v: k for k, v in SIGNAL_ATTR.items()}
ATTR_BY_SLOT = tuple(s.semconv for s in _cat.SIGNALS)

# Retrieval decomposition components (REF correlator.go:179-194)
RETRIEVAL_COMPONENTS = (ATTR_DNS_LATENCY_MS, ATTR_CONNECT_LATENCY_MS, ATTR_TLS_HANDSHAKE_MS)


def signal_attr_key(signal: str):
    """REF correlator.go:143-172: (key, supported)."""
    key = SIGNAL_ATTR.get(signal)
    return (key, True) if key else ("", False)

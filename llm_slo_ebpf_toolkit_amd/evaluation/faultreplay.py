"""Deterministic fault-sample streams (REF pkg/faultreplay/generator.go:10-129).

``generate_fault_samples`` reproduces REF's label streams exactly (round-robin labels,
``mixed_multi`` cycling four label pairs, ids ``replay-inc-%04d``, 1 s spacing,
confidence 0.9, burn 2.0/2.4, window 5 min) -- REF's samples carry NO ``signals`` so its
Bayes falls back to the label map. ``with_signals=True`` (NEW) populates every sample's
``signals`` from the REF fault profiles with seeded jitter, so the posterior is
actually exercised.
"""

from __future__ import annotations

from typing import List, Optional

import numpy as np

from ..models.sample import FaultSample, map_fault_label
from ..signals import catalog
from ..signals.generator import profile_for_fault, FAULT_OVERRIDES
from ..utils.timeutil import SECOND

SCENARIO_FAULT_LABELS = {
    "provider_throttle": ["provider_throttle"],
    "dns_latency": ["dns_latency"],
    "cpu_throttle": ["cpu_throttle"],
    "memory_pressure": ["memory_pressure"],
    "network_partition": ["network_partition"],
    "mixed": ["provider_throttle", "dns_latency", "cpu_throttle", "memory_pressure", "network_partition"],
    # NEW GPU scenarios
    "gpu_contention": ["gpu_contention"],
    "rccl_latency": ["rccl_latency"],
}
MIXED_MULTI_PAIRS = [("provider_throttle", "dns_latency"), ("cpu_throttle", "memory_pressure"),
                     ("network_partition", "dns_latency"), ("provider_throttle", "network_partition")]


def supported_scenarios() -> List[str]:
    return ["provider_throttle", "dns_latency", "cpu_throttle", "memory_pressure", "network_partition", "mixed",
            "mixed_multi", "gpu_contention", "rccl_latency"]


def unique_domains(*domains: str) -> List[str]:
    out: List[str] = []
    for d in domains:
        if d and d != "unknown" and d not in out:
            out.append(d)
    return out or ["unknown"]


def _signals(labels, rng: np.random.Generator, jitter: float) -> dict:
    prof = profile_for_fault("")
    for lab in labels:
        for k, v in FAULT_OVERRIDES.get(lab, {}).items():
            prof[k] = max(prof[k], v)
    out = {}
    for name, v in prof.items():
        if name in ("tcp_retransmits_total", "connect_errors_total", "tls_handshake_fail_total"):
            out[name] = float(rng.poisson(v)) if v > 0 else 0.0
        else:
            out[name] = float(v * np.exp(rng.normal(0, jitter)))
    return out


def generate_fault_samples(scenario: str, count: int, start_ns: int, with_signals: bool = False, seed: int = 42,
                           jitter: float = 0.2) -> List[FaultSample]:
    if count < 1:
        raise ValueError("count must be >= 1")
    rng = np.random.default_rng(seed)
    out: List[FaultSample] = []
    if scenario == "mixed_multi":
        for i in range(count):
            a, b = MIXED_MULTI_PAIRS[i % len(MIXED_MULTI_PAIRS)]
            doms = unique_domains(map_fault_label(a), map_fault_label(b))
            s = FaultSample(incident_id=f"replay-inc-{i + 1:04d}", timestamp=start_ns + i * SECOND, cluster="local",
                            namespace="default", service="chat", fault_label=a, expected_domain=doms[0],
                            expected_domains=doms, confidence=0.9, burn_rate=2.4, window_minutes=5,
                            request_id=f"replay-req-{i + 1:04d}", trace_id=f"replay-trace-{i + 1:04d}")
            if with_signals:
                s.signals = _signals((a, b), rng, jitter)
            out.append(s)
        return out
    labels = SCENARIO_FAULT_LABELS.get(scenario)
    if labels is None:
        raise ValueError(f'unsupported scenario "{scenario}"')
    for i in range(count):
        lab = labels[i % len(labels)]
        s = FaultSample(incident_id=f"replay-inc-{i + 1:04d}", timestamp=start_ns + i * SECOND, cluster="local",
                        namespace="default", service="chat", fault_label=lab, expected_domain=map_fault_label(lab),
                        confidence=0.9, burn_rate=2.0, window_minutes=5, request_id=f"replay-req-{i + 1:04d}",
                        trace_id=f"replay-trace-{i + 1:04d}")
        if with_signals:
            s.signals = _signals((lab,), rng, jitter)
        out.append(s)
    return out

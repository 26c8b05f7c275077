"""Measured collector overhead (replaces REF's constant 2.2 % / 120 MB / 900 events/s,
pkg/benchmark/harness.go:71-80).

Two measurement modes, both reporting CPU as percent of ONE core (REF formula,
pkg/safety/overhead_guard.go:103) over a paced run:

* ``agent``: the host agent emit loop at its configured cadence -- synthetic sample ->
  4 SLO events + up to 16 probe events -> compiled-schema validation -> JSONL encode.
* ``gpu``: the agent's MI355X window path paced at ``rate_eps`` events/s (default 1M/s,
  BASELINE config 5): ring compaction + host encoding + one DMA + the window graph.
"""

from __future__ import annotations

import io
import json
import os
import time
from typing import Dict, Optional

from ..safety import read_rss_mb
from ..utils.timeutil import now_ns


def _agent_loop(duration_s: float, ticks_per_s: float) -> Dict[str, float]:
    from ..collector.pipeline import SampleMeta, build_synthetic_sample, normalize_sample
    from ..contracts import validator
    from ..signals import catalog
    from ..signals.generator import Generator
    from ..signals.metadata import Metadata

    gen = Generator(catalog.MODE_GPU, list(catalog.SIGNAL_NAMES))
    meta = SampleMeta(node=os.uname().nodename)
    slo_schema = validator.compiled("slo-event")
    probe_schema = validator.compiled("probe-event")
    sink = io.StringIO()
    events = 0
    c0, w0 = time.process_time(), time.perf_counter()
    period = 1.0 / ticks_per_s
    nxt = w0
    i = 0
    while time.perf_counter() - w0 < duration_s:
        s = build_synthetic_sample("mixed", i, now_ns(), meta)
        for ev in normalize_sample(s):
            d = ev.to_dict()
            slo_schema.validate(d)
            sink.write(json.dumps({"kind": "slo", "payload": d}) + "\n")
            events += 1
        for ev in gen.generate(s, Metadata(node=meta.node, namespace="default", pod="agent", container="agent",
                                            pid=os.getpid(), tid=os.getpid(), trace_id=s.trace_id)):
            d = ev.to_dict()
            probe_schema.validate(d)
            sink.write(json.dumps({"kind": "probe", "payload": d}) + "\n")
            events += 1
        if sink.tell() > 1 << 20:
            sink.seek(0)
            sink.truncate()
        i += 1
        nxt += period
        time.sleep(max(0.0, nxt - time.perf_counter()))
    cpu, wall = time.process_time() - c0, time.perf_counter() - w0
    return {"cpu_pct": 100.0 * cpu / wall, "events_per_second": events / wall, "dropped": 0}


def _gpu_loop(duration_s: float, rate_eps: float, window_s: float) -> Dict[str, float]:
    """The agent's GPU window path at ``rate_eps``: a forked replay producer (the kernel's
    stand-in, not measured) writes into emulated rings; this process cuts a window every
    ``window_s``, assembles it natively and submits it to the native engine."""
    from ..collector import bpf
    from ..pipeline.window import RingWindowSource, WindowPipeline

    n = max(1024, int(rate_eps * window_s))
    groups = 32
    names = bpf.RingNames.of(f"/mislo-ovh-{os.getpid()}")
    kw = dict(events_per_window=n, spans_per_window=max(64, n // 64), n_services=groups)
    ring, user, spans = bpf.create_rings(names, 4 * 24 * n, 4 * n, 4 * kw["spans_per_window"])
    prod = bpf.start_replay_producer(names, kw, rate_eps, int(window_s * 1000), n_images=2)
    try:
        pipe = WindowPipeline(n + n // 4, kw["spans_per_window"], groups, 0, None, model="bayes", learn=False,
                              user_cap=max(1024, n // 2))
        src = RingWindowSource(pipe, ring, user, spans)
        pipe.eng.set_pods(*bpf.pod_metadata(kw))
        src.step(groups, with_labels=False)
        src.drain()
        c0, w0 = time.process_time(), time.perf_counter()
        nxt = w0
        k = events = 0
        while time.perf_counter() - w0 < duration_s:
            nxt += window_s
            time.sleep(max(0.0, nxt - time.perf_counter()))
            src.step(groups, with_labels=False)
            events += int(src.last["n_events"])
            k += 1
        src.drain()
        cpu, wall = time.process_time() - c0, time.perf_counter() - w0
    finally:
        prod.terminate()
        if "pipe" in locals():
            pipe.eng.close()
    return {"cpu_pct": 100.0 * cpu / wall, "events_per_second": events / wall, "dropped": 0}


def measure(duration_s: float = 1.0, mode: Optional[str] = None, rate_eps: float = 1e6, window_s: float = 1.0,
            ticks_per_s: float = 10.0) -> Dict[str, float]:
    if mode is None:
        try:
            from ..ops import load_agent

            # import only (no HIP call): the GPU loop forks its producer before the runtime starts
            load_agent(init=False)
            mode = "gpu" if os.path.exists("/dev/kfd") else "agent"
        except Exception:  # pragma: no cover
            mode = "agent"
    if mode == "gpu":
        r = _gpu_loop(duration_s, rate_eps, window_s)
    else:
        r = _agent_loop(duration_s, ticks_per_s)
    r.update({"timestamp": now_ns(), "node": os.uname().nodename, "rss_mb": read_rss_mb(os.getpid()), "mode": mode})
    return r

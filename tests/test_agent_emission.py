"""When and what the window agent emits (agent/daemon.py).

* REF emits on the tick it samples (/root/reference/cmd/agent/main.go:515-604); the window agent
  emits window k as soon as its chain is done (``emit_wait_ms``), not one window later at cut k+1.
* REF posts its webhook inside the tick (main.go:567-585, exporter.go:63-85: 5 s timeout x 3
  attempts, 1 s + 2 s backoff); the window agent's deliveries run on their own thread behind a
  bounded queue, so a hung endpoint never moves the window clock.
* Only incidents with SLO impact become IncidentAttributions (and pages); a healthy node emits none.
"""

import io
import os
import time

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.agent.daemon import Agent, AgentOptions


def _opts(tag, **kw):
    # small windows: the host oracle engine (CPU) finishes each in tens of ms, well inside the period
    base = dict(engine="cpu", source="replay", gpus=1, window_events=2048, window_spans=128, window_groups=8,
                window_ms=300, metrics_bind="", output="stdout", ring_name=f"/mislo-emit-{tag}-{os.getpid()}",
                config="", min_confidence=0.0, scenario="full", disable_overhead_guard=True)
    base.update(kw)
    return AgentOptions(**base)


def _run(o, windows):
    out = io.StringIO()
    a = Agent(o, out_stream=out)
    try:
        rc = a.run_windows(max_windows=windows)
    finally:
        a.close()
    return a, rc, [ln for ln in out.getvalue().splitlines() if ln.strip()]


@pytest.mark.timeout(120)
def test_a_hung_webhook_never_moves_the_window_clock(http_recorder):
    def hang(_path):
        time.sleep(5.0)
        return b"{}"

    srv = http_recorder([(200, hang)] * 64)
    o = _opts("hung", webhook_url=srv.url + "/hook", webhook_queue=2, window_ms=300)
    t0 = time.monotonic()
    a, rc, lines = _run(o, 8)
    assert rc == 0 and lines, "the replay's faulted groups breach the SLO: attributions expected"
    # every cut within 50 ms of its schedule, though each delivery hangs 5 s (x3 attempts)
    skew = list(a.cut_skew_ms)[1:]
    assert skew and max(skew) < 50.0, skew
    assert time.monotonic() - t0 < 8 * 0.3 + 15.0  # close() waits for the queue at most 5 s
    assert len(srv.requests) >= 1  # the sender thread did reach the endpoint
    assert a.webhook_q.dropped > 0  # the bounded queue overflowed instead of blocking
    from llm_slo_ebpf_toolkit_amd.export.prometheus import parse_exposition

    m = parse_exposition(a.metrics.registry.exposition())
    assert m['llm_slo_agent_dropped_events_total{reason="emit"}'] > 0


@pytest.mark.timeout(120)
def test_a_healthy_node_emits_no_attribution_and_no_page(http_recorder):
    srv = http_recorder()
    o = _opts("healthy", webhook_url=srv.url + "/hook", scenario="healthy")
    a, rc, lines = _run(o, 6)
    assert rc == 0
    assert lines == [] and a.attributions_emitted == 0
    assert srv.requests == []
    from llm_slo_ebpf_toolkit_amd.export.prometheus import parse_exposition

    m = parse_exposition(a.metrics.registry.exposition())
    kept = {k: v for k, v in m.items() if k.startswith("llm_slo_agent_incidents_scored_total")}
    assert sum(v for k, v in kept.items() if 'emitted="false"' in k) > 0, kept
    assert sum(v for k, v in kept.items() if 'emitted="true"' in k) == 0, kept


@pytest.mark.timeout(120)
def test_window_k_is_emitted_before_cut_k_plus_1():
    o = _opts("early", window_ms=500, emit_wait_ms=250)
    a, rc, lines = _run(o, 6)
    assert rc == 0 and lines
    lag = list(a.emit_lag_ms)
    assert len(lag) >= 5, lag
    # cut -> attributions on the output: the CPU engine's window time, well below the 500 ms period
    assert np.median(lag) < 250.0, lag
    late = _opts("late", window_ms=500, emit_wait_ms=0)
    b, rc, _ = _run(late, 6)
    assert rc == 0 and np.median(list(b.emit_lag_ms)) >= 450.0, list(b.emit_lag_ms)

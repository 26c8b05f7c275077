"""Correlation tiers, enrichment, fanout, retry storms and the labelled-pair gate."""

import os

import pytest

from llm_slo_ebpf_toolkit_amd.contracts import semconv
from llm_slo_ebpf_toolkit_amd.correlation import (Correlator, RetryStormDetector, SignalRef, SpanRecord, SpanRef,
                                                  decompose_retrieval, enrich_dns, evaluate_gate,
                                                  evaluate_labeled_pairs, load_labeled_pairs, match)
from llm_slo_ebpf_toolkit_amd.utils.timeutil import MS, SECOND

T0 = 1_771_000_000 * SECOND
CONN = "10.0.0.1:1234->10.0.0.2:53/udp"


def span():
    return SpanRef(trace_id="trace-1", service="chat", node="node-a", pod="pod-a", pid=42, conn_tuple=CONN,
                   timestamp=T0)


@pytest.mark.parametrize("sig,conf,tier", [
    (SignalRef("dns_latency_ms", trace_id="trace-1", timestamp=T0 + SECOND), 1.0, "trace_id_exact"),
    (SignalRef("dns_latency_ms", pod="pod-a", pid=42, timestamp=T0 + 50 * MS), 0.9, "pod_pid_100ms"),
    (SignalRef("dns_latency_ms", pod="pod-a", conn_tuple=CONN, timestamp=T0 + 200 * MS), 0.8, "pod_conn_250ms"),
    (SignalRef("dns_latency_ms", service="chat", node="node-a", timestamp=T0 + 400 * MS), 0.65,
     "service_node_500ms"),
])
def test_tier_matrix(sig, conf, tier):
    d = match(span(), sig)
    assert d.matched and d.confidence == conf and d.tier == tier


def test_window_edges_are_inclusive_and_zero_time_never_matches():
    s = span()
    assert match(s, SignalRef("x", pod="pod-a", pid=42, timestamp=T0 + 100 * MS)).tier == "pod_pid_100ms"
    assert match(s, SignalRef("x", pod="pod-a", pid=42, timestamp=T0 + 100 * MS + 1)).matched is False
    assert match(s, SignalRef("x", trace_id="trace-1", timestamp=T0 - 2 * SECOND)).matched
    assert not match(s, SignalRef("x", trace_id="trace-1", timestamp=T0 - 2 * SECOND - 1)).matched
    assert not match(s, SignalRef("x", trace_id="trace-1", timestamp=0)).matched
    # precedence: trace beats pod/pid even when both hold
    assert match(s, SignalRef("x", trace_id="trace-1", pod="pod-a", pid=42, timestamp=T0)).tier == "trace_id_exact"
    # empty fields never satisfy equality
    assert not match(SpanRef(timestamp=T0), SignalRef("x", timestamp=T0)).matched
    # custom narrow outer window bounds every tier
    assert not match(s, SignalRef("x", pod="pod-a", pid=42, timestamp=T0 + 60 * MS), window_ns=50 * MS).matched


def test_enrich_dns_threshold():
    out, d = enrich_dns(None, SpanRef(service="chat", node="node-a", timestamp=T0),
                        SignalRef("dns_latency_ms", service="chat", node="node-a", timestamp=T0 + 100 * MS,
                                  value=181.0))
    assert d.matched and out == {}
    out, d = enrich_dns(None, SpanRef(trace_id="t", timestamp=T0),
                        SignalRef("dns_latency_ms", trace_id="t", timestamp=T0 + 200 * MS, value=190.0))
    assert out[semconv.ATTR_DNS_LATENCY_MS] == 190.0 and out[semconv.ATTR_CORRELATION_CONF] == 1.0
    out, d = enrich_dns(None, SpanRef(trace_id="t", timestamp=T0),
                        SignalRef("tcp_retransmits_total", trace_id="t", timestamp=T0, value=3))
    assert out == {} and not d.matched


def test_fanout_cap_and_debug_counters():
    s = span()
    sigs = [SignalRef("dns_latency_ms", trace_id="trace-1", timestamp=T0 + i * MS, value=float(10 + i))
            for i in range(5)]
    sigs.append(SignalRef("runqueue_delay_ms", service="chat", node="node-a", timestamp=T0, value=99))  # low conf
    sigs.append(SignalRef("mystery_signal", trace_id="trace-1", timestamp=T0, value=1))                  # unsupported
    sigs.append(SignalRef("cpu_steal_pct", pod="pod-z", timestamp=T0, value=1))                         # unmatched
    res = Correlator().enrich_attributes({}, s, sigs)
    assert len(res.candidates) == 3
    assert [c.signal.value for c in res.candidates] == [10.0, 11.0, 12.0]  # |dt| ascending
    assert res.debug.fanout_dropped == 2
    assert res.debug.low_confidence == 1
    assert res.debug.unsupported_type == 1
    assert res.debug.unmatched == 1
    assert res.attributes[semconv.ATTR_DNS_LATENCY_MS] == 12.0  # max-merge of kept values
    assert res.attributes[semconv.ATTR_CORRELATION_CONF] == 1.0


def test_stable_order_for_ties_and_base_max_merge():
    s = span()
    sigs = [SignalRef("dns_latency_ms", trace_id="trace-1", timestamp=T0 + 5 * MS, value=v) for v in (3.0, 9.0, 1.0, 7.0)]
    res = Correlator(max_join_fanout=2).enrich_attributes({semconv.ATTR_DNS_LATENCY_MS: 5.0}, s, sigs)
    assert [c.signal.value for c in res.candidates] == [3.0, 9.0]
    assert res.attributes[semconv.ATTR_DNS_LATENCY_MS] == 9.0
    res = Correlator(max_join_fanout=1).enrich_attributes({semconv.ATTR_DNS_LATENCY_MS: 5.0}, s, sigs)
    assert res.attributes[semconv.ATTR_DNS_LATENCY_MS] == 5.0  # existing larger base value is kept


def test_process_batch_and_retrieval_decomposition():
    spans = [SpanRecord(trace_id="a", timestamp=T0), SpanRecord(trace_id="b", timestamp=T0)]
    sigs = [SignalRef("dns_latency_ms", trace_id="a", timestamp=T0, value=20),
            SignalRef("connect_latency_ms", trace_id="a", timestamp=T0, value=30),
            SignalRef("tls_handshake_ms", trace_id="a", timestamp=T0, value=50)]
    b = Correlator().process_batch(spans, sigs)
    assert b.spans[0].attributes[semconv.ATTR_RETRIEVAL_KERNEL_MS] == 100
    assert semconv.ATTR_RETRIEVAL_KERNEL_MS not in b.spans[1].attributes
    assert b.debug.unmatched == 3
    attrs = {}
    assert decompose_retrieval(attrs) == 0 and attrs == {}


def test_retry_storm_window():
    det = RetryStormDetector(window_ns=10 * SECOND, threshold=3)
    assert not det.record("p", T0)
    assert not det.record("p", T0 + SECOND)
    assert det.record("p", T0 + 2 * SECOND)
    assert det.count("p", T0 + 11 * SECOND) == 2  # only T0 is strictly before the cutoff T0+1s
    assert not det.is_storm("p", T0 + 11 * SECOND)
    assert det.count("q", T0) == 0
    det.reset()
    assert det.count("p", T0) == 0


def test_labeled_pairs_gate(fixtures_dir):
    pairs = load_labeled_pairs(os.path.join(fixtures_dir, "ref_labeled_pairs.jsonl"))
    rep, preds = evaluate_labeled_pairs(pairs)
    assert (rep.true_positive, rep.false_positive, rep.false_negative, rep.true_negative) == (40, 0, 0, 15)
    assert rep.precision == rep.recall == rep.f1 == 1.0 and rep.tier_accuracy == 1.0
    assert evaluate_gate(rep, 0.9, 0.85).passed
    assert not evaluate_gate(rep, 1.01, 0.85).passed
    assert len(preds) == 55 and all(p.correct for p in preds)


def test_load_labeled_pairs_empty(tmp_path):
    p = tmp_path / "empty.jsonl"
    p.write_text("\n\n")
    with pytest.raises(ValueError):
        load_labeled_pairs(str(p))

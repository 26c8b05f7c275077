"""Record layouts: REF 40-byte records, 64-byte EVENT/SPAN, 32-byte compact EVENT32."""

import numpy as np

from llm_slo_ebpf_toolkit_amd.collector import records
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator


def _win(seed=2):
    cfg = ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=8, events_per_window=3000,
                       spans_per_window=200, seed=seed)
    return ReplayGenerator(cfg).next_window()


def test_layout_sizes():
    assert records.EVENT.itemsize == 64
    assert records.EVENT32.itemsize == 32
    assert records.SPAN.itemsize == 64
    assert records.REF_EVENT.itemsize == 40


def test_ref_record_roundtrip():
    from llm_slo_ebpf_toolkit_amd.signals.metadata import Metadata

    raw = records.encode_ref_record(11, 12, 1234, 1, 5_000_000, 4000, 53, 0x0100007F, 110)
    meta = Metadata(node="n1", namespace="ns", pod="p", container="c", trace_id="t", span_id="s")
    ev = records.decode_ref_record(raw, meta, 99)
    assert ev.pid == 11 and ev.tid == 12 and ev.ts_unix_nano == 99
    assert ev.signal == "dns_latency_ms" and abs(ev.value - 5.0) < 1e-12 and ev.errno == 110
    assert ev.conn_tuple.dst_port == 53 and ev.conn_tuple.dst_ip == "127.0.0.1"
    assert ev.node == "n1" and ev.trace_id == "t"


def test_compact_preserves_join_structure():
    win = _win()
    it = records.ConnInterner()
    table = records.pod_table(win.events, win.spans)
    ev32 = records.to_compact(win.events, it)
    sp32 = records.compact_spans(win.spans, it)
    full = oracle.decode_events(win.events)
    comp = oracle.decode_compact(ev32, table)
    np.testing.assert_array_equal(full.slot, comp.slot)
    np.testing.assert_array_equal(full.svcnode, comp.svcnode)
    # milli-unit fixed point: |err| <= 0.0005 of the output unit (+ f32 rounding)
    np.testing.assert_allclose(comp.val, full.val, atol=6e-4, rtol=1e-6)
    # interning preserves connection equality, so tiers/keys are identical
    a = oracle.join(full, win.spans, win.n_groups)
    b = oracle.join(comp, sp32, win.n_groups)
    np.testing.assert_array_equal(a.top3, b.top3)
    np.testing.assert_array_equal(a.cnt, b.cnt)
    assert a.debug == b.debug


def test_interner_is_stable_and_zero_preserving():
    it = records.ConnInterner()
    x = np.array([0, 99, 5, 99, 0], dtype=np.uint64)
    ids = it.ids(x)
    assert ids[0] == 0 and ids[4] == 0 and ids[1] == ids[3] and ids[1] != ids[2]
    again = it.ids(np.array([5, 99], dtype=np.uint64))
    assert again[0] == ids[2] and again[1] == ids[1]

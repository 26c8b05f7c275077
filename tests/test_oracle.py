"""The window oracle (the GPU kernels' spec) agrees with REF-semantics scalar correlation."""

import numpy as np

from llm_slo_ebpf_toolkit_amd.contracts import semconv
from llm_slo_ebpf_toolkit_amd.correlation import Correlator, SignalRef, SpanRecord
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
from llm_slo_ebpf_toolkit_amd.signals import catalog


def _window(seed=11, n=1500, s=60):
    cfg = ReplayConfig(scenario="full", n_nodes=2, pods_per_node=4, n_services=4, events_per_window=n,
                       spans_per_window=s, seed=seed)
    return ReplayGenerator(cfg).next_window()


def _refs(win, d):
    sigs = []
    for i in range(win.n_events):
        sl = int(d.slot[i])
        name = catalog.SIGNAL_NAMES[sl] if sl != 255 else "unknown_signal"
        sn = int(d.svcnode[i])
        sigs.append(SignalRef(signal=name, trace_id=str(int(d.trace[i])) if d.trace[i] else "",
                              service=str(sn >> 16) if sn >> 16 else "", node=str(sn & 0xFFFF) if sn & 0xFFFF else "",
                              pod=str(int(d.pod[i])) if d.pod[i] else "", pid=int(d.pid[i]),
                              conn_tuple=str(int(d.conn[i])) if d.conn[i] else "", timestamp=int(d.ts[i]),
                              value=float(d.val[i])))
    spans = []
    for sp in win.spans:
        spans.append(SpanRecord(trace_id=str(int(sp["trace_h"])) if sp["trace_h"] else "",
                                service=str(int(sp["svc_id"])) if sp["svc_id"] else "",
                                node=str(int(sp["node_id"])) if sp["node_id"] else "",
                                pod=str(int(sp["pod_id"])) if sp["pod_id"] else "", pid=int(sp["pid"]),
                                conn_tuple=str(int(sp["conn_h"])) if sp["conn_h"] else "",
                                timestamp=int(sp["ts_ns"])))
    return spans, sigs


def test_oracle_equals_scalar_correlator():
    win = _window()
    d = oracle.decode_events(win.events)
    res = oracle.join(d, win.spans, win.n_groups, group_mode=0)
    spans, sigs = _refs(win, d)
    batch = Correlator().process_batch(spans, sigs)
    dbg = batch.debug
    assert (dbg.unmatched, dbg.low_confidence, dbg.fanout_dropped, dbg.unsupported_type) == (
        res.debug["unmatched"], res.debug["low_confidence"], res.debug["fanout_dropped"],
        res.debug["unsupported_type"])
    for s, rec in enumerate(batch.spans):
        for slot in range(16):
            key = semconv.ATTR_BY_SLOT[slot]
            a = rec.attributes.get(key)
            o = res.attrs[s, slot]
            if a is None:
                assert np.isnan(o)
            else:
                assert np.float32(a) == o
        conf = rec.attributes.get(semconv.ATTR_CORRELATION_CONF, 0.0)
        assert np.float32(conf) == res.conf[s]


def test_oracle_low_threshold_and_small_window():
    win = _window(seed=12, n=800, s=40)
    d = oracle.decode_events(win.events)
    spans, sigs = _refs(win, d)
    for window_ms, thr in ((2000, 0.6), (150, 0.7), (80, 0.85)):
        res = oracle.join(d, win.spans, win.n_groups, window_ms=window_ms, threshold=thr, group_mode=0)
        b = Correlator(window_ms=window_ms, enrichment_threshold=thr).process_batch(spans, sigs)
        assert b.debug.low_confidence == res.debug["low_confidence"]
        assert b.debug.unmatched == res.debug["unmatched"]
        assert b.debug.fanout_dropped == res.debug["fanout_dropped"]


def test_replay_window_shapes():
    win = _window(n=5000, s=100)
    assert win.n_events == 5000 and win.n_spans == 100
    assert np.all(np.diff(win.events["ts_ns"]) >= 0)
    assert win.group_labels.shape == (win.n_groups,)


def _same_join(a, b):
    np.testing.assert_array_equal(a.top3, b.top3)
    np.testing.assert_array_equal(a.cnt, b.cnt)
    np.testing.assert_array_equal(a.attrs, b.attrs)
    np.testing.assert_array_equal(a.conf, b.conf)
    np.testing.assert_array_equal(a.gsum, b.gsum)
    np.testing.assert_array_equal(a.gcnt, b.gcnt)
    np.testing.assert_array_equal(a.feat, b.feat)
    assert a.debug == b.debug


def test_indexed_join_is_the_bruteforce_join():
    """oracle.join (per-key time-sorted indexes: each span looks only at rows that share one of
    its tier keys within the tier's reach) gives the brute-force all-pairs join bit for bit --
    top-3 keys, counts, attributes, confidences, group sums, features and every debug counter --
    across scenarios, both group modes, the 100 ms / 2 s windows and imported halo rows."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_replay_images

    for seed, scen in ((11, "full"), (12, "mixed"), (13, "baseline")):
        cfg = ReplayConfig(scenario=scen, n_nodes=2, pods_per_node=8, n_services=8, events_per_window=4000,
                           spans_per_window=200, seed=seed)
        g = ReplayGenerator(cfg)
        wins = [g.next_window() for _ in range(2)]
        for w in wins:
            d = oracle.decode_events(w.events)
            for kw in ({}, {"window_ms": 100.0}, {"group_mode": 0}, {"threshold": 0.6, "fanout": 2}):
                _same_join(oracle.join(d, w.spans, w.n_groups, **kw), oracle.join_bruteforce(d, w.spans, w.n_groups, **kw))
        # the ring path: framed records + user rows, then the previous window's rows as imports
        imgs = build_replay_images(wins, user_rec=24)
        table, tmap = oracle.CtxTable(), oracle.TraceMap()
        prev = oracle.empty_rows()
        for w, img in zip(wins, imgs):
            oracle.apply_ring_defs(img.framed, table, tmap, {})
            d = oracle.decode_window(img.framed, img.user, table, tmap, img.bases)
            dd = oracle.concat(d, prev)
            sp = oracle.spans_native(img.spans, tmap)
            _same_join(oracle.join(dd, sp, w.n_groups), oracle.join_bruteforce(dd, sp, w.n_groups))
            prev = d

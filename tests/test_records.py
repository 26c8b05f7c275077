"""Record layouts: REF 40-byte records, 64-byte EVENT/SPAN, 32-byte EVENT32, 20-byte EVENT20."""

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
    assert records.EVENT20.itemsize == 20
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


def test_wire20_preserves_decode_and_join():
    win = _win(seed=4)
    ev = win.events.copy()
    ev["ts_ns"][5] = 0  # zero timestamps survive as the TS_ZERO sentinel (never join)
    conns, ctxs = records.ConnInterner(), records.CtxInterner()
    ev20, t_base = records.to_wire20(ev, conns, ctxs)
    sp = records.compact_spans(win.spans, conns)
    assert ev20["ts_off"][5] == records.TS_ZERO and t_base == int(ev["ts_ns"][ev["ts_ns"] != 0].min())
    full = oracle.decode_events(ev)
    d = oracle.decode_w20(ev20, t_base, ctxs.table())
    for f in ("ts", "slot", "svcnode", "pod", "pid", "trace"):
        np.testing.assert_array_equal(getattr(full, f), getattr(d, f), err_msg=f)
    np.testing.assert_allclose(d.val, full.val, atol=6e-4, rtol=1e-6)
    # the same interned conn ids as EVENT32, so every join key and tier is identical
    c32 = oracle.decode_compact(records.to_compact(ev, conns), records.pod_table(ev, win.spans))
    np.testing.assert_array_equal(c32.conn, d.conn)
    a = oracle.join(full, win.spans, win.n_groups)
    b = oracle.join(d, sp, win.n_groups)
    np.testing.assert_array_equal(a.top3, b.top3)
    np.testing.assert_array_equal(a.cnt, b.cnt)
    assert a.debug == b.debug


def test_ctx_interner_append_only_and_wide_window_rejected():
    xi = records.CtxInterner()
    z = np.zeros(3, dtype=np.uint32)
    ids = xi.ids(np.array([0, 7, 7]), np.array([0, 100, 101]), z, np.array([0, 65537, 65537]))
    assert ids[0] == 0 and ids[1] != ids[2] and len(xi) == 3
    tab = xi.table().view(np.uint32)
    assert tuple(tab[ids[2]]) == (7, 101, 0, 65537) and tuple(tab[0]) == (0, 0, 0, 0)
    again = xi.ids(np.array([7, 9]), np.array([101, 1]), np.zeros(2), np.array([65537, 1]))
    assert again[0] == ids[2] and again[1] == 3 and np.array_equal(xi.table()[:3], tab.view(np.int32))
    win = _win()
    ev = win.events.copy()
    ev["ts_ns"][0] = ev["ts_ns"][1:].min() + (1 << 32)
    import pytest

    with pytest.raises(ValueError):
        records.to_wire20(ev, records.ConnInterner(), records.CtxInterner())


def test_native_encoder_matches_numpy_reference():
    """runtime/csrc/wire.cpp == records.to_wire20 / to_wire16 up to id numbering."""
    pytest = __import__("pytest")
    try:
        enc20, enc16 = records.native_encoder(), records.native_encoder()
    except RuntimeError:
        pytest.skip("native runtime not built")
    win = _win(seed=6)
    ev = win.events.copy()
    ev["ts_ns"][7] = 0
    buf = np.zeros(ev.shape[0] * 20, dtype=np.uint8)
    t_base = enc20.encode(ev, buf, 20)
    n20 = buf.view(records.EVENT20)
    conns, ctxs = records.ConnInterner(), records.CtxInterner()
    r20, tb = records.to_wire20(ev, conns, ctxs)
    assert t_base == tb
    for f in ("ts_off", "value_milli", "trace_h"):
        np.testing.assert_array_equal(n20[f], r20[f], err_msg=f)
    a = oracle.decode_w20(n20, t_base, enc20.ctx_table())
    b = oracle.decode_w20(r20, tb, ctxs.table())
    for f in ("ts", "slot", "pod", "pid", "svcnode", "trace"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    # same connection equivalence classes (ids may be numbered differently)
    pairs = set(zip(a.conn.tolist(), b.conn.tolist()))
    assert len(pairs) == len(set(a.conn.tolist())) == len(set(b.conn.tolist()))
    # EVENT16: trace ids shared with the spans reproduce the 64-byte join exactly
    buf16 = np.zeros(ev.shape[0] * 16, dtype=np.uint8)
    tb16 = enc16.encode(ev, buf16, 16)
    sp16 = np.zeros_like(win.spans)
    enc16.encode_spans(win.spans, sp16, True)
    d16 = oracle.decode_w16(buf16.view(records.EVENT16), tb16, enc16.ctx_table())
    full = oracle.join(oracle.decode_events(ev), win.spans, win.n_groups)
    j16 = oracle.join(d16, sp16, win.n_groups)
    np.testing.assert_array_equal(full.top3, j16.top3)
    np.testing.assert_array_equal(full.cnt, j16.cnt)
    assert full.debug == j16.debug
    # numpy EVENT16 reference agrees too
    r16, _ = records.to_wire16(ev, records.ConnInterner(), records.CtxInterner(), records.TraceInterner())
    assert r16.dtype == records.EVENT16


def test_pooled_encode_window_is_byte_identical_to_sequential():
    """wire.cpp encode_window (3-phase worker pool) == encode() + encode_spans(), ids included,
    across windows (ids persist), thread counts, a window whose first event is not its
    earliest (timestamp rebase), zero timestamps, and connections first seen in spans."""
    pytest = __import__("pytest")
    try:
        seq, par = records.native_encoder(), records.native_encoder()
    except RuntimeError:
        pytest.skip("native runtime not built")
    for wire in (16, 20):
        seq, par = records.native_encoder(), records.native_encoder()
        for k, threads in enumerate((1, 3, 8, 5)):
            win = _win(seed=11 + k)
            ev, sp = win.events.copy(), win.spans.copy()
            if k == 1:
                ev = ev[::-1].copy()  # first record is the latest
            if k == 2:
                ev["ts_ns"][::97] = 0
                sp["conn_h"][::5] = np.arange(sp.shape[0])[::5].astype(np.uint64) * 7919 + 1  # span-only conns
            oa, ob = np.zeros(ev.shape[0] * wire, np.uint8), np.zeros(ev.shape[0] * wire, np.uint8)
            sa, sb = np.zeros_like(sp), np.zeros_like(sp)
            ta = seq.encode(ev, oa, wire)
            seq.encode_spans(sp, sa, wire == 16)
            tb = par.encode_window(ev, ob, wire, sp, sb, threads, 256)  # ~12 event + 6 span chunks
            seq.end_window()
            par.end_window()
            assert ta == tb
            np.testing.assert_array_equal(oa, ob, err_msg=f"wire {wire} window {k}")
            np.testing.assert_array_equal(sa.view(np.uint8), sb.view(np.uint8))
            np.testing.assert_array_equal(seq.ctx_table(), par.ctx_table())
            assert (seq.n_conns, seq.n_traces) == (par.n_conns, par.n_traces)
    # a window too wide for 32-bit offsets is refused before any table changes
    ev = _win(seed=3).events.copy()
    ev["ts_ns"][5] = ev["ts_ns"].max() + (1 << 33)
    n0 = par.n_ctx
    with pytest.raises(ValueError):
        par.encode_window(ev, np.zeros(ev.shape[0] * 16, np.uint8), 16, sp, np.zeros_like(sp), 4, 256)
    assert par.n_ctx == n0


def test_integer_milli_rule():
    """records.milli_int (and the probes' in-kernel mislo_milli): half-to-even, saturating;
    equal to the float rule rint(v * scale * 1000) away from exact halves."""
    shift = records.milli_shift_table()
    assert shift[1] == -3 and shift[2] == 3 and shift[6] == 0 and shift[200] == 3
    v = np.array([0, 499, 500, 501, 1500, 2500, 2501, 10 ** 15, 7], dtype=np.uint64)
    np.testing.assert_array_equal(records.milli_int(v, np.full(v.shape, -3)),
                                  [0, 0, 0, 1, 2, 2, 3, 10 ** 12 if 10 ** 12 < 2 ** 32 else 2 ** 32 - 1, 0])
    np.testing.assert_array_equal(records.milli_int(v[:4], np.full(4, 3)), [0, 499000, 500000, 501000])
    np.testing.assert_array_equal(records.milli_int(np.array([2 ** 40], np.uint64), np.array([0])), [2 ** 32 - 1])
    rng = np.random.default_rng(0)
    raw = rng.integers(0, 5 * 10 ** 9, 20000, dtype=np.uint64)
    raw = raw[raw % 1000 != 500]
    np.testing.assert_array_equal(records.milli_int(raw, np.full(raw.shape, -3)),
                                  np.clip(np.rint(raw.astype(np.float64) * 1e-6 * 1000.0), 0, 2 ** 32 - 1))


def test_native_event32_matches_numpy_compact():
    """Native EVENT32 (what the probes emit; bench --wire 32) == records.to_compact up to
    connection id numbering; spans mapped by the same encoder share the ids."""
    pytest = __import__("pytest")
    try:
        enc = records.native_encoder()
    except RuntimeError:
        pytest.skip("native runtime not built")
    win = _win(seed=9)
    ev = win.events
    buf = np.zeros(ev.shape[0] * 32, np.uint8)
    assert enc.encode(ev, buf, 32) == 0
    n32 = buf.view(records.EVENT32)
    r32 = records.to_compact(ev, records.ConnInterner())
    for f in ("ts_ns", "trace_h", "value_milli", "pid", "pod_id"):
        np.testing.assert_array_equal(n32[f], r32[f], err_msg=f)
    np.testing.assert_array_equal(n32["type_conn"] & 0xFF, r32["type_conn"] & 0xFF)
    a, b = (n32["type_conn"] >> 8).tolist(), (r32["type_conn"] >> 8).tolist()
    assert len(set(zip(a, b))) == len(set(a)) == len(set(b))
    assert (np.array(a) == 0).tolist() == (np.array(b) == 0).tolist()
    sp = np.zeros_like(win.spans)
    enc.encode_spans(win.spans, sp, False)
    ev_ids = dict(zip(records._conn_keys(ev).tolist(), a))
    for h, cid in zip(win.spans["conn_h"].tolist(), sp["conn_h"].tolist()):
        if h in ev_ids:
            assert cid == ev_ids[h]
    np.testing.assert_array_equal(sp["trace_h"], win.spans["trace_h"])


def test_event24_native_numpy_and_join():
    """EVENT24 (the probes' context-interned ring record): native == records.to_wire24 up to id
    numbering, and its decode joins exactly like the 64-byte records."""
    pytest = __import__("pytest")
    try:
        enc = records.native_encoder()
    except RuntimeError:
        pytest.skip("native runtime not built")
    win = _win(seed=12)
    ev = win.events
    buf = np.zeros(ev.shape[0] * 24, np.uint8)
    assert enc.encode(ev, buf, 24) == 0
    n24 = buf.view(records.EVENT24)
    ctxs = records.CtxInterner()
    r24 = records.to_wire24(ev, records.ConnInterner(), ctxs)
    for f in ("ts_ns", "trace_h", "value_milli"):
        np.testing.assert_array_equal(n24[f], r24[f], err_msg=f)
    a = oracle.decode_w24(n24, enc.ctx_table())
    b = oracle.decode_w24(r24, ctxs.table())
    for f in ("ts", "slot", "pod", "pid", "svcnode", "trace"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    sp = np.zeros_like(win.spans)
    enc.encode_spans(win.spans, sp, False)
    full = oracle.join(oracle.decode_events(ev), win.spans, win.n_groups)
    j24 = oracle.join(a, sp, win.n_groups)
    np.testing.assert_array_equal(full.top3, j24.top3)
    np.testing.assert_array_equal(full.cnt, j24.cnt)
    assert full.debug == j24.debug


def test_event20t_native_numpy_and_join():
    """EVENT20T (the probes' default ring record: kernel-interned contexts and trace ids, 20 bytes
    at 20-byte strides): native == records.to_wire20t up to id numbering, spans carry the same
    trace ids, and its decode joins exactly like the 64-byte records."""
    pytest = __import__("pytest")
    try:
        enc = records.native_encoder()
    except RuntimeError:
        pytest.skip("native runtime not built")
    assert records.EVENT20T.itemsize == 20 and records.wire_bytes(records.WIRE_20T) == 20
    assert records.wire_code(records.EVENT20T) == records.WIRE_20T and records.wire_code(records.EVENT20) == 20
    win = _win(seed=13)
    ev = win.events
    buf = np.zeros(ev.shape[0] * 20, np.uint8)
    assert enc.encode(ev, buf, records.WIRE_20T) == 0
    n20 = buf.view(records.EVENT20T)
    conns, ctxs, traces = records.ConnInterner(), records.CtxInterner(), records.TraceInterner()
    r20 = records.to_wire20t(ev, conns, ctxs, traces)
    for f in ("ts_ns", "value_milli"):
        np.testing.assert_array_equal(n20[f], r20[f], err_msg=f)
    # trace ids: same partition of the events (0 exactly for untraced ones)
    np.testing.assert_array_equal(n20["trace_id"] == 0, ev["trace_h"] == 0)
    pairs = set(zip(n20["trace_id"].tolist(), ev["trace_h"].tolist()))
    assert len(pairs) == len(set(ev["trace_h"].tolist()))
    a = oracle.decode_w20t(n20, enc.ctx_table())
    b = oracle.decode_w20t(r20, ctxs.table())
    for f in ("ts", "slot", "pod", "pid", "svcnode"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    sp = np.zeros_like(win.spans)
    enc.encode_spans(win.spans, sp, True)
    ids = dict(zip(ev["trace_h"].tolist(), n20["trace_id"].tolist()))
    for h, t in zip(win.spans["trace_h"].tolist(), sp["trace_h"].tolist()):
        if h in ids:
            assert t == ids[h]
    full = oracle.join(oracle.decode_events(ev), win.spans, win.n_groups)
    j20 = oracle.join(a, sp, win.n_groups)
    np.testing.assert_array_equal(full.top3, j20.top3)
    np.testing.assert_array_equal(full.cnt, j20.cnt)
    assert full.debug == j20.debug
    jr = oracle.join(b, records.wire_spans(win.spans, conns, traces), win.n_groups)
    np.testing.assert_array_equal(full.top3, jr.top3)
    assert full.debug == jr.debug


def test_event16_epoch_tags_decode_like_one_base():
    """EVENT16 as the probes write it with -DMISLO_RING_EVENT16: offsets from the epoch the agent
    last published, tagged with it (4 bases per window). Decoding with the window's bases gives
    the timestamps and trace ids of the single-base encoding, and joins identically."""
    pytest = __import__("pytest")
    try:
        enc = records.native_encoder()
    except RuntimeError:
        pytest.skip("native runtime not built")
    win = _win(seed=14)
    ev = win.events.copy()
    ev["ts_ns"][7] = 0
    buf = np.zeros(ev.shape[0], dtype=records.EVENT16)
    t_base = enc.encode(ev, buf.view(np.uint8).reshape(-1), 16)
    assert int((buf["trace_id"] >> np.uint32(30)).max()) == 0  # host encoding: tag 0
    tagged, bases = records.retag_epochs(buf, t_base, 256_000_000)
    tags = tagged["trace_id"] >> np.uint32(30)
    assert set(np.unique(tags).tolist()) == {0, 1, 2, 3}
    assert int(tagged["ts_off"][7]) == records.TS_ZERO
    one = oracle.decode_w16(buf, t_base, enc.ctx_table())
    four = oracle.decode_w16(tagged, t_base, enc.ctx_table(), bases=bases)
    for f in ("ts", "slot", "pod", "pid", "svcnode", "trace", "val"):
        np.testing.assert_array_equal(getattr(one, f), getattr(four, f), err_msg=f)
    np.testing.assert_array_equal(four.ts, np.where(ev["ts_ns"] == 0, 0, ev["ts_ns"]))
    c = records.counts_row(10, 2, 1, 0, bases, 5)
    assert c.shape == (records.COUNTS_LEN,) and int(c[6]) == 5
    got = [int(np.uint64(c[lo].astype(np.uint32)) | (np.uint64(c[lo + 1].astype(np.uint32)) << np.uint64(32)))
           for lo in (4, 8, 10, 12)]
    assert got == list(bases)


def test_epoch_clock_protocol_across_cuts():
    """Agent/probe epoch protocol: records stamped against any of the last 4 published epochs
    (a probe that read the epoch before a cut writes after it) decode to their exact timestamps
    with the bases the window ships."""
    clk = records.EpochClock()
    t0 = 1_700_000_000_123_456_789
    cfgs = [clk.publish(t0 + k * 1_000_000_007) for k in range(6)]  # 6 cuts: tags wrap
    bases = clk.bases()
    rng = np.random.default_rng(3)
    for k in range(2, 6):  # records stamped against epochs k, k-1, k-2 (late writers)
        for lag in range(3):
            cfg = cfgs[k - lag]
            ts = (cfg & ~3) + int(rng.integers(0, 2_500_000_000))
            off, tag = records.EpochClock.stamp(ts, cfg)
            assert tag == (k - lag) & 3
            if k == 5:  # the window after the last cut carries bases of epochs 2..5
                assert bases[tag] + off == ts
    assert records.EpochClock.stamp(0, cfgs[0]) == (records.TS_ZERO, cfgs[0] & 3)


def test_span20_native_matches_numpy_reference():
    """SPAN20 (20-byte spans on the event interners): native encode_spans20 == records.to_span20
    field for field once context ids are resolved through each side's context table, and trace
    ids agree with the events' EVENT20T trace ids."""
    pytest = __import__("pytest")
    try:
        enc = records.native_encoder()
    except RuntimeError:
        pytest.skip("native runtime not built")
    win = _win(seed=15)
    ev, sp = win.events, win.spans
    buf = np.zeros(ev.shape[0] * 20, np.uint8)
    enc.encode(ev, buf, records.WIRE_20T)
    n20 = buf.view(records.EVENT20T)
    s_nat = np.zeros(sp.shape[0], dtype=records.SPAN20)
    enc.encode_spans20(sp, s_nat.view(np.uint8).reshape(-1))
    conns, ctxs, traces = records.ConnInterner(), records.CtxInterner(), records.TraceInterner()
    records.to_wire20t(ev, conns, ctxs, traces)
    s_ref = records.to_span20(sp, conns, ctxs, traces)
    np.testing.assert_array_equal(s_nat["ts_ns"], sp["ts_ns"])
    np.testing.assert_array_equal(s_nat["group_id"], sp["group_id"])
    np.testing.assert_array_equal(s_nat["ts_ns"], s_ref["ts_ns"])
    tn, tr = enc.ctx_table().view(np.uint32), ctxs.table().view(np.uint32)
    rows_n, rows_r = tn[s_nat["ctx_id"]], tr[s_ref["ctx_id"]]
    for col in (0, 1, 3):  # pod, pid, svc|node (col 2 = conn id: numbering differs, checked below)
        np.testing.assert_array_equal(rows_n[:, col], rows_r[:, col])
    np.testing.assert_array_equal(rows_n[:, 0], sp["pod_id"])
    # same trace -> same id as the events carry; same conn hash -> same conn id as events
    ev_trace = dict(zip(ev["trace_h"].tolist(), n20["trace_id"].tolist()))
    for h, t in zip(sp["trace_h"].tolist(), s_nat["trace_id"].tolist()):
        assert (t == 0) == (h == 0)
        if h in ev_trace:
            assert t == ev_trace[h]
    ev_conn = dict(zip(records._conn_keys(ev).tolist(), tn[n20["ctx_type"] >> np.uint32(8)][:, 2].tolist()))
    for h, cid in zip(sp["conn_h"].tolist(), rows_n[:, 2].tolist()):
        if h in ev_conn and h:
            assert cid == ev_conn[h]
    c = records.counts_row(1, 1, 1, span_bytes=20)
    assert int(c[7]) == 20 and int(records.counts_row(1, 1, 1)[7]) == 0

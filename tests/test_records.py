"""Record layouts: REF 40-byte records, 64-byte EVENT/SPAN, the 16-byte EVENT16 the BPF ring
carries (8 to a 136-byte ring record), SPAN20; the integer fixed-point rule and the epoch
protocol (the ring path itself: tests/test_bpfring.py)."""

import pytest
import numpy as np

from llm_slo_ebpf_toolkit_amd.collector import records


def test_layout_sizes():
    assert records.EVENT.itemsize == 64
    assert records.EVENT16.itemsize == 16
    assert records.SPAN.itemsize == 64
    assert records.SPAN20.itemsize == 20
    assert records.REF_EVENT.itemsize == 40
    assert records.REC_STRIDE == 136 and records.BATCH_SLOTS == 8  # 8-slot batch records
    assert records.WIRE_DTYPES == {64: records.EVENT, 16: records.EVENT16}


def test_conn32_is_a_nonzero_fold():
    k = np.array([0, 1, 0xFFFFFFFF00000000, 0x123456789ABCDEF0], dtype=np.uint64)
    c = records.conn32_np(k)
    assert c[0] == 0 and (c[1:] % 2 == 1).all()
    assert [records.conn32(int(x)) for x in k] == c.tolist()


def test_ref_record_roundtrip():
    from llm_slo_ebpf_toolkit_amd.signals.metadata import Metadata

    raw = records.encode_ref_record(11, 12, 1234, 1, 5_000_000, 4000, 53, 0x0100007F, 110)
    meta = Metadata(node="n1", namespace="ns", pod="p", container="c", trace_id="t", span_id="s")
    ev = records.decode_ref_record(raw, meta, 99)
    assert ev.pid == 11 and ev.tid == 12 and ev.ts_unix_nano == 99
    assert ev.signal == "dns_latency_ms" and abs(ev.value - 5.0) < 1e-12 and ev.errno == 110
    assert ev.conn_tuple.dst_port == 53 and ev.conn_tuple.dst_ip == "127.0.0.1"
    assert ev.node == "n1" and ev.trace_id == "t"


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


def test_user24_roundtrip_against_user32():
    """USER24 keeps everything the decode reads of USER32: timestamps within +-2.4 h of the
    window's base come back exact (0 stays 0), pid / pod / type / value / trace unchanged."""
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

    w = ReplayGenerator(ReplayConfig(scenario="full", events_per_window=4096, spans_per_window=64, seed=5)).next_window()
    ev = w.events.copy()
    ev["ts_ns"][:3] = 0
    ev["ts_ns"][3] = int(w.t0_ns) + 2 * 3600 * 10**9      # 2 h after the base
    ev["ts_ns"][4] = int(w.t0_ns) - 2 * 3600 * 10**9      # 2 h before
    u24 = records.to_user24(ev)
    assert u24.itemsize == 24
    back = records.user24_to_user32(u24, int(w.t0_ns))
    u32 = records.to_user32(ev)
    for f in ("ts_ns", "trace_h", "value_milli", "pod_id", "pid", "signal_type"):
        assert np.array_equal(back[f], u32[f]), f
    assert (back["flags"] == u32["flags"]).all()  # has_gpu
    assert records.to_user(ev, 24).tobytes() == u24.tobytes()
    bad = ev[:1].copy()
    bad["pid"] = 1 << 22
    with pytest.raises(ValueError):
        records.to_user24(bad)


def test_user24_windows_decode_like_user32():
    """The probe-model images of the same replay windows with USER24 and USER32 user rings decode
    (pipeline/oracle.py, the GPU decode's reference) to identical rows: USER24 loses nothing the
    window decode reads, with timestamps resolved against the window's newest epoch base."""
    from llm_slo_ebpf_toolkit_amd.pipeline import oracle
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_replay_images

    def decoded(rec):
        g = ReplayGenerator(ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=8,
                                         events_per_window=3000, spans_per_window=100, seed=9))
        wins = [g.next_window() for _ in range(3)]
        imgs = build_replay_images(wins, user_rec=rec)
        sn = (g.pod_svc.astype(np.uint32) << np.uint32(16)) | g.pod_node.astype(np.uint32)
        pod_sn = dict(zip(g.pod_ids.tolist(), sn.tolist()))
        table, tmap = oracle.CtxTable(), oracle.TraceMap()
        out = []
        for img in imgs:
            assert img.user.dtype.itemsize == rec and len(img.user)
            oracle.apply_ring_defs(img.framed, table, tmap, pod_sn)
            out.append(oracle.decode_window(img.framed, img.user, table, tmap, img.bases, pod_sn=pod_sn))
        return out

    for a, b in zip(decoded(24), decoded(32)):
        for f in a.__dataclass_fields__:
            assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_user16_roundtrip_and_continuation_slots():
    """USER16 is USER24 without the trace hash: an untraced record is one 16-byte slot, a traced one
    two (the record with pid_sig bit 31, then {trace lo, trace hi, USER16_CONT, 0}); decoded, the
    records equal USER24's and the continuation slots are holes."""
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

    w = ReplayGenerator(ReplayConfig(scenario="full", events_per_window=4096, spans_per_window=64, seed=5)).next_window()
    ev = w.events[w.events["signal_type"] < 127].copy()
    ev["trace_h"][::4] = np.arange(len(ev[::4]), dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)
    ev["trace_h"][1::4] = 0
    u16 = records.to_user16(ev)
    traced = ev["trace_h"] != 0
    assert u16.itemsize == 16 and len(u16) == len(ev) + int(traced.sum())
    v, cont = records.user16_to_user24(u16)
    assert int(cont.sum()) == int(traced.sum())
    u24 = records.to_user24(ev)
    for f in u24.dtype.names:
        assert np.array_equal(v[~cont][f], u24[f]), f
    assert records.to_user(ev, 16).tobytes() == u16.tobytes()
    bad = ev[:1].copy()
    bad["signal_type"] = 127
    with pytest.raises(ValueError):
        records.to_user16(bad)


def test_user16_windows_decode_like_user24():
    """The oracle decode of the same windows with USER16 and USER24 user rings: identical rows once
    the continuation slots (holes) are taken out, traced records keeping their traces."""
    from llm_slo_ebpf_toolkit_amd.pipeline import oracle
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_replay_images, kernel_event_mask

    def decoded(rec):
        g = ReplayGenerator(ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=8,
                                         events_per_window=3000, spans_per_window=100, seed=9))
        wins = [g.next_window() for _ in range(2)]
        for w in wins:
            gpu = np.nonzero(~kernel_event_mask(w.events))[0][::2]
            w.events["trace_h"][gpu] = w.spans["trace_h"][np.arange(len(gpu)) % len(w.spans)]
        imgs = build_replay_images(wins, user_rec=rec)
        sn = (g.pod_svc.astype(np.uint32) << np.uint32(16)) | g.pod_node.astype(np.uint32)
        pod_sn = dict(zip(g.pod_ids.tolist(), sn.tolist()))
        table, tmap = oracle.CtxTable(), oracle.TraceMap()
        out = []
        for img in imgs:
            oracle.apply_ring_defs(img.framed, table, tmap, pod_sn)
            d = oracle.decode_window(img.framed, img.user, table, tmap, img.bases, pod_sn=pod_sn)
            n_k = records.framed_rows(img.framed)
            keep = np.ones(len(d.ts), bool)
            if rec == 16:
                cont = img.user["pid_sig"] == np.uint32(records.USER16_CONT)
                assert cont.any()
                keep[n_k:] = ~cont
                assert (d.slot[n_k:][cont] == oracle.NO_SLOT).all() and (d.ts[n_k:][cont] == 0).all()
            out.append(oracle.take(d, keep))
        return out

    for a, b in zip(decoded(16), decoded(24)):
        for f in a.__dataclass_fields__:
            assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_user24_window_without_epoch_is_refused():
    """WindowPipeline.submit refuses USER24 records with no epoch base to resolve them against
    (checked before the engine is touched, so this runs without a GPU)."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline

    pipe = WindowPipeline.__new__(WindowPipeline)  # no engine: the check comes first
    with pytest.raises(ValueError):
        pipe.submit([], [(0x1000, 24)], [], 1, bases=(0, 0, 0, 0), user_rec=24)

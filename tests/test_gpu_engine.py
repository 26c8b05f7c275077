"""GPU engine vs the CPU oracle on small replay windows (exact keys/tiers/counts)."""

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes, SufficientStats
from llm_slo_ebpf_toolkit_amd.ops.engine import signal_rows as rows
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

pytestmark = pytest.mark.gpu


def small_window(seed=1, n=4096, s=256, services=8, scenario="full"):
    cfg = ReplayConfig(scenario=scenario, n_nodes=2, pods_per_node=8, n_services=services, events_per_window=n,
                       spans_per_window=s, seed=seed)
    return ReplayGenerator(cfg).next_window()


@pytest.fixture(scope="module")
def engine():
    from llm_slo_ebpf_toolkit_amd.ops.engine import GpuEngine

    return GpuEngine(sig_cap=8192, span_cap=512, group_cap=64)


def test_extension_is_native(engine):
    import llm_slo_ebpf_toolkit_amd.ops as ops

    assert ops.available()
    assert engine.mod.__file__.endswith(".so")


@pytest.mark.parametrize("group_mode", [1, 0])
def test_decode_join_matches_oracle(engine, group_mode):
    win = small_window()
    engine.set_join_params(2000.0, 0.7, 3, group_mode)
    engine.set_model(NaiveBayes.ref())
    out = engine.process(win.events, win.spans, win.n_groups, win.group_labels)
    e = engine.eng
    d = oracle.decode_events(win.events)
    N, S = win.n_events, win.n_spans
    np.testing.assert_array_equal(rows(e, N)["slot"], d.slot.astype(np.uint32))
    np.testing.assert_array_equal(rows(e, N)["val"], d.val)
    np.testing.assert_array_equal(out.hist, oracle.histograms(d))
    np.testing.assert_array_equal(e.misc[2:18].cpu().numpy(), oracle.value_sums_milli(d))
    ref = oracle.join(d, win.spans, win.n_groups, group_mode=group_mode)
    top3 = e.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    np.testing.assert_array_equal(e.cnt[:S].cpu().numpy(), ref.cnt)
    np.testing.assert_array_equal(e.attrs[:S].cpu().numpy(), ref.attrs)
    np.testing.assert_array_equal(e.conf[:S].cpu().numpy(), ref.conf)
    for k in ("candidates", "low_confidence", "fanout_dropped", "unmatched", "unsupported_type", "spans_enriched"):
        assert out.debug[k] == ref.debug[k], k
    np.testing.assert_array_equal(e.gsum[: win.n_groups].cpu().numpy(), ref.gsum)
    np.testing.assert_array_equal(e.gcnt[: win.n_groups].cpu().numpy(), ref.gcnt)
    np.testing.assert_array_equal(out.feat, ref.feat)


def test_low_threshold_enumerates_service_node_tier(engine):
    win = small_window(seed=3, n=2048, s=128)
    engine.set_join_params(2000.0, 0.6, 3, 1)
    engine.set_model(NaiveBayes.ref())
    out = engine.process(win.events, win.spans, win.n_groups, win.group_labels)
    d = oracle.decode_events(win.events)
    ref = oracle.join(d, win.spans, win.n_groups, threshold=0.6)
    S = win.n_spans
    top3 = engine.eng.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    for k in ("candidates", "low_confidence", "unmatched"):
        assert out.debug[k] == ref.debug[k], k
    engine.set_join_params(2000.0, 0.7, 3, 1)


def test_posterior_matches_cpu_model(engine):
    win = small_window(seed=5)
    for model in (NaiveBayes.ref(),):
        engine.set_model(model)
        out = engine.process(win.events, win.spans, win.n_groups, win.group_labels)
        post_cpu = model.posteriors(out.feat.astype(np.float64))
        np.testing.assert_allclose(out.post[:, :10], post_cpu, rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(out.pred, np.argmax(model.logits(out.feat.astype(np.float64)), axis=1))
        bits = model.evidence_bits(out.feat.astype(np.float64))
        np.testing.assert_array_equal(out.evbits[:, :10], bits)
        conf = np.zeros((16, 16), dtype=np.int64)
        np.add.at(conf, (win.group_labels, out.pred), 1)
        np.testing.assert_array_equal(out.confusion, conf)


def test_stats_matches_cpu(engine):
    win = small_window(seed=7)
    model = NaiveBayes.ref()
    engine.set_model(model)
    engine.stage(win.events, win.spans, win.n_groups, win.group_labels)
    engine.upload()
    engine.run(True, learn=True)
    out = engine.outputs()
    st = SufficientStats()
    st.add(out.feat.astype(np.float64), win.group_labels)
    gpu = engine.eng.stats.cpu().numpy()
    cnt = engine.eng.stats_count.cpu().numpy()
    np.testing.assert_allclose(cnt[:10], st.count, rtol=1e-12)
    np.testing.assert_allclose(gpu[:16, :10], st.elevated_sum, rtol=1e-12)
    np.testing.assert_allclose(gpu[16:, :10], st.x_sum, rtol=1e-9)
    np.testing.assert_allclose(gpu[16:, 16:], st.xx, rtol=1e-9)


def test_ref_record_decode(engine):
    import torch
    from llm_slo_ebpf_toolkit_amd.collector import records

    recs = [records.encode_ref_record(7, 8, 1_000_000_000 + i, t, v, 4000 if t in (1, 4) else 0, 53 if t == 1 else 0)
            for i, (t, v) in enumerate([(1, 220_000_000), (2, 3), (6, 1500), (9, 51_000_000), (42, 1)])]
    buf = np.frombuffer(b"".join(recs), dtype=np.uint8)
    dev = torch.zeros(engine.sig_cap * 40, dtype=torch.uint8, device="cuda")
    dev[: buf.size] = torch.from_numpy(buf.copy()).cuda()
    engine.eng.counts[:4].copy_(torch.tensor([5, 0, 0, 0], dtype=torch.int32))
    engine.eng.reset_window()
    engine.eng.decode_ref(dev, 3, (1 << 16) | 2, 0)
    torch.cuda.synchronize()
    val = rows(engine.eng, 5)["val"]
    slot = rows(engine.eng, 5)["slot"]
    # REF convertValue (ringbuf.go:229-238): unknown types fall into the ns -> ms default
    np.testing.assert_allclose(val, [220.0, 3.0, 1500.0, 51.0, 1e-6], rtol=1e-6)
    assert list(slot) == [0, 1, 7, 11, 255]
    assert int(engine.eng.misc[0].item()) == 1


def test_compact_wire_matches_oracle(engine):
    from llm_slo_ebpf_toolkit_amd.collector import records

    win = small_window(seed=11)
    engine.set_join_params(2000.0, 0.7, 3, 1)
    engine.set_model(NaiveBayes.ref())
    interner = records.ConnInterner()
    table = records.pod_table(win.events, win.spans)
    ev32 = records.to_compact(win.events, interner)
    sp = records.compact_spans(win.spans, interner)
    engine.set_pod_table(table)
    out = engine.process(ev32, sp, win.n_groups, win.group_labels)
    e = engine.eng
    d = oracle.decode_compact(ev32, table)
    N, S = win.n_events, win.n_spans
    np.testing.assert_array_equal(rows(e, N)["slot"], d.slot.astype(np.uint32))
    np.testing.assert_array_equal(rows(e, N)["val"], d.val)
    np.testing.assert_array_equal(rows(e, N)["svcnode"], d.svcnode)
    ref = oracle.join(d, sp, win.n_groups)
    top3 = e.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    np.testing.assert_array_equal(e.attrs[:S].cpu().numpy(), ref.attrs)
    for k in ("candidates", "low_confidence", "fanout_dropped", "unmatched", "unsupported_type", "spans_enriched"):
        assert out.debug[k] == ref.debug[k], k
    np.testing.assert_array_equal(e.gsum[: win.n_groups].cpu().numpy(), ref.gsum)
    np.testing.assert_array_equal(e.gcnt[: win.n_groups].cpu().numpy(), ref.gcnt)
    np.testing.assert_array_equal(out.feat, ref.feat)


def test_wire20_matches_oracle(engine):
    from llm_slo_ebpf_toolkit_amd.collector import records

    win = small_window(seed=17)
    engine.set_join_params(2000.0, 0.7, 3, 1)
    engine.set_model(NaiveBayes.ref())
    conns, ctxs = records.ConnInterner(), records.CtxInterner()
    ev = win.events.copy()
    ev["ts_ns"][3] = 0
    ev20, t_base = records.to_wire20(ev, conns, ctxs)
    sp = records.compact_spans(win.spans, conns)
    engine.set_ctx_table(ctxs.table())
    engine.stage(ev20, sp, win.n_groups, win.group_labels, t_base=t_base)
    engine.upload()
    engine.run(True, False)
    out = engine.outputs()
    e = engine.eng
    d = oracle.decode_w20(ev20, t_base, ctxs.table())
    N, S = win.n_events, win.n_spans
    np.testing.assert_array_equal(rows(e, N)["ts"], d.ts)
    np.testing.assert_array_equal(rows(e, N)["slot"], d.slot.astype(np.uint32))
    np.testing.assert_array_equal(rows(e, N)["val"], d.val)
    np.testing.assert_array_equal(rows(e, N)["pid"], d.pid)
    np.testing.assert_array_equal(rows(e, N)["svcnode"], d.svcnode)
    ref = oracle.join(d, sp, win.n_groups)
    top3 = e.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    np.testing.assert_array_equal(e.attrs[:S].cpu().numpy(), ref.attrs)
    for k in ("candidates", "low_confidence", "fanout_dropped", "unmatched", "unsupported_type", "spans_enriched"):
        assert out.debug[k] == ref.debug[k], k
    np.testing.assert_array_equal(e.gsum[: win.n_groups].cpu().numpy(), ref.gsum)
    np.testing.assert_array_equal(out.feat, ref.feat)
    assert int(e.misc[1].item()) == 1  # the zero timestamp


def test_wire20t_matches_oracle(engine):
    """EVENT20T (the probes' default 20-byte ring record, interned trace ids, 4-byte aligned at
    20-byte strides) -> GPU decode + join == numpy oracle, zero timestamp included."""
    from llm_slo_ebpf_toolkit_amd.collector import records

    win = small_window(seed=21)
    engine.set_join_params(2000.0, 0.7, 3, 1)
    engine.set_model(NaiveBayes.ref())
    conns, ctxs, traces = records.ConnInterner(), records.CtxInterner(), records.TraceInterner()
    ev = win.events.copy()
    ev["ts_ns"][5] = 0
    e20 = records.to_wire20t(ev, conns, ctxs, traces)
    sp = records.wire_spans(win.spans, conns, traces)
    engine.set_ctx_table(ctxs.table())
    engine.stage(e20, sp, win.n_groups, win.group_labels)
    assert engine.wire == records.WIRE_20T
    engine.upload()
    engine.run(True, False)
    out = engine.outputs()
    e = engine.eng
    d = oracle.decode_w20t(e20, ctxs.table())
    N, S = win.n_events, win.n_spans
    np.testing.assert_array_equal(rows(e, N)["ts"], d.ts)
    np.testing.assert_array_equal(rows(e, N)["slot"], d.slot.astype(np.uint32))
    np.testing.assert_array_equal(rows(e, N)["val"], d.val)
    np.testing.assert_array_equal(rows(e, N)["pid"], d.pid)
    np.testing.assert_array_equal(rows(e, N)["svcnode"], d.svcnode)
    ref = oracle.join(d, sp, win.n_groups)
    top3 = e.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    np.testing.assert_array_equal(e.attrs[:S].cpu().numpy(), ref.attrs)
    for k in ("candidates", "low_confidence", "fanout_dropped", "unmatched", "unsupported_type", "spans_enriched"):
        assert out.debug[k] == ref.debug[k], k
    np.testing.assert_array_equal(out.feat, ref.feat)
    assert int(e.misc[1].item()) == 1  # the zero timestamp


def test_wire16_epoch_tags_match_oracle(engine):
    """EVENT16 with 2-bit epoch tags (the probes' -DMISLO_RING_EVENT16 record): the decode kernel
    picks each record's base from counts[4..5] / [8..13]; decode + join == numpy oracle."""
    from llm_slo_ebpf_toolkit_amd.collector import records

    win = small_window(seed=25)
    engine.set_join_params(2000.0, 0.7, 3, 1)
    engine.set_model(NaiveBayes.ref())
    conns, ctxs, traces = records.ConnInterner(), records.CtxInterner(), records.TraceInterner()
    ev = win.events.copy()
    ev["ts_ns"][2] = 0
    e16, t_base = records.to_wire16(ev, conns, ctxs, traces)
    e16, bases = records.retag_epochs(e16, t_base, 200_000_000)
    assert len(set((e16["trace_id"] >> np.uint32(30)).tolist())) > 1
    sp = records.wire_spans(win.spans, conns, traces)
    engine.set_ctx_table(ctxs.table())
    engine.stage(e16, sp, win.n_groups, win.group_labels, bases=bases)
    engine.upload()
    engine.run(True, False)
    out = engine.outputs()
    e = engine.eng
    d = oracle.decode_w16(e16, t_base, ctxs.table(), bases=bases)
    N, S = win.n_events, win.n_spans
    np.testing.assert_array_equal(rows(e, N)["ts"], d.ts)
    np.testing.assert_array_equal(d.ts, ev["ts_ns"])
    np.testing.assert_array_equal(rows(e, N)["slot"], d.slot.astype(np.uint32))
    ref = oracle.join(d, sp, win.n_groups)
    top3 = e.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    for k in ("candidates", "low_confidence", "fanout_dropped", "unmatched", "unsupported_type", "spans_enriched"):
        assert out.debug[k] == ref.debug[k], k
    np.testing.assert_array_equal(out.feat, ref.feat)


def test_wire16_native_matches_oracle(engine):
    """Native encoder (EVENT16, interned trace ids) -> GPU decode + join == numpy oracle."""
    from llm_slo_ebpf_toolkit_amd.collector import records

    win = small_window(seed=19)
    engine.set_join_params(2000.0, 0.7, 3, 1)
    engine.set_model(NaiveBayes.ref())
    enc = records.native_encoder()
    buf = np.zeros(win.n_events * 16, dtype=np.uint8)
    t_base = enc.encode(win.events, buf, 16)
    sp = np.zeros_like(win.spans)
    enc.encode_spans(win.spans, sp, True)
    ev16 = buf.view(records.EVENT16)
    engine.set_ctx_table(enc.ctx_table())
    engine.stage(ev16, sp, win.n_groups, win.group_labels, t_base=t_base)
    engine.upload()
    engine.run(True, False)
    out = engine.outputs()
    e = engine.eng
    d = oracle.decode_w16(ev16, t_base, enc.ctx_table())
    S = win.n_spans
    np.testing.assert_array_equal(rows(e, win.n_events)["ts"], d.ts)
    ref = oracle.join(d, sp, win.n_groups)
    top3 = e.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    np.testing.assert_array_equal(out.feat, ref.feat)
    # interning is exact: the same join as on the full 64-byte records
    full = oracle.join(oracle.decode_events(win.events), win.spans, win.n_groups)
    np.testing.assert_array_equal(ref.top3, full.top3)
    assert ref.debug == full.debug


def test_split_pre_post_equals_run_window(engine):
    """Global-incident-scope split (pre -> [group all-reduce] -> post) == one-shot window;
    and n_local excludes imported records from the counters but not from the join."""
    import torch

    win = small_window(seed=13)
    engine.set_join_params(2000.0, 0.7, 3, 1)
    engine.set_model(NaiveBayes.ref())
    out = engine.process(win.events, win.spans, win.n_groups, win.group_labels)
    e = engine.eng
    feat_a, post_a, pk_a = out.feat.copy(), out.post.copy(), e.packet.cpu().numpy().copy()
    e.run_window_pre(engine.ev_dev, engine.sp_dev, win.n_groups, 64)
    e.run_window_post(win.n_groups, True, False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(e.feat[: win.n_groups].cpu().numpy(), feat_a)
    np.testing.assert_array_equal(e.post[: win.n_groups].cpu().numpy(), post_a)
    np.testing.assert_array_equal(e.packet.cpu().numpy(), pk_a)
    # n_local: count only the first half of the events
    half = win.n_events // 2
    e.counts[:4].copy_(torch.tensor([win.n_events, win.n_spans, win.n_groups, half], dtype=torch.int32))
    e.run_window(engine.ev_dev, engine.sp_dev, win.n_groups, True, False, 64)
    torch.cuda.synchronize()
    d = oracle.decode_events(win.events[:half])
    np.testing.assert_array_equal(e.hist.cpu().numpy().astype(np.int64), oracle.histograms(d))
    np.testing.assert_array_equal(e.misc[2:18].cpu().numpy(), oracle.value_sums_milli(d))
    top3 = e.top3[: 3 * win.n_spans].cpu().numpy().view(np.uint64).reshape(win.n_spans, 3)
    ref = oracle.join(oracle.decode_events(win.events), win.spans, win.n_groups)
    np.testing.assert_array_equal(top3, ref.top3)
    e.counts[:4].copy_(torch.tensor([win.n_events, win.n_spans, win.n_groups, 0], dtype=torch.int32))


def test_device_refit_matches_host_learned_model(engine):
    """k_refit_nb == NaiveBayes.learned on the same sufficient statistics."""
    import torch

    from llm_slo_ebpf_toolkit_amd.models.bayes import N_DOMAINS
    from llm_slo_ebpf_toolkit_amd.ops.engine import MODEL_DTYPE, model_bytes

    win = small_window(seed=17)
    engine.set_model(NaiveBayes.ref())
    out = engine.process(win.events, win.spans, win.n_groups, win.group_labels, learn=True)
    st = SufficientStats()
    st.add(out.feat.astype(np.float64), win.group_labels)
    acc = np.zeros(1040)
    S = np.zeros((32, 32))
    S[:16, :N_DOMAINS] = st.elevated_sum
    acc[:1024] = S.ravel()
    acc[1024:1024 + N_DOMAINS] = st.count
    p0 = np.zeros((16, 16))
    p0[:, :N_DOMAINS] = NaiveBayes.random_init_table(42)
    host = NaiveBayes.learned(st, seed=42)
    engine.eng.set_model_bytes(torch.from_numpy(model_bytes(NaiveBayes.learned(SufficientStats(), seed=42))))
    engine.eng.refit_nb(torch.from_numpy(acc).cuda(), torch.from_numpy(p0.ravel()).cuda(), 2.0, 1.0, N_DOMAINS)
    torch.cuda.synchronize()
    dev = np.frombuffer(engine.eng.model.cpu().numpy().tobytes(), dtype=MODEL_DTYPE)[0]
    ref = np.frombuffer(model_bytes(host).tobytes(), dtype=MODEL_DTYPE)[0]
    np.testing.assert_allclose(dev["w"], ref["w"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(dev["bias"][:N_DOMAINS], ref["bias"][:N_DOMAINS], rtol=1e-13)
    assert np.isneginf(dev["bias"][N_DOMAINS:]).all()
    np.testing.assert_array_equal(dev["dom_mask"], ref["dom_mask"])
    assert dev["table_mask"] == ref["table_mask"] and dev["mode"] == 0


def test_pipeline_wire20_equals_wire32():
    """The pipelined engine gives bit-identical window totals on 32-, 20- and 16-byte records
    (native encoder, append-only context table uploads, graphs, device refit)."""
    import torch

    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline, stage_window

    cfg = ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=8, events_per_window=6000,
                       spans_per_window=300, seed=23)
    gen = ReplayGenerator(cfg)
    wins = [gen.next_window() for _ in range(3)]
    sums = {}
    for wire in (32, 21, 20, 16):
        it, enc = records.ConnInterner(), records.native_encoder()
        staged = [stage_window(torch, w.events, w.spans, w.n_groups, w.group_labels, 8, w.group_domains, wire=wire,
                               interner=it, encoder=enc) for w in wins]
        pipe = WindowPipeline(8192, 512, 8, 0, None, model="bayes_learned")
        for i in range(6):
            pipe.submit(staged[i % 3])
        sums[wire] = pipe.summary()
    for wire in (21, 20, 16):
        for k in ("confusion", "hist", "status", "dbg", "misc"):
            np.testing.assert_array_equal(sums[wire][k], sums[32][k], err_msg=f"{wire} {k}")


@pytest.mark.gpu
def test_wire_stager_matches_prestaged_windows():
    """bench.py's per-step staging (WireStager: probe-native EVENT32 / EVENT24 / EVENT20T rings + span mapping,
    pooled 16/20-byte encoding, pinned 64-byte ring) reproduces the totals of windows staged
    up front with stage_window."""
    import torch

    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline, WireStager, stage_window

    cfg = ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=8, events_per_window=6000,
                       spans_per_window=300, seed=29)
    gen = ReplayGenerator(cfg)
    wins = [gen.next_window() for _ in range(3)]
    pods = records.pod_table(np.concatenate([w.events for w in wins]), np.concatenate([w.spans for w in wins]))

    def totals_prestaged(wire):
        it, enc = records.ConnInterner(), records.native_encoder()
        staged = [stage_window(torch, w.events, w.spans, w.n_groups, w.group_labels, 8, w.group_domains, wire=wire,
                               interner=it, encoder=enc) for w in wins]
        pipe = WindowPipeline(8192, 512, 8, 0, None, model="bayes_learned")
        for i in range(7):
            pipe.submit(staged[i % 3])
        return pipe.summary()

    def totals_stager(wire):
        pipe = WindowPipeline(8192, 512, 8, 0, None, model="bayes_learned")
        st = WireStager(torch, pipe, 8192, 512, 8, wire=16 if wire == "16t" else wire, threads=4)
        if wire == 64:
            ring = [(torch.from_numpy(w.events.view(np.uint8).reshape(-1)).pin_memory(),
                     torch.from_numpy(w.spans.view(np.uint8).reshape(-1)).pin_memory()) for w in wins]
        elif wire in (21, 24, 32):
            ring = [(st.probe_records(w.events), None) for w in wins]
        elif wire == "16t":  # EVENT16 probe ring, epoch-tagged
            r16 = [st.probe_ring16(w.events, epoch_ns=300_000_000) for w in wins]
            ring = [(t, b) for t, b in r16]
        else:
            ring = [(None, None)] * 3
        for i in range(7):
            w = wins[i % 3]
            if wire == "16t":
                pipe.submit(st.stage(w.events, w.spans, w.n_groups, w.group_labels, w.group_domains,
                                     ev_pinned=ring[i % 3][0], bases=ring[i % 3][1]))
            else:
                pipe.submit(st.stage(w.events, w.spans, w.n_groups, w.group_labels, w.group_domains,
                                     ev_pinned=ring[i % 3][0], sp_pinned=ring[i % 3][1], pod_table=pods))
        return pipe.summary()

    keys = ("confusion", "hist", "status", "dbg", "misc")
    ref32 = totals_prestaged(32)
    for wire in (32, 24, 21, 20, 16, "16t"):
        got = totals_stager(wire)
        for k in keys:
            np.testing.assert_array_equal(got[k], ref32[k], err_msg=f"stager {wire} {k}")
    ref64, got64 = totals_prestaged(64), totals_stager(64)
    for k in keys:
        np.testing.assert_array_equal(got64[k], ref64[k], err_msg=f"stager 64 {k}")

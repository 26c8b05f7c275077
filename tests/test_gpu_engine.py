"""GPU engine vs the CPU oracle on small replay windows (exact keys/tiers/counts)."""

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes, SufficientStats
from llm_slo_ebpf_toolkit_amd.ops.engine import signal_rows as rows

rows_ = rows
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

pytestmark = pytest.mark.gpu


def small_window(seed=1, n=4096, s=256, services=8, scenario="full"):
    cfg = ReplayConfig(scenario=scenario, n_nodes=2, pods_per_node=8, n_services=services, events_per_window=n,
                       spans_per_window=s, seed=seed)
    return ReplayGenerator(cfg).next_window()


@pytest.fixture(scope="module")
def engine():
    from llm_slo_ebpf_toolkit_amd.ops.engine import KernelHarness

    return KernelHarness(sig_cap=8192, span_cap=512, group_cap=64)


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


def test_wire16_epoch_tags_match_oracle(engine):
    """EVENT16 as the probes write it (probe model: epoch published at each of 4 cuts, records
    stamped with the epoch in force) + host-encoded spans: decode picks each record's base by its
    tag; decode + join == numpy oracle, and == the join of the 64-byte originals."""
    from llm_slo_ebpf_toolkit_amd.collector import records

    win = small_window(seed=25)
    engine.set_join_params(2000.0, 0.7, 3, 1)
    engine.set_model(NaiveBayes.ref())
    ev = win.events[np.argsort(win.events["ts_ns"], kind="stable")].copy()
    ev["ts_ns"][2] = 0
    cfg = np.zeros(128, dtype=np.uint64)
    clock, model = records.EpochClock(), records.ProbeModel(cfg, cpus=1)  # one CPU: slots keep the event order
    first = int(ev["ts_ns"][ev["ts_ns"] > 0].min())
    cfg[124] = clock.publish(first)  # epoch 0 (tag 0), then one epoch per 250 ms cut
    bounds = [first + j * 250_000_000 for j in (1, 2, 3)]
    parts = [model.encode(ev[ev["ts_ns"] < bounds[0]])]
    for j, c in enumerate(bounds):
        cfg[124] = clock.publish(c)
        hi = bounds[j + 1] if j + 1 < len(bounds) else 1 << 62
        parts.append(model.encode(ev[(ev["ts_ns"] >= c) & (ev["ts_ns"] < hi)]))
    enc = np.concatenate(parts)
    e16 = enc[(enc["ctx_type"] & 0xFF) < 0xF0]
    assert len(set((e16["trace_id"] >> np.uint32(30)).tolist())) > 1
    tab = records.HostEncoderModel()
    for p, sn in zip(ev["pod_id"], (ev["svc_id"].astype(np.uint32) << 16) | ev["node_id"]):
        tab.set_pod(int(p), int(sn))
    tab.apply_defs(enc[(enc["ctx_type"] & 0xFF) >= 0xF0])
    sp20 = tab.encode_spans(win.spans)
    ids, rows = tab.take_rows()
    engine.set_ctx_rows(ids, rows)
    engine.stage(e16, sp20, win.n_groups, win.group_labels, bases=clock.bases())
    engine.upload()
    engine.run(True, False)
    out = engine.outputs()
    e = engine.eng
    table = oracle.CtxTable(ids, rows)
    d = oracle.decode_w16(e16, table, clock.bases())
    N, S = len(e16), win.n_spans
    np.testing.assert_array_equal(rows_(e, N)["ts"], d.ts)
    np.testing.assert_array_equal(d.ts, ev["ts_ns"])
    np.testing.assert_array_equal(rows_(e, N)["slot"], d.slot.astype(np.uint32))
    np.testing.assert_array_equal(rows_(e, N)["svcnode"], d.svcnode)
    ref = oracle.join(d, oracle.decode_span20(sp20, table), win.n_groups)
    top3 = e.top3[: 3 * S].cpu().numpy().view(np.uint64).reshape(S, 3)
    np.testing.assert_array_equal(top3, ref.top3)
    for k in ("candidates", "low_confidence", "fanout_dropped", "unmatched", "unsupported_type", "spans_enriched"):
        assert out.debug[k] == ref.debug[k], k
    np.testing.assert_array_equal(out.feat, ref.feat)
    full = oracle.join(oracle.decode_events(ev), win.spans, win.n_groups)
    assert full.debug["candidates"] == ref.debug["candidates"]
    assert int(e.misc[1].item()) == 1  # the zero timestamp


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




def test_record_window_through_the_shipped_engine():
    """ops.engine.GpuEngine: a window of 64-byte EVENT / SPAN records through the agent's
    WindowEngine (page-locked rings -> DMA -> decode -> LDS join -> MFMA posterior) matches the
    oracle on the same records (connections folded to conn32 as the native engine does)."""
    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.ops.engine import GpuEngine

    w = small_window(seed=9)
    eng = GpuEngine(8192, 512, 8)
    model = NaiveBayes.ref()
    eng.set_model(model)
    for _ in range(2):  # the rings and buffers are reused window after window
        out = eng.process(w.events, w.spans, w.n_groups, w.group_labels)
        d = oracle.decode_events(w.events)
        d.conn = records.conn32_np(d.conn).astype(np.uint64)
        ref = oracle.join(d, oracle.spans_native(w.spans), w.n_groups)
        np.testing.assert_array_equal(out.feat, ref.feat)
        np.testing.assert_array_equal(out.hist, oracle.histograms(d))
        assert out.debug["candidates"] == ref.debug["candidates"]
        np.testing.assert_array_equal(out.pred, np.argmax(model.logits(ref.feat.astype(np.float64)), axis=1))
        assert out.confusion.sum() == w.n_groups
    eng.close()

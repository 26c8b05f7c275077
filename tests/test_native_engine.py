"""Native window engine (ops/csrc/engine.hip, no PyTorch) fed zero-copy from the rings: probe
model -> framed BPF ring records -> page-locked ring -> DMA -> on-device definitions (context
rows, trace map) -> decode of framed + user-space records -> LDS join -> MFMA posterior.
Every window is checked against the numpy oracle run on exactly the ring bytes, and the join
against the 64-byte originals; a record left busy in the ring is re-submitted exactly once."""

import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector import records as R
from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

pytestmark = pytest.mark.gpu


def windows(n_win=3, seed=31, n=6000, s=300, services=8):
    cfg = ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=services, events_per_window=n,
                       spans_per_window=s, seed=seed)
    g = ReplayGenerator(cfg)
    return [g.next_window() for _ in range(n_win)], g


def rings(tag, user_rec=64):
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    return (rt.Ringbuf.create_shm(f"/mislo-gt-{os.getpid()}-{tag}", 1 << 22), rt.HostRing(1 << 14, user_rec),
            rt.HostRing(1 << 12, 64))


def feed(img, rb, user, spans):
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut

    assert rb.append_framed(img.framed)
    assert user.push(img.user) == len(img.user)
    assert spans.push(img.spans) == len(img.spans)
    return Cut(kernel=rb.producer_pos, user=user.head, spans=spans.head, bases=img.bases)


def pod_meta(gen):
    sn = (gen.pod_svc.astype(np.uint32) << np.uint32(16)) | gen.pod_node.astype(np.uint32)
    return gen.pod_ids.astype(np.uint32), sn


def test_extension_is_native():
    from llm_slo_ebpf_toolkit_amd.ops import load_agent

    mod = load_agent()
    assert mod.__file__.endswith(".so") and mod.device_count() >= 1


@pytest.mark.parametrize("user_rec", [64, 32, 24, 16])
def test_ring_windows_match_oracle(user_rec):
    """user_rec 32 / 24 / 16: the user-space ring holds USER32 / USER24 records / USER16 slots (the rocprof
    tool's compact forms, svc|node from the device pod table; USER16 with traced records, whose trace
    rides in a continuation slot)."""
    _check_ring_windows(user_rec, f"oracle{user_rec}")


@pytest.mark.parametrize("mode", ["one_chain", "one_stream"])
def test_stream_layouts_match_oracle(monkeypatch, mode):
    """The engine's stream layouts compute the same windows: the default (the span side on its own
    stream), one chain on the compute stream (MISLO_SPAN_STREAM=0: the probe's work list built in the
    signal scatter's launch) and the one-queue agent's single stream (MISLO_ONE_STREAM=1, copies on
    the compute stream too)."""
    monkeypatch.setenv("MISLO_SPAN_STREAM" if mode == "one_chain" else "MISLO_ONE_STREAM", "0" if mode == "one_chain" else "1")
    _check_ring_windows(24, f"layout-{mode}")


def _check_ring_windows(user_rec, tag):
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows()
    if user_rec == 16:  # a third of the GPU signals' records tagged with a request's trace (two slots each)
        from llm_slo_ebpf_toolkit_amd.pipeline.window import kernel_event_mask

        for w in wins:
            gpu = np.nonzero(~kernel_event_mask(w.events))[0][::3]
            w.events["trace_h"][gpu] = w.spans["trace_h"][np.arange(len(gpu)) % len(w.spans)]
    imgs = build_replay_images(wins, user_rec=user_rec)
    pipe = WindowPipeline(16384, 512, 8, model="bayes", learn=False, user_cap=4096)
    rb, user, spans = rings(tag, user_rec)
    src = RingWindowSource(pipe, rb, user, spans)
    assert all(src.direct.values())  # the rings are page-locked: DMA straight from them
    pods, sn = pod_meta(gen)
    pipe.eng.set_pods(pods, sn)
    pod_sn = dict(zip(pods.tolist(), sn.tolist()))
    table, tmap = oracle.CtxTable(), oracle.TraceMap()
    model = NaiveBayes.ref()
    for w, img in zip(wins, imgs):
        cut = feed(img, rb, user, spans)
        r = src.stage(cut, w.n_groups, img.labels)
        k = r["k"]
        assert r["n_kernel"] == R.framed_rows(img.framed) and r["n_user"] == len(img.user)
        oracle.apply_ring_defs(img.framed, table, tmap, pod_sn)
        d = oracle.decode_window(img.framed, img.user, table, tmap, img.bases, pod_sn=pod_sn)
        ref = oracle.join(d, oracle.spans_native(img.spans, tmap), w.n_groups)
        pk = pipe.packet(k)
        res = pipe.results(k, w.n_groups)
        np.testing.assert_array_equal(pk["hist"].astype(np.int64), oracle.histograms(d))
        np.testing.assert_array_equal(pk["misc"][2:18].astype(np.int64), oracle.value_sums_milli(d))
        assert pk["ring_state"]["first_busy"] == -1
        n_rec = int((img.user["pid_sig"] != R.USER16_CONT).sum()) if user_rec == 16 else len(img.user)
        if user_rec == 16:
            assert n_rec < len(img.user)  # continuation slots are rows, not records
        assert pk["ring_state"]["events"] == R.framed_event_count(img.framed) + n_rec
        dbg = dict(zip(("candidates", "low_raw", "overlap", "fanout_dropped", "spans_enriched"),
                       pk["dbg"][:5].astype(np.int64).tolist()))
        for key in ("candidates", "fanout_dropped", "spans_enriched"):
            assert dbg[key] == ref.debug[key], key
        np.testing.assert_array_equal(res["feat"], ref.feat)
        feat = res["feat"].astype(np.float64)
        np.testing.assert_allclose(res["post"][:, :10], model.posteriors(feat), rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(res["pred"], np.argmax(model.logits(feat), axis=1))
        conf = np.zeros((16, 16), dtype=np.int64)
        np.add.at(conf, (img.labels, res["pred"]), 1)
        np.testing.assert_array_equal(pk["confusion"].astype(np.int64), conf)
        # per-incident TTFT SLO accounting (device-counted) == the spans
        exp = np.zeros((w.n_groups, 2), dtype=np.int64)
        np.add.at(exp[:, 0], w.spans["group_id"], 1)
        np.add.at(exp[:, 1], w.spans["group_id"], (w.spans["ttft_ms"] > 800.0).astype(np.int64))
        np.testing.assert_array_equal(res["sli"].astype(np.int64), exp)
        # the join on the 64-byte originals sees the same candidates
        full = oracle.join(oracle.decode_events(w.events), w.spans, w.n_groups)
        assert full.debug["candidates"] == ref.debug["candidates"]
        assert full.debug["spans_enriched"] == ref.debug["spans_enriched"]
        total, comp = pipe.window_ms(k)
        assert total > 0 and comp > 0
    src.drain()
    assert rb.consumer_pos == rb.producer_pos and user.size == 0 and spans.size == 0
    assert pipe.eng.staged_bytes == 0 and pipe.eng.direct_bytes > 0


def test_busy_record_is_resubmitted_exactly_once():
    """A batch record still being written at the cut (busy bit) stops the GPU's decode of that
    window there; the rest of the range is re-submitted with the next window and counted once."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut, RingWindowSource, WindowPipeline

    rb, user, spans = rings("busy")
    pipe = WindowPipeline(4096, 64, 4, model="bayes", learn=False, user_cap=64)
    src = RingWindowSource(pipe, rb, user, spans)
    base = 1_700_000_000_000_000_000
    rb.cfg_set(124, base)
    ev = np.zeros(300, dtype=R.EVENT)
    ev["signal_type"] = 1          # dns_latency_ms
    ev["value"] = 5_000_000        # 5 ms
    ev["ts_ns"] = base + np.arange(300) * 1000
    from llm_slo_ebpf_toolkit_amd.runtime import load

    sim = load().ProbeSim(rb, R.milli_shift_table())
    sim.submit(ev[:96])            # 12 full batch records (all on CPU 0)
    at = rb.reserve(R.REC_PAYLOAD)  # a CPU still writing batch 12 (events 96..103)
    sim.submit(ev[104:200])        # 12 more batches
    k0 = src.stage(Cut(kernel=rb.producer_pos, user=0, spans=0, bases=(base, 0, 0, 0)), 4)["k"]
    src.reap(keep=0)
    assert pipe.packet(k0)["ring_state"]["first_busy"] == 96  # the busy batch's first row
    assert pipe.packet(k0)["hist"].sum() == 96
    assert rb.consumer_pos == 12 * R.REC_STRIDE and src.resubmitted == 13 * R.BATCH_SLOTS
    rb.write(at, sim.encode(ev[96:104]).reshape(-1))
    rb.commit(at)
    sim.submit(ev[200:300])
    k1 = src.stage(Cut(kernel=rb.producer_pos, user=0, spans=0, bases=(base, 0, 0, 0)), 4)["k"]
    src.drain()
    assert pipe.packet(k1)["ring_state"]["first_busy"] == -1
    assert pipe.packet(k1)["hist"].sum() == 204  # the 104 re-submitted + 100 new, each once
    tot = pipe.summary()["hist"].sum()
    assert tot == 300
    assert rb.consumer_pos == rb.producer_pos


def test_pipelined_learning_with_graphs_and_device_refit():
    """bayes_learned: graphs captured per buffer, the device refit folds window k-nb before
    window k; eager and graph runs agree bit for bit."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows(n_win=3, seed=37)
    imgs = build_replay_images(wins)
    sums = []
    for graphs in (False, True):
        pipe = WindowPipeline(16384, 512, 8, model="bayes_learned", use_graphs=graphs, user_cap=4096)
        rb, user, spans = rings(f"learn{graphs}")
        src = RingWindowSource(pipe, rb, user, spans)
        pipe.eng.set_pods(*pod_meta(gen))
        for i in range(8):
            img = imgs[i % 3]
            src.stage(feed(img, rb, user, spans), img.n_groups, img.labels)
        src.drain()
        summ = pipe.summary()
        assert summ["confusion"].sum() == 8 * imgs[0].n_groups
        assert pipe.windows_folded == 8 - pipe.nb
        if graphs:
            assert pipe.eng.graphs >= 3
        sums.append(summ)
        pipe.eng.close()
    for key in ("confusion", "hist", "status", "dbg", "misc"):
        np.testing.assert_array_equal(sums[0][key], sums[1][key], err_msg=key)


def test_halo_and_remote_rows_join_like_the_oracle():
    """Halo and imported rows: window k also joins (never counts) the rows of earlier windows --
    resident on the device in their generation slots -- that lie within the halo of every later
    window's latest local record, and the rows the other GPUs exchanged in the same window
    (injected here as the all-gather would deliver them: XRec blocks, no identity), through the
    engine's two-part chain. Features, candidates and counters match the oracle run over
    [window rows | halo | other GPUs' rows] in the same row order (parallel/exchange.py
    ExchangeModel), and the device's generation state (rows, anchors, cut-offs) is the oracle's."""
    from llm_slo_ebpf_toolkit_amd.parallel.exchange import ExchangeModel
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows(n_win=3, seed=43)
    imgs = build_replay_images(wins)
    halo_ms, icap = 2000.0, 16384
    pipe = WindowPipeline(16384, 512, 8, model="bayes", learn=False, user_cap=4096, halo_ms=halo_ms, import_cap=icap,
                          xchg_cap=64)
    rb, user, spans = rings("halo")
    src = RingWindowSource(pipe, rb, user, spans)
    pods, sn = pod_meta(gen)
    pipe.eng.set_pods(pods, sn)
    pod_sn = dict(zip(pods.tolist(), sn.tolist()))
    table, tmap = oracle.CtxTable(), oracle.TraceMap()
    xm = ExchangeModel(0, 1, halo_ms, icap, 0, halo_windows=3)
    n_halo, tmaxes = [], []
    for j, (w, img) in enumerate(zip(wins, imgs)):
        n_remote = 0
        if j == 2:  # another GPU saw slow DNS lookups on the first 40 traced requests of this window
            sp = w.spans[w.spans["trace_h"] != 0][:40]
            remote = oracle.Decoded(sp["ts_ns"].astype(np.int64) + 1_000_000, np.full(len(sp), 150.0, np.float32),
                                    np.zeros(len(sp), np.uint8), np.full(len(sp), 2, np.uint8),
                                    np.zeros(len(sp), np.uint32), np.zeros(len(sp), np.uint32),
                                    np.zeros(len(sp), np.uint32), sp["trace_h"].astype(np.uint64),
                                    np.zeros(len(sp), np.uint64))
            pipe.inject_remote(oracle.exchange_blocks([remote, oracle.empty_rows()], 64), world=2, me=1)
            xm.injected = remote
            n_remote = len(remote.ts)
        r = src.stage(feed(img, rb, user, spans), w.n_groups, img.labels)
        k = r["k"]
        oracle.apply_ring_defs(img.framed, table, tmap, pod_sn)
        d_loc = oracle.decode_window(img.framed, img.user, table, tmap, img.bases)
        n_loc = len(d_loc.ts)
        n_halo.append(len(xm.halo().ts))
        ref = xm.join(d_loc, oracle.spans_native(img.spans), w.n_groups)
        pk = pipe.packet(k)
        res = pipe.results(k, w.n_groups)
        np.testing.assert_array_equal(pk["hist"].astype(np.int64), oracle.histograms(d_loc))  # imports never count
        assert pk["ring_state"]["events"] == R.framed_event_count(img.framed) + len(img.user)
        dbg = pk["dbg"][:5].astype(np.int64).tolist()
        # rows[0..1], tmax, gens, cur, filled, cut[4], rows per age[4], remote per buffer
        st = pipe.eng.import_state()
        tmaxes.append(oracle.window_tmax(d_loc, n_loc))
        assert st[0] == n_loc and st[1] == n_loc + n_remote, (j, st)
        assert st[2] == tmaxes[-1], (j, st)
        assert st[3] == 4 and st[4] == j % 4 and st[5] == j + 1, (j, st)
        cuts = [max(tmaxes[j - i] for i in range(1, a + 1)) - int(halo_ms * 1e6) for a in range(1, j + 1)]
        assert st[7:7 + j] == cuts and st[6] == -(1 << 63), (j, st, cuts)
        assert st[10] == n_loc + n_remote, (j, st)
        assert (dbg[0], dbg[4]) == (ref.debug["candidates"], ref.debug["spans_enriched"]), (j, n_halo, dbg)
        np.testing.assert_array_equal(res["feat"], ref.feat, err_msg=f"window {j}")
    assert n_halo[0] == 0 and n_halo[1] > 0 and n_halo[2] > 0, n_halo
    src.drain()
    pipe.eng.close()


def test_checkpoint_resume_restores_every_finished_window(tmp_path):
    """Checkpoint / resume: after 6 learned windows (the device refit folds nb behind), the
    checkpoint holds the statistics of all 6; a fresh pipeline restored from it refits on the
    device and scores the next window with exactly that model (= NaiveBayes.learned of the
    same statistics), and the fold counter continues."""
    from llm_slo_ebpf_toolkit_amd.models.bayes import SufficientStats
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows(n_win=4, seed=47)
    imgs = build_replay_images(wins)
    pods = pod_meta(gen)

    def make(tag):
        pipe = WindowPipeline(16384, 512, 8, model="bayes_learned", user_cap=4096)
        rb, user, spans = rings(tag)
        src = RingWindowSource(pipe, rb, user, spans)
        pipe.eng.set_pods(*pods)
        return pipe, src, (rb, user, spans)

    a, src_a, ra = make("ckpt-a")
    total = np.zeros(int(a.mod.STATS_LEN))
    for i in range(6):
        img = imgs[i % 3]
        k = src_a.stage(feed(img, ra[0], ra[1], ra[2]), img.n_groups, img.labels)["k"]
        a.wait(k)
        total += a.eng.packet(k)[int(a.mod.STATS_OFF):int(a.mod.STATS_OFF) + int(a.mod.STATS_LEN)]
    src_a.drain()
    path = str(tmp_path / "state.safetensors")
    a.save_checkpoint(path, {"agent_windows": 6})
    b, src_b, rb_ = make("ckpt-b")
    meta = b.load_checkpoint(path)
    assert meta["agent_windows"] == 6 and meta["windows_folded_device"] == 6
    np.testing.assert_allclose(b.eng.stats_acc(), total, rtol=1e-12, atol=1e-9)
    img = imgs[3]
    kb = src_b.stage(feed(img, rb_[0], rb_[1], rb_[2]), img.n_groups, img.labels, learn=False)["k"]
    res = b.results(kb, img.n_groups)
    s = SufficientStats(count=total[1024:1024 + 10].copy(), elevated_sum=total[:1024].reshape(32, 32)[:16, :10].copy(),
                        x_sum=total[:1024].reshape(32, 32)[16:, :10].copy(), xx=total[:1024].reshape(32, 32)[16:, 16:].copy())
    model = NaiveBayes.learned(s, seed=42)
    np.testing.assert_allclose(res["post"][:, :10], model.posteriors(res["feat"].astype(np.float64)), rtol=1e-9,
                               atol=1e-12)
    src_b.drain()
    assert b.windows_folded == 6
    a.eng.close()
    b.eng.close()


def test_group_sharding_on_device_matches_the_whole_stream():
    """agent --gpus N on one GPU's worth of checks: engines configured as shard 0/2 and 1/2 decode
    the same ring bytes, each keeps only its services' records and incident groups (decode.hip
    shard_owns); their histograms add up to the whole-stream engine's and their local groups'
    features, SLO counts and posteriors are the whole-stream engine's, group for group."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows(n_win=2, seed=53)
    imgs = build_replay_images(wins, user_rec=24)
    pods = pod_meta(gen)
    out = {}
    for shard in ((0, 1), (0, 2), (1, 2)):
        G = len(range(shard[0], 8, shard[1]))
        pipe = WindowPipeline(16384, 512, 8, model="bayes", learn=False, user_cap=4096, shard=shard, halo_ms=2000.0,
                              import_cap=8192)
        rb, user, spans = rings(f"shard{shard[0]}{shard[1]}", 24)
        src = RingWindowSource(pipe, rb, user, spans)
        pipe.eng.set_pods(*pods)
        res = []
        for img in imgs:
            k = src.stage(feed(img, rb, user, spans), G, None)["k"]
            res.append((pipe.packet(k), pipe.results(k, G)))
        src.drain()
        pipe.eng.close()
        out[shard] = res
    for j in range(len(imgs)):
        whole, a, b = out[(0, 1)][j], out[(0, 2)][j], out[(1, 2)][j]
        np.testing.assert_array_equal(whole[0]["hist"], a[0]["hist"] + b[0]["hist"])
        assert whole[0]["ring_state"]["events"] == a[0]["ring_state"]["events"] + b[0]["ring_state"]["events"]
        assert a[0]["ring_state"]["other_shard"] == b[0]["ring_state"]["events"]
        for r, part in ((0, a), (1, b)):
            np.testing.assert_array_equal(part[1]["feat"], whole[1]["feat"][r::2], err_msg=f"window {j} shard {r}")
            np.testing.assert_array_equal(part[1]["sli"], whole[1]["sli"][r::2])
            np.testing.assert_allclose(part[1]["post"], whole[1]["post"][r::2], rtol=1e-12, atol=1e-15)


def test_soft_label_statistics_temperature_refit_and_scoring():
    """Learning on the device with soft labels (a multi-fault incident's mass spread over its
    domain set, label_code) gives the host's SufficientStats; the refit with a temperature and a
    minimum domain mass is NaiveBayes.learned(..., temperature, min_count); scoring REF's 55
    rows through the engine's posterior kernel matches the host model."""
    from llm_slo_ebpf_toolkit_amd.models.bayes import SufficientStats, label_code, soft_labels
    from llm_slo_ebpf_toolkit_amd.models.train import ref55_report, host_scorer
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows(n_win=3, seed=59)
    imgs = build_replay_images(wins)
    pipe = WindowPipeline(16384, 512, 8, model="bayes_learned", user_cap=4096)
    rb, user, spans = rings("softlab")
    src = RingWindowSource(pipe, rb, user, spans)
    pipe.eng.set_pods(*pod_meta(gen))
    host = SufficientStats()
    rng = np.random.default_rng(5)
    for img in imgs:
        codes = np.array([label_code(int(l), [int(l), int(rng.integers(0, 5))] if rng.random() < 0.5 else [])
                          for l in img.labels], dtype=np.int32)
        k = src.stage(feed(img, rb, user, spans), img.n_groups, codes)["k"]
        res = pipe.results(k, img.n_groups)
        host.add(res["feat"].astype(np.float64), soft_labels(codes))
    src.drain()
    # the device has folded the windows the prequential refit reached; the last nb are in their packets
    arrays, meta = pipe.state()
    st = arrays["stats_acc"]
    np.testing.assert_allclose(st[1024:1024 + 10], host.count, rtol=1e-12)
    np.testing.assert_allclose(st[:1024].reshape(32, 32)[:16, :10], host.elevated_sum, rtol=1e-12, atol=1e-12)
    # refit from exactly these statistics with a temperature and a minimum domain mass
    pipe.eng.restore(st, np.zeros(0, np.uint8), len(imgs))
    pipe.eng.set_refit(2.0, 1.0, 1.0 / 2.5, 1.0)
    pipe.eng.refit_now()
    model = NaiveBayes.learned(host, seed=42, temperature=2.5, min_count=1.0)
    fx = os.path.join(os.path.dirname(__file__), "fixtures", "ref_multi_fault_samples.jsonl")

    def dev(feat):
        r = pipe.eng.score(np.ascontiguousarray(feat, dtype=np.float32), None)
        return r["post"][:, :10], r["pred"]

    f = np.random.default_rng(3).uniform(0, 300, (40, 16)).astype(np.float32)
    p_dev, pred_dev = dev(f)
    np.testing.assert_allclose(p_dev, model.posteriors(f.astype(np.float64)), rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(pred_dev, np.argmax(model.logits(f.astype(np.float64)), axis=1))
    assert ref55_report(fx, dev) == ref55_report(fx, host_scorer(model))
    pipe.eng.close()


@pytest.mark.gpu
def test_two_fault_refit_and_marginals_match_the_host_model():
    """2-fault posterior on the device: the image carries the pair structure, k_refit_nb
    rebuilds the noisy-OR pair columns from the statistics (bayes.with_pairs), and the posterior
    kernel's per-domain marginals / argmax equal the host model's; REF's 55 rows score the same."""
    from llm_slo_ebpf_toolkit_amd.models.bayes import SufficientStats, label_code, soft_labels, with_pairs
    from llm_slo_ebpf_toolkit_amd.models.train import ref55_report, host_scorer
    from llm_slo_ebpf_toolkit_amd.ops.engine import MODEL_DTYPE, model_bytes
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows(n_win=3, seed=61)
    imgs = build_replay_images(wins)
    pipe = WindowPipeline(16384, 512, 8, model="bayes_learned", user_cap=4096)
    rb, user, spans = rings("pairs")
    src = RingWindowSource(pipe, rb, user, spans)
    pipe.eng.set_pods(*pod_meta(gen))
    host = SufficientStats()
    rng = np.random.default_rng(7)
    for img in imgs:
        codes = np.array([label_code(int(l), [int(l), int(rng.integers(0, 5))] if rng.random() < 0.5 else [])
                          for l in img.labels], dtype=np.int32)
        k = src.stage(feed(img, rb, user, spans), img.n_groups, codes)["k"]
        host.add(pipe.results(k, img.n_groups)["feat"].astype(np.float64), soft_labels(codes))
    src.drain()
    st = pipe.state()[0]["stats_acc"]
    T, rho = 2.5, 0.3
    model = with_pairs(NaiveBayes.learned(host, seed=42, temperature=T, min_count=1.0), rho, T)
    pipe.eng.restore(st, model_bytes(model), len(imgs))
    pipe.eng.set_refit(2.0, 1.0, 1.0 / T, 1.0)
    pipe.eng.refit_now()
    dev_img = np.frombuffer(np.asarray(pipe.eng.model_bytes(), dtype=np.uint8).tobytes(), dtype=MODEL_DTYPE)[0]
    ref_img = np.frombuffer(model_bytes(model).tobytes(), dtype=MODEL_DTYPE)[0]
    assert int(dev_img["n_pairs"]) == len(model.pairs)
    np.testing.assert_allclose(dev_img["w2"], ref_img["w2"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(dev_img["bias2"], ref_img["bias2"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(dev_img["bias"], ref_img["bias"], rtol=1e-9, atol=1e-12)

    def dev(feat):
        r = pipe.eng.score(np.ascontiguousarray(feat, dtype=np.float32), None)
        return r["post"][:, :10], r["pred"]

    f = np.random.default_rng(4).uniform(0, 300, (48, 16)).astype(np.float32)
    p_dev, pred_dev = dev(f)
    np.testing.assert_allclose(p_dev, model.posteriors(f.astype(np.float64)), rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(pred_dev, model.predict(f.astype(np.float64)))
    fx = os.path.join(os.path.dirname(__file__), "fixtures", "ref_multi_fault_samples.jsonl")
    assert ref55_report(fx, dev) == ref55_report(fx, host_scorer(model))
    pipe.eng.close()


def test_headline_shape_windows_match_the_oracle():
    """The bench's window shape (BASELINE config 5): 1,048,576 events with the probes' framed
    definitions + USER24 rows, 16,384 spans, 64 incident groups, the agent's 2000 ms halo, over
    two consecutive windows (the second joins the first's resident rows). This is the shape that
    runs the multi-block part scans, the long-list span sort and full LDS partitions, which the
    8192-event tests never reach. Histograms, value sums, ring accounting, join counters,
    features, SLI counts, confusion are exact; posteriors within 1e-9."""
    import time

    from llm_slo_ebpf_toolkit_amd.parallel.exchange import ExchangeModel
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images
    from llm_slo_ebpf_toolkit_amd.runtime import load

    t0 = time.time()
    cfg = ReplayConfig(scenario="full", events_per_window=1 << 20, spans_per_window=16384, n_services=64, seed=42,
                       fault_hold=2)
    gen = ReplayGenerator(cfg)
    wins = [gen.next_window() for _ in range(2)]
    imgs = build_replay_images(wins, user_rec=24)
    sig_cap = max(R.framed_rows(i.framed) + len(i.user) for i in imgs)
    halo_ms = 2000.0
    pipe = WindowPipeline(sig_cap, 16384, 64, model="bayes", learn=False, user_cap=1 << 18, halo_ms=halo_ms)
    rt = load()
    rb = rt.Ringbuf.create_shm(f"/mislo-gt-{os.getpid()}-headline", 1 << 26)
    user, spans = rt.HostRing(1 << 19, 24), rt.HostRing(1 << 16, 64)  # two windows in flight
    src = RingWindowSource(pipe, rb, user, spans)
    pods, sn = pod_meta(gen)
    pipe.eng.set_pods(pods, sn)
    pod_sn = dict(zip(pods.tolist(), sn.tolist()))
    table, tmap = oracle.CtxTable(), oracle.TraceMap()
    xm = ExchangeModel(0, 1, halo_ms, 0, 0, halo_windows=3)
    model = NaiveBayes.ref()
    print(f"generated in {time.time() - t0:.1f} s; sig_cap {sig_cap}", flush=True)
    for j, (w, img) in enumerate(zip(wins, imgs)):
        r = src.stage(feed(img, rb, user, spans), w.n_groups, img.labels)
        k = r["k"]
        assert r["n_kernel"] == R.framed_rows(img.framed) and r["n_user"] == len(img.user)
        pk = pipe.packet(k)
        res = pipe.results(k, w.n_groups)
        t1 = time.time()
        oracle.apply_ring_defs(img.framed, table, tmap, pod_sn)
        d = oracle.decode_window(img.framed, img.user, table, tmap, img.bases, pod_sn=pod_sn)
        ref = xm.join(d, oracle.spans_native(img.spans, tmap), w.n_groups)
        print(f"window {j}: {len(d.ts)} rows, oracle in {time.time() - t1:.1f} s, {ref.debug}", flush=True)
        np.testing.assert_array_equal(pk["hist"].astype(np.int64), oracle.histograms(d))
        np.testing.assert_array_equal(pk["misc"][2:18].astype(np.int64), oracle.value_sums_milli(d))
        assert pk["ring_state"]["first_busy"] == -1
        assert pk["ring_state"]["events"] == R.framed_event_count(img.framed) + len(img.user)
        dbg = dict(zip(("candidates", "low_raw", "overlap", "fanout_dropped", "spans_enriched"),
                       pk["dbg"][:5].astype(np.int64).tolist()))
        for key in ("candidates", "fanout_dropped", "spans_enriched"):
            assert dbg[key] == ref.debug[key], (j, key, dbg, ref.debug)
        np.testing.assert_array_equal(res["feat"], ref.feat, err_msg=f"window {j}")
        feat = res["feat"].astype(np.float64)
        np.testing.assert_allclose(res["post"][:, :10], model.posteriors(feat), rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(res["pred"], np.argmax(model.logits(feat), axis=1))
        conf = np.zeros((16, 16), dtype=np.int64)
        np.add.at(conf, (img.labels, res["pred"]), 1)
        np.testing.assert_array_equal(pk["confusion"].astype(np.int64), conf)
        exp = np.zeros((w.n_groups, 2), dtype=np.int64)
        np.add.at(exp[:, 0], w.spans["group_id"], 1)
        np.add.at(exp[:, 1], w.spans["group_id"], (w.spans["ttft_ms"] > 800.0).astype(np.int64))
        np.testing.assert_array_equal(res["sli"].astype(np.int64), exp)
        if j == 1:  # the second window joined the first's rows through the halo
            assert pipe.eng.import_state()[5] == 2
    src.drain()
    pipe.eng.close()


def test_expert_prior_floor_and_capped_unknown_refit_matches_the_host_model():
    """The shipped training configuration on the device: REF's expert table as the Beta prior
    (alpha 10), the likelihood floor of the "unknown" column and its capped prior
    (models/train.py learned_kwargs), with the 2-fault columns -- k_refit_nb builds the same image
    as NaiveBayes.learned(..., init, floor, cap_domain) + with_pairs, and scores the same."""
    from llm_slo_ebpf_toolkit_amd.models import train as mtrain
    from llm_slo_ebpf_toolkit_amd.models.bayes import SufficientStats, label_code, soft_labels, with_pairs
    from llm_slo_ebpf_toolkit_amd.ops.engine import MODEL_DTYPE, model_bytes
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images

    wins, gen = windows(n_win=3, seed=67)
    imgs = build_replay_images(wins)
    pipe = WindowPipeline(16384, 512, 8, model="bayes_learned", user_cap=4096)
    rb, user, spans = rings("expert")
    src = RingWindowSource(pipe, rb, user, spans)
    pipe.eng.set_pods(*pod_meta(gen))
    host = SufficientStats()
    for img in imgs:
        codes = np.asarray(img.labels, dtype=np.int32)
        k = src.stage(feed(img, rb, user, spans), img.n_groups, codes)["k"]
        host.add(pipe.results(k, img.n_groups)["feat"].astype(np.float64), soft_labels(codes))
    src.drain()
    st = pipe.state()[0]["stats_acc"]
    cfg = mtrain.TrainConfig()
    kw = mtrain.learned_kwargs(cfg)
    T, rho = 2.5, 0.3
    model = with_pairs(NaiveBayes.learned(host, temperature=T, **kw), rho, T)
    uncapped = NaiveBayes.learned(host, temperature=T, **dict(kw, cap_domain=None))
    pipe.eng.restore(st, model_bytes(model), len(imgs))
    pipe.set_prior(kw["init"], kw["floor"], kw["cap_domain"], kw["ceil"])
    pipe.eng.set_refit(cfg.alpha, cfg.prior_pseudo, 1.0 / T, cfg.min_count, pipe.cap_dom(), pipe.lik_ceil())
    pipe.eng.refit_now()
    dev_img = np.frombuffer(np.asarray(pipe.eng.model_bytes(), dtype=np.uint8).tobytes(), dtype=MODEL_DTYPE)[0]
    ref_img = np.frombuffer(model_bytes(model).tobytes(), dtype=MODEL_DTYPE)[0]
    for f in ("w", "bias", "w2", "bias2"):
        np.testing.assert_allclose(dev_img[f], ref_img[f], rtol=1e-9, atol=1e-12, err_msg=f)
    live = np.isfinite(model.bias)  # an inactive domain's evidence mask is never read
    np.testing.assert_array_equal(dev_img["dom_mask"][:10][live], ref_img["dom_mask"][:10][live])
    from llm_slo_ebpf_toolkit_amd.signals import catalog

    u = catalog.DOMAIN_INDEX["unknown"]
    capped = NaiveBayes.learned(host, temperature=T, **kw)
    assert capped.bias[u] < uncapped.bias[u]  # the windows' many healthy groups: the cap bites

    def dev(feat):
        r = pipe.eng.score(np.ascontiguousarray(feat, dtype=np.float32), None)
        return r["post"][:, :10], r["pred"]

    f = np.random.default_rng(8).uniform(0, 300, (48, 16)).astype(np.float32)
    p_dev, pred_dev = dev(f)
    np.testing.assert_allclose(p_dev, model.posteriors(f.astype(np.float64)), rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(pred_dev, model.predict(f.astype(np.float64)))
    pipe.eng.close()

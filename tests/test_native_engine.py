"""Native window engine (ops/csrc/engine.hip, no PyTorch) fed by the kernel-ring path:
probe model -> framed BPF ring records -> compacting consumer + id tables + window assembler ->
one DMA -> captured HIP graph of decode / LDS join / MFMA posterior. Every window is checked
against the numpy oracle run on exactly the bytes that crossed PCIe, and the join against the
64-byte originals."""

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
    return [g.next_window() for _ in range(n_win)]


def setup_source(pipe, tag, threads=4):
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    rb = rt.Ringbuf.create_shm(f"/mislo-gt-{os.getpid()}-{tag}", 1 << 22)
    user = rt.HostRing(1 << 14, 64)
    spans = rt.HostRing(1 << 12, 64)
    return RingWindowSource(pipe, rb, user, spans, threads=threads), rb, user, spans


def feed(img, rb, user, spans):
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut

    assert rb.append_framed(img.framed)
    assert user.push(img.user) == len(img.user)
    assert spans.push(img.spans) == len(img.spans)
    return Cut(kernel=rb.producer_pos, user=user.head, spans=spans.head, bases=img.bases)


def test_extension_is_native():
    from llm_slo_ebpf_toolkit_amd.ops import load_agent

    mod = load_agent()
    assert mod.__file__.endswith(".so") and mod.device_count() >= 1


def test_ring_windows_match_oracle():
    from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline, build_replay_images

    wins = windows()
    imgs = build_replay_images(wins)
    pipe = WindowPipeline(8192, 512, 8, model="bayes", learn=False, row_cap=4096)
    src, rb, user, spans = setup_source(pipe, "oracle")
    for w in wins:
        sn = (w.events["svc_id"].astype(np.uint32) << np.uint32(16)) | w.events["node_id"].astype(np.uint32)
        src.tables.set_pods(w.events["pod_id"], sn)
    table = oracle.CtxTable()
    model = NaiveBayes.ref()
    L = pipe.layout
    for w, img in zip(wins, imgs):
        cut = feed(img, rb, user, spans)
        r = src.stage(cut, w.n_groups, img.labels)
        slot = pipe.eng.slot_view(pipe.k).copy()  # exactly what the DMA carries
        k = pipe.submit(r["dma_bytes"], w.n_groups, with_labels=True, learn=False)
        n, nr = r["n_events"], r["n_rows"]
        ev = slot[L["ev_off"]:L["ev_off"] + 16 * n].view(R.EVENT16)
        p = L["ev_off"] + 16 * n
        ids = slot[p:p + 4 * nr].view(np.uint32)
        q = p + (4 * nr + 15) // 16 * 16
        table.add(ids, slot[q:q + 16 * nr].view(np.uint32).reshape(-1, 4))
        d = oracle.decode_w16(ev, table, img.bases)
        sp = oracle.decode_span20(slot[L["sp_off"]:L["sp_off"] + 20 * r["n_spans"]].view(R.SPAN20), table)
        ref = oracle.join(d, sp, w.n_groups)
        pk = pipe.packet(k)
        res = pipe.results(k, w.n_groups)
        np.testing.assert_array_equal(pk["hist"].astype(np.int64), oracle.histograms(d))
        np.testing.assert_array_equal(pk["misc"][2:18].astype(np.int64), oracle.value_sums_milli(d))
        dbg = {key: v for key, v in zip(("candidates", "low_raw", "overlap", "fanout_dropped", "spans_enriched"),
                                          pk["dbg"][:5].astype(np.int64))}
        assert dbg["candidates"] == ref.debug["candidates"]
        assert dbg["fanout_dropped"] == ref.debug["fanout_dropped"]
        assert dbg["spans_enriched"] == ref.debug["spans_enriched"]
        np.testing.assert_array_equal(res["feat"], ref.feat)
        feat = res["feat"].astype(np.float64)
        np.testing.assert_allclose(res["post"][:, :10], model.posteriors(feat), rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(res["pred"], np.argmax(model.logits(feat), axis=1))
        conf = np.zeros((16, 16), dtype=np.int64)
        np.add.at(conf, (img.labels, res["pred"]), 1)
        np.testing.assert_array_equal(pk["confusion"].astype(np.int64), conf)
        # the join on the 64-byte originals sees the same candidates
        full = oracle.join(oracle.decode_events(w.events), w.spans, w.n_groups)
        assert full.debug["candidates"] == ref.debug["candidates"]
        assert full.debug["spans_enriched"] == ref.debug["spans_enriched"]
        total, comp = pipe.window_ms(k)
        assert total > 0 and comp > 0


def test_pipelined_learning_with_graphs_and_device_refit():
    """bayes_learned: graphs captured per buffer, the device refit folds window k-nb before
    window k; totals equal the per-window packets; eager and graph runs agree."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline, build_replay_images

    wins = windows(n_win=3, seed=37)
    imgs = build_replay_images(wins)
    sums = []
    for graphs in (False, True):
        pipe = WindowPipeline(8192, 512, 8, model="bayes_learned", use_graphs=graphs, row_cap=4096)
        src, rb, user, spans = setup_source(pipe, f"learn{graphs}")
        packets = []
        for i in range(8):
            img = imgs[i % 3]
            cut = feed(img, rb, user, spans)
            r = src.stage(cut, img.n_groups, img.labels)
            packets.append(pipe.submit(r["dma_bytes"], img.n_groups, with_labels=True))
        summ = pipe.summary()
        assert summ["confusion"].sum() == 8 * imgs[0].n_groups
        assert pipe.windows_folded == 8 - pipe.nb
        tot = sum(pipe.packet(k)["confusion"] for k in packets[-3:])  # last nb packets still resident
        assert tot.sum() == 3 * imgs[0].n_groups
        if graphs:
            assert pipe.eng.graphs >= 3
        sums.append(summ)
    for key in ("confusion", "hist", "status", "dbg", "misc"):
        np.testing.assert_array_equal(sums[0][key], sums[1][key], err_msg=key)

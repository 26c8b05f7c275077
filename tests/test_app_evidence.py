"""Application evidence (models/bayes.py AppEvidence, ops/csrc/mislo_launch.h AppModel): an
incident group's retrieval time beyond the kernel-attributed share -- REF's DecomposeRetrieval
(pkg/otel/processor/ebpfcorrelator/correlator.go:179-194) at group level, fed by the spans'
llm.slo.retrieval.* breakdown (REF demo/rag-service/main.go:393-397) -- scored as one more binary
naive-Bayes signal with source "application" (REF incident-attribution.schema.json:41-56).

CPU tests pin the host model's math; the GPU test checks the engine (span decode's group sums,
the K3 kernel's residual, logits and evidence bit) against it."""

import math
import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector import records as R
from llm_slo_ebpf_toolkit_amd.models.bayes import (APP_BIT, AppEvidence, NaiveBayes, app_counts, marginalize,
                                                   with_pairs)
from llm_slo_ebpf_toolkit_amd.models import train as mtrain
from llm_slo_ebpf_toolkit_amd.signals import catalog

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")
RETR = catalog.DOMAIN_INDEX["retrieval_backend"]


def _feat(rows):
    f = np.full((len(rows), 16), np.nan, np.float32)
    for i, r in enumerate(rows):
        for k, v in r.items():
            f[i, catalog.BY_NAME[k].slot] = v
    return f


def test_residual_is_mean_retrieval_minus_kernel_share():
    # group 0: 2 spans, 300 ms of retrieval in 10 us units; kernel share dns 10 + tls 5 (connect absent)
    cnt = np.array([[2, 30000], [0, 0], [1, 2000]], np.uint32)
    feat = _feat([{"dns_latency_ms": 10.0, "tls_handshake_ms": 5.0}, {}, {"connect_latency_ms": 350.0}])
    r = AppEvidence.residual(cnt, feat)
    assert r[0] == pytest.approx(135.0) and math.isnan(r[1]) and r[2] == pytest.approx(20.0 - 350.0)
    st = AppEvidence.expert(100.0).state(cnt, feat)
    assert st.tolist() == [1, -1, 0]


def test_app_counts_match_the_span_decode_rule():
    sp = np.zeros(6, R.SPAN)
    sp["group_id"] = [0, 0, 1, 1, 2, 5]
    sp["retr_ms"] = [150.004, 20.0, 0.0, np.nan, -3.0, 40.0]
    c = app_counts(sp, 4)
    assert c.tolist() == [[2, 15000 + 2000], [0, 0], [0, 0], [0, 0]]  # rint(150.004 * 100) = 15000


def test_app_evidence_is_one_more_naive_bayes_signal():
    """logit_d = log pi_d + sum_s log P(e_s | d) + log P(e_app | d): the closed form, computed
    signal by signal, equals the linear-logit model with the channel attached."""
    m = NaiveBayes.gpu()
    m.app = AppEvidence.expert(100.0)
    ref_lik = np.asarray(catalog.extended_likelihood_matrix())
    feat = _feat([{"dns_latency_ms": 200.0}, {"runqueue_delay_ms": 30.0}, {}])
    for st in ([1, 1, 1], [0, 0, 0], [1, 0, -1]):
        st = np.array(st)
        post = m.posteriors(feat.astype(np.float64), st)
        for g in range(3):
            lg = np.zeros(10)
            for d in range(10):
                lg[d] = math.log(0.1)
                for s in range(16):
                    p = min(max(ref_lik[s][d], 0.01), 0.99)
                    e = not math.isnan(feat[g, s]) and feat[g, s] >= catalog.SIGNALS[s].elevated
                    lg[d] += math.log(p if e else min(max(1 - ref_lik[s][d], 0.01), 0.99))
                if st[g] >= 0:
                    pa = catalog.APP_RETRIEVAL_LIKELIHOOD[catalog.ALL_DOMAINS[d]]
                    lg[d] += math.log(pa if st[g] == 1 else 1 - pa)
            z = np.exp(lg - lg.max())
            np.testing.assert_allclose(post[g], z / z.sum(), rtol=1e-12)
        bits = m.evidence_bits(feat.astype(np.float64), st)
        assert bool(bits[0, RETR] >> APP_BIT & 1) == (st[0] == 1)
        assert not (bits[:, catalog.DOMAIN_INDEX["unknown"]] >> APP_BIT & 1).any()


def test_absent_application_evidence_changes_nothing_on_refs_rows():
    """REF's 55 rows carry no retrieval breakdown: with the channel attached every score is the
    table's own (the signal is summed out, not read as 'not elevated')."""
    from llm_slo_ebpf_toolkit_amd.models.sample import load_samples_jsonl

    samples = load_samples_jsonl(os.path.join(FIX, "ref_multi_fault_samples.jsonl"))
    feat = np.array([catalog.feature_vector(s.signals) for s in samples], dtype=np.float64)
    for m in (NaiveBayes.ref(), with_pairs(NaiveBayes.gpu(), 0.2)):
        base = m.posteriors(feat)
        m.app = AppEvidence.expert()
        np.testing.assert_array_equal(m.posteriors(feat, np.full(len(feat), -1)), base)
        np.testing.assert_array_equal(m.predict(feat, np.full(len(feat), -1)), m.predict(feat))


def test_a_lone_retrieval_stall_is_retrieval_backend_and_network_keeps_egress():
    """The live config-3 shapes under the shipped learned 2-fault model marginalised to what the
    box observes: a vector-DB stall with no kernel signal reads retrieval_backend (round 5: unknown,
    the domain was dropped as unobservable); the network fault, whose kernel share covers the
    retrieval time, stays network_egress; a healthy group with a normal retrieval time stays unknown;
    a CPU fault stays cpu_throttle although the starved service's retrieval time is long."""
    model, _img, meta = mtrain.load_model(os.path.join(os.path.dirname(FIX), "..", "config", "models",
                                                       "mislo-learned.safetensors"))
    T = float(meta.get("temperature", 1.0))
    obs = ["dns_latency_ms", "tcp_retransmits_total", "connect_latency_ms", "connect_errors_total",
           "tls_handshake_ms", "tls_handshake_fail_total", "runqueue_delay_ms", "cpu_steal_pct"]
    plain = marginalize(model, obs, T)
    assert not np.isfinite(plain.bias[RETR])  # round 5: unobservable, never attributed
    model.app = AppEvidence.expert(100.0, temperature=T)
    m = marginalize(model, obs, T)
    assert np.isfinite(m.bias[RETR])
    feat = _feat([{}, {"connect_latency_ms": 350.0, "dns_latency_ms": 180.0, "tcp_retransmits_total": 12.0,
                       "connect_errors_total": 3.0, "tls_handshake_fail_total": 2.0},
                  {}, {"runqueue_delay_ms": 28.0, "cpu_steal_pct": 9.0}])
    cnt = np.array([[10, 10 * 18500], [10, 10 * 18500], [10, 10 * 3000], [10, 10 * 16000]], np.uint32)
    st = m.app.state(cnt, feat)
    assert st.tolist() == [1, 0, 0, 1]
    pred = [catalog.ALL_DOMAINS[d] for d in m.predict(feat.astype(np.float64), st)]
    assert pred == ["retrieval_backend", "network_egress", "unknown", "cpu_throttle"]


def test_cpu_ring_engine_scores_the_application_evidence():
    """agent --engine cpu: the host engine's group counts, states, posteriors and evidence bits."""
    from llm_slo_ebpf_toolkit_amd.ops.engine import app_from_bytes, app_model_bytes
    from llm_slo_ebpf_toolkit_amd.pipeline.cpu import CpuRingEngine

    m = with_pairs(NaiveBayes.gpu(), 0.2)
    m.app = AppEvidence.expert(100.0)
    img = app_model_bytes(m)
    back = app_from_bytes(img)
    w, b = m.app.terms()
    np.testing.assert_array_equal(back.terms()[0], w)
    np.testing.assert_array_equal(back.pair_terms(m.pairs)[1], m.app.pair_terms(m.pairs)[1])
    eng = CpuRingEngine(group_cap=4, span_cap=16)
    from llm_slo_ebpf_toolkit_amd.ops.engine import model_bytes

    eng.set_model_bytes(model_bytes(m))
    eng.set_app_model(img)
    sp = np.zeros(4, R.SPAN)
    sp["ts_ns"] = 1_700_000_000_000_000_000 + np.arange(4)
    sp["group_id"] = [0, 0, 1, 2]
    sp["retr_ms"] = [180.0, 190.0, 25.0, 0.0]
    buf = np.ascontiguousarray(sp).view(np.uint8)
    eng.submit(0, [], [], [(buf.ctypes.data, buf.nbytes)], 3, None, (0, 0, 0, 0), False, False, 64)
    res = eng.results(0, 3)
    assert res["app"].tolist() == [[2, 37000], [1, 2500], [0, 0]]
    st = m.app.state(res["app"], res["feat"])
    assert st.tolist() == [1, 0, -1]
    assert res["pred"][0] == RETR and (res["evbits"][0, RETR] >> APP_BIT) & 1
    np.testing.assert_allclose(res["post"][:, :10], m.posteriors(res["feat"].astype(np.float64), st))


def _stall_spans(w, stall=(0,), healthy=(1,)):
    """Retrieval breakdowns on the replay's spans: a stall far above any kernel share (the replay's
    fault profiles put connect latency at 350 ms) in ``stall``, a healthy time in ``healthy``; every
    third span flagged late (SPAN_LATE)."""
    sp = w.spans.copy()
    g = sp["group_id"]
    sp["retr_ms"] = 0.0
    for x in stall:
        sp["retr_ms"][g == x] = np.float32(5000.0) + (np.arange((g == x).sum()) % 7).astype(np.float32)
    for x in healthy:
        sp["retr_ms"][g == x] = np.float32(22.5)
    sp["flags"][::3] = R.SPAN_LATE
    return sp


@pytest.mark.gpu
@pytest.mark.parametrize("pairs", [False, True])
def test_engine_application_evidence_matches_the_host_model(pairs):
    """The native engine: per-group retrieval counts exact (k_decode_spans), residual state,
    posteriors (rtol 1e-9) and the evidence bit equal to the host model's; score() with counts
    too."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import RingWindowSource, WindowPipeline, build_replay_images
    from tests.test_native_engine import feed, pod_meta, rings, windows

    wins, gen = windows(n_win=2, seed=5)
    for w in wins:
        w.spans = _stall_spans(w)
    imgs = build_replay_images(wins, user_rec=24)
    m = NaiveBayes.gpu()
    if pairs:
        m = with_pairs(m, 0.2)
    pipe = WindowPipeline(16384, 512, 8, model="bayes_gpu", learn=False, user_cap=4096)
    pipe.set_model(m)
    pipe.set_app(AppEvidence.expert(100.0))
    rb, user, spans = rings(f"app{int(pairs)}", 24)
    src = RingWindowSource(pipe, rb, user, spans)
    pods, sn = pod_meta(gen)
    pipe.eng.set_pods(pods, sn)
    seen_elevated = False
    for w, img in zip(wins, imgs):
        r = src.stage(feed(img, rb, user, spans), w.n_groups, img.labels)
        res = pipe.results(r["k"], w.n_groups)
        np.testing.assert_array_equal(res["app"], app_counts(w.spans, w.n_groups))
        # late breaches (SPAN_LATE): counted apart from the window's own requests
        breach = w.spans["ttft_ms"] > np.float32(800.0)
        late = breach & (w.spans["flags"] == R.SPAN_LATE)
        exp = np.zeros((w.n_groups, 2), np.int64)
        np.add.at(exp[:, 0], w.spans["group_id"][~late], 1)
        np.add.at(exp[:, 1], w.spans["group_id"][breach & ~late], 1)
        np.testing.assert_array_equal(res["sli"].astype(np.int64), exp)
        exp_late = np.zeros(w.n_groups, np.int64)
        np.add.at(exp_late, w.spans["group_id"][late], 1)
        np.testing.assert_array_equal(res["late"][:, 0].astype(np.int64), exp_late)
        feat = res["feat"].astype(np.float64)
        st = m.app.state(res["app"], res["feat"])
        seen_elevated |= bool((st == 1).any())
        np.testing.assert_allclose(res["post"][:, :10], m.posteriors(feat, st), rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(res["pred"], m.predict(feat, st))
        np.testing.assert_array_equal(res["evbits"][:, :10], m.evidence_bits(feat, st))
        sc = pipe.eng.score(res["feat"], None, res["app"])
        np.testing.assert_allclose(sc["post"][:, :10], m.posteriors(feat, st), rtol=1e-9, atol=1e-12)
        np.testing.assert_array_equal(sc["evbits"][:, :10], m.evidence_bits(feat, st))
    assert seen_elevated
    pipe.eng.close()

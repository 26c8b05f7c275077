"""Attribution parity with REF's Bayes math on REF's own dataset, learned models, metrics."""

import math
import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd import models
from llm_slo_ebpf_toolkit_amd.contracts import validator
from llm_slo_ebpf_toolkit_amd.models.bayes import LDA, NaiveBayes, SufficientStats, samples_to_arrays
from llm_slo_ebpf_toolkit_amd.signals import catalog


@pytest.fixture(scope="module")
def ref55(fixtures_dir=os.path.join(os.path.dirname(__file__), "fixtures")):
    return models.load_samples_jsonl(os.path.join(fixtures_dir, "ref_multi_fault_samples.jsonl"))


def _single(samples, preds):
    return [(s, p) for s, p in zip(samples, preds) if s.expected_domain]


def test_ref_bayes_reproduces_published_numbers(ref55):
    preds = models.build_attributions(ref55, "bayes")
    assert models.accuracy(ref55, preds) == pytest.approx(29 / 55)  # 0.5273: multi rows map to unknown
    single = _single(ref55, preds)
    actual = [s.actual_domain() for s, _ in single]
    pred = [p.predicted_fault_domain for _, p in single]
    assert sum(a == b for a, b in zip(actual, pred)) == 29
    assert models.macro_f1(actual, pred) == pytest.approx(0.9818181818)
    assert models.macro_f1(actual, pred, include_predicted=True) == pytest.approx(0.8181818181)
    multi = [(s, p) for s, p in zip(ref55, preds) if not s.expected_domain]
    assert models.partial_accuracy([s for s, _ in multi], [p for _, p in multi]) == 1.0
    assert models.coverage_accuracy([s for s, _ in multi], [p for _, p in multi], 0.10) == pytest.approx(2 / 3)
    # the only single-fault miss is mf-04 provider_throttle -> provider_error (0.546 vs 0.179)
    miss = [(s, p) for s, p in single if s.actual_domain() != p.predicted_fault_domain]
    assert len(miss) == 1 and miss[0][0].incident_id == "mf-04"
    hyp = {h.domain: h.posterior for h in miss[0][1].fault_hypotheses}
    assert hyp["provider_error"] == pytest.approx(0.546, abs=5e-4)
    assert hyp["provider_throttle"] == pytest.approx(0.179, abs=5e-4)


def _ref_scalar_posteriors(signals):
    """Literal re-derivation of REF Attribute (bayesian.go:218-284) for cross-checking."""
    lik = catalog.ref_likelihoods()
    thr = {s.name: s.elevated for s in catalog.SIGNALS[:12]}
    elevated = {k for k, v in signals.items() if k in thr and v >= thr[k]}
    logp = {}
    for d in catalog.REF_DOMAINS:
        lp = math.log(1 / 8)
        for sig, row in lik.items():
            p = row[d]
            lp += math.log(min(max(p if sig in elevated else 1 - p, 0.01), 0.99))
        logp[d] = lp
    m = max(logp.values())
    z = m + math.log(sum(math.exp(v - m) for v in logp.values()))
    return {d: math.exp(v - z) for d, v in logp.items()}


def test_linear_form_equals_scalar_ref_math(ref55):
    model = NaiveBayes.ref()
    for s in ref55:
        ref = _ref_scalar_posteriors(s.signals)
        got = {p.domain: p.posterior for p in model.attribute(s.signals)}
        for d in catalog.REF_DOMAINS:
            assert got[d] == pytest.approx(ref[d], rel=1e-12, abs=1e-15)


def test_posteriors_sum_to_one_and_evidence():
    model = NaiveBayes.ref()
    post = model.attribute({"dns_latency_ms": 220, "connect_latency_ms": 130})
    assert sum(p.posterior for p in post) == pytest.approx(1.0, abs=1e-9)
    assert post[0].domain == "network_dns"
    assert post[0].evidence == ["connect_latency_ms", "dns_latency_ms"]
    cpu = model.attribute({"runqueue_delay_ms": 28, "cpu_steal_pct": 9, "cfs_throttled_ms": 170})
    assert cpu[0].domain == "cpu_throttle"
    mem = model.attribute({"cfs_throttled_ms": 90, "mem_reclaim_latency_ms": 25, "disk_io_latency_ms": 60,
                           "runqueue_delay_ms": 14})
    assert mem[0].domain == "memory_pressure"
    prov = model.attribute({"connect_latency_ms": 95, "tls_handshake_ms": 90, "syscall_latency_ms": 300,
                            "connect_errors_total": 2})
    assert prov[0].domain == "provider_throttle"
    # GPU signals are unknown to the REF table and must not change REF posteriors
    a = model.attribute({"dns_latency_ms": 220})
    b = model.attribute({"dns_latency_ms": 220, "gpu_queue_delay_ms": 500})
    assert [p.posterior for p in a] == [p.posterior for p in b]


def test_rule_fallback_without_signals():
    s = models.FaultSample(incident_id="i", fault_label="dns_latency", confidence=0.9, burn_rate=2, window_minutes=5)
    att = NaiveBayes.ref().attribute_sample(s)
    assert att.predicted_fault_domain == "network_dns" and att.fault_hypotheses == []
    assert [e.signal for e in att.evidence] == ["fault_label", "mapped_domain", "llm.ebpf.correlation_confidence",
                                                "llm.ebpf.dns.latency_ms"]
    assert att.evidence[3].value == 180.0
    validator.validate("incident-attribution", att)


def test_label_map():
    assert models.map_fault_label("network_partition") == "network_egress"
    assert models.map_fault_label("retrieval_slowdown") == "retrieval_backend"
    assert models.map_fault_label("whatever") == "unknown"


def test_learned_and_lda_fix_mf04(ref55):
    # train on REF profile-shaped synthetic samples (replay world), test on REF's dataset
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
    from llm_slo_ebpf_toolkit_amd.pipeline import oracle

    gen = ReplayGenerator(ReplayConfig(scenario="full", n_nodes=1, pods_per_node=16, n_services=16,
                                       events_per_window=6000, spans_per_window=300, seed=3))
    st = SufficientStats()
    for _ in range(6):
        w = gen.next_window()
        d = oracle.decode_events(w.events)
        res = oracle.join(d, w.spans, w.n_groups)
        keep = ~np.all(np.isnan(res.feat), axis=1)
        st.add(res.feat[keep].astype(np.float64), w.group_labels[keep])
    single = [s for s in ref55 if s.expected_domain]
    vals, labels = samples_to_arrays(single)
    for model in (NaiveBayes.learned(st), LDA.fit(st)):
        pred = np.argmax(model.logits(vals), axis=1)
        acc = float(np.mean(pred == labels))
        assert acc >= 0.9, (model.name, acc)


def test_stats_pack_roundtrip():
    st = SufficientStats()
    rng = np.random.default_rng(0)
    v = rng.uniform(0, 100, size=(20, 16))
    v[rng.random((20, 16)) < 0.3] = np.nan
    st.add(v, rng.integers(0, 10, size=20))
    st2 = SufficientStats.unpack(st.pack())
    np.testing.assert_allclose(st2.xx, st.xx)
    assert st.pack().shape[0] == SufficientStats.PACKED_LEN


def test_confusion_and_macro_f1_helpers():
    conf = models.metrics.confusion_from_arrays([0, 0, 1, 2], [0, 1, 1, 2], 3)
    assert conf.tolist() == [[1, 1, 0], [0, 1, 0], [0, 0, 1]]
    assert models.macro_f1_from_confusion(conf) == pytest.approx(models.macro_f1(["a", "a", "b", "c"],
                                                                                  ["a", "b", "b", "c"]))


def test_bayes_gpu_names_gpu_domains_and_keeps_ref_rows():
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes
    from llm_slo_ebpf_toolkit_amd.signals import catalog

    m = NaiveBayes.gpu()
    v = np.full((1, catalog.N_SLOTS), np.nan)
    v[0, catalog.BY_NAME["gpu_queue_delay_ms"].slot] = 5.0
    top = m.attribute({"gpu_queue_delay_ms": 5.0})[0]
    assert top.domain == "gpu_contention" and "gpu_queue_delay_ms" in top.evidence
    assert m.attribute({"rccl_collective_ms": 30.0, "xgmi_link_latency_us": 60.0})[0].domain == "gpu_interconnect"
    assert m.attribute({"dns_latency_ms": 300.0})[0].domain == "network_dns"
    # REF's rows over REF's domains are REF's table
    ref = NaiveBayes.ref()
    for s in catalog.REF_DOMAINS:
        d = catalog.DOMAIN_INDEX[s]
        for name in catalog.SIGNAL_NAMES[:12]:
            slot = catalog.BY_NAME[name].slot
            assert m.weights[slot, d] == ref.weights[slot, d]


def test_confusion_report_matches_list_metrics():
    """confusion_report (the bench's held-out report) agrees with the list-based per-class
    report and REF's one-vs-rest rates on the same predictions."""
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.evaluation.benchmark import one_vs_rest_rates
    from llm_slo_ebpf_toolkit_amd.models.metrics import confusion_report, per_class_report

    labels = ["a", "b", "unknown", "c"]
    actual = ["a", "a", "b", "b", "b", "c", "c", "a"]
    pred = ["a", "b", "b", "unknown", "b", "c", "a", "a"]
    cm = np.zeros((4, 4))
    for x, y in zip(actual, pred):
        cm[labels.index(x), labels.index(y)] += 1
    rep = confusion_report(cm, labels)
    ref = {r.label: r for r in per_class_report(actual, pred, labels)}
    for r in rep["per_class"]:
        assert r["precision"] == pytest.approx(ref[r["label"]].precision, abs=1e-4)
        assert r["recall"] == pytest.approx(ref[r["label"]].recall, abs=1e-4)
        assert r["f1"] == pytest.approx(ref[r["label"]].f1, abs=1e-4)
    rates = one_vs_rest_rates(actual, pred)
    assert rep["false_positive_rate"] == pytest.approx(rates["false_positive_rate"], abs=1e-4)
    assert rep["false_negative_rate"] == pytest.approx(rates["false_negative_rate"], abs=1e-4)
    assert rep["abstain_rate"] == pytest.approx(1 / 8)  # b -> unknown, of 8 faulted incidents
    cm2 = cm.copy()
    cm2[labels.index("unknown"), labels.index("unknown")] += 4  # correct no-fault incidents
    assert confusion_report(cm2, labels)["abstain_rate"] == pytest.approx(1 / 8)

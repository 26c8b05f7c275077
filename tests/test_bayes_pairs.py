"""The 2-fault posterior (models/bayes.py with_pairs) and signal marginalisation (marginalize):
checked against brute-force Bayes over the hypothesis space, and on REF's 55 labelled rows."""

import itertools
import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.models import train
from llm_slo_ebpf_toolkit_amd.models.bayes import (PAIR_LIST, NaiveBayes, label_code, marginalize, with_pairs,
                                                   with_temperature)
from llm_slo_ebpf_toolkit_amd.ops.engine import model_bytes, model_from_bytes
from llm_slo_ebpf_toolkit_amd.signals import catalog

FX = os.path.join(os.path.dirname(__file__), "fixtures", "ref_multi_fault_samples.jsonl")


def brute_force(m, values, rho, observed=None):
    """P(hypothesis | evidence) from the probability tables themselves: priors (1-rho) pi_d and
    rho pi_a pi_b / Z, likelihoods p (singles) and noisy-OR (pairs), product over the observed
    table signals."""
    p, logpi, table = [np.asarray(x) for x in train_tables(m)]
    pi = np.exp(logpi - np.logaddexp.reduce(logpi[np.isfinite(logpi)]))
    slots = [s for s in range(16) if table[s] and (observed is None or s in observed)]
    e = m.elevated(values[None, :])[0]
    hyps, prior, lik = [], [], []
    for d in range(len(pi)):
        if pi[d] > 0:
            hyps.append((d,))
            prior.append((1 - rho) * pi[d])
    z = sum(pi[a] * pi[b] for a, b in PAIR_LIST)
    for a, b in PAIR_LIST:
        if pi[a] > 0 and pi[b] > 0:
            hyps.append((a, b))
            prior.append(rho * pi[a] * pi[b] / z)
    for h in hyps:
        q = p[:, h[0]] if len(h) == 1 else 1 - (1 - p[:, h[0]]) * (1 - p[:, h[1]])
        q = np.clip(q, 0.01, 0.99)
        lik.append(np.prod([q[s] if e[s] else 1 - q[s] for s in slots]))
    post = np.array(prior) * np.array(lik)
    post /= post.sum()
    marg = np.zeros(m.weights.shape[1])
    for h, v in zip(hyps, post):
        for d in h:
            marg[d] += v
    return marg


def train_tables(m):
    from llm_slo_ebpf_toolkit_amd.models.bayes import _raw_tables

    return _raw_tables(m, 1.0)


@pytest.mark.parametrize("rho", [0.05, 0.3])
def test_pair_marginals_equal_brute_force_bayes(rho):
    base = NaiveBayes.ref()
    m = with_pairs(base, rho)
    rng = np.random.default_rng(1)
    for _ in range(20):
        v = np.where(rng.random(16) < 0.5, rng.uniform(0, 400, 16), np.nan)
        np.testing.assert_allclose(m.posteriors(v[None, :])[0], brute_force(base, v, rho), rtol=1e-9, atol=1e-12)


def test_marginalising_a_signal_drops_its_factor():
    base = NaiveBayes.ref()
    obs = ["dns_latency_ms", "tcp_retransmits_total", "runqueue_delay_ms"]
    slots = {catalog.BY_NAME[s].slot for s in obs}
    m = marginalize(with_pairs(base, 0.2), obs, drop_unobservable=False)
    rng = np.random.default_rng(2)
    for _ in range(20):
        v = rng.uniform(0, 400, 16)
        np.testing.assert_allclose(m.posteriors(v[None, :])[0], brute_force(base, v, 0.2, slots), rtol=1e-9,
                                   atol=1e-12)
        # values of unobserved signals change nothing
        w = v.copy()
        w[[s for s in range(16) if s not in slots]] = 0.0
        np.testing.assert_allclose(m.posteriors(v[None, :]), m.posteriors(w[None, :]), rtol=1e-12)
    assert not m.evidence_mask[[s for s in range(16) if s not in slots]].any()


def test_domains_no_observable_signal_indicates_are_not_attributed():
    """A node whose sources produce only the network signals cannot tell CPU, memory, provider or
    GPU faults from a healthy service: those domains (and their pairs) are inactive, so a window
    with nothing elevated is "unknown", not the domain with the largest prior."""
    base = with_pairs(NaiveBayes.gpu(), 0.2)
    obs = ["dns_latency_ms", "tcp_retransmits_total", "connect_latency_ms"]
    m = marginalize(base, obs)
    active = {catalog.ALL_DOMAINS[d] for d in np.flatnonzero(np.isfinite(m.bias))}
    assert active == {"network_dns", "network_egress", "provider_throttle", "unknown"}, active
    assert not np.isfinite(m.pair_b[(m.pairs == catalog.DOMAIN_INDEX["cpu_throttle"]).any(axis=1)]).any()
    v = np.full((1, 16), np.nan)
    assert catalog.ALL_DOMAINS[int(m.predict(v)[0])] == "unknown"
    v[0, catalog.BY_NAME["dns_latency_ms"].slot] = 250.0
    assert catalog.ALL_DOMAINS[int(m.predict(v)[0])] == "network_dns"


def test_single_fault_limit_and_temperature_commute():
    base = NaiveBayes.ref()
    v = np.random.default_rng(3).uniform(0, 300, (30, 16))
    tiny = with_pairs(base, 1e-14)
    np.testing.assert_allclose(tiny.posteriors(v), base.posteriors(v), atol=1e-6)
    np.testing.assert_array_equal(tiny.predict(v), base.predict(v))
    # the pair columns at a temperature are the tempered noisy-OR tables
    T = 2.5
    a = with_pairs(with_temperature(base, T), 0.3, T)
    b = with_temperature(with_pairs(base, 0.3), T)
    np.testing.assert_allclose(a.pair_w, b.pair_w, rtol=1e-12)
    np.testing.assert_allclose(a.pair_b, b.pair_b, rtol=1e-12)


def test_image_round_trip_keeps_the_pairs():
    m = with_pairs(NaiveBayes.gpu(), 0.25)
    back = model_from_bytes(model_bytes(m))
    v = np.random.default_rng(4).uniform(0, 300, (25, 16))
    np.testing.assert_array_equal(back.posteriors(v), m.posteriors(v))
    assert back.pair_rho == 0.25 and len(back.pairs) == len(PAIR_LIST) == 36


def test_ref55_two_fault_coverage_beats_ref_without_losing_single_fault_f1():
    ref = train.ref55_report(FX, train.host_scorer(NaiveBayes.ref()))
    two = train.ref55_report(FX, train.host_scorer(with_pairs(NaiveBayes.ref(), 0.3)))
    assert two["single_fault_macro_f1"] == ref["single_fault_macro_f1"] == 0.9818
    assert two["multi_fault_partial_accuracy"] == 1.0
    assert ref["multi_fault_coverage_accuracy"] == 0.6667
    assert two["multi_fault_coverage_accuracy"] > 0.9


def test_pair_prior_and_hypothesis_targets():
    codes = np.array([3, label_code(1, [1, 2]), label_code(2, [1, 2, 3]), -1, 7])
    assert train.pair_prior(codes) == pytest.approx((2 + 1) / (4 + 2))
    Y1, Y2 = train.hypothesis_targets(codes)
    assert Y1[0, 3] == 1 and Y1[4, 7] == 1 and Y1[3].sum() == 0 and Y2[3].sum() == 0
    assert Y2[1, PAIR_LIST.index((1, 2))] == 1
    trip = [PAIR_LIST.index(p) for p in itertools.combinations((1, 2, 3), 2)]
    np.testing.assert_allclose(Y2[2, trip], 1 / 3)

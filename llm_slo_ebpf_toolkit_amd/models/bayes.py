"""Attribution models as linear-logit posteriors over the 16-slot feature layout.

Every model here reduces to ``logits = X @ W + b`` followed by a log-sum-exp
normalisation, which is exactly what the MFMA posterior kernel (``ops.posterior``)
evaluates for a whole batch of incidents at once:

* ``NaiveBayes.ref()`` -- REF-exact naive Bayes (pkg/attribution/bayesian.go:39-343):
  uniform priors over the 8 REF domains, the 12x8 likelihood table, binary evidence
  ``value >= threshold`` (bayesian.go:194-207), every table signal contributes
  (absent = not elevated, bayesian.go:237-240), clamp [0.01, 0.99], LSE, evidence =
  elevated signals with P(elevated|d) >= 0.5, stable sort by posterior, hypotheses
  < 0.01 dropped, top-1 overrides the label map, empty ``signals`` -> rule fallback.
  In linear form: X = e (0/1), W = log p - log(1-p), b = log prior + sum log(1-p).
* ``NaiveBayes.learned(stats)`` -- the same model with priors/likelihoods re-estimated
  from labelled sufficient statistics (Beta/Dirichlet smoothing towards a seeded
  random-init table), the "random-init priors" north-star configuration.
* ``LDA.fit(stats)`` -- the covariance-corrected model: shared-covariance Gaussian
  class conditionals on log1p(signal) features; W = S^-1 mu_d,
  b = -1/2 mu_d^T S^-1 mu_d + log pi_d. Its scatter matrix is the MFMA covariance step.

* ``with_pairs(model, rho)`` -- the 2-fault posterior: the hypothesis space grows from the
  single domains to every pair of fault domains, each pair a noisy-OR of its members'
  likelihoods (P(e_s | {a, b}) = 1 - (1 - p_sa)(1 - p_sb)) with prior mass ``rho`` shared over
  the pairs in proportion to pi_a pi_b. A pair is one more linear-logit column, so the MFMA
  kernel scores all 10 + 36 hypotheses in the same product; the output per domain is its
  *marginal* P(d in the incident | evidence) = P({d}) + sum of the pairs holding d (REF's
  single-label posterior, pipeline.go:140-185, has no way to say "both").

All CPU math is float64 numpy (the oracle); the GPU path evaluates the same W/b.
"""

from __future__ import annotations

import functools
import itertools
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..contracts.types import FaultHypothesis, IncidentAttribution
from ..signals import catalog
from .sample import FaultSample, build_attribution

N_SLOTS = catalog.N_SLOTS
N_DOMAINS = len(catalog.ALL_DOMAINS)       # 10 (8 REF + 2 GPU)
N_REF_DOMAINS = len(catalog.REF_DOMAINS)   # 8
THRESHOLDS = np.array([s.elevated for s in catalog.SIGNALS], dtype=np.float64)
# Nominal ("healthy") values used to impute absent signals for continuous models:
# REF base signal profile (pkg/signals/generator.go:244-259) + GPU nominals.
NOMINAL = np.array([12, 0.2, 4, 18, 0, 22, 0, 0.6, 5, 0.5, 2, 5, 0.5, 40, 3, 1.0], dtype=np.float64)
NEG_INF = -np.inf
MAX_PAIRS = 48                             # ops/csrc/mislo_launch.h kMaxPairs (3 MFMA column tiles)
# 2-fault hypotheses: every pair of fault domains ("unknown" is the no-fault hypothesis)
PAIR_LIST: Tuple[Tuple[int, int], ...] = tuple(itertools.combinations(
    [d for d, n in enumerate(catalog.ALL_DOMAINS) if n != "unknown"], 2))
assert len(PAIR_LIST) <= MAX_PAIRS


def clamp_likelihood(p):
    return np.clip(p, 0.01, 0.99)


@dataclass
class Posterior:
    domain: str
    posterior: float
    evidence: List[str]


APP_BIT = 16  # ops/csrc/mislo_launch.h kAppBit: the application evidence's bit in evbits


@functools.lru_cache(maxsize=4096)
def _evidence_names(bits: int) -> tuple:
    """Signal names of an evidence bitmask over the 16 slots (and the application bit), sorted
    (REF's evidence order)."""
    names = [catalog.SIGNAL_NAMES[s] for s in range(N_SLOTS) if bits >> s & 1]
    if bits >> APP_BIT & 1:
        names.append(catalog.APP_RETRIEVAL_SIGNAL)
    return tuple(sorted(names))


@dataclass
class AppEvidence:
    """Application-source evidence: one binary signal beside the 16 kernel slots (the device twin
    is ops/csrc/mislo_launch.h ``AppModel``, evaluated inside the K3 posterior kernel).

    The signal is an incident group's retrieval time that the kernel does not account for. It is
    REF's ``DecomposeRetrieval`` (pkg/otel/processor/ebpfcorrelator/correlator.go:179-194) taken
    to group level: the mean application-reported retrieval time of the group's spans (REF's
    ``llm.slo.retrieval.{vectordb,network,dns}_ms``, demo/rag-service/main.go:393-397) minus the
    kernel-attributed share, the group's mean joined dns + connect + TLS latency. REF's schema
    lets such evidence come from the application (incident-attribution.schema.json:41-56).

    A group none of whose spans carries a breakdown contributes nothing: the signal is summed out,
    not read as "not elevated", so REF's rows score exactly as before. Otherwise the domain logit
    gains ``log P(!e|d) + e * logit P(e|d)`` (at the model's temperature), e = residual >= threshold."""
    p: Optional[np.ndarray]            # [D] P(residual elevated | domain)
    threshold_ms: float = catalog.APP_RETRIEVAL_THRESHOLD_MS
    temperature: float = 1.0
    # the device image's terms as given (from_image: the CPU engine scores what the GPU would)
    image_terms: Optional[Tuple[np.ndarray, ...]] = None

    @staticmethod
    def expert(threshold_ms: float = catalog.APP_RETRIEVAL_THRESHOLD_MS, temperature: float = 1.0) -> "AppEvidence":
        p = np.array([catalog.APP_RETRIEVAL_LIKELIHOOD[d] for d in catalog.ALL_DOMAINS], dtype=np.float64)
        return AppEvidence(p, float(threshold_ms), float(temperature))

    @staticmethod
    def from_image(w: np.ndarray, b: np.ndarray, w2: np.ndarray, b2: np.ndarray, thr_ms: float,
                   dom_mask: int) -> "AppEvidence":
        mask = np.array([(int(dom_mask) >> d) & 1 for d in range(len(w))], dtype=bool)
        return AppEvidence(None, float(thr_ms), 1.0, (np.asarray(w, np.float64), np.asarray(b, np.float64),
                                                      np.asarray(w2, np.float64), np.asarray(b2, np.float64), mask))

    def evidence_mask(self, D: int) -> np.ndarray:
        """[D] bool: domains whose evidence the elevated signal is (P(e|d) >= 0.5)."""
        if self.image_terms is not None:
            return self.image_terms[4][:D]
        return self.p[:D] >= 0.5

    def terms(self) -> Tuple[np.ndarray, np.ndarray]:
        """(w [D], b [D]): logit P(e|d) and log P(!e|d), divided by the temperature."""
        if self.image_terms is not None:
            return self.image_terms[0], self.image_terms[1]
        pe, pn = clamp_likelihood(self.p), clamp_likelihood(1.0 - self.p)
        return (np.log(pe) - np.log(pn)) / self.temperature, np.log(pn) / self.temperature

    def pair_terms(self, pairs: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """The 2-fault columns' terms: noisy-OR of the members (``with_pairs``)."""
        if self.image_terms is not None:
            P = len(pairs)
            return self.image_terms[2][:P], self.image_terms[3][:P]
        pe = clamp_likelihood(self.p)
        a, b = np.asarray(pairs)[:, 0], np.asarray(pairs)[:, 1]
        q = clamp_likelihood(1.0 - (1.0 - pe[a]) * (1.0 - pe[b]))
        qn = clamp_likelihood(1.0 - q)
        return (np.log(q) - np.log(qn)) / self.temperature, np.log(qn) / self.temperature

    @staticmethod
    def residual(app_cnt: np.ndarray, feat: np.ndarray) -> np.ndarray:
        """[G] residual ms (NaN: no breakdown) from the groups' [G, 2] counts (spans, sum in 10 us
        units) and features, in the device's operation order (posterior.hip app_state)."""
        cnt = np.asarray(app_cnt, dtype=np.uint32).reshape(-1, 2)
        f = np.asarray(feat, dtype=np.float32).reshape(-1, N_SLOTS)
        n = cnt[:, 0].astype(np.float64)
        with np.errstate(invalid="ignore", divide="ignore"):
            mean = cnt[:, 1].astype(np.float64) / APP_UNITS_PER_MS / n
        kern = np.zeros(len(n))
        for s in (0, 3, 5):  # dns + connect + tls, in that order
            v = f[:, s].astype(np.float64)
            kern = kern + np.where(np.isnan(v), 0.0, v)
        return np.where(n > 0, mean - kern, np.nan)

    def state(self, app_cnt: np.ndarray, feat: np.ndarray) -> np.ndarray:
        """[G] int: -1 absent, 0 present, 1 elevated."""
        r = self.residual(app_cnt, feat)
        with np.errstate(invalid="ignore"):
            return np.where(np.isnan(r), -1, (r >= self.threshold_ms).astype(np.int64))


APP_UNITS_PER_MS = 100.0  # ops/csrc/mislo_launch.h kAppUnitsPerMs (10 us fixed point)


def app_counts(spans: np.ndarray, n_groups: int, mine: Optional[np.ndarray] = None,
               groups: Optional[np.ndarray] = None) -> np.ndarray:
    """[G, 2] uint32 application retrieval counts of a window's SPAN records, as k_decode_spans
    accumulates them: spans with 0 < retr_ms < 1e7 (spans, rint(retr_ms * 100) summed, u32)."""
    out = np.zeros((int(n_groups), 2), np.uint32)
    if len(spans) == 0 or n_groups <= 0:
        return out
    r = np.asarray(spans["retr_ms"], dtype=np.float32)
    g = np.asarray(spans["group_id"] if groups is None else groups, dtype=np.int64)
    with np.errstate(invalid="ignore"):
        ok = (r > np.float32(0)) & (r < np.float32(1e7)) & (g >= 0) & (g < n_groups)
    if mine is not None:
        ok &= mine
    units = np.rint(r[ok].astype(np.float64) * APP_UNITS_PER_MS).astype(np.uint64)
    np.add.at(out[:, 0], g[ok], np.uint32(1))
    s = np.zeros(int(n_groups), np.uint64)
    np.add.at(s, g[ok], units)
    out[:, 1] = (s & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    return out


@dataclass
class LinearPosteriorModel:
    """logits[b, d] = X[b] @ W[:, d] + bias[d]; domains with bias -inf are inactive."""
    name: str
    weights: np.ndarray                 # [16, D] float64
    bias: np.ndarray                    # [D]     float64 (-inf = inactive domain)
    evidence_mask: np.ndarray           # [16, D] bool
    feature_mode: str = "binary"        # "binary" (e = v >= thr) | "continuous"
    thresholds: np.ndarray = field(default_factory=lambda: THRESHOLDS.copy())
    mean: Optional[np.ndarray] = None   # continuous: feature centring
    table_mask: Optional[np.ndarray] = None  # binary: which slots the model knows
    # 2-fault hypotheses (with_pairs): [16, P] weights, [P] bias (-inf = inactive), [P, 2] members
    pair_w: Optional[np.ndarray] = None
    pair_b: Optional[np.ndarray] = None
    pairs: Optional[np.ndarray] = None
    pair_rho: float = 0.0
    # application evidence (AppEvidence); the methods below take the groups' states (-1/0/1,
    # AppEvidence.state) as ``app``
    app: Optional[AppEvidence] = None

    def _app_add(self, app: Optional[np.ndarray], B: int) -> Tuple[Optional[np.ndarray], Optional[np.ndarray]]:
        """(single [B, D], pair [B, P]) logit terms of the application evidence, or None."""
        if self.app is None or app is None:
            return None, None
        st = np.asarray(app, dtype=np.int64).reshape(-1)[:B]
        w, b = self.app.terms()
        pres = (st >= 0)[:, None]
        add = np.where(pres, b[None, :self.weights.shape[1]] + np.where((st == 1)[:, None], w[None, :self.weights.shape[1]], 0.0), 0.0)
        add2 = None
        if self.pairs is not None:
            w2, b2 = self.app.pair_terms(self.pairs)
            add2 = np.where(pres, b2[None, :] + np.where((st == 1)[:, None], w2[None, :], 0.0), 0.0)
        return add, add2

    def features(self, values: np.ndarray) -> np.ndarray:
        """values: [B, 16] with NaN for absent signals -> model features X [B, 16]."""
        values = np.asarray(values, dtype=np.float64)
        if self.feature_mode == "binary":
            with np.errstate(invalid="ignore"):
                e = (values >= self.thresholds[None, :]) & ~np.isnan(values)
            x = e.astype(np.float64)
            if self.table_mask is not None:
                x = x * self.table_mask[None, :]
            return x
        v = np.where(np.isnan(values), NOMINAL[None, :], values)
        x = np.log1p(np.maximum(v, 0.0))
        if self.mean is not None:
            x = x - self.mean[None, :]
        return x

    def elevated(self, values: np.ndarray) -> np.ndarray:
        values = np.asarray(values, dtype=np.float64)
        with np.errstate(invalid="ignore"):
            e = (values >= self.thresholds[None, :]) & ~np.isnan(values)
        if self.table_mask is not None:
            e &= self.table_mask[None, :].astype(bool)
        return e

    def logits(self, values: np.ndarray, app: Optional[np.ndarray] = None) -> np.ndarray:
        lg = self.features(values) @ self.weights + self.bias[None, :]
        add, _ = self._app_add(app, lg.shape[0])
        return lg if add is None else lg + add

    def hypothesis_posteriors(self, values: np.ndarray, app: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        """(P(single d) [B, D], P(pair h) [B, P]) -- the normalised hypothesis distribution (no
        pairs: [B, 0])."""
        x = self.features(values)
        lg = x @ self.weights + self.bias[None, :]
        l2 = (x @ self.pair_w + self.pair_b[None, :]) if self.pairs is not None else np.zeros((lg.shape[0], 0))
        add, add2 = self._app_add(app, lg.shape[0])
        if add is not None:
            lg = lg + add
            if add2 is not None:
                l2 = l2 + add2
        allv = np.concatenate([lg, l2], axis=1)
        m = np.max(allv, axis=1, keepdims=True)
        with np.errstate(invalid="ignore"):
            z = m + np.log(np.sum(np.exp(allv - m), axis=1, keepdims=True))
        return np.exp(lg - z), np.exp(l2 - z)

    def posteriors(self, values: np.ndarray, app: Optional[np.ndarray] = None) -> np.ndarray:
        """Per domain: the posterior (single-fault model) or the marginal P(d in the incident)
        (2-fault model)."""
        if self.pairs is None:
            lg = self.logits(values, app)
            m = np.max(lg, axis=1, keepdims=True)
            with np.errstate(invalid="ignore"):
                ex = np.exp(lg - m)
            z = m + np.log(np.sum(ex, axis=1, keepdims=True))
            return np.exp(lg - z)
        p1, p2 = self.hypothesis_posteriors(values, app)
        marg = p1.copy()
        for h, (a, b) in enumerate(self.pairs.tolist()):
            marg[:, a] += p2[:, h]
            marg[:, b] += p2[:, h]
        return marg

    def predict(self, values: np.ndarray, app: Optional[np.ndarray] = None) -> np.ndarray:
        """Top-1 domain: argmax of the logits (single-fault) or of the marginals (2-fault);
        ties -> the lowest domain index, as the kernel."""
        if self.pairs is None:
            return np.argmax(self.logits(values, app), axis=1)
        return np.argmax(self.posteriors(values, app), axis=1)

    def evidence_bits(self, values: np.ndarray, app: Optional[np.ndarray] = None) -> np.ndarray:
        """[B, D] uint32 bitmask over slots: elevated & P(elevated|d) >= 0.5; bit APP_BIT: the
        application evidence elevated & P(e|d) >= 0.5."""
        e = self.elevated(values)
        D = self.weights.shape[1]
        bits = np.zeros((e.shape[0], D), dtype=np.uint32)
        for s in range(N_SLOTS):
            col = e[:, s:s + 1] & self.evidence_mask[s][None, :]
            bits |= (col.astype(np.uint32) << np.uint32(s))
        if self.app is not None and app is not None:
            st = np.asarray(app, dtype=np.int64).reshape(-1)[:e.shape[0]]
            col = (st == 1)[:, None] & self.app.evidence_mask(D)[None, :]
            bits |= (col.astype(np.uint32) << np.uint32(APP_BIT))
        return bits

    def attribute(self, signals: Dict[str, float]) -> List[Posterior]:
        """Single-sample API with REF ordering semantics (stable sort, domain order ties)."""
        vec = np.array([catalog.feature_vector(signals)], dtype=np.float64)
        return self.ranked(self.posteriors(vec)[0], self.evidence_bits(vec)[0])

    def ranked(self, post: np.ndarray, bits: np.ndarray) -> List[Posterior]:
        """Posterior row + evidence bitmask row (numpy or the GPU kernel's) -> sorted hypotheses.
        Rows become Python lists once (the agent ranks every incident of every window)."""
        D = self.weights.shape[1]
        live = np.isfinite(self.bias[:D]).tolist()
        pl = np.asarray(post, dtype=np.float64)[:D].tolist()
        bl = np.asarray(bits).astype(np.int64)[:D].tolist()
        out: List[Posterior] = [Posterior(dom, pl[d], list(_evidence_names(bl[d])))
                                for d, dom in enumerate(catalog.ALL_DOMAINS[:D]) if live[d]]
        out.sort(key=lambda p: -p.posterior)  # Python sort is stable == sort.SliceStable
        return out

    def attribute_sample(self, sample: FaultSample) -> IncidentAttribution:
        if not sample.signals:
            return build_attribution(sample)
        return self.attribution_from_ranked(sample, self.attribute(sample.signals))

    def attribution_from_posterior(self, sample: FaultSample, post: np.ndarray,
                                   bits: np.ndarray) -> IncidentAttribution:
        if not sample.signals:
            return build_attribution(sample)
        return self.attribution_from_ranked(sample, self.ranked(post, bits))

    @staticmethod
    def attribution_from_ranked(sample: FaultSample, posts: List[Posterior]) -> IncidentAttribution:
        base = build_attribution(sample)
        base.fault_hypotheses = [FaultHypothesis(p.domain, p.posterior, p.evidence)
                                 for p in posts if p.posterior >= 0.01]
        if posts:
            base.predicted_fault_domain = posts[0].domain
            base.confidence = posts[0].posterior
        return base

    def to_arrays(self) -> Dict[str, np.ndarray]:
        return {"weights": self.weights, "bias": self.bias, "evidence_mask": self.evidence_mask,
                "thresholds": self.thresholds,
                "mean": self.mean if self.mean is not None else np.zeros(N_SLOTS),
                "table_mask": self.table_mask if self.table_mask is not None else np.ones(N_SLOTS)}


class NaiveBayes:
    """Factory for binary-evidence naive Bayes in linear-logit form."""

    @staticmethod
    def from_tables(priors: Dict[str, float], likelihoods: Dict[str, Dict[str, float]],
                    domains: Sequence[str] = catalog.REF_DOMAINS, name: str = "bayes") -> LinearPosteriorModel:
        D = N_DOMAINS
        W = np.zeros((N_SLOTS, D))
        b = np.full(D, NEG_INF)
        mask = np.zeros((N_SLOTS, D), dtype=bool)
        table = np.zeros(N_SLOTS)
        for dom in domains:
            d = catalog.DOMAIN_INDEX[dom]
            prior = priors.get(dom, 0.0)
            if prior <= 0:
                prior = 1e-10
            b[d] = math.log(prior)
        for sig, row in likelihoods.items():
            spec = catalog.BY_NAME.get(sig)
            if spec is None:
                continue
            s = spec.slot
            table[s] = 1.0
            for dom in domains:
                d = catalog.DOMAIN_INDEX[dom]
                p = row.get(dom)
                if p is None:  # REF likelihoodFor: missing domain entry -> 0.5 uninformative
                    pe = pn = 0.5
                else:
                    pe, pn = clamp_likelihood(p), clamp_likelihood(1.0 - p)
                    mask[s, d] = p >= 0.5
                W[s, d] = math.log(pe) - math.log(pn)
                b[d] += math.log(pn)
        return LinearPosteriorModel(name, W, b, mask, "binary", THRESHOLDS.copy(), None, table)

    @staticmethod
    def ref() -> LinearPosteriorModel:
        doms = catalog.REF_DOMAINS
        priors = {d: 1.0 / len(doms) for d in doms}
        return NaiveBayes.from_tables(priors, catalog.ref_likelihoods(), doms, "bayes")

    @staticmethod
    def gpu() -> LinearPosteriorModel:
        """REF's table extended to the 16 signals x 10 domains (catalog.extended_likelihood_matrix:
        REF rows and columns unchanged, plus the 4 GPU signals and the 2 GPU domains), uniform
        priors: an expert model that can name gpu_contention / gpu_interconnect without labels
        (the agent never learns online, REF's table cannot see GPU signals)."""
        doms = catalog.ALL_DOMAINS
        m = catalog.extended_likelihood_matrix()
        lik = {catalog.SIGNAL_NAMES[s]: dict(zip(doms, m[s])) for s in range(N_SLOTS)}
        return NaiveBayes.from_tables({d: 1.0 / len(doms) for d in doms}, lik, doms, "bayes_gpu")

    @staticmethod
    def random_init_table(seed: int = 42, domains: Sequence[str] = catalog.ALL_DOMAINS) -> np.ndarray:
        rng = np.random.default_rng(seed)
        return rng.uniform(0.05, 0.95, size=(N_SLOTS, len(domains)))

    @staticmethod
    def expert_table(domains: Sequence[str] = catalog.ALL_DOMAINS) -> np.ndarray:
        """[16, D] P(elevated | domain) of REF's expert table (bayesian.go:67-190), extended to
        the GPU signals and domains (catalog.extended_likelihood_matrix)."""
        m = np.asarray(catalog.extended_likelihood_matrix(), dtype=np.float64)
        return m[:, [catalog.DOMAIN_INDEX[d] for d in domains]]

    @staticmethod
    def unknown_floor(domains: Sequence[str] = catalog.ALL_DOMAINS) -> np.ndarray:
        """[16, D] minimum likelihoods: the ``unknown`` column of REF's table (every signal
        elevated by chance 5-10 % of the time), zero elsewhere. Healthy replay incidents never
        show an elevated signal, so the learned P(e | unknown) falls to REF's clamp (0.01) and one
        elevated signal then costs "no fault" more than a whole fault domain's missing symptoms
        (REF row mf-51, a lone DNS elevation, read as unknown). The floor keeps "unknown" what it
        is in REF: the hypothesis that whatever is elevated is noise."""
        f = np.zeros((N_SLOTS, len(domains)))
        if "unknown" in domains:
            u = list(domains).index("unknown")
            f[:, u] = NaiveBayes.expert_table(domains)[:, u]
        return f

    @staticmethod
    def learned(stats: "SufficientStats", alpha: float = 2.0, seed: int = 42,
                init: Optional[np.ndarray] = None, domains: Sequence[str] = catalog.ALL_DOMAINS,
                prior_pseudo: float = 1.0, temperature: float = 1.0, min_count: float = 0.0,
                floor: Optional[np.ndarray] = None, cap_domain: Optional[str] = None,
                ceil: Optional[float] = None) -> LinearPosteriorModel:
        """Posterior-mean estimates: p_sd = (c_sd + alpha*p0_sd) / (n_d + alpha), with p0 a
        seeded random-init table (north star: random-init priors) or REF's expert table
        (``expert_table``: a domain without labelled mass keeps REF's column); pi_d ~ Dirichlet(1).
        ``floor`` [16, D] bounds every likelihood from below (``unknown_floor``), ``ceil`` from
        above (REF's table spans [0.05, 0.95]: no symptom's presence or absence is near-certain
        evidence); the prior of
        ``cap_domain`` is capped at the largest prior of the other active domains (the no-fault
        class, the most frequent label, must not win on its prior alone).
        ``temperature`` T divides every logit (calibration: same argmax, flatter posteriors for
        T > 1); a domain with less than ``min_count`` labelled mass is inactive. The device refit
        (ops/csrc/posterior.hip k_refit_nb) computes exactly this."""
        p0 = init if init is not None else NaiveBayes.random_init_table(seed, domains)
        idx = [catalog.DOMAIN_INDEX[d] for d in domains]
        n = stats.count[idx]
        c = stats.elevated_sum[:, idx]
        p = (c + alpha * p0) / (n[None, :] + alpha)
        if floor is not None:
            p = np.maximum(p, floor)
        if ceil is not None:
            p = np.minimum(p, float(ceil))
        priors_arr = (n + prior_pseudo) / (n.sum() + prior_pseudo * len(idx))
        if cap_domain is not None and cap_domain in domains:
            u = list(domains).index(cap_domain)
            others = [i for i in range(len(idx)) if i != u and n[i] >= min_count]
            if others:
                priors_arr[u] = min(priors_arr[u], max(priors_arr[i] for i in others))
        priors = {d: float(priors_arr[i]) for i, d in enumerate(domains)}
        lik = {catalog.SIGNAL_NAMES[s]: {d: float(p[s, i]) for i, d in enumerate(domains)}
               for s in range(N_SLOTS)}
        m = NaiveBayes.from_tables(priors, lik, domains, "bayes_learned")
        for i, d in enumerate(domains):
            if n[i] < min_count:
                m.bias[catalog.DOMAIN_INDEX[d]] = NEG_INF
        return with_temperature(m, temperature)


def with_temperature(m: LinearPosteriorModel, temperature: float) -> LinearPosteriorModel:
    """The model with every logit divided by ``temperature`` (inactive domains stay -inf)."""
    if temperature == 1.0:
        return m
    if not temperature > 0:
        raise ValueError("temperature must be > 0")
    inv = 1.0 / float(temperature)
    bias = np.where(np.isfinite(m.bias), m.bias * inv, m.bias)
    out = LinearPosteriorModel(m.name, m.weights * inv, bias, m.evidence_mask.copy(), m.feature_mode,
                               m.thresholds.copy(), None if m.mean is None else m.mean.copy(),
                               None if m.table_mask is None else m.table_mask.copy())
    if m.pairs is not None:
        out.pair_w, out.pairs, out.pair_rho = m.pair_w * inv, m.pairs.copy(), m.pair_rho
        out.pair_b = np.where(np.isfinite(m.pair_b), m.pair_b * inv, m.pair_b)
    if m.app is not None and m.app.p is not None:
        out.app = AppEvidence(m.app.p.copy(), m.app.threshold_ms, m.app.temperature * float(temperature))
    return out


def _raw_tables(m: LinearPosteriorModel, temperature: float):
    """(P(e | d) [16, D], log prior [D] (-inf inactive), table slots [16] bool) of a binary naive
    Bayes in linear-logit form at ``temperature``: W = logit(p) and pe + pn = 1 after REF's
    clamp, so p = sigmoid(T W) and log pi_d = T b_d - sum_s log(1 - p_sd)."""
    T = float(temperature)
    table = (m.table_mask if m.table_mask is not None else np.ones(N_SLOTS)).astype(bool)
    raw = m.weights * T
    p = 1.0 / (1.0 + np.exp(-raw))
    logpn = -np.logaddexp(0.0, raw)
    with np.errstate(invalid="ignore"):
        logpi = np.where(np.isfinite(m.bias), m.bias * T - (logpn * table[:, None]).sum(axis=0), NEG_INF)
    return p, logpi, table


def with_pairs(m: LinearPosteriorModel, rho: float, temperature: float = 1.0) -> LinearPosteriorModel:
    """The 2-fault model of a binary naive Bayes (see the module docstring): single hypotheses
    keep their likelihoods with prior (1 - rho) pi_d; pair {a, b} gets the noisy-OR likelihood
    and prior rho pi_a pi_b / sum over active pairs. ``temperature`` is the one the model's
    weights are already divided by (the pair columns get the same). The device refit
    (posterior.hip k_refit_nb) builds the identical tables."""
    if m.feature_mode != "binary":
        raise ValueError("the 2-fault model is defined for binary naive Bayes")
    if not 0.0 < rho < 1.0:
        raise ValueError("rho must be in (0, 1)")
    T = float(temperature)
    p, logpi, table = _raw_tables(m, T)
    fin = np.isfinite(logpi)
    logpi = np.where(fin, logpi - np.log(np.exp(logpi[fin]).sum()), NEG_INF)
    P = len(PAIR_LIST)
    pw = np.zeros((N_SLOTS, P))
    pb = np.full(P, NEG_INF)
    pr = np.array([logpi[a] + logpi[b] for a, b in PAIR_LIST])
    act = np.isfinite(pr)
    pnorm = math.log(np.exp(pr[act]).sum()) if act.any() else 0.0
    for h, (a, b) in enumerate(PAIR_LIST):
        if not act[h]:
            continue
        q = clamp_likelihood(1.0 - (1.0 - p[:, a]) * (1.0 - p[:, b]))
        qn = clamp_likelihood(1.0 - q)
        pw[:, h] = np.where(table, np.log(q) - np.log(qn), 0.0) / T
        pb[h] = (math.log(rho) + pr[h] - pnorm + float(np.log(qn)[table].sum())) / T
    bias = np.where(np.isfinite(m.bias), m.bias + math.log1p(-rho) / T, m.bias)
    out = LinearPosteriorModel(m.name, m.weights.copy(), bias, m.evidence_mask.copy(), m.feature_mode,
                               m.thresholds.copy(), None, None if m.table_mask is None else m.table_mask.copy())
    out.pair_w, out.pair_b, out.pairs, out.pair_rho = pw, pb, np.array(PAIR_LIST, dtype=np.int64), float(rho)
    out.app = m.app
    return out


def marginalize(m: LinearPosteriorModel, observable: Sequence[str], temperature: float = 1.0,
                drop_unobservable: bool = True) -> LinearPosteriorModel:
    """The binary naive-Bayes model scoring only the ``observable`` signals: every other table
    signal is summed out of the likelihood (its factor P(e_s | d) marginalises to 1) instead of
    being read as "not elevated". An agent whose sources cannot produce a signal at all (no
    probe for it on this node, a degraded capability mode, no GPU tool) must not count its
    absence as evidence against the domains it would indicate.

    In the linear-logit form a table signal contributes ``e * W[s, d]`` plus ``log P(not e | d)``
    folded into the bias, with ``W = logit(P(e | d))``; so summing it out is ``W[s, :] = 0`` and
    ``bias[d] += softplus(W[s, d])``, both at the model's ``temperature`` (stored weights and bias
    are divided by it). With ``drop_unobservable`` a domain none of the observable signals indicates
    is deactivated (below); without it the result is the exact marginal of the full model."""
    if m.feature_mode != "binary":
        raise ValueError("only binary naive-Bayes models marginalise signal by signal")
    keep = {catalog.BY_NAME[s].slot for s in observable if s in catalog.BY_NAME}
    unknown = [s for s in observable if s not in catalog.BY_NAME]
    if unknown:
        raise ValueError(f"unknown signals {unknown}")
    T = float(temperature)
    W, b = m.weights.copy(), m.bias.copy()
    table = m.table_mask.copy() if m.table_mask is not None else np.ones(N_SLOTS)
    mask = m.evidence_mask.copy()
    fin = np.isfinite(b)
    pw = m.pair_w.copy() if m.pairs is not None else None
    pb = m.pair_b.copy() if m.pairs is not None else None
    pfin = np.isfinite(pb) if pb is not None else None
    for s in range(N_SLOTS):
        if s in keep or not table[s]:
            continue
        b[fin] += (np.logaddexp(0.0, W[s] * T) / T)[fin]
        W[s] = 0.0
        if pw is not None:  # the pair columns are naive-Bayes columns too
            pb[pfin] += (np.logaddexp(0.0, pw[s] * T) / T)[pfin]
            pw[s] = 0.0
        mask[s] = False
        table[s] = 0.0
    # a fault domain that no observable signal indicates (P(e | d) >= 0.5 and at least twice
    # P(e | unknown)) cannot be told apart from "unknown" on this node: with its evidence summed
    # out it would win on its prior alone whenever nothing is elevated. It is not attributed.
    if drop_unobservable and "unknown" in catalog.DOMAIN_INDEX and keep:
        u = catalog.DOMAIN_INDEX["unknown"]
        raw = m.weights * T
        p = 1.0 / (1.0 + np.exp(-raw))
        obs = np.array(sorted(keep))
        for d in range(W.shape[1]):
            if d == u or not fin[d]:
                continue
            if m.app is not None and m.app.p is not None and m.app.p[d] >= 0.5 and m.app.p[d] >= 2.0 * m.app.p[u]:
                continue  # the application evidence indicates it (AppEvidence)
            if not np.any((p[obs, d] >= 0.5) & (p[obs, d] >= 2.0 * p[obs, u])):
                b[d] = NEG_INF
                if pb is not None:
                    pb[(m.pairs[:, 0] == d) | (m.pairs[:, 1] == d)] = NEG_INF
    out = LinearPosteriorModel(m.name, W, b, mask, m.feature_mode, m.thresholds.copy(), None, table)
    if pw is not None:
        out.pair_w, out.pair_b, out.pairs, out.pair_rho = pw, pb, m.pairs.copy(), m.pair_rho
    out.app = m.app
    return out


def label_code(primary: int, domains: Sequence[int] = ()) -> int:
    """int32 incident label the engine takes (posterior.hip): bits 0-7 the primary domain,
    bits 8-23 the domain set of a multi-fault incident (its statistics spread evenly over the
    set; the confusion matrix counts the primary)."""
    ds = sorted(set(int(d) for d in domains) | {int(primary)})
    if len(ds) <= 1:
        return int(primary)
    return int(primary) | (sum(1 << d for d in ds) << 8)


def soft_labels(codes: np.ndarray, n_domains: int = N_DOMAINS) -> np.ndarray:
    """label codes [B] -> soft label rows [B, n_domains] (0 rows for codes < 0)."""
    codes = np.asarray(codes, dtype=np.int64)
    Y = np.zeros((len(codes), n_domains))
    for b, c in enumerate(codes.tolist()):
        if c < 0:
            continue
        dset = (c >> 8) & 0xFFFF
        if dset:
            ds = [d for d in range(16) if dset >> d & 1 and d < n_domains]
            Y[b, ds] = 1.0 / len(ds)
        elif (c & 0xFF) < n_domains:
            Y[b, c & 0xFF] = 1.0
    return Y


class LDA:
    @staticmethod
    def fit(stats: "SufficientStats", shrinkage: float = 0.05, domains: Sequence[str] = catalog.ALL_DOMAINS,
            prior_pseudo: float = 1.0) -> LinearPosteriorModel:
        D = N_DOMAINS
        idx = [catalog.DOMAIN_INDEX[d] for d in domains]
        n = stats.count.astype(np.float64)
        N = max(float(n[idx].sum()), 1.0)
        mean_all = stats.x_sum.sum(axis=1) / N                  # [16]
        mu = np.zeros((N_SLOTS, D))
        for d in idx:
            if n[d] > 0:
                mu[:, d] = stats.x_sum[:, d] / n[d]
            else:
                mu[:, d] = mean_all
        # pooled within-class scatter: S2 - sum_d n_d mu_d mu_d^T
        within = stats.xx.copy()
        for d in idx:
            if n[d] > 0:
                within -= n[d] * np.outer(mu[:, d], mu[:, d])
        dof = max(N - len([d for d in idx if n[d] > 0]), 1.0)
        cov = within / dof
        cov = (1 - shrinkage) * cov + shrinkage * (np.trace(cov) / N_SLOTS + 1e-6) * np.eye(N_SLOTS)
        prec = np.linalg.inv(cov)
        muc = mu - mean_all[:, None]
        W = np.zeros((N_SLOTS, D))
        b = np.full(D, NEG_INF)
        for d in idx:
            W[:, d] = prec @ muc[:, d]
            pi = (n[d] + prior_pseudo) / (N + prior_pseudo * len(idx))
            b[d] = -0.5 * muc[:, d] @ prec @ muc[:, d] + math.log(pi)
        # evidence: a slot supports d when the class mean sits above the elevated threshold
        thr = np.log1p(THRESHOLDS) - mean_all
        mask = muc >= thr[:, None]
        return LinearPosteriorModel("lda", W, b, mask, "continuous", THRESHOLDS.copy(), mean_all, None)


@dataclass
class SufficientStats:
    """Labelled sufficient statistics (CPU oracle of the MFMA statistics kernel).

    count[d]            = #samples labelled d
    elevated_sum[s, d]  = sum_b y_bd * e_bs        (E^T Y)
    x_sum[s, d]         = sum_b y_bd * x_bs        (X^T Y, x = log1p(value), NOMINAL-imputed)
    xx[s, t]            = sum_b x_bs x_bt          (X^T X, the covariance step)
    """
    count: np.ndarray = field(default_factory=lambda: np.zeros(N_DOMAINS))
    elevated_sum: np.ndarray = field(default_factory=lambda: np.zeros((N_SLOTS, N_DOMAINS)))
    x_sum: np.ndarray = field(default_factory=lambda: np.zeros((N_SLOTS, N_DOMAINS)))
    xx: np.ndarray = field(default_factory=lambda: np.zeros((N_SLOTS, N_SLOTS)))

    def add(self, values: np.ndarray, labels: np.ndarray, weights: Optional[np.ndarray] = None) -> None:
        """values [B,16] (NaN = absent), labels [B] domain index (or [B,D] soft labels)."""
        values = np.asarray(values, dtype=np.float64)
        B = values.shape[0]
        labels = np.asarray(labels)
        if labels.ndim == 1:
            Y = np.zeros((B, N_DOMAINS))
            Y[np.arange(B), labels.astype(np.int64)] = 1.0
        else:
            Y = labels.astype(np.float64)
        if weights is not None:
            Y = Y * np.asarray(weights, dtype=np.float64)[:, None]
        with np.errstate(invalid="ignore"):
            E = ((values >= THRESHOLDS[None, :]) & ~np.isnan(values)).astype(np.float64)
        X = np.log1p(np.maximum(np.where(np.isnan(values), NOMINAL[None, :], values), 0.0))
        self.count += Y.sum(axis=0)
        self.elevated_sum += E.T @ Y
        self.x_sum += X.T @ Y
        self.xx += X.T @ X

    def merge(self, other: "SufficientStats") -> "SufficientStats":
        return SufficientStats(self.count + other.count, self.elevated_sum + other.elevated_sum,
                               self.x_sum + other.x_sum, self.xx + other.xx)

    def pack(self) -> np.ndarray:
        return np.concatenate([self.count.ravel(), self.elevated_sum.ravel(), self.x_sum.ravel(),
                               self.xx.ravel()])

    @classmethod
    def unpack(cls, flat: np.ndarray) -> "SufficientStats":
        flat = np.asarray(flat, dtype=np.float64)
        o = 0
        count = flat[o:o + N_DOMAINS]; o += N_DOMAINS
        es = flat[o:o + N_SLOTS * N_DOMAINS].reshape(N_SLOTS, N_DOMAINS); o += N_SLOTS * N_DOMAINS
        xs = flat[o:o + N_SLOTS * N_DOMAINS].reshape(N_SLOTS, N_DOMAINS); o += N_SLOTS * N_DOMAINS
        xx = flat[o:o + N_SLOTS * N_SLOTS].reshape(N_SLOTS, N_SLOTS)
        return cls(count.copy(), es.copy(), xs.copy(), xx.copy())

    PACKED_LEN = N_DOMAINS + 2 * N_SLOTS * N_DOMAINS + N_SLOTS * N_SLOTS


def samples_to_arrays(samples: Sequence[FaultSample]) -> Tuple[np.ndarray, np.ndarray]:
    vals = np.array([catalog.feature_vector(s.signals) for s in samples], dtype=np.float64)
    labels = np.array([catalog.DOMAIN_INDEX.get(s.actual_domain(), catalog.DOMAIN_INDEX["unknown"])
                       for s in samples], dtype=np.int64)
    return vals, labels


def get_model(name: str, stats: Optional[SufficientStats] = None, seed: int = 42) -> LinearPosteriorModel:
    if name in ("bayes", "", None):
        return NaiveBayes.ref()
    if name == "bayes_gpu":
        return NaiveBayes.gpu()
    if name == "bayes_learned":
        if stats is None:
            raise ValueError("bayes_learned needs sufficient statistics")
        return NaiveBayes.learned(stats, seed=seed)
    if name == "lda":
        if stats is None:
            raise ValueError("lda needs sufficient statistics")
        return LDA.fit(stats)
    raise ValueError(f"unknown model {name!r}")

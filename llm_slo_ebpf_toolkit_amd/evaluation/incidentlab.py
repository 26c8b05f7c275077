"""Incident lab: declarative fault scenarios that are actually executed.

REF ships seven scenario YAMLs (test/incident-lab/scenarios/*.yaml) that no code reads
(SURVEY §2.10 #68). Here each scenario drives the window engine end to end:

    phases (baseline -> fault -> recovery), each N windows of seeded replay traffic
      -> K1 decode / K2 join / K3 posterior (GPU engine, or the CPU oracle engine)
      -> per-phase metrics -> assertions (metric, op, value, phase)

Metrics per phase:
  ``attribution_accuracy``  share of faulted incident groups whose top domain is one of
                            the scenario's expected domains
  ``detected_groups``       faulted groups predicted as an expected domain (count)
  ``false_alarm_rate``      share of healthy groups predicted as an expected domain
  ``enrichment_rate``       spans enriched by >= 1 kernel/GPU signal (REF DebugStats)
  ``<signal>_p95``          p95 of a signal from the decode kernel's histograms
                            (Prometheus ``le`` semantics, histogram_quantile)
  ``ttft_p95_ms``, ``error_rate_mean``  from the synthetic SLI samples of the phase
"""

from __future__ import annotations

import glob
import operator
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np
import yaml

from ..collector.pipeline import SCENARIO_SEQUENCE, SampleMeta, build_synthetic_sample
from ..models.bayes import NaiveBayes
from ..pipeline.replay import SCENARIOS, ReplayConfig, ReplayGenerator
from ..signals import catalog
from .slo import histogram_quantile, mean, quantile

OPS = {">": operator.gt, ">=": operator.ge, "<": operator.lt, "<=": operator.le, "==": operator.eq}
PHASES = ("baseline", "fault", "recovery")
HERE = os.path.dirname(os.path.abspath(__file__))
SCENARIO_DIR = os.path.join(os.path.dirname(os.path.dirname(HERE)), "test", "incident-lab", "scenarios")


@dataclass
class Assertion:
    metric: str
    op: str
    value: float
    phase: str = "fault"


@dataclass
class Scenario:
    name: str
    description: str
    replay_scenario: str
    expected_domains: List[str]
    primary_signal: str
    windows: Dict[str, int]
    seed: int = 42
    events_per_window: int = 20000
    spans_per_window: int = 1024
    services: int = 16
    sample_count: int = 24
    model: str = "learned"             # learned (calibrated online, like the agent) | bayes (REF table)
    calibration_windows: int = 4
    assertions: List[Assertion] = field(default_factory=list)


def load_scenario(path: str) -> Scenario:
    with open(path, "r", encoding="utf-8") as fh:
        d = yaml.safe_load(fh)
    h = d.get("harness") or {}
    exp = d.get("expected") or {}
    sc = Scenario(
        name=d["name"], description=(d.get("description") or "").strip(),
        replay_scenario=d.get("fault", {}).get("replay_scenario", d["name"]),
        expected_domains=list(exp.get("domains") or []), primary_signal=exp.get("primary_signal", ""),
        windows={p: int((h.get("phases") or {}).get(p, {}).get("windows", 1)) for p in PHASES},
        seed=int(h.get("seed", 42)), events_per_window=int(h.get("events_per_window", 20000)),
        spans_per_window=int(h.get("spans_per_window", 1024)), services=int(h.get("services", 16)),
        sample_count=int(h.get("sample_count", 24)), model=str(d.get("model", "learned")),
        calibration_windows=int(h.get("calibration_windows", 4)),
        assertions=[Assertion(a["metric"], a["operator"], float(a["value"]), a.get("phase", "fault"))
                    for a in d.get("assertions") or []])
    if sc.replay_scenario not in SCENARIOS:
        raise ValueError(f"{path}: unknown replay scenario {sc.replay_scenario!r}")
    for a in sc.assertions:
        if a.op not in OPS or a.phase not in PHASES:
            raise ValueError(f"{path}: bad assertion {a}")
    for dom in sc.expected_domains:
        if dom not in catalog.ALL_DOMAINS:
            raise ValueError(f"{path}: unknown domain {dom!r}")
    return sc


def discover(directory: str = SCENARIO_DIR) -> List[str]:
    return sorted(glob.glob(os.path.join(directory, "*.yaml")))


def calibrated_model(sc: Scenario):
    """Learned naive Bayes from labelled calibration windows of every fault (the agent's
    online refit, run ahead of the scenario on an independent seed)."""
    from ..models.bayes import SufficientStats
    from ..pipeline.cpu import CpuWindowEngine

    stats = SufficientStats()
    eng = CpuWindowEngine(NaiveBayes.ref())
    gen = ReplayGenerator(ReplayConfig(scenario="full", n_nodes=2, pods_per_node=16, n_services=sc.services,
                                       events_per_window=sc.events_per_window, spans_per_window=sc.spans_per_window,
                                       seed=sc.seed + 7919, p_fault=0.7))
    for _ in range(max(1, sc.calibration_windows)):
        w = gen.next_window()
        r = eng.run(w.events, w.spans, w.n_groups)
        stats.add(r.feat.astype(np.float64), w.group_labels)
    return NaiveBayes.learned(stats, seed=sc.seed)


class _Engine:
    """GPU window engine when available (device="gpu"/"auto"), else the CPU oracle engine."""

    def __init__(self, sc: Scenario, device: str):
        self.model = calibrated_model(sc) if sc.model == "learned" else NaiveBayes.ref()
        self.gpu = None
        if device in ("gpu", "auto"):
            try:
                import torch

                if torch.cuda.is_available():
                    from ..ops.engine import GpuEngine

                    self.gpu = GpuEngine(sc.events_per_window + 4096, sc.spans_per_window, sc.services)
                    self.gpu.set_model(self.model)
            except Exception:
                if device == "gpu":
                    raise
                self.gpu = None
        if device == "gpu" and self.gpu is None:
            raise RuntimeError("device=gpu but no MI355X / HIP extension available")
        if self.gpu is None:
            from ..pipeline.cpu import CpuWindowEngine

            self.cpu = CpuWindowEngine(self.model)

    def run(self, w):
        """-> (pred[G], hist[16,16], spans_enriched)"""
        if self.gpu is not None:
            out = self.gpu.process(w.events, w.spans, w.n_groups)
            return out.pred, out.hist, out.debug["spans_enriched"]
        r = self.cpu.run(w.events, w.spans, w.n_groups)
        p = self.cpu.unpack(r.packet)
        return r.pred, p["hist"], r.join.debug["spans_enriched"]


def run_scenario(sc: Scenario, device: str = "auto") -> Dict[str, Any]:
    eng = _Engine(sc, device)
    expected = {catalog.DOMAIN_INDEX[d] for d in sc.expected_domains}
    results: Dict[str, Dict[str, float]] = {}
    edges = {s.name: [e for e in s.buckets] for s in catalog.SIGNALS}
    for pi, phase in enumerate(PHASES):
        faulted = phase == "fault"
        cfg = ReplayConfig(scenario=sc.replay_scenario if faulted else "baseline", n_nodes=2, pods_per_node=16,
                           n_services=sc.services, events_per_window=sc.events_per_window,
                           spans_per_window=sc.spans_per_window, seed=sc.seed + 101 * pi,
                           p_fault=1.0 if faulted else 0.0)
        gen = ReplayGenerator(cfg)
        hist = np.zeros((16, 16), dtype=np.int64)
        hit = total_f = false_alarm = total_h = enriched = spans = 0
        for _ in range(sc.windows[phase]):
            w = gen.next_window()
            pred, h, enr = eng.run(w)
            hist += np.asarray(h, dtype=np.int64)
            enriched += int(enr)
            spans += w.n_spans
            for g in range(w.n_groups):
                is_fault = bool(w.group_faults[g])
                p_ok = int(pred[g]) in expected
                if is_fault:
                    total_f += 1
                    hit += p_ok
                else:
                    total_h += 1
                    false_alarm += p_ok
        m: Dict[str, float] = {
            "attribution_accuracy": hit / total_f if total_f else 0.0, "detected_groups": float(hit),
            "false_alarm_rate": false_alarm / total_h if total_h else 0.0,
            "enrichment_rate": enriched / spans if spans else 0.0,
        }
        for s in catalog.SIGNALS:
            cum = np.cumsum(hist[s.slot]).astype(float)
            m[f"{s.name}_p95"] = histogram_quantile(0.95, edges[s.name], list(cum)) if cum[-1] else 0.0
        label = "baseline"
        if faulted:
            label = sc.replay_scenario if sc.replay_scenario in SCENARIO_SEQUENCE else "mixed"
        meta = SampleMeta()
        samples = [build_synthetic_sample(label, i, 0, meta)
                   for i in range(sc.sample_count)]
        m["ttft_p95_ms"] = quantile([x.ttft_ms for x in samples], 0.95)
        m["error_rate_mean"] = mean([x.error_rate for x in samples])
        results[phase] = m
    checks = []
    for a in sc.assertions:
        got = results[a.phase].get(a.metric)
        ok = got is not None and OPS[a.op](got, a.value)
        checks.append({"metric": a.metric, "op": a.op, "value": a.value, "phase": a.phase, "actual": got,
                       "pass": bool(ok)})
    return {"scenario": sc.name, "engine": "gpu" if eng.gpu is not None else "cpu", "phases": results,
            "assertions": checks, "pass": all(c["pass"] for c in checks)}


def run_all(directory: str = SCENARIO_DIR, device: str = "auto", only: Optional[List[str]] = None):
    out = []
    for p in discover(directory):
        sc = load_scenario(p)
        if only and sc.name not in only:
            continue
        out.append(run_scenario(sc, device))
    return out

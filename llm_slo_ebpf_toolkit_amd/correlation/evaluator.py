"""Labelled-pair correlation evaluation and the P/R gate.

REF pkg/correlation/evaluator.go:13-196: precision/recall/F1 over labelled
(span, signal, expected_match, expected_tier) pairs at a window/threshold, tier
accuracy over true positives with an expected tier, mean confidence of predicted
positives, and a min-precision / min-recall gate.
"""

from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from ..utils.timeutil import MS, format_rfc3339_ns, now_ns
from .match import (DEFAULT_ENRICHMENT_THRESHOLD, DEFAULT_WINDOW_NS, SignalRef, SpanRef, match)


@dataclass
class LabeledPair:
    case_id: str
    span: SpanRef
    signal: SignalRef
    expected_match: bool
    expected_tier: str = ""

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "LabeledPair":
        return cls(d.get("case_id", ""), SpanRef.from_dict(d.get("span") or {}),
                   SignalRef.from_dict(d.get("signal") or {}), bool(d.get("expected_match", False)),
                   d.get("expected_tier", "") or "")


@dataclass
class Prediction:
    case_id: str
    expected: bool
    predicted: bool
    confidence: float
    tier: str
    correct: bool
    signal: str
    expected_tier: str = ""


@dataclass
class EvalReport:
    generated_at: int = 0
    sample_size: int = 0
    true_positive: int = 0
    false_positive: int = 0
    false_negative: int = 0
    true_negative: int = 0
    precision: float = 0.0
    recall: float = 0.0
    f1: float = 0.0
    tier_accuracy: float = 0.0
    mean_confidence: float = 0.0
    window_ms: int = 0
    threshold: float = 0.0
    min_precision_required: float = 0.0
    min_recall_required: float = 0.0
    passed_gate: bool = False

    def to_dict(self) -> Dict[str, Any]:
        out = {
            "generated_at": format_rfc3339_ns(self.generated_at), "sample_size": self.sample_size,
            "true_positive": self.true_positive, "false_positive": self.false_positive,
            "false_negative": self.false_negative, "true_negative": self.true_negative,
            "precision": self.precision, "recall": self.recall, "f1": self.f1,
            "tier_accuracy": self.tier_accuracy, "mean_confidence": self.mean_confidence,
            "window_ms": self.window_ms, "threshold": self.threshold,
        }
        if self.min_precision_required:
            out["min_precision_required"] = self.min_precision_required
        if self.min_recall_required:
            out["min_recall_required"] = self.min_recall_required
        if self.passed_gate:
            out["passed_gate"] = True
        return out


@dataclass
class GateResult:
    passed: bool
    message: str


def load_labeled_pairs(path: str) -> List[LabeledPair]:
    pairs: List[LabeledPair] = []
    with open(path, "r", encoding="utf-8") as fh:
        for line in fh:
            line = line.strip()
            if not line:
                continue
            try:
                pairs.append(LabeledPair.from_dict(json.loads(line)))
            except (ValueError, KeyError) as exc:
                raise ValueError(f"parse labeled pair: {exc}") from exc
    if not pairs:
        raise ValueError(f"no labeled pairs loaded from {path}")
    return pairs


def _safe_div(num: int, den: int) -> float:
    return 0.0 if den == 0 else num / den


def evaluate_labeled_pairs(pairs: List[LabeledPair], window_ns: int = DEFAULT_WINDOW_NS,
                           threshold: float = DEFAULT_ENRICHMENT_THRESHOLD
                           ) -> Tuple[EvalReport, List[Prediction]]:
    if window_ns <= 0:
        window_ns = DEFAULT_WINDOW_NS
    if threshold <= 0:
        threshold = DEFAULT_ENRICHMENT_THRESHOLD
    rep = EvalReport(generated_at=now_ns(), sample_size=len(pairs), window_ms=window_ns // MS,
                     threshold=threshold)
    preds: List[Prediction] = []
    tier_correct = tier_cmp = 0
    conf_sum = 0.0
    conf_n = 0
    for p in pairs:
        dec = match(p.span, p.signal, window_ns)
        predicted = dec.matched and dec.confidence >= threshold
        preds.append(Prediction(p.case_id, p.expected_match, predicted, dec.confidence, dec.tier,
                                predicted == p.expected_match, p.signal.signal, p.expected_tier))
        if predicted:
            conf_sum += dec.confidence
            conf_n += 1
        if p.expected_match and predicted:
            rep.true_positive += 1
        elif not p.expected_match and predicted:
            rep.false_positive += 1
        elif p.expected_match and not predicted:
            rep.false_negative += 1
        else:
            rep.true_negative += 1
        if p.expected_match and p.expected_tier and predicted:
            tier_cmp += 1
            if p.expected_tier == dec.tier:
                tier_correct += 1
    rep.precision = _safe_div(rep.true_positive, rep.true_positive + rep.false_positive)
    rep.recall = _safe_div(rep.true_positive, rep.true_positive + rep.false_negative)
    if rep.precision + rep.recall > 0:
        rep.f1 = 2 * (rep.precision * rep.recall) / (rep.precision + rep.recall)
    if tier_cmp:
        rep.tier_accuracy = tier_correct / tier_cmp
    if conf_n:
        rep.mean_confidence = conf_sum / conf_n
    return rep, preds


def evaluate_gate(report: EvalReport, min_precision: float, min_recall: float) -> GateResult:
    if report.precision < min_precision:
        return GateResult(False, f"precision gate failed: got {report.precision:.4f} required {min_precision:.4f}")
    if report.recall < min_recall:
        return GateResult(False, f"recall gate failed: got {report.recall:.4f} required {min_recall:.4f}")
    return GateResult(True, "correlation gate passed")

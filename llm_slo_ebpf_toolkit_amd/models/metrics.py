"""Attribution dispatch and evaluation metrics.

REF pkg/attribution/pipeline.go:13-185: mode dispatch (bayes default, unknown -> bayes),
confusion matrix keyed by (actual, predicted), Accuracy, PartialAccuracy,
CoverageAccuracy. NEW adds per-class precision/recall/F1 and macro-F1 -- the
north-star metric REF's report template asks for (docs/benchmarks/reports/template.md:20-28)
but never computes.
"""

from __future__ import annotations

from collections import Counter
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from ..contracts.types import IncidentAttribution
from .bayes import LinearPosteriorModel, NaiveBayes, SufficientStats, get_model
from .sample import FaultSample, build_attribution

MODE_BAYES = "bayes"
MODE_RULE = "rule"
MODES = ("bayes", "bayes_gpu", "bayes_learned", "lda", "rule")


def normalize_mode(mode: str) -> str:
    m = (mode or "").strip().lower()
    return m if m in MODES else MODE_BAYES


def build_attributions(samples: Sequence[FaultSample], mode: str = MODE_BAYES,
                       model: Optional[LinearPosteriorModel] = None,
                       stats: Optional[SufficientStats] = None) -> List[IncidentAttribution]:
    m = normalize_mode(mode)
    if m == MODE_RULE:
        return [build_attribution(s) for s in samples]
    if model is None:
        model = get_model(m, stats)
    return [model.attribute_sample(s) for s in samples]


def confusion_matrix(samples: Sequence[FaultSample],
                     predictions: Sequence[IncidentAttribution]) -> Dict[Tuple[str, str], int]:
    out: Counter = Counter()
    for s, p in zip(samples, predictions):
        out[(s.actual_domain(), p.predicted_fault_domain)] += 1
    return dict(out)


def accuracy(samples, predictions) -> float:
    if not predictions:
        return 0.0
    ok = sum(1 for s, p in zip(samples, predictions) if s.actual_domain() == p.predicted_fault_domain)
    return ok / len(predictions)


def partial_accuracy(samples, predictions) -> float:
    if not predictions:
        return 0.0
    ok = sum(1 for s, p in zip(samples, predictions) if p.predicted_fault_domain in s.expected_set())
    return ok / len(predictions)


def coverage_accuracy(samples, predictions, threshold: float = 0.10) -> float:
    if not predictions:
        return 0.0
    total = 0.0
    n = 0
    for s, p in zip(samples, predictions):
        exp = s.expected_set()
        hyp = {h.domain for h in p.fault_hypotheses if h.posterior >= threshold}
        hyp.add(p.predicted_fault_domain)
        total += sum(1 for d in exp if d in hyp) / len(exp)
        n += 1
    return total / n if n else 0.0


@dataclass
class ClassReport:
    label: str
    precision: float
    recall: float
    f1: float
    support: int
    predicted: int


def per_class_report(actual: Iterable[str], predicted: Iterable[str],
                     labels: Optional[Sequence[str]] = None) -> List[ClassReport]:
    actual = list(actual)
    predicted = list(predicted)
    if labels is None:
        labels = sorted(set(actual))
    out = []
    for lab in labels:
        tp = sum(1 for a, p in zip(actual, predicted) if a == lab and p == lab)
        sup = sum(1 for a in actual if a == lab)
        npred = sum(1 for p in predicted if p == lab)
        prec = tp / npred if npred else 0.0
        rec = tp / sup if sup else 0.0
        f1 = 2 * prec * rec / (prec + rec) if prec + rec > 0 else 0.0
        out.append(ClassReport(lab, prec, rec, f1, sup, npred))
    return out


def macro_f1(actual: Iterable[str], predicted: Iterable[str], include_predicted: bool = False) -> float:
    """Macro-F1 over ground-truth classes (default) or ground-truth U predicted classes."""
    actual = list(actual)
    predicted = list(predicted)
    labels = set(actual)
    if include_predicted:
        labels |= set(predicted)
    rep = per_class_report(actual, predicted, sorted(labels))
    return sum(r.f1 for r in rep) / len(rep) if rep else 0.0


def confusion_from_arrays(actual_idx, pred_idx, n_classes: int):
    import numpy as np

    m = np.zeros((n_classes, n_classes), dtype=np.int64)
    np.add.at(m, (np.asarray(actual_idx), np.asarray(pred_idx)), 1)
    return m


def confusion_report(conf, labels: Sequence[str], abstain_label: str = "unknown") -> dict:
    """conf[actual, predicted] -> per-class precision / recall / F1 / support (classes with
    support or predictions), the one-vs-rest false-positive and false-negative rates averaged
    over those classes (REF harness definitions, evaluation/benchmark.py), and the abstain rate:
    the share of faulted incidents (ground truth other than ``abstain_label``) predicted
    ``abstain_label`` (REF target <= 15 %; a no-fault incident predicted so is correct, not an
    abstention)."""
    import numpy as np

    conf = np.asarray(conf, dtype=np.float64)
    n = conf.sum()
    tp = np.diag(conf)
    sup, npred = conf.sum(axis=1), conf.sum(axis=0)
    per, fprs, fnrs = [], [], []
    for i, lab in enumerate(labels):
        if sup[i] == 0 and npred[i] == 0:
            continue
        prec = tp[i] / npred[i] if npred[i] else 0.0
        rec = tp[i] / sup[i] if sup[i] else 0.0
        f1 = 2 * prec * rec / (prec + rec) if prec + rec > 0 else 0.0
        per.append({"label": lab, "precision": round(float(prec), 4), "recall": round(float(rec), 4),
                    "f1": round(float(f1), 4), "support": int(sup[i])})
        fp, fn = npred[i] - tp[i], sup[i] - tp[i]
        tn = n - tp[i] - fp - fn
        if tp[i] + fn:
            fnrs.append(fn / (tp[i] + fn))
        if fp + tn:
            fprs.append(fp / (fp + tn))
    ab = list(labels).index(abstain_label) if abstain_label in labels else -1
    return {"per_class": per,
            "false_positive_rate": round(float(np.mean(fprs)), 4) if fprs else 0.0,
            "false_negative_rate": round(float(np.mean(fnrs)), 4) if fnrs else 0.0,
            "abstain_rate": round(float((conf[:, ab].sum() - conf[ab, ab]) / (n - sup[ab])), 4)
            if ab >= 0 and n > sup[ab] else 0.0}


def macro_f1_from_confusion(conf, present_only: bool = True) -> float:
    """conf[actual, predicted]; macro over classes with support (ground-truth classes)."""
    import numpy as np

    conf = np.asarray(conf, dtype=np.float64)
    tp = np.diag(conf)
    sup = conf.sum(axis=1)
    npred = conf.sum(axis=0)
    prec = np.divide(tp, npred, out=np.zeros_like(tp), where=npred > 0)
    rec = np.divide(tp, sup, out=np.zeros_like(tp), where=sup > 0)
    f1 = np.divide(2 * prec * rec, prec + rec, out=np.zeros_like(tp), where=(prec + rec) > 0)
    mask = sup > 0 if present_only else (sup + npred) > 0
    return float(f1[mask].mean()) if mask.any() else 0.0

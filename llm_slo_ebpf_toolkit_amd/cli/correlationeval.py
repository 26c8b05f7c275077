"""`correlationeval`: labelled span/signal pairs -> P/R/F1 report + gate
(REF cmd/correlationeval/main.go:24-143). Exit 1 when the gate fails."""

from __future__ import annotations

import csv
import json
import os
import sys
from typing import List, Optional

from ..correlation.evaluator import evaluate_gate, evaluate_labeled_pairs, load_labeled_pairs
from ..utils.timeutil import MS
from ._common import GoFlags, eprint, ensure_parent, is_version_request, print_version, project_root

DEFAULT_INPUT = os.path.join("tests", "fixtures", "ref_labeled_pairs.jsonl")


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    p = GoFlags("correlationeval", "evaluate span/signal correlation on labelled pairs")
    p.flag("input", DEFAULT_INPUT, "labeled correlation dataset JSONL")
    p.flag("out", os.path.join("artifacts", "correlation", "eval_summary.json"), "summary JSON output path")
    p.flag("predictions-out", os.path.join("artifacts", "correlation", "predictions.csv"),
           "predictions CSV output path")
    p.flag("window-ms", 2000, "correlation window in milliseconds")
    p.flag("threshold", 0.7, "minimum confidence to count as positive correlation")
    p.flag("min-precision", 0.90, "minimum precision gate")
    p.flag("min-recall", 0.85, "minimum recall gate")
    a = p.parse_args(argv)
    path = a.input
    if path == DEFAULT_INPUT and not os.path.exists(path):
        path = os.path.join(project_root(), DEFAULT_INPUT)
    try:
        pairs = load_labeled_pairs(path)
    except Exception as exc:  # noqa: BLE001
        eprint(f"load labeled dataset failed: {exc}")
        return 1
    report, preds = evaluate_labeled_pairs(pairs, a.window_ms * MS, a.threshold)
    gate = evaluate_gate(report, a.min_precision, a.min_recall)
    report.min_precision_required = a.min_precision
    report.min_recall_required = a.min_recall
    report.passed_gate = gate.passed
    ensure_parent(a.out)
    with open(a.out, "w", encoding="utf-8") as fh:
        json.dump(report.to_dict(), fh, indent=2)
    ensure_parent(a.predictions_out)
    with open(a.predictions_out, "w", newline="", encoding="utf-8") as fh:
        w = csv.writer(fh)
        w.writerow(["case_id", "signal", "expected_match", "predicted_match", "confidence", "tier", "expected_tier",
                    "is_correct"])
        for pr in preds:
            w.writerow([pr.case_id, pr.signal, str(pr.expected).lower(), str(pr.predicted).lower(),
                        f"{pr.confidence:.4f}", pr.tier, pr.expected_tier, str(pr.correct).lower()])
    print(f"correlation gate: {'PASS' if gate.passed else 'FAIL'} | precision={report.precision:.4f} "
          f"recall={report.recall:.4f} f1={report.f1:.4f} sample_size={report.sample_size}")
    print(f"summary: {a.out}")
    print(f"predictions: {a.predictions_out}")
    if not gate.passed:
        eprint(gate.message)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""`attributor`: FaultSample JSONL -> schema-valid IncidentAttribution JSONL
(REF cmd/attributor/main.go:37-327).

Flags match REF (--input --out --summary-out --confusion-out --schema --config
--attribution-mode --webhook-*). Additive: ``--attribution-mode`` also accepts
``bayes_learned`` / ``lda`` (models/bayes.py), and ``--device gpu`` scores the batch with
the MFMA posterior kernel (ops/csrc/posterior.hip) instead of numpy; the summary gains
macro-F1 and per-class P/R/F1, which REF's report template asks for.
"""

from __future__ import annotations

import csv
import json
import os
import sys
from collections import Counter
from typing import List, Optional

from ..contracts import config as toolkitcfg
from ..contracts import validator
from ..export.webhook import WebhookExporter, parse_format
from ..models import metrics
from ..models.sample import FaultSample, load_samples_jsonl
from ..utils.timeutil import format_rfc3339_s, now_ns
from ._common import GoFlags, eprint, ensure_parent, is_version_request, jsonl_line, open_output, print_version


def default_sample() -> FaultSample:
    return FaultSample(incident_id="inc-1", timestamp=now_ns(), cluster="local", namespace="default",
                       service="chat", fault_label="provider_throttle", expected_domain="provider_throttle",
                       confidence=0.9, burn_rate=2.0, window_minutes=5, request_id="req-1", trace_id="trace-1")


def write_confusion_csv(path: str, samples, predictions) -> None:
    ensure_parent(path)
    m = metrics.confusion_matrix(samples, predictions)
    with open(path, "w", newline="", encoding="utf-8") as fh:
        w = csv.writer(fh)
        w.writerow(["actual", "predicted", "count"])
        for (act, pred) in sorted(m):
            w.writerow([act, pred, m[(act, pred)]])


def gpu_attributions(samples: List[FaultSample], mode: str):
    """Score the batch with the HIP posterior kernel; returns IncidentAttributions."""
    import numpy as np
    import torch

    from ..models.bayes import get_model, samples_to_arrays
    from ..ops.engine import GpuEngine

    model = get_model(metrics.normalize_mode(mode))
    vals, _ = samples_to_arrays(samples)
    eng = GpuEngine(8, 8, max(1, len(samples)))
    eng.set_model(model)
    e = eng.eng
    e.feat[: len(samples)].copy_(torch.from_numpy(vals.astype(np.float32)))
    e.counts[:4].copy_(torch.tensor([0, 0, len(samples), 0], dtype=torch.int32))
    e.bind_io(e.counts, e.labels, e.packet)
    e.posterior(False)
    post = e.post[: len(samples)].cpu().numpy()
    bits = e.evbits[: len(samples)].cpu().numpy().view(np.uint32)
    return [model.attribution_from_posterior(s, post[i], bits[i]) for i, s in enumerate(samples)]


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    cfg_path = toolkitcfg.resolve_config_path(argv, os.path.join("config", "toolkit.yaml"))
    try:
        cfg = toolkitcfg.load(cfg_path)
    except Exception as exc:  # noqa: BLE001 - REF logs and continues with defaults
        eprint(f"warning: failed to load config {cfg_path}: {exc} (using defaults)")
        cfg = toolkitcfg.default()
    p = GoFlags("attributor", "fault samples -> incident attributions")
    p.flag("input", "", "JSONL file containing fault samples")
    p.flag("out", "-", "Attribution JSONL output path ('-' for stdout)")
    p.flag("summary-out", "", "Optional JSON summary output path")
    p.flag("confusion-out", "", "Optional confusion matrix CSV output path")
    p.flag("schema", os.path.join("docs", "contracts", "v1", "incident-attribution.schema.json"),
           "Incident attribution JSON schema path")
    p.flag("config", cfg_path, "toolkit config path")
    p.flag("attribution-mode", metrics.MODE_BAYES, "attribution mode: bayes|rule|bayes_learned|lda")
    p.flag("webhook-enabled", bool(cfg.webhook.enabled), "enable webhook delivery")
    p.flag("webhook-url", cfg.webhook.url, "webhook endpoint URL")
    p.flag("webhook-secret", cfg.webhook.secret, "webhook secret for HMAC signature")
    p.flag("webhook-format", cfg.webhook.format, "webhook format: generic|pagerduty|opsgenie")
    p.flag("webhook-timeout-ms", int(cfg.webhook.timeout_ms), "webhook timeout in milliseconds")
    p.flag("webhook-strict", False, "fail command when webhook delivery fails")
    p.flag("device", "cpu", "posterior device: cpu|gpu (MFMA posterior kernel)", choices=("cpu", "gpu"))
    a = p.parse_args(argv)
    if a.config.strip() != cfg_path.strip():
        try:
            cfg = toolkitcfg.load(a.config)
        except Exception as exc:  # noqa: BLE001
            eprint(f"warning: failed to load config {a.config}: {exc} (continuing with previous defaults)")

    try:
        samples = load_samples_jsonl(a.input) if a.input else [default_sample()]
    except Exception as exc:  # noqa: BLE001
        eprint(f"failed to load samples: {exc}")
        return 1
    mode = a.attribution_mode
    if a.device == "gpu" and metrics.normalize_mode(mode) != metrics.MODE_RULE:
        preds = gpu_attributions(samples, mode)
    else:
        preds = metrics.build_attributions(samples, mode)
    schema = a.schema if os.path.exists(a.schema) else "incident-attribution"
    for pr in preds:
        try:
            validator.validate(schema, pr)
        except validator.ValidationError as exc:
            eprint(f"schema validation failed: {exc}")
            return 1
    out, close = open_output(a.out)
    try:
        for pr in preds:
            out.write(jsonl_line(pr))
    finally:
        close()
    if a.confusion_out:
        write_confusion_csv(a.confusion_out, samples, preds)

    errs = 0
    if a.webhook_enabled:
        if not a.webhook_url.strip():
            msg = "webhook delivery enabled but webhook-url is empty"
            if a.webhook_strict:
                eprint(msg)
                return 1
            eprint(f"warning: {msg}")
        else:
            try:
                fmt = parse_format(a.webhook_format)
            except ValueError as exc:
                eprint(f"invalid webhook-format: {exc}")
                return 2
            exp = WebhookExporter(a.webhook_url, a.webhook_secret, fmt, a.webhook_timeout_ms)
            for pr in preds:
                try:
                    exp.send(pr)
                except Exception as exc:  # noqa: BLE001
                    errs += 1
                    if a.webhook_strict:
                        eprint(f"webhook delivery failed: {exc}")
                        return 1
                    eprint(f"warning: webhook delivery failed for incident {pr.incident_id}: {exc}")

    if a.summary_out:
        actual = [s.actual_domain() for s in samples]
        predicted = [p_.predicted_fault_domain for p_ in preds]
        single = [(x, y) for s, x, y in zip(samples, actual, predicted) if s.expected_domain]
        summary = {
            "generated_at": format_rfc3339_s(now_ns()), "total_samples": len(samples),
            "accuracy": metrics.accuracy(samples, preds), "attribution_mode": mode,
            "predicted_domain_counts": dict(Counter(predicted)), "webhook_enabled": bool(a.webhook_enabled),
            "webhook_strict": bool(a.webhook_strict), "webhook_delivery_errors": errs,
            "partial_accuracy": metrics.partial_accuracy(samples, preds),
            "coverage_accuracy": metrics.coverage_accuracy(samples, preds),
            "single_fault_macro_f1": metrics.macro_f1([x for x, _ in single], [y for _, y in single]) if single else 0.0,
            "per_class": [c.__dict__ for c in metrics.per_class_report([x for x, _ in single],
                                                                      [y for _, y in single])] if single else [],
            "device": a.device,
        }
        if a.input:
            summary["input_path"] = a.input
        if a.out:
            summary["output_path"] = a.out
        if a.confusion_out:
            summary["confusion_path"] = a.confusion_out
        ensure_parent(a.summary_out)
        with open(a.summary_out, "w", encoding="utf-8") as fh:
            json.dump(summary, fh, indent=2)
    return 0


if __name__ == "__main__":
    sys.exit(main())

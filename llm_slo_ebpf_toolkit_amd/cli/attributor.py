"""`attributor`: FaultSample JSONL -> schema-valid IncidentAttribution JSONL
(REF cmd/attributor/main.go:37-327).

Flags match REF (--input --out --summary-out --confusion-out --schema --config
--attribution-mode --webhook-*). Additive:

* ``--device gpu`` scores the batch with the window engine's MFMA posterior kernel
  (ops/csrc/posterior.hip through WindowEngine.score) instead of numpy;
* ``--model-path FILE`` scores with a trained model file (models/train.py), the file the agent
  loads with the same flag;
* ``--train --out FILE`` trains that file: from ``--input`` (labelled FaultSamples with signals;
  a multi-fault row's mass spread over its expected domains) or, without it, from the fixed
  fault-replay training set (single and compound faults of REF's profiles) whose incident
  features the window engine's CPU oracle computes from the records; calibrated by a held-out
  temperature. ``--summary-out`` then reports the fit and REF's 55-row scores of the new model.

The summary gains macro-F1, per-class P/R/F1, partial and coverage accuracy.
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

# the model `attributor --train` shipped with the toolkit (agent --model-path in the DaemonSet)
SHIPPED_MODEL = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                             "config", "models", "mislo-learned.safetensors")


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


def gpu_attributions(samples: List[FaultSample], model):
    """Score the batch with the window engine's posterior kernel (WindowEngine.score, the
    agent's engine); returns IncidentAttributions."""
    import numpy as np

    from ..models.bayes import samples_to_arrays
    from ..ops import load_agent
    from ..ops.engine import model_bytes

    vals, _ = samples_to_arrays(samples)
    eng = load_agent().WindowEngine(sig_cap=1024, span_cap=64, group_cap=64, user_cap=64, n_buffers=2,
                                    max_ahead=2, use_graphs=False, device_refit=False)
    try:
        eng.set_model_bytes(model_bytes(model))
        r = eng.score(np.ascontiguousarray(vals, dtype=np.float32), None)
    finally:
        eng.close()
    post, bits = r["post"], r["evbits"].view(np.uint32)
    return [model.attribution_from_posterior(s, post[i], bits[i]) for i, s in enumerate(samples)]


def train_main(a) -> int:
    """attributor --train: fit, calibrate and write a model file (agent --model-path)."""
    import numpy as np

    from ..models import train as mtrain
    from ..models.bayes import label_code
    from ..signals import catalog

    cfg = mtrain.TrainConfig(windows=a.train_windows, events_per_window=a.train_events,
                             spans_per_window=a.train_spans, seed=a.seed, init=a.train_prior)
    if a.input:
        rows = [s for s in load_samples_jsonl(a.input) if s.signals and s.expected_set()]
        if not rows:
            eprint(f"{a.input}: no labelled rows with signals")
            return 1
        feats = np.array([catalog.feature_vector(s.signals) for s in rows], dtype=np.float32)
        codes = np.array([label_code(catalog.DOMAIN_INDEX[s.expected_set()[0]],
                                     [catalog.DOMAIN_INDEX[d] for d in s.expected_set()]) for s in rows], np.int32)
        tm = mtrain.fit(feats, codes, np.arange(len(rows)), cfg)
        tm.meta.update({"engine": "labelled-samples", "input": a.input, "config": cfg.__dict__})
    else:
        tm = mtrain.train_cpu(cfg)
        tm.meta["heldout"] = mtrain.heldout_report(tm.model, cfg)
    fx = a.ref55 if a.ref55 and os.path.exists(a.ref55) else ""
    if fx:
        tm.meta["ref55"] = mtrain.ref55_report(fx, mtrain.host_scorer(tm.model))
    if a.out in ("", "-"):
        eprint("--train needs --out FILE")
        return 2
    mtrain.save_model(a.out, tm)
    if a.summary_out:
        ensure_parent(a.summary_out)
        with open(a.summary_out, "w", encoding="utf-8") as fh:
            json.dump({"model": a.out, **tm.meta}, fh, indent=2, default=str)
    eprint(f"trained {a.out}: T = {tm.temperature:.3f}, active domains {tm.meta.get('active_domains')}")
    return 0


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
    p.flag("model-path", "", "score with a trained model file (attributor --train / the agent's --model-path)")
    p.flag("train", False, "train a model file (--out) from --input labelled samples or the fault-replay set")
    p.flag("train-windows", 48, "--train without --input: fault-replay training windows")
    p.flag("train-events", 16384, "--train: events per training window")
    p.flag("train-spans", 1024, "--train: spans per training window")
    p.flag("seed", 42, "--train: replay and random-init seed")
    p.flag("train-prior", "expert", "--train: the likelihoods' Beta prior, expert (REF's table) or random (seeded)",
           choices=("expert", "random"))
    p.flag("ref55", os.path.join("tests", "fixtures", "ref_multi_fault_samples.jsonl"),
           "--train: REF's 55 labelled rows to score the new model on (skipped if absent)")
    a = p.parse_args(argv)
    if a.train:
        return train_main(a)
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
    model = None
    if not a.model_path and metrics.normalize_mode(mode) == "bayes_learned":
        # the shipped trained model (config/models/mislo-learned.safetensors) unless another is given
        a.model_path = SHIPPED_MODEL
    if a.model_path:
        from ..models.train import load_model

        try:
            model = load_model(a.model_path)[0]
        except (OSError, ValueError) as exc:
            eprint(f"failed to load model: {exc}")
            return 1
        mode = f"model:{os.path.basename(a.model_path)}"
    elif metrics.normalize_mode(mode) != metrics.MODE_RULE:
        from ..models.bayes import get_model

        if metrics.normalize_mode(mode) == "lda":
            eprint(f"attribution-mode {mode} is learned: give --model-path (attributor --train writes one)")
            return 1
        model = get_model(metrics.normalize_mode(mode))
    if model is not None and a.device == "gpu":
        preds = gpu_attributions(samples, model)
    elif model is not None:
        preds = [model.attribute_sample(s) for s in samples]
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

"""M5 release gates on synthetic run directories (REF pkg/releasegate/gate_test.go:21-499)."""

import csv
import json
import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector.pipeline import RawSample
from llm_slo_ebpf_toolkit_amd.evaluation import releasegate as rg
from llm_slo_ebpf_toolkit_amd.utils.timeutil import SECOND

SCEN = ["dns_latency"]


def write_run(root, scenario, run, ttft, tps, errs, cpu_rows=(("node-a", 2.0),)):
    d = os.path.join(root, scenario, f"run-{run}")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "raw_samples.jsonl"), "w") as fh:
        for i, (t, p, e) in enumerate(zip(ttft, tps, errs)):
            s = RawSample(timestamp=(i + 1) * SECOND, cluster="local", namespace="default", workload="w", service="s",
                          node="n", request_id=f"run-{run}-req-{i}", trace_id=f"run-{run}-trace-{i}", ttft_ms=t,
                          request_latency_ms=2 * t, token_throughput_tps=p, error_rate=e, fault_label=scenario)
            fh.write(json.dumps(s.to_dict()) + "\n")
    with open(os.path.join(d, "collector_overhead.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["timestamp", "node", "collector_cpu_pct", "collector_memory_mb", "events_per_second",
                    "dropped_events"])
        for i, (node, cpu) in enumerate(cpu_rows):
            w.writerow([f"1970-01-01T00:00:0{i + 1}Z", node, f"{cpu:.3f}", "120", "900", "0"])


def series(n, base, spread, seed):
    rng = np.random.default_rng(seed)
    return list(base + rng.uniform(-spread, spread, n))


def populate(tmp, cand_ttft=200.0, base_ttft=200.0, n=40, runs=3, cand_cpu=2.0, tok_spread=0.5):
    cand = str(tmp / "cand")
    base = str(tmp / "cand" / "baseline")
    for r in range(1, runs + 1):
        write_run(cand, SCEN[0], r, series(n, cand_ttft, 5, r), series(n, 30, tok_spread, 100 + r),
                  [0.01] * n, [("node-a", cand_cpu), ("node-b", cand_cpu * 0.9)])
        write_run(base, SCEN[0], r, series(n, base_ttft, 5, 50 + r), series(n, 30, 0.5, 200 + r), [0.01] * n)
    return cand, base


def cfg(cand, base, **kw):
    c = rg.Config(candidate_root=cand, baseline_root=base, scenarios=list(SCEN))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_evaluate_pass(tmp_path):
    cand, base = populate(tmp_path)
    s = rg.evaluate(cfg(cand, base))
    assert s["pass"], s.get("failures")
    assert s["overhead"]["max_node_p95_node"] == "node-a"
    md = rg.render_markdown(s)
    assert "# M5 Gate Summary" in md and "`PASS`" in md


def test_overhead_fail(tmp_path):
    cand, base = populate(tmp_path, cand_cpu=4.2)
    s = rg.evaluate(cfg(cand, base))
    assert not s["pass"] and not s["overhead"]["pass"]
    assert any(f.startswith("B5 overhead gate failed") for f in s["failures"])


def test_variance_token_fail(tmp_path):
    cand = str(tmp_path / "cand")
    base = str(tmp_path / "cand" / "baseline")
    for r, tok in zip((1, 2, 3), (10.0, 30.0, 50.0)):
        write_run(cand, SCEN[0], r, series(40, 200, 5, r), [tok] * 40, [0.01] * 40)
        write_run(base, SCEN[0], r, series(40, 200, 5, 50 + r), [30.0] * 40, [0.01] * 40)
    s = rg.evaluate(cfg(cand, base))
    assert not s["variance"]["pass"]
    assert "tokens variance" in s["variance"]["scenarios"][0]["failure_reason"]


def test_significance_fail(tmp_path):
    cand, base = populate(tmp_path, cand_ttft=260.0, base_ttft=200.0)
    s = rg.evaluate(cfg(cand, base))
    sig = s["significance"]["scenarios"][0]
    assert not s["significance"]["pass"] and sig["ttft_regression_pct"] > 5
    assert sig["mann_whitney_p_value"] < 0.05 and sig["bootstrap_delta_ci95"][0] > 0
    assert abs(sig["cliffs_delta"]) >= 0.147


def test_significance_min_samples_fail(tmp_path):
    cand, base = populate(tmp_path, n=8)
    s = rg.evaluate(cfg(cand, base))
    sig = s["significance"]["scenarios"][0]
    assert not sig["pass"] and "insufficient samples" in sig["failure_reason"]


def test_baseline_manifest_required(tmp_path):
    cand, base = populate(tmp_path)
    s = rg.evaluate(cfg(cand, base, require_baseline_manifest=True))
    assert not s["baseline"]["pass"] and "manifest missing" in s["baseline"]["failure_reason"]


def test_baseline_same_source_passes_gracefully(tmp_path):
    cand, base = populate(tmp_path)
    with open(os.path.join(base, "manifest.json"), "w") as fh:
        json.dump({"source_ref": "v0.3.0", "source_commit": "abc123"}, fh)
    s = rg.evaluate(cfg(cand, base, require_baseline_manifest=True, candidate_commit="abc123"))
    assert s["baseline"]["pass"] and s["baseline"]["same_source"]
    assert "skipping regression comparison" in s["baseline"]["failure_reason"]


def test_missing_runs_raises(tmp_path):
    with pytest.raises(ValueError):
        rg.evaluate(cfg(str(tmp_path / "nothing"), str(tmp_path / "nothing2")))

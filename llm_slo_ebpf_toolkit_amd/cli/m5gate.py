"""`m5gate`: M5 release gates -> JSON + Markdown; exit 1 on fail (REF cmd/m5gate/main.go:22-239).

Additive: ``--device gpu`` runs the E3 statistics through the K5 HIP kernels
(ops/gatestats.py); results are identical to the CPU path by construction.
"""

from __future__ import annotations

import json
import os
import sys
from typing import List, Optional

from ..evaluation import releasegate
from ._common import GoFlags, eprint, ensure_parent, is_version_request, print_version, split_csv


def _first(*vals: str) -> str:
    for v in vals:
        if v and v.strip():
            return v.strip()
    return ""


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    wb = os.path.join("artifacts", "weekly-benchmark")
    p = GoFlags("m5gate", "evaluate M5 release gates")
    p.flag("candidate-root", wb, "candidate benchmark root")
    p.flag("baseline-root", os.path.join(wb, "baseline"), "baseline benchmark root")
    p.flag("baseline-manifest", os.path.join(wb, "baseline", "manifest.json"), "baseline manifest path")
    p.flag("candidate-ref", _first(os.environ.get("GITHUB_REF_NAME", ""), os.environ.get("GITHUB_REF", ""), "local"),
           "candidate git ref")
    p.flag("candidate-commit", _first(os.environ.get("GITHUB_SHA", ""), "local"), "candidate git commit")
    p.flag("require-baseline-manifest", False, "require baseline manifest and source independence check")
    p.flag("scenarios", ",".join(releasegate.DEFAULT_SCENARIOS), "comma-separated scenario list")
    p.flag("max-overhead-pct", 3.0, "B5 max collector CPU overhead percent")
    p.flag("max-variance-pct", 10.0, "D3 max rerun variance percent")
    p.flag("min-runs", 3, "D3 minimum reruns per scenario")
    p.flag("ttft-regression-pct", 5.0, "E3 max p95 TTFT regression percent")
    p.flag("alpha", 0.05, "E3 significance alpha")
    p.flag("bootstrap-iters", 1000, "E3 bootstrap iterations")
    p.flag("seed", 42, "bootstrap RNG seed")
    p.flag("min-samples", 30, "E3 minimum samples required per scenario for both candidate and baseline")
    p.flag("min-cliffs-delta", 0.147, "E3 minimum absolute Cliff's delta for a practical regression")
    p.flag("out-json", os.path.join(wb, "m5_gate_summary.json"), "output JSON summary path")
    p.flag("out-md", os.path.join(wb, "m5_gate_summary.md"), "output markdown summary path")
    p.flag("device", "cpu", "E3 statistics device: cpu|gpu", choices=("cpu", "gpu"))
    a = p.parse_args(argv)
    cfg = releasegate.Config(
        candidate_root=a.candidate_root, baseline_root=a.baseline_root, baseline_manifest_path=a.baseline_manifest,
        candidate_ref=a.candidate_ref, candidate_commit=a.candidate_commit,
        require_baseline_manifest=a.require_baseline_manifest, scenarios=split_csv(a.scenarios),
        max_overhead_pct=a.max_overhead_pct, max_variance_pct=a.max_variance_pct, min_runs_per_scenario=a.min_runs,
        regression_pct_limit=a.ttft_regression_pct, significance_alpha=a.alpha,
        bootstrap_iterations=a.bootstrap_iters, bootstrap_seed=a.seed, min_samples_per_scenario=a.min_samples,
        min_cliffs_delta_for_failure=a.min_cliffs_delta, use_gpu=a.device == "gpu")
    try:
        s = releasegate.evaluate(cfg)
    except Exception as exc:  # noqa: BLE001
        eprint(f"m5 gate evaluation failed: {exc}")
        return 1
    ensure_parent(a.out_json)
    with open(a.out_json, "w", encoding="utf-8") as fh:
        json.dump(s, fh, indent=2)
    ensure_parent(a.out_md)
    with open(a.out_md, "w", encoding="utf-8") as fh:
        fh.write(releasegate.render_markdown(s))
    word = "PASS" if s["pass"] else "FAIL"
    o = s["overhead"]
    print(f"m5 gate: {word}")
    print(f"summary json: {a.out_json}")
    print(f"summary md: {a.out_md}")
    print(f"B5 overhead node p95 max: {o['max_node_p95_pct']:.4f}% on {o['max_node_p95_node']} "
          f"(limit {o['threshold_pct']:.4f}%)")
    if s["baseline"].get("same_source"):
        print(f"note: {s['baseline'].get('failure_reason', '')}")
    if not s["pass"]:
        for f in s.get("failures", []):
            print(f"- {f}")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""M5 release gates: baseline provenance, B5 overhead, D3 rerun variance, E3 significance.

REF pkg/releasegate/gate.go:21-946, same defaults (3 % overhead, 10 % CV, >= 3 runs,
5 % p95 regression, alpha 0.05, 1000 bootstrap iterations, seed 42, >= 30 samples,
|Cliff's delta| >= 0.147), same decision rules:

* B5 passes iff max node-p95 CPU% <= threshold AND mean CPU% <= threshold (:357);
* D3 per scenario: CV% of per-run TTFT p95 / tokens p50 / error-rate mean <= threshold;
* E3 fails a scenario iff regression% > limit AND Mann-Whitney p < alpha AND bootstrap
  p95-delta CI low > 0 AND |Cliff's delta| >= min (:559-585).

Statistics: Mann-Whitney U with average tie ranks, tie-corrected variance and
continuity correction (:816-891); Cliff's delta (:893-911); bootstrap CI of the p95
difference (:917-946). Go's math/rand stream cannot be bit-reproduced in Python; the
bootstrap uses a seeded counter-based stream (splitmix64, seed 42) that the numpy path
and the ``ops.gatestats`` HIP kernel (K5: all iterations x resamples in one launch, LDS
multiplicity histograms instead of per-resample sorts) evaluate identically.
"""

from __future__ import annotations

import csv
import json
import math
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..collector.pipeline import RawSample
from ..utils.timeutil import format_rfc3339_ns, now_ns
from .slo import cv_pct, mean, quantile, stddev

DEFAULT_SCENARIOS = ["dns_latency", "cpu_throttle", "provider_throttle", "memory_pressure", "network_partition",
                     "mixed", "mixed_multi"]


@dataclass
class Config:
    candidate_root: str = ""
    baseline_root: str = ""
    baseline_manifest_path: str = ""
    candidate_ref: str = ""
    candidate_commit: str = ""
    require_baseline_manifest: bool = False
    scenarios: List[str] = field(default_factory=list)
    max_overhead_pct: float = 0.0
    max_variance_pct: float = 0.0
    min_runs_per_scenario: int = 0
    regression_pct_limit: float = 0.0
    significance_alpha: float = 0.0
    bootstrap_iterations: int = 0
    bootstrap_seed: int = 0
    min_samples_per_scenario: int = 0
    min_cliffs_delta_for_failure: float = 0.0
    use_gpu: bool = False


def normalize_config(c: Config) -> Config:
    if not c.candidate_root:
        c.candidate_root = os.path.join("artifacts", "weekly-benchmark")
    if not c.baseline_root:
        c.baseline_root = os.path.join(c.candidate_root, "baseline")
    if not c.baseline_manifest_path:
        c.baseline_manifest_path = os.path.join(c.baseline_root, "manifest.json")
    if not c.scenarios:
        c.scenarios = list(DEFAULT_SCENARIOS)
    if c.max_overhead_pct <= 0:
        c.max_overhead_pct = 3
    if c.max_variance_pct <= 0:
        c.max_variance_pct = 10
    if c.min_runs_per_scenario <= 0:
        c.min_runs_per_scenario = 3
    if c.regression_pct_limit <= 0:
        c.regression_pct_limit = 5
    if c.significance_alpha <= 0 or c.significance_alpha >= 1:
        c.significance_alpha = 0.05
    if c.bootstrap_iterations <= 0:
        c.bootstrap_iterations = 1000
    if c.bootstrap_seed == 0:
        c.bootstrap_seed = 42
    if c.min_samples_per_scenario <= 0:
        c.min_samples_per_scenario = 30
    if c.min_cliffs_delta_for_failure <= 0:
        c.min_cliffs_delta_for_failure = 0.147
    return c


# ---------------------------------------------------------------------------------------
# statistics
# ---------------------------------------------------------------------------------------

def normal_cdf(z: float) -> float:
    return 0.5 * (1 + math.erf(z / math.sqrt(2)))


def mann_whitney_p(x: Sequence[float], y: Sequence[float]) -> float:
    nx, ny = len(x), len(y)
    if nx == 0 or ny == 0:
        return 1.0
    vals = np.concatenate([np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)])
    grp = np.concatenate([np.zeros(nx, dtype=np.int8), np.ones(ny, dtype=np.int8)])
    order = np.argsort(vals, kind="stable")
    sv = vals[order]
    ranks = np.empty(len(sv))
    tie_sum = 0.0
    i = 0
    n = len(sv)
    while i < n:
        j = i + 1
        while j < n and sv[j] == sv[i]:
            j += 1
        ranks[i:j] = (i + 1 + j) / 2.0
        t = j - i
        if t > 1:
            tie_sum += t ** 3 - t
        i = j
    rank_x = float(ranks[grp[order] == 0].sum())
    nxf, nyf = float(nx), float(ny)
    u1 = rank_x - nxf * (nxf + 1) / 2.0
    u2 = nxf * nyf - u1
    u = min(u1, u2)
    N = nxf + nyf
    mean_u = nxf * nyf / 2.0
    var_u = (nxf * nyf / 12.0) * ((N + 1.0) - tie_sum / (N * (N - 1.0)))
    if var_u <= 0:
        return 1.0
    z = u - mean_u
    z = (z - 0.5) / math.sqrt(var_u) if z > 0 else (z + 0.5) / math.sqrt(var_u)
    p = 2 * (1 - normal_cdf(abs(z)))
    return min(max(p, 0.0), 1.0)


def cliffs_delta(x: Sequence[float], y: Sequence[float]) -> float:
    if len(x) == 0 or len(y) == 0:
        return 0.0
    xa = np.asarray(x, dtype=np.float64)
    ys = np.sort(np.asarray(y, dtype=np.float64))
    # greater = #y < x ; lower = #y > x   (O((n+m) log m) instead of O(n*m))
    greater = np.searchsorted(ys, xa, side="left").sum()
    lower = (len(ys) - np.searchsorted(ys, xa, side="right")).sum()
    return float(greater - lower) / float(len(xa) * len(ys))


def bootstrap_delta_ci(cand: Sequence[float], base: Sequence[float], quant: float, iterations: int,
                       seed: int = 42, use_gpu: bool = False) -> Tuple[float, float]:
    if len(cand) == 0 or len(base) == 0 or iterations < 10:
        return 0.0, 0.0
    from ..ops import gatestats

    c = np.asarray(cand, dtype=np.float64)
    b = np.asarray(base, dtype=np.float64)
    # counter-based resampling stream shared by the numpy path and the K5 HIP kernel, so
    # the CPU and GPU gates agree bit for bit (ops/gatestats.py)
    deltas = gatestats.bootstrap_quantile_delta(c, b, quant, iterations, seed, use_gpu=use_gpu)
    deltas = np.sort(deltas)
    lo = max(int(math.floor(0.025 * (len(deltas) - 1))), 0)
    hi = min(int(math.ceil(0.975 * (len(deltas) - 1))), len(deltas) - 1)
    return float(deltas[lo]), float(deltas[hi])


# ---------------------------------------------------------------------------------------
# gate evaluation
# ---------------------------------------------------------------------------------------

def discover_runs(scenario_root: str) -> List[str]:
    if not os.path.isdir(scenario_root):
        return []
    runs = sorted(os.path.join(scenario_root, e) for e in os.listdir(scenario_root)
                  if e.startswith("run-") and os.path.isdir(os.path.join(scenario_root, e)))
    if runs:
        return runs
    if os.path.exists(os.path.join(scenario_root, "raw_samples.jsonl")):
        return [scenario_root]
    return []


def load_raw_samples(path: str) -> List[RawSample]:
    out = []
    with open(path, "r", encoding="utf-8") as fh:
        for line in fh:
            line = line.strip()
            if line:
                out.append(RawSample.from_dict(json.loads(line)))
    if not out:
        raise ValueError(f"no raw samples in {path}")
    return out


def load_collector_cpu(path: str) -> List[Tuple[str, float]]:
    with open(path, newline="") as fh:
        rows = list(csv.reader(fh))
    if len(rows) < 2:
        raise ValueError(f"overhead csv {path} has no data rows")
    hdr = rows[0]
    if "collector_cpu_pct" not in hdr:
        raise ValueError(f"collector_cpu_pct column missing in {path}")
    ci = hdr.index("collector_cpu_pct")
    ni = hdr.index("node") if "node" in hdr else -1
    out = []
    for r in rows[1:]:
        if ci >= len(r):
            continue
        node = r[ni].strip() if 0 <= ni < len(r) and r[ni].strip() else "unknown"
        out.append((node, float(r[ci].strip())))
    if not out:
        raise ValueError(f"no collector_cpu_pct values in {path}")
    return out


def evaluate_baseline(c: Config) -> Dict[str, object]:
    res = {"pass": True, "manifest_required": c.require_baseline_manifest, "manifest_path": c.baseline_manifest_path,
           "candidate_ref": c.candidate_ref, "candidate_commit": c.candidate_commit, "same_source": False}
    exists = os.path.exists(c.baseline_manifest_path)
    if c.require_baseline_manifest and not exists:
        res["pass"] = False
        res["failure_reason"] = f"required baseline manifest missing: {c.baseline_manifest_path}"
        return res
    if not exists:
        return res
    with open(c.baseline_manifest_path) as fh:
        man = json.load(fh)
    sref, scommit = (man.get("source_ref") or "").strip(), (man.get("source_commit") or "").strip()
    res["source_ref"], res["source_commit"] = sref, scommit
    same_commit = bool(scommit and c.candidate_commit and scommit == c.candidate_commit)
    same_ref = bool(sref and c.candidate_ref and sref == c.candidate_ref)
    res["same_source"] = same_commit or same_ref
    if res["same_source"]:
        res["failure_reason"] = (f"baseline source_commit matches candidate commit ({scommit}); skipping regression comparison"
                                 if same_commit else
                                 f"baseline source_ref matches candidate ref ({sref}); skipping regression comparison")
    return res


def evaluate_overhead(c: Config) -> Dict[str, object]:
    values: List[float] = []
    by_node: Dict[str, List[float]] = {}
    files = 0
    for sc in c.scenarios:
        runs = discover_runs(os.path.join(c.candidate_root, sc))
        if not runs:
            raise ValueError(f"no run directories found for scenario {sc}")
        for r in runs:
            for node, v in load_collector_cpu(os.path.join(r, "collector_overhead.csv")):
                values.append(v)
                by_node.setdefault(node, []).append(v)
            files += 1
    if not values:
        raise ValueError(f"no overhead values found in candidate root {c.candidate_root}")
    res: Dict[str, object] = {"threshold_pct": c.max_overhead_pct, "files_checked": files, "sample_count": len(values),
                              "max_observed_pct": max(values), "mean_observed_pct": mean(values),
                              "node_p95_observed": {}}
    max_node, max_p95 = "", 0.0
    for node, vals in by_node.items():
        p95 = quantile(vals, 0.95)
        res["node_p95_observed"][node] = p95
        if not max_node or p95 > max_p95:
            max_node, max_p95 = node, p95
    res["max_node_p95_node"], res["max_node_p95_pct"] = max_node, max_p95
    res["pass"] = max_p95 <= c.max_overhead_pct and res["mean_observed_pct"] <= c.max_overhead_pct
    if not res["pass"]:
        if max_p95 > c.max_overhead_pct:
            res["failure_reason"] = f"node {max_node} p95 overhead {max_p95:.4f} exceeds {c.max_overhead_pct:.4f}"
        else:
            res["failure_reason"] = f"mean overhead {res['mean_observed_pct']:.4f} exceeds {c.max_overhead_pct:.4f}"
    return res


def evaluate_variance(c: Config) -> Dict[str, object]:
    out = {"pass": True, "threshold_pct": c.max_variance_pct, "min_runs": c.min_runs_per_scenario, "scenarios": []}
    for sc in c.scenarios:
        runs = discover_runs(os.path.join(c.candidate_root, sc))
        r: Dict[str, object] = {"scenario": sc, "run_count": len(runs)}
        if len(runs) < c.min_runs_per_scenario:
            r["pass"] = False
            r["failure_reason"] = f"requires at least {c.min_runs_per_scenario} runs"
            out["pass"] = False
            out["scenarios"].append(r)
            continue
        ttft, tok, err = [], [], []
        for run in runs:
            raw = load_raw_samples(os.path.join(run, "raw_samples.jsonl"))
            ttft.append(quantile([s.ttft_ms for s in raw], 0.95))
            tok.append(quantile([s.token_throughput_tps for s in raw], 0.50))
            err.append(mean([s.error_rate for s in raw]))
        r.update({"ttft_p95_values": ttft, "mean_ttft_p95": mean(ttft), "stddev_ttft_p95": stddev(ttft),
                  "variance_pct": cv_pct(ttft), "tokens_p50_values": tok, "mean_tokens_p50": mean(tok),
                  "stddev_tokens_p50": stddev(tok), "tokens_variance_pct": cv_pct(tok),
                  "error_rate_mean_values": err, "mean_error_rate_mean": mean(err),
                  "stddev_error_rate_mean": stddev(err), "error_rate_variance_pct": cv_pct(err)})
        ok = (r["variance_pct"] <= c.max_variance_pct and r["tokens_variance_pct"] <= c.max_variance_pct
              and r["error_rate_variance_pct"] <= c.max_variance_pct)
        r["pass"] = ok
        if not ok:
            parts = []
            if r["variance_pct"] > c.max_variance_pct:
                parts.append(f"ttft variance {r['variance_pct']:.4f}% exceeds {c.max_variance_pct:.4f}%")
            if r["tokens_variance_pct"] > c.max_variance_pct:
                parts.append(f"tokens variance {r['tokens_variance_pct']:.4f}% exceeds {c.max_variance_pct:.4f}%")
            if r["error_rate_variance_pct"] > c.max_variance_pct:
                parts.append(f"error-rate variance {r['error_rate_variance_pct']:.4f}% exceeds {c.max_variance_pct:.4f}%")
            r["failure_reason"] = "; ".join(parts)
            out["pass"] = False
        out["scenarios"].append(r)
    return out


def evaluate_significance(c: Config) -> Dict[str, object]:
    out = {"pass": True, "regression_pct_limit": c.regression_pct_limit, "alpha": c.significance_alpha,
           "bootstrap_iterations": c.bootstrap_iterations, "min_samples_per_scenario": c.min_samples_per_scenario,
           "min_cliffs_delta_for_failure": c.min_cliffs_delta_for_failure, "scenarios": []}
    for idx, sc in enumerate(c.scenarios):
        cruns = discover_runs(os.path.join(c.candidate_root, sc))
        if not cruns:
            raise ValueError(f"no candidate runs found for {sc}")
        bruns = discover_runs(os.path.join(c.baseline_root, sc))
        if not bruns:
            raise ValueError(f"no baseline runs found for {sc} in {c.baseline_root}")
        cs = [s for r in cruns for s in load_raw_samples(os.path.join(r, "raw_samples.jsonl"))]
        bs = [s for r in bruns for s in load_raw_samples(os.path.join(r, "raw_samples.jsonl"))]
        ct, bt = [s.ttft_ms for s in cs], [s.ttft_ms for s in bs]
        cp95, bp95 = quantile(ct, 0.95), quantile(bt, 0.95)
        reg = ((cp95 - bp95) / bp95) * 100 if bp95 > 0 else 0.0
        enough = len(ct) >= c.min_samples_per_scenario and len(bt) >= c.min_samples_per_scenario
        r: Dict[str, object] = {
            "scenario": sc, "candidate_n": len(ct), "baseline_n": len(bt), "candidate_ttft_p95": cp95,
            "baseline_ttft_p95": bp95, "ttft_regression_pct": reg,
            "candidate_tokens_p50": quantile([s.token_throughput_tps for s in cs], 0.5),
            "baseline_tokens_p50": quantile([s.token_throughput_tps for s in bs], 0.5),
            "mann_whitney_p_value": 1.0, "bootstrap_delta_ci95": [0.0, 0.0], "cliffs_delta": 0.0,
            "practical_effect_pass": False, "minimum_samples_reached": enough, "pass": True,
        }
        if not enough:
            r["pass"] = False
            r["failure_reason"] = (f"insufficient samples: candidate={len(ct)} baseline={len(bt)} "
                                   f"requires >={c.min_samples_per_scenario}")
            out["pass"] = False
            out["scenarios"].append(r)
            continue
        if c.use_gpu:  # K5 rank counts on the device: ranks, ties and Cliff's delta in one pass
            from ..ops import gatestats

            p, cd, _ = gatestats.stats_from_rank_counts(gatestats.rank_counts(ct, bt), len(ct), len(bt))
        else:
            p, cd = mann_whitney_p(ct, bt), cliffs_delta(ct, bt)
        sub_seed = c.bootstrap_seed + idx  # one deterministic stream per scenario
        lo, hi = bootstrap_delta_ci(ct, bt, 0.95, c.bootstrap_iterations, sub_seed, c.use_gpu)
        r.update({"mann_whitney_p_value": p, "bootstrap_delta_ci95": [lo, hi], "cliffs_delta": cd,
                  "practical_effect_pass": abs(cd) >= c.min_cliffs_delta_for_failure})
        is_reg = reg > c.regression_pct_limit and p < c.significance_alpha and lo > 0
        if is_reg and not r["practical_effect_pass"]:
            r["failure_reason"] = (f"statistical regression detected ({reg:.4f}%, p={p:.6f}, CI95[{lo:.4f}, {hi:.4f}]) "
                                   f"but |Cliff's delta| {abs(cd):.4f} < {c.min_cliffs_delta_for_failure:.4f} practical threshold")
        if is_reg and r["practical_effect_pass"]:
            r["pass"] = False
            r["failure_reason"] = (f"ttft regression {reg:.4f}% exceeds {c.regression_pct_limit:.4f}% with p={p:.6f} "
                                   f"CI95[{lo:.4f}, {hi:.4f}] and Cliff's delta {cd:.4f}")
            out["pass"] = False
        out["scenarios"].append(r)
    return out


def evaluate(cfg: Config) -> Dict[str, object]:
    c = normalize_config(cfg)
    s: Dict[str, object] = {"generated_at": format_rfc3339_ns(now_ns()), "candidate_root": c.candidate_root,
                            "baseline_root": c.baseline_root, "scenarios": list(c.scenarios)}
    s["baseline"] = evaluate_baseline(c)
    s["overhead"] = evaluate_overhead(c)
    s["variance"] = evaluate_variance(c)
    s["significance"] = evaluate_significance(c)
    s["pass"] = all(s[k]["pass"] for k in ("baseline", "overhead", "variance", "significance"))
    fails = []
    if not s["baseline"]["pass"]:
        fails.append("baseline gate failed: " + (s["baseline"].get("failure_reason") or
                                                 "baseline provenance validation failed"))
    if not s["overhead"]["pass"]:
        o = s["overhead"]
        fails.append("B5 overhead gate failed: " + (o.get("failure_reason") or
                     f"node p95 {o['max_node_p95_pct']:.4f} on {o['max_node_p95_node']} exceeded {o['threshold_pct']:.4f}"))
    if not s["variance"]["pass"]:
        fails.append("D3 rerun variance gate failed")
    if not s["significance"]["pass"]:
        fails.append("E3 significance gate failed")
    if fails:
        s["failures"] = fails
    return s


def _word(b: bool) -> str:
    return "PASS" if b else "FAIL"


def render_markdown(s: Dict[str, object]) -> str:
    b, o, v, g = s["baseline"], s["overhead"], s["variance"], s["significance"]
    nz = lambda x: x if (x or "").strip() else "-"  # noqa: E731
    lines = [
        "# M5 Gate Summary", "", f"- Overall: `{_word(s['pass'])}`", f"- Generated at: `{s['generated_at']}`",
        f"- Candidate root: `{s['candidate_root']}`", f"- Baseline root: `{s['baseline_root']}`", "",
        "## Baseline Provenance", "", f"- Status: `{_word(b['pass'])}`",
        f"- Manifest required: `{str(b['manifest_required']).lower()}`", f"- Manifest path: `{b['manifest_path']}`",
        f"- Baseline source ref: `{nz(b.get('source_ref'))}`", f"- Baseline source commit: `{nz(b.get('source_commit'))}`",
        f"- Candidate ref: `{nz(b.get('candidate_ref'))}`", f"- Candidate commit: `{nz(b.get('candidate_commit'))}`", "",
        "## B5 Overhead", "", f"- Status: `{_word(o['pass'])}`",
        f"- Max observed CPU overhead (%): `{o['max_observed_pct']:.4f}`",
        f"- Mean observed CPU overhead (%): `{o['mean_observed_pct']:.4f}`",
        f"- Max node p95 CPU overhead (%): `{o['max_node_p95_pct']:.4f}` (`{nz(o['max_node_p95_node'])}`)",
        f"- Threshold (%): `{o['threshold_pct']:.4f}`", f"- Samples: `{o['sample_count']}`", "",
        "## D3 Rerun Variance", "", f"- Status: `{_word(v['pass'])}`", f"- Threshold (%): `{v['threshold_pct']:.4f}`", "",
    ]
    for sc in v["scenarios"]:
        lines.append(f"- `{sc['scenario']}`: status=`{_word(sc['pass'])}`, runs=`{sc['run_count']}`, "
                     f"ttft_variance_pct=`{sc.get('variance_pct', 0):.4f}`, "
                     f"tokens_variance_pct=`{sc.get('tokens_variance_pct', 0):.4f}`, "
                     f"error_rate_variance_pct=`{sc.get('error_rate_variance_pct', 0):.4f}`, "
                     f"mean_ttft_p95=`{sc.get('mean_ttft_p95', 0):.4f}`")
        if sc.get("failure_reason"):
            lines.append(f"  failure: `{sc['failure_reason']}`")
    lines += ["", "## E3 Significance", "", f"- Status: `{_word(g['pass'])}`",
              f"- TTFT regression threshold (%): `{g['regression_pct_limit']:.4f}`", f"- Alpha: `{g['alpha']:.4f}`",
              f"- Bootstrap iterations: `{g['bootstrap_iterations']}`", "",
              f"- Minimum samples per scenario: `{g['min_samples_per_scenario']}`",
              f"- Minimum |Cliff's delta| for failure: `{g['min_cliffs_delta_for_failure']:.4f}`", ""]
    for sc in g["scenarios"]:
        ci = sc["bootstrap_delta_ci95"]
        lines.append(f"- `{sc['scenario']}`: status=`{_word(sc['pass'])}`, candidate_n=`{sc['candidate_n']}`, "
                     f"baseline_n=`{sc['baseline_n']}`, candidate_p95=`{sc['candidate_ttft_p95']:.4f}`, "
                     f"baseline_p95=`{sc['baseline_ttft_p95']:.4f}`, regression_pct=`{sc['ttft_regression_pct']:.4f}`, "
                     f"p=`{sc['mann_whitney_p_value']:.6f}`, ci95_delta=[`{ci[0]:.4f}`,`{ci[1]:.4f}`], "
                     f"cliffs_delta=`{sc['cliffs_delta']:.4f}`")
        if sc.get("failure_reason"):
            lines.append(f"  failure: `{sc['failure_reason']}`")
    if s.get("failures"):
        lines += ["", "## Failures", ""] + [f"- {f}" for f in s["failures"]]
    return "\n".join(lines) + "\n"

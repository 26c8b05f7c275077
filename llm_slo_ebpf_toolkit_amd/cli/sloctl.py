"""`sloctl`: operator CLI (REF cmd/sloctl/main.go:14-125, cmd/sloctl/cdgate.go:19-165).

  sloctl prereq check [--output text|json] [--strict] [--require-gpu]
  sloctl cdgate check [--config PATH] [--prometheus-url URL] [--ttft-p95-ms N]
                      [--error-rate N] [--burn-rate N] [--fail-open] [--output text|json] [--timeout S]
  sloctl schema export [--root DIR]        (additive: regenerate the contract files)
  sloctl lab run [--scenario NAME,...] [--dir DIR] [--device auto|cpu|gpu] [--out FILE]
                                           (additive: execute incident-lab scenarios)
"""

from __future__ import annotations

import json
import os
import sys
from typing import List, Optional

from ..contracts import config as toolkitcfg
from ..contracts import schemas
from ..evaluation import prereq
from ..export import cdgate
from ..utils.timeutil import format_rfc3339_s
from ._common import GoFlags, eprint, is_version_request, print_version

USAGE = """Usage:
  sloctl prereq check [--output text|json] [--strict] [--require-gpu]
  sloctl cdgate check [--config PATH] [--prometheus-url URL] [--ttft-p95-ms N] [--error-rate N] [--burn-rate N] [--fail-open] [--output text|json]
  sloctl schema export [--root DIR]
  sloctl lab run [--scenario NAME,...] [--dir DIR] [--device auto|cpu|gpu] [--out FILE]"""

CDGATE_USAGE = """Usage:
  sloctl cdgate check [flags]

Flags:
  --config          Toolkit config path (default: config/toolkit.yaml)
  --prometheus-url  Prometheus base URL (default: http://prometheus:9090)
  --ttft-p95-ms     TTFT p95 threshold in ms (default: 800)
  --error-rate      Error rate threshold 0-1 (default: 0.05)
  --burn-rate       Burn rate threshold (default: 2.0)
  --fail-open       Pass if Prometheus unreachable (default: true)
  --output          Output mode: text|json (default: text)
  --timeout         Query timeout in seconds (default: 10)"""


def prereq_check(args: List[str]) -> int:
    p = GoFlags("sloctl prereq check")
    p.flag("output", "text", "output mode: text|json")
    p.flag("strict", False, "treat warnings as failures")
    p.flag("require-gpu", False, "treat missing ROCm / MI355X prerequisites as blockers")
    a = p.parse_args(args)
    rep = prereq.run_local(a.require_gpu)
    if a.output == "json":
        print(prereq.to_json(rep))
    elif a.output == "text":
        print(prereq.text_report(rep))
    else:
        eprint(f'unsupported output mode "{a.output}"')
        return 2
    ok = prereq.strict_pass(rep) if a.strict else rep.pass_
    return 0 if ok else 1


def cdgate_check(args: List[str], querier_factory=None) -> int:
    default_path = os.path.join("config", "toolkit.yaml")
    cfg_path = toolkitcfg.resolve_config_path(args, default_path)
    try:
        cfg = toolkitcfg.load(cfg_path)
    except Exception as exc:  # noqa: BLE001
        eprint(f"warning: failed to load config {cfg_path}: {exc} (using defaults)")
        cfg = toolkitcfg.default()
    d = toolkitcfg.default().cdgate
    cg = cfg.cdgate
    p = GoFlags("sloctl cdgate check")
    p.flag("config", cfg_path, "toolkit config path")
    p.flag("prometheus-url", cg.prometheus_url or d.prometheus_url, "Prometheus base URL")
    p.flag("ttft-p95-ms", float(cg.ttft_p95_ms if cg.ttft_p95_ms > 0 else d.ttft_p95_ms), "TTFT p95 threshold (ms)")
    p.flag("error-rate", float(cg.error_rate if cg.error_rate > 0 else d.error_rate), "Error rate threshold (0-1)")
    p.flag("burn-rate", float(cg.burn_rate if cg.burn_rate > 0 else d.burn_rate), "Burn rate threshold")
    p.flag("fail-open", bool(cg.fail_open), "Pass gate if Prometheus is unreachable")
    p.flag("output", "text", "Output mode: text|json")
    p.flag("timeout", 10, "Query timeout in seconds")
    a = p.parse_args(args)
    if a.config.strip() != cfg_path.strip():
        try:
            toolkitcfg.load(a.config)
        except Exception as exc:  # noqa: BLE001
            eprint(f"warning: failed to load config {a.config}: {exc}")
    q = (querier_factory or (lambda url, t: cdgate.HTTPQuerier(url, t)))(a.prometheus_url, float(a.timeout))
    res = cdgate.evaluate_slo_gate(q, cdgate.Thresholds(a.ttft_p95_ms, a.error_rate, a.burn_rate))
    if res.error and a.fail_open:
        res.passed = True
        res.error += " (fail-open: passing despite query error)"
    if a.output == "json":
        print(json.dumps(res.to_dict(), indent=2))
    elif a.output == "text":
        print(f"timestamp: {format_rfc3339_s(res.timestamp)}")
        if res.error:
            print(f"error: {res.error}")
        print()
        if res.violations:
            print("violations:")
            for v in res.violations:
                print(f"  - {v.metric}: actual={v.actual:.4f} threshold={v.threshold:.4f}")
            print()
        print("result: PASS (all SLO metrics within thresholds)" if res.passed else
              "result: FAIL (one or more SLO metrics exceeded thresholds)")
    else:
        eprint(f'unsupported output mode "{a.output}"')
        return 2
    return 0 if res.passed else 1


def schema_export(args: List[str]) -> int:
    p = GoFlags("sloctl schema export")
    p.flag("root", ".", "repository root to write docs/contracts and config/ into")
    a = p.parse_args(args)
    for path in schemas.export_all(a.root):
        print(f"wrote {path}")
    return 0


def lab_run(args: List[str]) -> int:
    from ..evaluation import incidentlab
    from ._common import split_csv, write_json

    p = GoFlags("sloctl lab run")
    p.flag("scenario", "", "comma-separated scenario names (default: all)")
    p.flag("dir", incidentlab.SCENARIO_DIR, "scenario directory")
    p.flag("device", "auto", "engine device: auto|cpu|gpu")
    p.flag("out", "", "write the JSON report here")
    a = p.parse_args(args)
    reports = incidentlab.run_all(a.dir, a.device, split_csv(a.scenario) or None)
    if not reports:
        eprint("no scenarios matched")
        return 2
    for r in reports:
        print(f"[{'PASS' if r['pass'] else 'FAIL'}] {r['scenario']} (engine={r['engine']})")
        for c in r["assertions"]:
            act = "n/a" if c["actual"] is None else f"{c['actual']:.4f}"
            print(f"    {'ok ' if c['pass'] else 'BAD'} {c['phase']}: {c['metric']} {c['op']} {c['value']} (actual {act})")
    if a.out:
        write_json(a.out, reports)
    return 0 if all(r["pass"] for r in reports) else 1


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print(USAGE)
        return 2
    cmd, rest = argv[0], argv[1:]
    if is_version_request([cmd]):
        return print_version()
    if cmd in ("help", "-h", "--help"):
        print(USAGE)
        return 0
    table = {"prereq": {"check": prereq_check}, "cdgate": {"check": cdgate_check}, "schema": {"export": schema_export},
             "lab": {"run": lab_run}}
    if cmd not in table:
        eprint(f'unknown command "{cmd}"')
        print(USAGE)
        return 2
    if not rest or rest[0] not in table[cmd]:
        if rest:
            eprint(f'unknown {cmd} subcommand "{rest[0]}"')
        print(CDGATE_USAGE if cmd == "cdgate" else USAGE)
        return 2
    return table[cmd][rest[0]](rest[1:])


if __name__ == "__main__":
    sys.exit(main())

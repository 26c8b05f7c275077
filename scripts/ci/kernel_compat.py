#!/usr/bin/env python3
"""Kernel / node compatibility records for the privileged probe path, and the matrix page
(REF scripts/ci/kernel_compat_probe.sh + render_compatibility_report.sh).

    kernel_compat.py probe  --profile kernel-6-8 --out artifacts/compatibility/kernel-6-8.json
    kernel_compat.py render --input-dir artifacts/compatibility --out docs/compatibility.md

``probe`` records what the agent needs from a node: kernel release and BTF (CO-RE probes), the
``sloctl prereq check`` report (tooling, capabilities, bpffs, ROCm / KFD / gfx950), the agent's
``--probe-smoke`` (root only; ``skipped`` otherwise, as in REF) and, for the MI355X side, the GPUs
the amdgpu driver exposes and whether the unprivileged signal sources (schedstat, PSI) are
readable. ``STRICT=true`` fails the run on a failed prerequisite or probe smoke. ``render``
writes one matrix row per profile record found, whatever the profile labels are.
"""

from __future__ import annotations

import argparse
import datetime as _dt
import glob
import json
import os
import platform
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _run(args, timeout=120):
    env = dict(os.environ, PYTHONPATH=ROOT + (":" + os.environ["PYTHONPATH"] if os.environ.get("PYTHONPATH") else ""))
    try:
        p = subprocess.run(args, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
        return p.returncode, p.stdout, p.stderr
    except (OSError, subprocess.TimeoutExpired) as exc:
        return 127, "", str(exc)


def probe(profile: str, out: str) -> dict:
    sys.path.insert(0, ROOT)
    from llm_slo_ebpf_toolkit_amd.collector import procfs
    from llm_slo_ebpf_toolkit_amd.parallel.numa import visible_gpu_count

    d = os.path.dirname(os.path.abspath(out))
    os.makedirs(d, exist_ok=True)
    prereq_path = os.path.join(d, f"{profile}-prereq.json")
    rc, so, se = _run([sys.executable, "-m", "llm_slo_ebpf_toolkit_amd.cli.sloctl", "prereq", "check", "--output", "json"])
    with open(prereq_path, "w") as fh:
        fh.write(so)
    prereq = {"status": "pass" if rc == 0 else "fail", "detail": " ".join(se.split())[:2000],
              "json_path": os.path.basename(prereq_path)}
    if os.geteuid() == 0:
        rc2, so2, se2 = _run([sys.executable, "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--probe-smoke"])
        smoke = {"status": "pass" if rc2 == 0 else "fail", "detail": " ".join((so2 if rc2 == 0 else se2).split())[:2000]}
    else:
        smoke = {"status": "skipped", "detail": "agent probe smoke skipped (non-root)"}
    rec = {
        "profile": profile,
        "timestamp_utc": _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
        "host_os": platform.system(), "host_arch": platform.machine(), "kernel_release": platform.release(),
        "btf_available": os.path.exists("/sys/kernel/btf/vmlinux"),
        "prereq": prereq, "probe_smoke": smoke,
        "gpus_visible": visible_gpu_count(),
        "unprivileged_sources": {"schedstat": os.path.exists(f"/proc/{os.getpid()}/schedstat"),
                                 "psi_memory": procfs.psi_available()},
    }
    with open(out, "w") as fh:
        json.dump(rec, fh, indent=2)
    return rec


def render(input_dir: str, out: str, run_id: str) -> str:
    rows = []
    for path in sorted(glob.glob(os.path.join(input_dir, "*.json"))):
        if path.endswith("-prereq.json"):
            continue
        try:
            with open(path) as fh:
                r = json.load(fh)
        except (OSError, ValueError):
            continue
        if "profile" not in r:
            continue
        g = lambda *ks: _get(r, ks)  # noqa: E731
        rows.append(f"| `{r['profile']}` | {r.get('status', 'available')} | `{g('kernel_release')}` | "
                    f"`{str(g('btf_available')).lower()}` | `{g('prereq', 'status')}` | `{g('probe_smoke', 'status')}` | "
                    f"`{g('gpus_visible')}` | `{str(g('unprivileged_sources', 'psi_memory')).lower()}` |")
    now = _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
    text = "\n".join([
        "# Kernel Compatibility Matrix", "",
        "Compatibility checks of the privileged probe path (and the MI355X node prerequisites) per runner kernel "
        "profile.", "",
        f"- Generated at (UTC): {now}", f"- Source run: `{run_id}`", f"- Report source directory: `{input_dir}`", "",
        "## Matrix", "",
        "| Profile | Availability | Kernel release | BTF | `sloctl prereq` | `agent --probe-smoke` | GPUs | PSI |",
        "|---|---|---|---|---|---|---|---|",
        *(rows or ["| (no profile records) | | | | | | | |"]), "",
        "## Interpretation", "",
        "- `available`: the matrix job ran on a runner matching the profile label; `unavailable`: no online runner "
        "with that label was found in preflight.",
        "- `prereq=pass`: kernel, tooling, capability (and, with `--require-gpu`, ROCm / KFD / gfx950) checks passed.",
        "- `probe-smoke=pass`: the probe loader smoke succeeded; `skipped` without root.",
        "- GPUs: the GPUs the amdgpu driver exposes to the runner; PSI: memory pressure-stall accounting readable "
        "(the unprivileged sampler's memory signal).", "",
        "These are compatibility signals, not performance regressions; the benchmark workflows gate performance.", ""])
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as fh:
        fh.write(text)
    return text


def _get(r, ks):
    v = r
    for k in ks:
        if not isinstance(v, dict) or k not in v:
            return "n/a"
        v = v[k]
    return "n/a" if v is None else v


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("probe")
    p.add_argument("--profile", required=True)
    p.add_argument("--out", required=True)
    r = sub.add_parser("render")
    r.add_argument("--input-dir", default="artifacts/compatibility")
    r.add_argument("--out", default="docs/compatibility.md")
    a = ap.parse_args(argv)
    if a.cmd == "probe":
        rec = probe(a.profile, a.out)
        print(json.dumps(rec))
        if os.environ.get("STRICT", "false") == "true":
            if rec["prereq"]["status"] != "pass" or rec["probe_smoke"]["status"] == "fail":
                return 1
        return 0
    render(a.input_dir, a.out, os.environ.get("RUN_ID", "manual"))
    print(f"wrote {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""scripts/ci/kernel_compat.py (REF scripts/ci/kernel_compat_probe.sh + render_compatibility_report.sh)
and deploy/kind/bootstrap-tools.sh."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "ci"))

import kernel_compat  # noqa: E402


def test_probe_record_and_matrix(tmp_path):
    out = tmp_path / "kernel-x.json"
    rec = kernel_compat.probe("kernel-x", str(out))
    on_disk = json.loads(out.read_text())
    assert on_disk == json.loads(json.dumps(rec))
    assert rec["kernel_release"] == os.uname().release
    assert rec["prereq"]["status"] in ("pass", "fail")
    assert (tmp_path / "kernel-x-prereq.json").exists()
    assert rec["probe_smoke"]["status"] in ("pass", "fail", "skipped")
    # a second profile that did not run, and the rendered page
    (tmp_path / "kernel-y.json").write_text(json.dumps({"profile": "kernel-y", "status": "unavailable"}))
    text = kernel_compat.render(str(tmp_path), str(tmp_path / "compat.md"), "run-1")
    assert "| `kernel-x` | available |" in text and "| `kernel-y` | unavailable | `n/a` |" in text
    assert "kernel-x-prereq" not in text and "`run-1`" in text


def test_bootstrap_tools_reports_missing_tools():
    p = subprocess.run(["bash", os.path.join(ROOT, "deploy", "kind", "bootstrap-tools.sh")], capture_output=True,
                       text=True, timeout=120, env=dict(os.environ, AUTO_INSTALL="0"))
    assert p.returncode in (0, 1)
    assert ("all required tools are installed" in p.stdout) == (p.returncode == 0)
    if p.returncode:
        assert "missing tools:" in p.stdout and "AUTO_INSTALL=1" in p.stdout

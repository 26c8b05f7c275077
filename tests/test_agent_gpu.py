"""The agent daemon's GPU window loop end to end (REF cmd/agent/main.go:269-633 run loop):
a forked replay producer writes the BPF ring (probe model), the user-space GPU-signal ring and
the span ring; the agent cuts windows, the native engine attributes them, and the agent emits
one attribution per incident group per window, then exits cleanly (engine closed, producer
reaped) -- run as a child process, as an operator would start it."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_agent_replay_windows_and_clean_exit(tmp_path):
    out = tmp_path / "attr.jsonl"
    n_win, groups = 3, 32
    cmd = [sys.executable, "-u", "-m", "llm_slo_ebpf_toolkit_amd.cli.agent", "--engine", "gpu", "--source", "replay",
           "--count", str(n_win), "--window-ms", "300", "--window-events", "65536", "--window-spans", "2048",
           "--window-groups", str(groups), "--output", "jsonl", "--output-path", str(out), "--metrics-bind", "",
           "--scenario", "full"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-2000:]
    rows = [json.loads(x) for x in out.read_text().splitlines() if x.strip()]
    assert len(rows) == n_win * groups
    doms = {r["predicted_fault_domain"] for r in rows}
    assert len(doms) >= 3  # the replay's full scenario spans several fault domains
    assert all(0.0 <= r["confidence"] <= 1.0 for r in rows)

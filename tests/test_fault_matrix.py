"""scripts/chaos/run_fault_matrix.sh: the release gate's collector_overhead.csv comes from the window
agent that ships (tools/agent_overhead.py with the ConfigMap's toolkit.yaml and the shipped model),
not from the synthetic tick loop (REF pkg/releasegate/gate.go:303-376 reads the CSV)."""

import csv
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
def test_fault_matrix_overhead_csv_is_the_window_agents(tmp_path):
    env = dict(os.environ, SCENARIOS="cpu_throttle", RUNS="1", COUNT="6", ENGINE="cpu", OVERHEAD_RATE="2e4",
               OVERHEAD_SECONDS="2", OUT=str(tmp_path / "wk"), NODE_NAME="node-x")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "chaos", "run_fault_matrix.sh")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    run = tmp_path / "wk" / "cpu_throttle" / "run-1"
    rows = list(csv.DictReader(open(run / "collector_overhead.csv")))
    assert len(rows) == 1 and rows[0]["node"] == "node-x"
    assert float(rows[0]["collector_cpu_pct"]) > 0 and float(rows[0]["collector_memory_mb"]) > 50
    meas = json.load(open(run / "agent_overhead.json"))
    assert meas["exit_code"] == 0 and meas["windows_in_interval"] >= 1
    assert meas["shipped_config"]["config"] == "deploy/k8s/configmap.yaml:toolkit.yaml"
    assert meas["shipped_config"]["model"] == "config/models/mislo-learned.safetensors"
    assert "window engine: cpu" in meas["agent_log_tail"]
    from llm_slo_ebpf_toolkit_amd.evaluation.releasegate import load_collector_cpu

    assert [n for n, _v in load_collector_cpu(str(run / "collector_overhead.csv"))] == ["node-x"]

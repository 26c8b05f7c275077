"""Incident-lab scenarios execute (REF's YAMLs are never read), and the deploy assets are
consistent with what the agent exports."""

import glob
import json
import os
import re

import pytest
import yaml

from llm_slo_ebpf_toolkit_amd.agent.metrics import AgentMetrics
from llm_slo_ebpf_toolkit_amd.cli import sloctl
from llm_slo_ebpf_toolkit_amd.evaluation import incidentlab

from conftest import ROOT


def test_all_scenarios_load():
    paths = incidentlab.discover()
    names = {incidentlab.load_scenario(p).name for p in paths}
    assert {"dns_latency", "cpu_throttle", "memory_pressure", "provider_throttle", "network_partition", "mixed",
            "mixed_multi", "gpu_contention", "rccl_latency"} <= names


@pytest.mark.parametrize("name", ["dns_latency", "gpu_contention", "mixed_multi"])
def test_scenario_runs_and_passes_on_cpu(name):
    sc = incidentlab.load_scenario(os.path.join(incidentlab.SCENARIO_DIR, name + ".yaml"))
    r = incidentlab.run_scenario(sc, device="cpu")
    assert r["engine"] == "cpu" and r["pass"], r["assertions"]
    assert set(r["phases"]) == {"baseline", "fault", "recovery"}


def test_sloctl_lab_run(tmp_path, capsys):
    out = tmp_path / "lab.json"
    assert sloctl.main(["lab", "run", "--scenario", "cpu_throttle", "--device", "cpu", "--out", str(out)]) == 0
    assert "[PASS] cpu_throttle" in capsys.readouterr().out
    assert json.load(open(out))[0]["scenario"] == "cpu_throttle"


def _yaml_docs(pattern):
    docs = []
    for p in glob.glob(os.path.join(ROOT, pattern), recursive=True):
        with open(p) as fh:
            docs += [d for d in yaml.safe_load_all(fh) if d]
    return docs


def test_daemonset_mounts_gpu_devices_and_probes():
    ds = [d for d in _yaml_docs("deploy/k8s/*.yaml") if d.get("kind") == "DaemonSet"][0]
    spec = ds["spec"]["template"]["spec"]
    paths = {v["hostPath"]["path"] for v in spec["volumes"] if "hostPath" in v}
    assert {"/dev/kfd", "/dev/dri", "/sys/fs/bpf"} <= paths
    c = spec["containers"][0]
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz" and c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert any(a.startswith("--engine=") for a in c["args"])
    cm = [d for d in _yaml_docs("deploy/k8s/*.yaml") if d.get("kind") == "ConfigMap"][0]
    from llm_slo_ebpf_toolkit_amd.contracts import validator

    validator.validate("toolkit-config", yaml.safe_load(cm["data"]["toolkit.yaml"]))


def _agent_metric_names():
    m = AgentMetrics("probe", "core_full", [], [])
    names = set()
    for line in m.registry.exposition().splitlines():
        if line.startswith("# TYPE"):
            names.add(line.split()[2])
    # demo rag-service metrics (demo/rag_service.py) and histogram series suffixes
    names |= {"llm_slo_ttft_ms", "llm_slo_tokens_per_sec", "llm_slo_retrieval_dns_ms", "llm_slo_requests_total",
              "llm_slo_errors_total", "llm_slo_burn_rate", "llm_slo_correlation_total"}
    return names


def _metrics_in(expr):
    out = set()
    for tok in re.findall(r"\b(llm_[a-z0-9_]+)", expr):
        out.add(re.sub(r"_(bucket|sum|count)$", "", tok))
    return out


def test_alerts_and_dashboards_reference_exported_metrics():
    known = _agent_metric_names()
    alerts = [d for d in _yaml_docs("deploy/observability/*.yaml") if d.get("metadata", {}).get("name") ==
              "prometheus-alerts"][0]
    rules = yaml.safe_load(alerts["data"]["alerts.yaml"])["groups"][0]["rules"]
    names = {r["alert"] for r in rules}
    assert {"TTFTBudgetBurning", "ErrorRateHigh", "CorrelationDegraded", "AgentHeartbeatStale", "OverheadHigh",
            "LLMHighTTFTWithDNSKernelSignal"} <= names
    for r in rules:
        assert _metrics_in(r["expr"]) <= known, (r["alert"], _metrics_in(r["expr"]) - known)
    for p in glob.glob(os.path.join(ROOT, "dashboards", "*.json")):
        d = json.load(open(p))
        for panel in d["panels"]:
            for t in panel["targets"]:
                assert _metrics_in(t["expr"]) <= known, (p, t["expr"])


def test_helm_chart_files_present():
    base = os.path.join(ROOT, "charts", "llm-slo-agent")
    chart = yaml.safe_load(open(os.path.join(base, "Chart.yaml")))
    assert chart["name"] == "llm-slo-agent"
    vals = yaml.safe_load(open(os.path.join(base, "values.yaml")))
    from llm_slo_ebpf_toolkit_amd.contracts import validator

    cfg = dict(vals["config"], apiVersion="toolkit.llm-slo.dev/v1alpha1", kind="ToolkitConfig")
    validator.validate("toolkit-config", cfg)
    assert os.path.exists(os.path.join(base, "templates", "daemonset.yaml"))

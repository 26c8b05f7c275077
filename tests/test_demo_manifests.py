"""Demo / deployment manifests stay consistent with the code they run (REF demo/*/k8s,
test/integration-kind): every agent flag the DaemonSet passes exists, the services' OTLP
endpoint is the agent's receiver port, the rocprofiler tool path and ring name match the
agent's defaults, and the pod identity the services export is what the receiver maps."""

import os
import re

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(rel):
    with open(os.path.join(ROOT, rel)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def _container(rel):
    return _load(rel)[0]["spec"]["template"]["spec"]["containers"][0]


def test_daemonset_flags_exist_and_receiver_is_exposed():
    from llm_slo_ebpf_toolkit_amd.cli import agent

    c = _container("deploy/k8s/daemonset.yaml")
    names = {a.split("=", 1)[0].lstrip("-") for a in c["args"]}
    src = open(agent.__file__).read()
    for n in names:
        assert f'("{n}"' in src, n
    assert any(a.startswith("--otlp-receiver-bind=") and a.endswith(":4318") for a in c["args"])
    assert any(a.startswith("--state-dir=") for a in c["args"])
    assert {"containerPort": 4318, "name": "otlp-http"} in c["ports"]


def test_services_export_spans_to_the_node_agent():
    from llm_slo_ebpf_toolkit_amd.agent.daemon import AgentOptions
    from llm_slo_ebpf_toolkit_amd.collector.bpf import RingNames

    for rel in ("deploy/demo/rag-service/deployment.yaml", "deploy/demo/llm/deployment.yaml"):
        env = {e["name"]: e for e in _container(rel)["env"]}
        assert re.search(r":4318/v1/traces$", env["OTEL_EXPORTER_OTLP_TRACES_ENDPOINT"]["value"]), rel
        assert env["POD_UID"]["valueFrom"]["fieldRef"]["fieldPath"] == "metadata.uid", rel
    env = {e["name"]: e for e in _container("deploy/demo/llm/deployment.yaml")["env"]}
    tool = env["ROCP_TOOL_LIBRARIES"]["value"]
    assert tool.startswith("/opt/llm-slo/")
    assert os.path.exists(os.path.join(ROOT, "llm_slo_ebpf_toolkit_amd", "probes", "rocprof", "mislo_rocprof.cpp"))
    assert env["MISLO_RING"]["value"] == RingNames.of(AgentOptions().ring_name).user


def test_kind_smokes_and_runner_scripts_parse():
    import subprocess

    for rel in ("test/integration-kind/smoke.sh", "test/integration-kind/observability-smoke.sh",
                "infra/runner/mi355x/runner-loop.sh", "infra/runner/mi355x/preflight.sh"):
        subprocess.run(["bash", "-n", os.path.join(ROOT, rel)], check=True)
    for rel in (".github/workflows/e2e-evidence-report.yml", ".github/workflows/runner-health.yml"):
        wf = _load(rel)[0]
        assert wf["jobs"], rel

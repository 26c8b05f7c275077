"""`schemavalidate`: compile the 4 contract schemas, validate sample payloads, validate
config/toolkit.yaml against its schema and with the loader (REF cmd/schemavalidate/main.go:31-250).

Uses the built-in compiled validator (contracts/validator.py; no jsonschema dependency).
Also checks that the on-disk schema files equal the programmatic contracts
(contracts/schemas.py), so the two can never drift.
"""

from __future__ import annotations

import json
import os
import sys
from typing import List, Optional

import yaml

from ..contracts import config as toolkitcfg
from ..contracts import schemas, validator
from ..contracts.types import ConnTuple, Evidence, FaultHypothesis, IncidentAttribution, ProbeEventV1, SLOEvent, \
    SLOImpact
from ..utils.timeutil import now_ns
from ._common import eprint, is_version_request, print_version, project_root

SCHEMA_FILES = dict(schemas.EXPORT_PATHS)


def check_schema_documents(root: str) -> None:
    for name, rel in SCHEMA_FILES.items():
        path = os.path.join(root, rel)
        with open(path, "r", encoding="utf-8") as fh:
            doc = json.load(fh)
        validator.CompiledSchema(doc)  # compile
        if doc != schemas.get(name):
            raise ValueError(f"schema {path} differs from the programmatic contract {name} "
                             f"(regenerate with `sloctl schema export`)")


def sample_payloads():
    t = now_ns()
    slo = SLOEvent(event_id="evt-schema-1", timestamp=t, cluster="local", namespace="default", workload="gateway",
                   service="rag-service", request_id="req-schema-1", trace_id="trace-schema-1", sli_name="ttft_ms",
                   sli_value=220, unit="ms", status="ok")
    inc = IncidentAttribution(
        incident_id="inc-schema-1", timestamp=t, cluster="local", namespace="default", service="rag-service",
        predicted_fault_domain="provider_throttle", confidence=0.92,
        evidence=[Evidence("llm.ebpf.tcp.retransmits", 7, "ebpf")], slo_impact=SLOImpact("ttft_ms", 2.4, 5),
        trace_ids=["trace-schema-1"], request_ids=["req-schema-1"],
        fault_hypotheses=[FaultHypothesis("provider_throttle", 0.8, ["tcp_retransmits_total"]),
                          FaultHypothesis("network_dns", 0.2, ["dns_latency_ms"])])
    probe = ProbeEventV1(ts_unix_nano=t, signal="dns_latency_ms", node="kind-worker", namespace="default",
                         pod="rag-service-0", container="rag-service", pid=101, tid=101,
                         conn_tuple=ConnTuple("10.244.0.2", "10.96.0.10", 41000, 53, "udp"), value=17.4, unit="ms",
                         status="ok", trace_id="trace-schema-1", span_id="span-schema-1")
    gpu_probe = ProbeEventV1(ts_unix_nano=t, signal="rccl_collective_ms", node="mi355x-0", namespace="default",
                             pod="llama-tp-0", container="server", pid=77, tid=78, value=0.42, unit="ms",
                             status="ok")
    return [("slo-event", slo), ("incident-attribution", inc), ("probe-event", probe), ("probe-event", gpu_probe)]


def check_contract_samples(root: str) -> None:
    for name, payload in sample_payloads():
        validator.validate(os.path.join(root, SCHEMA_FILES[name]), payload)


def check_config_schema(root: str) -> None:
    with open(os.path.join(root, "config", "toolkit.yaml"), "r", encoding="utf-8") as fh:
        data = yaml.safe_load(fh)
    validator.validate(os.path.join(root, SCHEMA_FILES["toolkit-config"]), data)


def check_config_loader(root: str) -> None:
    toolkitcfg.load(os.path.join(root, "config", "toolkit.yaml"))


CHECKS = [("schema document parse", check_schema_documents), ("contract sample payloads", check_contract_samples),
          ("toolkit config schema", check_config_schema), ("toolkit config loader", check_config_loader)]


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    root = os.environ.get("LLM_SLO_ROOT") or (os.getcwd() if os.path.isdir("docs/contracts") else project_root())
    for name, fn in CHECKS:
        try:
            fn(root)
        except Exception as exc:  # noqa: BLE001
            eprint(f"schema validation failed ({name}): {exc}")
            return 1
        print(f"ok: {name}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

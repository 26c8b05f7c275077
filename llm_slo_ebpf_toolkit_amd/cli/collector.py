"""`collector`: RawSample JSONL (file/stdin) or synthetic -> NormalizeSample -> schema
validation -> stdout / jsonl / OTLP sink (REF cmd/collector/main.go:25-238).

Stream mode when ``--count 0``. The OTLP sink batches log records (REF posts one per
event); ``--otlp-batch 1`` restores per-event posts.
"""

from __future__ import annotations

import sys
import time
from typing import List, Optional

from ..collector.pipeline import SampleMeta, build_synthetic_sample, generate_synthetic_samples, normalize_sample, \
    read_raw_samples
from ..contracts import validator
from ..export.otel import OTLPLogExporter
from ..utils.timeutil import now_ns
from ._common import GoFlags, eprint, ensure_parent, is_version_request, jsonl_line, print_version


class Sink:
    def __init__(self, mode: str, path: str, endpoint: str, timeout_ms: int, batch: int):
        self.mode = mode
        self.fh = None
        self.exp = None
        if mode == "stdout":
            self.fh = sys.stdout
        elif mode == "jsonl":
            ensure_parent(path)
            self.fh = open(path, "w", encoding="utf-8")
        elif mode == "otlp":
            self.exp = OTLPLogExporter(endpoint, "llm-slo-ebpf-toolkit", "llm-slo-ebpf-toolkit/collector",
                                       timeout_ms / 1000.0, max_batch=max(1, batch))
        else:
            raise ValueError(f'unsupported output mode "{mode}"')

    def emit(self, ev) -> None:
        if self.exp is not None:
            self.exp.add_slo(ev)
        else:
            self.fh.write(jsonl_line(ev))

    def flush(self) -> None:
        if self.exp is not None:
            self.exp.flush()
        elif self.fh is not None:
            self.fh.flush()

    def close(self) -> None:
        self.flush()
        if self.fh is not None and self.fh is not sys.stdout:
            self.fh.close()


def emit_samples(sink: Sink, samples) -> None:
    schema = validator.compiled("slo-event")
    for s in samples:
        for ev in normalize_sample(s):
            schema.validate(ev.to_dict())
            sink.emit(ev)
    sink.flush()


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    p = GoFlags("collector", "normalize raw samples into SLO events")
    p.flag("input", "-", "raw sample input JSONL path or '-' for stdin")
    p.flag("output", "stdout", "output mode: stdout|jsonl|otlp")
    p.flag("output-path", "artifacts/collector/slo-events.jsonl", "output path when output=jsonl")
    p.flag("otlp-endpoint", "http://otel-collector.observability.svc.cluster.local:4318/v1/logs",
           "OTLP/HTTP logs endpoint when output=otlp")
    p.flag("otlp-timeout-ms", 5000, "OTLP export timeout in milliseconds")
    p.flag("otlp-batch", 256, "log records per OTLP POST")
    p.flag("cluster", "local", "cluster name for synthetic generation")
    p.flag("namespace", "default", "namespace for synthetic generation")
    p.flag("workload", "gateway", "workload for synthetic generation")
    p.flag("service", "chat", "service for synthetic generation")
    p.flag("k8s-node", "unknown-node", "node name label")
    p.flag("scenario", "baseline", "synthetic scenario name")
    p.flag("count", 1, "synthetic sample count (0 = stream mode)")
    p.flag("interval-ms", 1000, "stream interval milliseconds when count=0")
    a = p.parse_args(argv)
    try:
        if a.input == "-":
            samples = [] if sys.stdin is None or sys.stdin.isatty() else read_raw_samples(sys.stdin)
        else:
            with open(a.input, "r", encoding="utf-8") as fh:
                samples = read_raw_samples(fh)
    except Exception as exc:  # noqa: BLE001
        eprint(f"failed to read samples: {exc}")
        return 1
    try:
        sink = Sink(a.output, a.output_path, a.otlp_endpoint, a.otlp_timeout_ms, a.otlp_batch)
    except Exception as exc:  # noqa: BLE001
        eprint(f"failed to open output: {exc}")
        return 1
    meta = SampleMeta(cluster=a.cluster, namespace=a.namespace, workload=a.workload, service=a.service,
                      node=a.k8s_node)
    try:
        if samples:
            emit_samples(sink, samples)
            return 0
        if a.count < 0:
            eprint("count must be >= 0")
            return 1
        if a.count > 0:
            emit_samples(sink, generate_synthetic_samples(a.scenario, a.count, now_ns(), meta))
            return 0
        if a.interval_ms <= 0:
            eprint("interval-ms must be > 0")
            return 1
        idx = 0
        nxt = time.monotonic()
        while True:
            emit_samples(sink, [build_synthetic_sample(a.scenario, idx, now_ns(), meta)])
            idx += 1
            nxt += a.interval_ms / 1000.0
            time.sleep(max(0.0, nxt - time.monotonic()))
    except KeyboardInterrupt:
        return 0
    except Exception as exc:  # noqa: BLE001
        eprint(f"emit failed: {exc}")
        return 1
    finally:
        try:
            sink.close()
        except Exception as exc:  # noqa: BLE001
            eprint(f"close output failed: {exc}")


if __name__ == "__main__":
    sys.exit(main())

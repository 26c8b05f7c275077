"""`faultinject`: synthetic RawSample JSONL for collector input (REF cmd/faultinject/main.go:22-68)."""

from __future__ import annotations

import sys
from typing import List, Optional

from ..collector.pipeline import SampleMeta, generate_synthetic_samples
from ..utils.timeutil import now_ns
from ._common import GoFlags, eprint, ensure_parent, is_version_request, jsonl_line, print_version


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    p = GoFlags("faultinject", "write synthetic raw samples")
    p.flag("scenario", "mixed", "fault injection scenario")
    p.flag("count", 24, "number of raw samples to emit")
    p.flag("out", "artifacts/fault-injection/raw_samples.jsonl", "output JSONL file for collector input")
    p.flag("cluster", "local", "cluster label")
    p.flag("namespace", "default", "namespace label")
    p.flag("workload", "gateway", "workload label")
    p.flag("service", "chat", "service label")
    p.flag("node", "kind-control-plane", "node label")
    a = p.parse_args(argv)
    meta = SampleMeta(cluster=a.cluster, namespace=a.namespace, workload=a.workload, service=a.service,
                      node=a.node)
    try:
        samples = generate_synthetic_samples(a.scenario, a.count, now_ns(), meta)
    except ValueError as exc:
        eprint(f"generate fault-injection samples failed: {exc}")
        return 1
    ensure_parent(a.out)
    with open(a.out, "w", encoding="utf-8") as fh:
        for s in samples:
            fh.write(jsonl_line(s))
    print(f"wrote {len(samples)} raw samples to {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

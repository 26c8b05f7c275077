"""`benchgen`: benchmark artefact bundle (REF cmd/benchgen/main.go:20-31 over
pkg/benchmark/harness.go). Unlike REF, overhead / events/s / detection delay in the
bundle are measured (evaluation/benchmark.py), not constants."""

from __future__ import annotations

import sys
from typing import List, Optional

from ..evaluation.benchmark import generate_artifacts
from ._common import GoFlags, eprint, is_version_request, print_version


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    p = GoFlags("benchgen", "generate the benchmark artefact bundle")
    p.flag("out", "artifacts/benchmarks", "output directory")
    p.flag("scenario", "provider_throttle", "fault scenario")
    p.flag("workload", "rag_mixed", "workload profile")
    p.flag("input", "", "optional JSONL fault sample input")
    p.flag("attribution-mode", "bayes", "attribution mode: bayes|rule|bayes_learned|lda")
    p.flag("measure-seconds", 1.0, "seconds of agent-loop CPU measurement for collector_overhead.csv")
    a = p.parse_args(argv)
    try:
        generate_artifacts(a.out, a.scenario, a.workload, a.input, a.attribution_mode,
                           measure_seconds=a.measure_seconds)
    except Exception as exc:  # noqa: BLE001
        eprint(f"benchmark generation failed: {exc}")
        return 1
    print(f"benchmark artifacts written to {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

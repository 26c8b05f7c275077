"""`faultreplay`: deterministic FaultSample JSONL streams (REF cmd/faultreplay/main.go:22-53).

Extra flags (additive): ``--with-signals`` populates kernel/GPU signal values from the
fault profiles so replays exercise the Bayes path, ``--seed`` for their jitter.
"""

from __future__ import annotations

import sys
from typing import List, Optional

from ..evaluation.faultreplay import generate_fault_samples
from ..utils.timeutil import now_ns
from ._common import GoFlags, eprint, ensure_parent, is_version_request, jsonl_line, print_version


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    p = GoFlags("faultreplay", "write deterministic fault-replay samples")
    p.flag("scenario", "mixed", "fault scenario")
    p.flag("count", 30, "number of samples to emit")
    p.flag("out", "artifacts/fault-replay/fault_samples.jsonl", "output JSONL path")
    p.flag("with-signals", False, "populate signal values from the fault profiles")
    p.flag("seed", 42, "seed for signal jitter (with --with-signals)")
    a = p.parse_args(argv)
    try:
        samples = generate_fault_samples(a.scenario, a.count, now_ns(), with_signals=a.with_signals, seed=a.seed)
    except ValueError as exc:
        eprint(f"failed to generate replay samples: {exc}")
        return 1
    ensure_parent(a.out)
    with open(a.out, "w", encoding="utf-8") as fh:
        for s in samples:
            fh.write(jsonl_line(s))
    print(f"wrote {len(samples)} replay samples to {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""`loadgen`: deterministic request trace JSONL (REF cmd/loadgen/main.go:32-103).

Same profiles, field names and value ranges (prompt class mix, retrieval_docs 2..9,
target_tokens 64..575, per-profile expected TTFT ranges); Go's math/rand stream is not
reproducible in Python, so the draws come from numpy PCG64 with the same seed.
"""

from __future__ import annotations

import json
import sys
from typing import List, Optional

import numpy as np

from ..utils.timeutil import SECOND, format_rfc3339_ns, now_ns
from ._common import GoFlags, eprint, ensure_parent, is_version_request, print_version

CLASSES = ("chat_short", "rag_medium", "context_long")
TTFT_RANGES = {"chat_short": (80, 70), "rag_medium": (140, 150), "context_long": (280, 250)}
DEFAULT_TTFT = (90, 220)


def prompt_class(profile: str, rng: np.random.Generator) -> str:
    if profile in ("chat_short", "rag_medium"):
        return profile
    return CLASSES[int(rng.integers(len(CLASSES)))]


def expected_ttft(profile: str, rng: np.random.Generator) -> int:
    lo, span = TTFT_RANGES.get(profile, DEFAULT_TTFT)
    return lo + int(rng.integers(span))


def generate(profile: str, duration_sec: int, rps: int, seed: int, start_ns: int):
    rng = np.random.default_rng(seed)
    for i in range(duration_sec * rps):
        yield {
            "timestamp": format_rfc3339_ns(start_ns + i * SECOND // rps),
            "profile": profile, "request_id": f"req-{i:06d}", "trace_id": f"trace-{i:06d}",
            "prompt_class": prompt_class(profile, rng), "retrieval_docs": 2 + int(rng.integers(8)),
            "target_tokens": 64 + int(rng.integers(512)), "expected_ttft_ms": expected_ttft(profile, rng),
        }


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    p = GoFlags("loadgen", "generate a deterministic request trace")
    p.flag("profile", "rag_mixed_20rps", "load profile")
    p.flag("duration-sec", 60, "generation duration in seconds")
    p.flag("rps", 20, "requests per second")
    p.flag("seed", 42, "deterministic seed")
    p.flag("out", "artifacts/loadgen/requests.jsonl", "output JSONL path")
    a = p.parse_args(argv)
    if a.duration_sec <= 0 or a.rps <= 0:
        eprint("duration-sec and rps must be > 0")
        return 1
    ensure_parent(a.out)
    n = 0
    with open(a.out, "w", encoding="utf-8") as fh:
        for ev in generate(a.profile, a.duration_sec, a.rps, a.seed, now_ns()):
            fh.write(json.dumps(ev) + "\n")
            n += 1
    print(f"wrote {n} requests to {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

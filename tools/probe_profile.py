"""Per-key-type cost split of the LDS join probe (join.hip k_probe) from its MISLO_PROBE_PROFILE
counters: work items, signals, staged span chunks and the clock64 cycles spent staging spans,
streaming signals and flushing candidates, summed over workgroups.

Needs the kernel-harness extension built with the counters (on the GPU box, into its scratch copy):

    MISLO_HIP_DEFINES=-DMISLO_PROBE_PROFILE python -c \\
        "from llm_slo_ebpf_toolkit_amd.ops import build; build.build_hip_ext(force=True)"
    python tools/probe_profile.py --events 2097152 --windows 4
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KEYS = ("trace", "pod+pid", "pod+conn", "svc+node")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1 << 21, help="rows per window (2 windows of rows = halo on)")
    ap.add_argument("--spans", type=int, default=16384)
    ap.add_argument("--windows", type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch

    from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes
    from llm_slo_ebpf_toolkit_amd.ops.engine import KernelHarness
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

    gen = ReplayGenerator(ReplayConfig(events_per_window=a.events, spans_per_window=a.spans, n_services=64))
    wins = [gen.next_window() for _ in range(a.windows)]
    h = KernelHarness(a.events, a.spans, 64)
    h.set_model(NaiveBayes.ref())
    prof_off = h.mod.PROBE_PROF_OFF
    acc = np.zeros((4, 8), dtype=np.uint64)
    for w in wins:
        h.process(w.events, w.spans, w.n_groups)
        torch.cuda.synchronize()
        work = h.eng.probe_work.cpu().numpy().view(np.uint32)
        acc += work[prof_off:prof_off + 64].view(np.uint64).reshape(4, 8)
        h.eng.probe_work.zero_()
    out = {}
    for k, name in enumerate(KEYS):
        items, sig, chunks, stage, sigc, flush, s1, s2 = (int(x) for x in acc[k, :8])
        out[name] = {"items": items, "signals": sig, "span_chunks": chunks, "stage_Mcycles": round(stage / 1e6, 2),
                     "signal_Mcycles": round(sigc / 1e6, 2), "flush_Mcycles": round(flush / 1e6, 2),
                     "stage_cycles_per_item": round(stage / max(items, 1)),
                     "signal_cycles_per_signal_per_wg": round(sigc / max(sig, 1), 1),
                     # thread 0's share of the signal loop, when the build counts it (round-5 variant
                     # builds): waiting for the next entry + its search, then the accounting
                     **({"search_Mcycles": round(s1 / 1e6, 2), "account_Mcycles": round(s2 / 1e6, 2)}
                        if s1 or s2 else {})}
    print(json.dumps({"windows": a.windows, "rows_per_window": a.events, "spans": a.spans, "per_key_type": out},
                     indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Diagnostic: is the window pipeline copy-bound, compute-bound or losing overlap?

Times, on one GPU and without a profiler, (1) the event H2D alone, (2) the captured window
kernel chain alone (graph replays on resident buffers), (3) both issued on their own streams
with no dependencies between them (the ideal overlap), and (4) the real pipeline (bench.py's
step). Prints one JSON line of microseconds per window.
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from llm_slo_ebpf_toolkit_amd.collector import records  # noqa: E402
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator  # noqa: E402
from llm_slo_ebpf_toolkit_amd.pipeline.window import WindowPipeline, WireStager  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1 << 20)
    ap.add_argument("--wire", type=int, default=16, choices=(16, 21, 24, 32),
                    help="16 = the epoch-tagged EVENT16 probe ring (4 epochs per window)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--buffers", type=int, default=3)
    a = ap.parse_args()
    cfg = ReplayConfig(scenario="full", events_per_window=a.events, spans_per_window=16384, n_services=64, seed=42)
    gen = ReplayGenerator(cfg)
    wins = [gen.next_window() for _ in range(2)]
    pipe = WindowPipeline(a.events, 16384, 64, 0, None, max_ahead=a.buffers, n_buffers=a.buffers)
    st = WireStager(torch, pipe, a.events, 16384, 64, wire=a.wire)
    if a.wire == 16:
        r16 = [st.probe_ring16(w.events, epoch_ns=256_000_000) for w in wins]
        ring, bases = [t for t, _ in r16], [b for _, b in r16]
    else:
        ring, bases = [st.probe_records(w.events) for w in wins], [None, None]
    pods = records.pod_table(np.concatenate([w.events for w in wins]), np.concatenate([w.spans for w in wins]))

    def stage(j):
        w = wins[j % 2]
        return st.stage(w.events, w.spans, w.n_groups, w.group_labels, w.group_domains, ev_pinned=ring[j % 2],
                        pod_table=pods, bases=bases[j % 2])

    for j in range(8):  # warm: graphs captured for both buffers
        pipe.submit(stage(j))
    pipe.drain()
    torch.cuda.synchronize()
    nb = a.events * records.wire_bytes(a.wire)
    cs, ks = pipe.copy_stream, pipe.compute_stream
    last = stage(0)
    pipe.submit(last)
    pipe.drain()

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(a.iters):
            fn(i)
        torch.cuda.synchronize()
        return 1e6 * (time.perf_counter() - t) / a.iters

    def copy_only(i):
        with torch.cuda.stream(cs):
            pipe.ev_dev[i % 2][:nb].copy_(ring[i % 2][:nb], non_blocking=True)

    def compute_only(i):
        with torch.cuda.stream(ks):
            pipe._run_window(0, last, True)

    def both(i):
        copy_only(i + 1)  # into the other buffer than the one computed on
        compute_only(i)

    res = {"copy_us": timed(copy_only), "compute_us": timed(compute_only), "both_independent_us": timed(both)}
    t = time.perf_counter()
    for j in range(a.iters):
        pipe.submit(stage(j))
    pipe.drain()
    torch.cuda.synchronize()
    res["pipeline_us"] = 1e6 * (time.perf_counter() - t) / a.iters
    print(json.dumps({"buffers": a.buffers, **{k: round(v, 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()

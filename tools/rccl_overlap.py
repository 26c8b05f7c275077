"""P3 evidence on a one-GPU box: the window engine with a one-rank RCCL communicator, windows
submitted back to back, so window k's collectives (comm stream) run while window k+1's kernels
(compute stream) do. SURVEY §2.4 P3: "RCCL all-reduce of window k overlapped with window k+1".

    # the run (under the kernel and RCCL API tracers)
    rocprofv3 --kernel-trace --rccl-trace --output-format csv -d gpurun_out/p3 -- python tools/rccl_overlap.py run
    # the summary (CPU): RCCL dispatches, how many overlap a later window's engine kernel, by how much
    python tools/rccl_overlap.py summary gpurun_out/p3 --out profiles/r5_rccl_p3/overlap.md

``run`` prefills the rings with every window first (the producer of bench.py runs ahead the
same way), then stages them back to back through RingWindowSource (3 buffers in flight), and
prints one JSON line: windows, ms per window, the engine's world.
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a) -> int:
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime per process: torch's)

    from llm_slo_ebpf_toolkit_amd.collector.records import framed_rows
    from llm_slo_ebpf_toolkit_amd.ops import load_agent, require_gpu_extension
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut, RingWindowSource, WindowPipeline, build_replay_images
    from llm_slo_ebpf_toolkit_amd.runtime import load

    require_gpu_extension()
    gen = ReplayGenerator(ReplayConfig(scenario="full", events_per_window=a.events, spans_per_window=a.spans,
                                       n_services=a.services, seed=a.seed, fault_hold=a.distinct))
    wins = [gen.next_window() for _ in range(a.distinct)]
    imgs = build_replay_images(wins)
    rt = load()
    tag = f"/mislo-p3-{os.getpid()}"
    win_bytes = max(len(i.framed) for i in imgs)
    ring_bytes = 1 << int(np.ceil(np.log2(win_bytes * (a.windows + 2))))
    rb = rt.Ringbuf.create_shm(tag + "-ev", ring_bytes)
    n_user = max(1, max(len(i.user) for i in imgs))
    user = rt.HostRing(1 << int(np.ceil(np.log2(n_user * (a.windows + 2)))), 64)
    spans = rt.HostRing(1 << int(np.ceil(np.log2(a.spans * (a.windows + 2)))), 64)
    comm = None if a.no_comm else (load_agent().unique_id(), 0, 1)
    sig_cap = max(framed_rows(i.framed) + len(i.user) for i in imgs)
    pipe = WindowPipeline(sig_cap, a.spans, a.services, 0, comm, model="bayes", learn=False, max_ahead=3, n_buffers=3,
                          user_cap=min(1 << int(np.ceil(np.log2(n_user))), sig_cap), halo_ms=2000.0,
                          import_cap=a.xchg, xchg_cap=a.xchg)
    src = RingWindowSource(pipe, rb, user, spans)
    sn = (gen.pod_svc.astype(np.uint32) << np.uint32(16)) | gen.pod_node.astype(np.uint32)
    pipe.eng.set_pods(gen.pod_ids.astype(np.uint32), sn)
    cuts = []
    for j in range(a.windows):  # the producer runs ahead: every window is in the rings first
        img = imgs[j % len(imgs)]
        assert rb.append_framed(img.framed)
        assert user.push(img.user) == len(img.user)
        assert spans.push(img.spans) == len(img.spans)
        cuts.append((Cut(kernel=rb.producer_pos, user=user.head, spans=spans.head, bases=img.bases), img))
    t0 = time.perf_counter()
    for c, img in cuts:
        src.stage(c, img.n_groups, img.labels)
    src.drain()
    dt = time.perf_counter() - t0
    e = pipe.eng
    last = a.windows - 1
    print(json.dumps({"windows": a.windows, "events_per_window": a.events, "ms_per_window": round(1e3 * dt / a.windows, 4),
                      "comm": comm is not None, "world": int(e.world), "xchg_cap": a.xchg,
                      "window_ms_dma_to_results_and_compute": [list(e.window_ms(k)) for k in range(last - 2, last + 1)],
                      "copy_ms": [list(e.copy_ms(k)) for k in range(last - 2, last + 1)],
                      "host_issue_us": round(e.host_issue_us, 1), "host_wait_us": round(e.host_wait_us, 1),
                      "host_dma_us": round(e.host_dma_issue_us, 1), "host_launch_us": round(e.host_launch_us, 1),
                      "host_pre_us": round(e.host_pre_us, 1), "host_tail_us": round(e.host_tail_us, 1),
                      "graphs": int(getattr(e, "graphs", -1))}), flush=True)
    pipe.eng.close()
    return 0


def load_trace(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Stream_Id", "?")))
    rows.sort()
    return rows


def load_rccl_api(d):
    """ncclAllReduce / ncclAllGather / ... calls from ``--rccl-trace`` (if it was on)."""
    import collections

    calls = collections.Counter()
    for path in glob.glob(os.path.join(d, "**", "*rccl_api_trace.csv"), recursive=True):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                calls[r.get("Function", r.get("Operation", "?"))] += 1
    return dict(calls)


def summary(a) -> int:
    """The comm stream is the one k_accumulate runs on (engine.hip: the packet accumulation behind
    the collectives), the compute stream the one k_probe runs on. Within a window the compute
    stream waits for the trace-row exchange; after the window's chain the comm stream runs its
    collectives while the compute stream moves on to the next window -- the overlap counted here."""
    rows = load_trace(a.dir)
    comm = {r[3] for r in rows if r[2].endswith("k_accumulate")}
    comp = {r[3] for r in rows if "k_probe<" in r[2] or r[2].endswith("k_probe")}
    cs = sorted(r for r in rows if r[3] in comm)
    cp = sorted(r for r in rows if r[3] in comp)
    hidden, busy, n_ov = 0, 0, 0
    j0 = 0
    for s, e, name, q in cs:
        busy += e - s
        while j0 < len(cp) and cp[j0][1] < s:
            j0 += 1
        ov = 0
        for s2, e2, _, _ in cp[j0:]:
            if s2 >= e:
                break
            ov += max(0, min(e, e2) - max(s, s2))
        hidden += min(ov, e - s)
        n_ov += ov > 0
    kinds = {}
    for s, e, name, q in cs:
        k = "rccl copy (one-rank collective)" if name.startswith("__amd_rocclr_copyBuffer") else name
        kinds[k] = kinds.get(k, 0) + 1
    # the window's DMAs (memory-copy trace) under the compute stream's kernels: window k+1's copy
    # running while window k computes
    copies = []
    for path in glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True):
        with open(path) as fh:
            copies += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(fh)
                       if "HOST_TO_DEVICE" in r.get("Direction", "")]
    copies.sort()
    c_busy = sum(e - s for s, e in copies)
    c_hidden = 0
    for s, e in copies:
        c_hidden += min(e - s, sum(max(0, min(e, e2) - max(s, s2)) for s2, e2, _, _ in cp if s2 < e and e2 > s))
    out = {"comm_stream": sorted(comm), "compute_stream": sorted(comp), "comm_stream_dispatches": len(cs),
           "comm_stream_dispatch_kinds": kinds, "comm_dispatches_overlapping_compute": n_ov,
           "comm_busy_us": round(busy / 1e3, 1), "comm_busy_hidden_under_compute_us": round(hidden / 1e3, 1),
           "hidden_fraction": round(hidden / busy, 4) if busy else None, "rccl_api_calls": load_rccl_api(a.dir),
           "h2d_copies": len(copies), "h2d_busy_us": round(c_busy / 1e3, 1),
           "h2d_busy_hidden_under_compute_us": round(c_hidden / 1e3, 1),
           "h2d_hidden_fraction": round(c_hidden / c_busy, 4) if c_busy else None}
    md = ["# P3: window k's collectives on the comm stream overlapping window k+1's kernels", "",
          "One-rank RCCL communicator (a one-GPU box), windows submitted back to back "
          "(`tools/rccl_overlap.py run` under `rocprofv3 --kernel-trace --rccl-trace`). RCCL runs a one-rank "
          "all-gather as a device copy kernel (`__amd_rocclr_copyBuffer`) on the stream it is given.", "",
          "```json", json.dumps(out, indent=2), "```", ""]
    text = "\n".join(md)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as fh:
            fh.write(text)
    print(json.dumps(out))
    return 0


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--windows", type=int, default=16)
    r.add_argument("--distinct", type=int, default=2)
    r.add_argument("--events", type=int, default=1 << 20)
    r.add_argument("--spans", type=int, default=16384)
    r.add_argument("--services", type=int, default=64)
    r.add_argument("--xchg", type=int, default=65536)
    r.add_argument("--seed", type=int, default=42)
    r.add_argument("--no-comm", action="store_true", help="no communicator (the one-GPU agent's engine)")
    s = sub.add_parser("summary")
    s.add_argument("dir")
    s.add_argument("--out", default="")
    a = ap.parse_args()
    return run(a) if a.cmd == "run" else summary(a)


if __name__ == "__main__":
    sys.exit(main())

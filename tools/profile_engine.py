"""rocprofv3 harness for the agent's window path: no PyTorch, no forked producer (the ring is
refilled in-process between windows, outside the engine's streams), so a profiler sees exactly
the native engine's DMAs and kernels.

    rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof -o run -- \\
        python tools/profile_engine.py --windows 12
"""

from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--windows", type=int, default=12)
    ap.add_argument("--events", type=int, default=1 << 20)
    ap.add_argument("--spans", type=int, default=16384)
    ap.add_argument("--services", type=int, default=64)
    ap.add_argument("--no-graphs", action="store_true")
    a = ap.parse_args()
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector.records import framed_rows
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut, RingWindowSource, WindowPipeline, build_replay_images
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    gen = ReplayGenerator(ReplayConfig(events_per_window=a.events, spans_per_window=a.spans, n_services=a.services))
    imgs = build_replay_images([gen.next_window() for _ in range(2)])
    n_user = max(len(i.user) for i in imgs)
    tag = f"/mislo-prof-{os.getpid()}"
    rb = rt.Ringbuf.create_shm(tag, 1 << 28)
    user = rt.HostRing(1 << int(np.ceil(np.log2(n_user * 4))), 64)
    spans = rt.HostRing(1 << int(np.ceil(np.log2(a.spans * 4))), 64)
    budget = max(framed_rows(i.framed) + len(i.user) for i in imgs)  # framed (events + definitions) + user
    pipe = WindowPipeline(budget, a.spans, a.services, 0, None, model="bayes_learned",
                          use_graphs=not a.no_graphs, user_cap=1 << int(np.ceil(np.log2(n_user))))
    pipe.eng.set_pods(gen.pod_ids.astype(np.uint32),
                      (gen.pod_svc.astype(np.uint32) << np.uint32(16)) | gen.pod_node.astype(np.uint32))
    src = RingWindowSource(pipe, rb, user, spans)
    t0 = time.perf_counter()
    for i in range(a.windows):
        img = imgs[i % 2]
        src.reap(keep=1)  # room in the rings for the next window
        while not rb.append_framed(img.framed, 8):
            src.reap(keep=0)
        user.push(img.user, 4)
        spans.push(img.spans)
        src.stage(Cut(rb.producer_pos, user.head, spans.head, img.bases), img.n_groups, img.labels)
    src.drain()
    dt = time.perf_counter() - t0
    s = pipe.summary()
    print(f"{a.windows} windows in {dt * 1e3:.1f} ms (ring refill in-process included); macro-F1 "
          f"{s['macro_f1']:.4f}; over budget {src.carried}; direct DMA {pipe.eng.direct_bytes / 1e6:.1f} MB, staged {pipe.eng.staged_bytes}",
          flush=True)
    pipe.eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())

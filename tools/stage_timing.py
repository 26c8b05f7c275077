"""Per-stage GPU timing of one replay window (diagnostic; not the headline bench)."""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes  # noqa: E402
from llm_slo_ebpf_toolkit_amd.ops.engine import GpuEngine  # noqa: E402
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1 << 20)
    ap.add_argument("--spans", type=int, default=16384)
    ap.add_argument("--services", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--wire", type=int, default=20, choices=(16, 20, 32, 64))
    ap.add_argument("--sort-ts", action="store_true", help="events in timestamp order (ring arrival order)")
    a = ap.parse_args()
    t = time.time()
    cfg = ReplayConfig(events_per_window=a.events, spans_per_window=a.spans, n_services=a.services)
    win = ReplayGenerator(cfg).next_window()
    print(f"gen {time.time() - t:.2f}s", flush=True)
    eng = GpuEngine(a.events, a.spans, a.services)
    eng.set_model(NaiveBayes.ref())
    ev, sp = win.events, win.spans
    if a.sort_ts:
        ev = ev[np.argsort(ev["ts_ns"], kind="stable")]
    if a.wire == 32:
        from llm_slo_ebpf_toolkit_amd.collector import records

        it = records.ConnInterner()
        eng.set_pod_table(records.pod_table(ev, sp))
        ev, sp = records.to_compact(ev, it), records.compact_spans(sp, it)
    t_base = 0
    if a.wire in (20, 16):
        from llm_slo_ebpf_toolkit_amd.collector import records

        enc = records.native_encoder()
        buf = np.zeros(ev.shape[0] * a.wire, dtype=np.uint8)
        t_base = enc.encode(ev, buf, a.wire)
        sp2 = np.zeros_like(sp)
        enc.encode_spans(sp, sp2, a.wire == 16)
        ev, sp = buf.view(records.WIRE_DTYPES[a.wire]), sp2
        eng.set_ctx_table(enc.ctx_table())
    eng.stage(ev, sp, win.n_groups, win.group_labels, t_base=t_base)
    eng.upload()
    torch.cuda.synchronize()
    e = eng.eng
    stages = {
        "reset": lambda: e.reset_window(),
        "decode": lambda: e.decode_wire(eng.ev_dev, a.wire),
        "join": lambda: e.join(eng.sp_dev, win.n_groups, None),
        "posterior": lambda: e.posterior(True),
        "stats": lambda: e.accumulate_stats(None),
        "pack": lambda: e.pack(),
    }
    times = {k: [] for k in stages}
    h2d = []
    for it in range(a.iters + 3):
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record()
        eng.upload()
        s1.record()
        torch.cuda.synchronize()
        if it >= 3:
            h2d.append(s0.elapsed_time(s1))
        for k, fn in stages.items():
            a0 = torch.cuda.Event(enable_timing=True)
            a1 = torch.cuda.Event(enable_timing=True)
            a0.record()
            fn()
            a1.record()
            torch.cuda.synchronize()
            if it >= 3:
                times[k].append(a0.elapsed_time(a1))
    res = {k: float(np.median(v)) for k, v in times.items()}
    res["h2d"] = float(np.median(h2d))
    tot = sum(v for k, v in res.items() if k != "h2d")
    res["total_ms"] = tot
    res["events_per_s_compute"] = a.events / (tot / 1e3)
    res["debug"] = eng.outputs().debug
    if os.environ.get("MISLO_HIP_DEFINES", "").find("MISLO_PROBE_PROFILE") >= 0:
        # probe cycle counters (diagnostic build): per key type, summed over every run
        pw = e.probe_work.cpu().numpy()
        pr = pw[4 + 4 * 1024 * 16:].view(np.uint64).reshape(4, 8).astype(np.float64)
        runs = a.iters + 3
        res["probe_profile"] = {
            name: {"items": pr[k, 0] / runs, "signals": pr[k, 1] / runs, "chunks": pr[k, 2] / runs,
                   "stage_kcyc_per_item": pr[k, 3] / max(pr[k, 0], 1) / 1e3,
                   "signal_kcyc_per_item": pr[k, 4] / max(pr[k, 0], 1) / 1e3,
                   "flush_kcyc_per_item": pr[k, 5] / max(pr[k, 0], 1) / 1e3}
            for k, name in enumerate(["trace", "pod_pid", "pod_conn", "svc_node"])}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

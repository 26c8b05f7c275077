"""The window source's handling of BPF ring records still being written at a cut (CPU engine:
the same busy-record stop and packet as the device, pipeline/cpu.py)."""

import os

import numpy as np

from llm_slo_ebpf_toolkit_amd.collector import records as R


def test_late_records_past_three_cuts_are_dropped_not_mis_stamped():
    """A record kept busy across cuts stops each window's decode there, so the tail behind it is
    re-submitted window after window. Its records carry the epoch tag of the window that first
    took them; from 3 windows later on that 2-bit tag names a newer epoch's base (a timestamp
    off by whole windows), so the source drops and counts them instead, and the ring moves on."""
    from llm_slo_ebpf_toolkit_amd.pipeline.window import Cut, RingWindowSource, WindowPipeline
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    rb = rt.Ringbuf.create_shm(f"/mislo-late-{os.getpid()}", 1 << 20)
    user, spans = rt.HostRing(1 << 10, 64), rt.HostRing(1 << 10, 64)
    pipe = WindowPipeline(4096, 64, 4, model="bayes", learn=False, user_cap=64, engine="cpu")
    src = RingWindowSource(pipe, rb, user, spans)
    base = 1_700_000_000_000_000_000
    rb.cfg_set(124, base)
    ev = np.zeros(300, dtype=R.EVENT)
    ev["signal_type"] = 1          # dns_latency_ms
    ev["value"] = 5_000_000
    ev["ts_ns"] = base + np.arange(300) * 1000
    sim = rt.ProbeSim(rb, R.milli_shift_table())
    sim.submit(ev[:100])
    rb.reserve(R.REC_PAYLOAD)      # a CPU's batch that is never finished (after 13 batches: 100 events)
    sim.submit(ev[101:200])
    hist = []
    for _ in range(5):
        k = src.stage(Cut(kernel=rb.producer_pos, user=0, spans=0, bases=(base, 0, 0, 0)), 4)["k"]
        src.reap(keep=0)
        hist.append(int(pipe.packet(k)["hist"].sum()))
    src.drain()
    # window 0 decodes the 100 events ahead of the busy batch; windows 1 and 2 re-submit the tail
    # (and stop at the busy batch again); window 3 would decode it 3 cuts late: dropped -- the
    # busy batch and the 13 batches behind it (99 events + 5 pads), in rows
    assert hist == [100, 0, 0, 0, 0], hist
    assert src.late_dropped == R.BATCH_SLOTS * (1 + 13) and not src.late
    assert rb.consumer_pos == rb.producer_pos

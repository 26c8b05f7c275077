"""Kernel -> agent ring path on the CPU: BPF ring buffer framing, the agent's compacting consumer,
the probe model, the agent's id tables and window assembly (REF pkg/collector/ringbuf.go:120-197
reads the same ring record by record; ringbuf_test.go:9-44 round-trips one record)."""

import mmap
import multiprocessing as mp
import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector import records as R
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator
from llm_slo_ebpf_toolkit_amd.runtime import load

rt = load()
PAGE = os.sysconf("SC_PAGE_SIZE")


def shm(tag: str, size: int):
    return rt.Ringbuf.create_shm(f"/mislo-test-{os.getpid()}-{tag}", size)


def window(seed=1, n=3000, s=200):
    cfg = ReplayConfig(scenario="full", n_nodes=2, pods_per_node=8, n_services=8, events_per_window=n,
                       spans_per_window=s, seed=seed)
    return ReplayGenerator(cfg).next_window()


def payload16(k: int, i: int):
    return np.array([i, 7 | ((i % 50) << 8), i * 3, k], dtype=np.uint32)


def batch(k: int, i: int):
    """Batch record i's 8 event slots (slot j carries event 8 i + j)."""
    return np.concatenate([payload16(k, 8 * i + j) for j in range(R.BATCH_SLOTS)])


RS = R.REC_STRIDE


def test_producer_writes_kernel_exact_framing():
    """reserve/commit/output lay records out exactly as kernel/bpf/ringbuf.c does: 8-byte
    header {len | busy, pg_off}, payload, 8-byte rounding; commit clears busy, discard sets it."""
    rb = shm("frame", 4 * PAGE)
    a = rb.reserve(R.REC_PAYLOAD)
    rb.write(a, batch(1, 0))
    b = rb.reserve(5)                   # 5 bytes -> 16-byte record (8 + 5 rounded up)
    rb.write(b, np.frombuffer(b"hello", dtype=np.uint8))
    c = rb.reserve(R.REC_PAYLOAD)
    data = rb.data_view()
    hdr = lambda off: data[off:off + 8].view(np.uint32)  # noqa: E731
    assert tuple(hdr(0)) == (R.REC_PAYLOAD | R.RB_BUSY, 3)  # data page 3 of the kernel's rb struct
    assert tuple(hdr(RS)) == (5 | R.RB_BUSY, 3)
    assert rb.producer_pos == RS + 16 + RS
    rb.commit(a)
    rb.commit(b, discard=True)
    assert tuple(hdr(0)) == (R.REC_PAYLOAD, 3)
    assert tuple(hdr(RS)) == (5 | R.RB_DISCARD, 3)
    # numpy model of the same bytes (the batch the test wrote) == the ring bytes
    exp = R.frame(batch(1, 0).view(R.EVENT16))
    exp[4:8] = np.array([3], dtype=np.uint32).view(np.uint8)
    np.testing.assert_array_equal(data[:RS], exp)
    ev, defs, disc, busy = R.unframe(data[:rb.producer_pos])
    assert len(ev) == R.BATCH_SLOTS and disc == 1 and busy  # c is still being written
    rb.commit(c)
    assert not R.unframe(data[:rb.producer_pos])[3]


def test_consumer_wraps_skips_discards_and_stops_at_busy():
    """Small ring, many laps: the consumer returns every committed 16-byte record once, in
    order, skips discards, never passes a busy record, and frees space as it goes."""
    rb = shm("wrap", 4 * PAGE)                # 16 KiB: 120 batch records per lap
    con = rt.RingbufConsumer(rb, 4)
    out = np.zeros((4096, 4), dtype=np.uint32)
    rng = np.random.default_rng(3)
    expect, got, seq = [], [], 0
    pending = []
    for lap in range(12):
        for _ in range(int(rng.integers(30, 90))):
            at = rb.reserve(R.REC_PAYLOAD)
            if at == 0:
                break
            p = batch(lap, seq)
            seq += 1
            rb.write(at, p)
            pending.append((at, p, rng.random() < 0.05))
        keep = int(rng.integers(0, 4))  # leave a few records busy at the tail
        for at, p, disc in pending[:len(pending) - keep]:
            rb.commit(at, disc)
            if not disc:
                expect += [tuple(r) for r in p.reshape(-1, 4)]
        pending = pending[len(pending) - keep:]
        st, defs = con.consume(out, out.shape[0])
        got += [tuple(r) for r in out[:st["events"]]]
        assert st["busy_stop"] == (keep > 0)
        assert rb.consumer_pos == st["end_pos"]
        assert len(defs) == 0
    for at, p, disc in pending:
        rb.commit(at, disc)
        if not disc:
            expect += [tuple(r) for r in p.reshape(-1, 4)]
    st, _ = con.consume(out, out.shape[0])
    got += [tuple(r) for r in out[:st["events"]]]
    assert got == expect
    assert rb.consumer_pos == rb.producer_pos
    assert rb.producer_pos > 4 * 4 * PAGE  # wrapped several times


def test_full_ring_drops_like_the_kernel():
    rb = shm("full", 4 * PAGE)
    n = 0
    while rb.output(batch(0, n)):
        n += 1
    assert n == (4 * PAGE - 1) // RS  # producer may run at most size - 1 bytes ahead
    assert rb.stats()["dropped"] == 1


def test_parallel_compaction_equals_serial_and_model():
    """Probe model -> framed image -> ring -> parallel consumer == serial consumer == numpy
    unframe of the model's bytes, definitions diverted in ring order."""
    w = window(seed=5, n=40000, s=500)
    cfg = np.zeros(128, dtype=np.uint64)
    cfg[R.ProbeModel.CFG_EPOCH] = (int(w.t0_ns) & ~3) | 1
    img = R.frame(R.ProbeModel(cfg).encode(w.events[:6000]))
    ev_ref, defs_ref, _, _ = R.unframe(img)
    assert len(defs_ref) > 50
    for threads in (1, 8):
        rb = shm(f"par{threads}", 1 << 20)
        assert rb.append_framed(img)
        out = np.zeros((16000, 4), dtype=np.uint32)
        st, defs = rt.RingbufConsumer(rb, threads).consume(out, 16000)
        assert st["pads"] > 0
        assert not st["serial"]
        np.testing.assert_array_equal(out[:st["events"]].view(R.EVENT16).reshape(-1), ev_ref)
        np.testing.assert_array_equal(defs.view(R.EVENT16).reshape(-1), defs_ref)


def test_foreign_record_size_takes_the_serial_walk():
    rb = shm("foreign", 1 << 16)
    for i in range(100):
        assert rb.output(batch(0, i))
    assert rb.output(np.zeros(32, dtype=np.uint8))  # another program's 32-byte record
    for i in range(100, 150):
        assert rb.output(batch(0, i))
    out = np.zeros((2048, 4), dtype=np.uint32)
    st, _ = rt.RingbufConsumer(rb, 8).consume(out, 2048)
    assert st["serial"] and st["foreign"] == 1 and st["events"] == 1200
    assert out[1199, 0] == 1199


def test_window_capacity_and_limit_leave_the_rest_queued():
    """Whole batches only: a window of 100 rows takes 12 batch records (96 events)."""
    rb = shm("cap", 1 << 16)
    for i in range(40):
        rb.output(batch(0, i))
    out = np.zeros((1000, 4), dtype=np.uint32)
    con = rt.RingbufConsumer(rb, 4)
    st, _ = con.consume(out, 100)                        # window capacity
    assert st["events"] == 96 and st["end_pos"] == 12 * RS
    st, _ = con.consume(out, 1000, limit=20 * RS)        # window cut
    assert st["events"] == 64 and out[0, 0] == 96
    st, _ = con.consume(out, 1000)
    assert st["events"] == 160 and out[159, 0] == 319


def test_native_probe_model_matches_numpy_model_and_floors():
    w = window(seed=7)
    rb = shm("sim", 1 << 20)
    base = (int(w.t0_ns) & ~3) | 2
    rb.cfg_set(rt.CFG_EPOCH, base)
    rb.cfg_set(2 + 3, 5_000_000)  # runqueue emit floor (the overhead guard raises floors)
    native = rt.ProbeSim(rb, R.milli_shift_table()).encode(w.events).view(R.EVENT16).reshape(-1)
    cfg = np.zeros(128, dtype=np.uint64)
    cfg[124], cfg[5] = base, 5_000_000
    ref = R.ProbeModel(cfg).encode(w.events)
    np.testing.assert_array_equal(native, ref)
    rq = (w.events["signal_type"] == 3) & (w.events["value"] < 5_000_000)
    assert rq.any()
    n_ev = int(((ref["ctx_type"] & 0xFF) < 0xF0).sum())
    assert n_ev == len(w.events) - int(rq.sum())


def test_probe_submit_through_ring_equals_encode():
    w = window(seed=9)
    a, b = shm("subA", 1 << 20), shm("subB", 1 << 20)
    for r in (a, b):
        r.cfg_set(rt.CFG_EPOCH, int(w.t0_ns) & ~3)
    rt.ProbeSim(a, R.milli_shift_table()).submit(w.events)
    img = rt.frame_records(rt.ProbeSim(b, R.milli_shift_table()).encode(w.events))
    n = a.producer_pos
    data = a.data_view()[:n].copy()
    # pg_off differs by position; everything else is byte-identical
    hdr = data.view(np.uint32).reshape(-1, RS // 4)
    assert (hdr[:, 1] == 3 + (np.arange(hdr.shape[0]) * RS) // PAGE).all()
    hdr[:, 1] = 0
    np.testing.assert_array_equal(data, img)


def test_epoch_tags_decode_records_written_across_cuts():
    """One epoch per window cut; records stamped up to 3 cuts late decode exactly."""
    w = window(seed=11, n=2000)
    clock = R.EpochClock()
    cfg = np.zeros(128, dtype=np.uint64)
    model = R.ProbeModel(cfg, cpus=1)  # one CPU: the slots keep the input order
    ev = w.events.copy()
    ev = ev[np.argsort(ev["ts_ns"])]
    cuts = [int(ev["ts_ns"][0]) + j * 200_000_000 for j in range(5)]
    parts = []
    for j, c in enumerate(cuts):  # records with ts in [cut j, cut j+1) are stamped with epoch j
        cfg[124] = clock.publish(c)
        hi = cuts[j + 1] if j + 1 < len(cuts) else 1 << 62
        parts.append(model.encode(ev[(ev["ts_ns"] >= c) & (ev["ts_ns"] < hi)]))
    enc = np.concatenate(parts)
    events = enc[(enc["ctx_type"] & 0xFF) < 0xF0]
    tags = set((events["trace_id"] >> np.uint32(30)).tolist())
    assert len(tags) == 4
    tab = R.HostEncoderModel()
    tab.apply_defs(enc[(enc["ctx_type"] & 0xFF) >= 0xF0])
    ids, rows = tab.take_rows()
    d = oracle.decode_w16(events, oracle.CtxTable(ids, rows), clock.bases())
    in_range = ev[ev["ts_ns"] >= cuts[0]]
    # epoch 0's base was overwritten by epoch 4 (same tag): those records are > 3 cuts late
    late = in_range["ts_ns"] < cuts[1]
    np.testing.assert_array_equal(d.ts[~late], in_range["ts_ns"][~late])


def test_agent_tables_match_model_and_rows_follow_pod_metadata():
    w = window(seed=13)
    cfg = np.zeros(128, dtype=np.uint64)
    cfg[124] = int(w.t0_ns) & ~3
    enc = R.ProbeModel(cfg).encode(w.events)
    defs = enc[(enc["ctx_type"] & 0xFF) >= 0xF0]
    nat, ref = R.native_tables(), R.HostEncoderModel()
    pods = np.unique(w.events["pod_id"])
    for t in (nat, ref):
        for p in pods[: len(pods) // 2]:
            t.set_pod(int(p), 0x00010001 * (int(p) % 7 + 1))
        t.apply_defs(defs)
        for p in pods[len(pods) // 2:]:   # metadata arriving after the definitions
            t.set_pod(int(p), 0x00010001 * (int(p) % 7 + 1))
    bases = [int(w.t0_ns), int(w.t0_ns) + 400_000_000, 0, int(w.t0_ns) - 1_000_000_000]
    np.testing.assert_array_equal(nat.encode_events(w.events, bases).view(R.EVENT16).reshape(-1),
                                  ref.encode_events(w.events, bases))
    np.testing.assert_array_equal(nat.encode_spans(w.spans).view(R.SPAN20), ref.encode_spans(w.spans))
    a_ids, a_rows = nat.take_rows(1 << 20)
    b_ids, b_rows = ref.take_rows()
    np.testing.assert_array_equal(a_ids, b_ids)
    np.testing.assert_array_equal(a_rows, b_rows)
    assert (a_ids[a_ids < R.KERNEL_CTX_LIMIT] > 0).all() and (a_ids >= R.KERNEL_CTX_LIMIT).any()
    # kernel trace definitions win over host-assigned ids
    tr = 0x1234567890ABCDEF  # a trace no kernel event carried
    host_id = nat.trace_id(tr)
    assert host_id >= R.KERNEL_TRACE_LIMIT
    nat.apply_defs(np.array([[77, R.DEF_TRACE, tr & 0xFFFFFFFF, tr >> 32]], dtype=np.uint32))
    assert nat.trace_id(tr) == 77


def test_event16_path_preserves_the_join_of_the_64_byte_originals():
    """Kernel path (probe model -> ring -> compaction -> tables) + host path (user-space
    records, spans): the decoded window equals the 64-byte originals on every join key, and
    the oracle join gives the same tiers / debug counters as on the originals."""
    w = window(seed=15, n=4000, s=256)
    from llm_slo_ebpf_toolkit_amd.pipeline.window import kernel_event_mask

    km = kernel_event_mask(w.events)
    cfg = np.zeros(128, dtype=np.uint64)
    clock = R.EpochClock()
    cfg[124] = clock.publish(int(w.events["ts_ns"].min()) - 10)
    enc = R.ProbeModel(cfg, cpus=1).encode(w.events[km])  # one CPU: row order = event order
    tab = R.HostEncoderModel()
    for p, sn in zip(w.events["pod_id"], (w.events["svc_id"].astype(np.uint32) << 16) | w.events["node_id"]):
        tab.set_pod(int(p), int(sn))
    tab.apply_defs(enc[(enc["ctx_type"] & 0xFF) >= 0xF0])
    k16 = enc[(enc["ctx_type"] & 0xFF) < 0xF0]
    u16 = tab.encode_events(w.events[~km], clock.bases())
    sp20 = tab.encode_spans(w.spans)
    ids, rows = tab.take_rows()
    table = oracle.CtxTable(ids, rows)
    d = oracle.decode_w16(np.concatenate([k16, u16]), table, clock.bases())
    orig = np.concatenate([w.events[km], w.events[~km]])
    o = oracle.decode_events(orig)
    np.testing.assert_array_equal(d.ts, o.ts)
    np.testing.assert_array_equal(d.pod, o.pod)
    np.testing.assert_array_equal(d.pid, o.pid)
    np.testing.assert_array_equal(d.svcnode, o.svcnode)
    np.testing.assert_array_equal(d.conn, R.conn32_np(o.conn).astype(np.uint64))
    np.testing.assert_array_equal(d.slot, o.slot)
    spans = oracle.decode_span20(sp20, table)
    a = oracle.join(d, spans, w.n_groups)
    ref_spans = w.spans.copy()
    ref_spans["conn_h"] = R.conn32_np(ref_spans["conn_h"])
    o.conn = R.conn32_np(o.conn).astype(np.uint64)
    o.trace = d.trace  # interned ids are a bijection of the hashes within the window
    ref_spans["trace_h"] = sp20["trace_id"]
    b = oracle.join(o, ref_spans, w.n_groups)
    assert a.debug == b.debug
    np.testing.assert_array_equal(a.top3, b.top3)
    np.testing.assert_array_equal(a.cnt, b.cnt)


def test_assembler_fills_the_slot_layout():
    w = window(seed=17, n=3000, s=150)
    from llm_slo_ebpf_toolkit_amd.pipeline.window import build_replay_images

    img = build_replay_images([w])[0]
    rb = shm("asm", 1 << 20)
    user = rt.HostRing(1 << 12, 64)
    spans = rt.HostRing(1 << 10, 64)
    assert rb.append_framed(img.framed)
    user.push(img.user)
    spans.push(img.spans)
    tables = R.native_tables()
    con = rt.RingbufConsumer(rb, 4)
    asm = rt.WindowAssembler(64, 512, 8192, 4096, tables, con, user, spans)
    L = asm.layout
    slot = np.zeros(L["bytes"], dtype=np.uint8)
    r = asm.assemble(slot.ctypes.data, list(img.bases), w.n_groups, img.labels)
    assert r["n_kernel"] == img.n_kernel and r["n_user"] == len(img.user) and r["n_spans"] == w.n_spans
    assert r["n_rows"] > 0 and r["rows_deferred"] == 0
    c = slot[:64].view(np.int32)
    assert c[0] == r["n_events"] and c[1] == w.n_spans and c[2] == w.n_groups and c[7] == 20 and c[14] == r["n_rows"]
    b0 = int(c[4].view(np.uint32)) | (int(c[5].view(np.uint32)) << 32)
    assert b0 == img.bases[0]
    np.testing.assert_array_equal(slot[64:64 + 4 * w.n_groups].view(np.int32), img.labels)
    ev = slot[L["ev_off"]:L["ev_off"] + 16 * r["n_events"]].view(R.EVENT16)
    ref_ev, _, _, _ = R.unframe(img.framed)
    np.testing.assert_array_equal(ev[: r["n_kernel"]], ref_ev)
    p = L["ev_off"] + 16 * r["n_events"]
    ids = slot[p:p + 4 * r["n_rows"]].view(np.uint32)
    assert len(set(ids.tolist())) == r["n_rows"]
    assert r["dma_bytes"] == p + ((4 * r["n_rows"] + 15) // 16) * 16 + 16 * r["n_rows"]
    assert rb.consumer_pos == rb.producer_pos and user.size == 0 and spans.size == 0


def _producer(name: str, k: int, n: int) -> None:
    r = load().Ringbuf.attach_shm(name)
    i = 0
    while i < n:  # batch records of 8 events
        if r.output(np.array([[i + j, 7, k, 0xC0FFEE] for j in range(8)], dtype=np.uint32)):
            i += 8


def test_multiprocess_producers_exactly_once():
    """4 producer processes racing on one ring (the kernel's per-CPU programs), one consumer:
    every record arrives exactly once and per-producer order is kept."""
    name = f"/mislo-test-{os.getpid()}-mp"
    rb = rt.Ringbuf.create_shm(name, 1 << 14)
    n = 20000
    ctx = mp.get_context("fork")
    procs = [ctx.Process(target=_producer, args=(name, k, n)) for k in range(4)]
    for p in procs:
        p.start()
    con = rt.RingbufConsumer(rb, 4)
    out = np.zeros((4096, 4), dtype=np.uint32)
    seen = {k: [] for k in range(4)}
    total = 0
    import time

    deadline = time.time() + 60
    while total < 4 * n and time.time() < deadline:
        st, _ = con.consume(out, out.shape[0])
        for row in out[: st["events"]]:
            seen[int(row[2])].append(int(row[0]))
        total += st["events"]
    for p in procs:
        p.join(10)
    assert total == 4 * n
    for k in range(4):
        assert seen[k] == list(range(n))


def test_host_ring_takes_over_a_lock_left_by_a_dead_producer():
    name = f"/mislo-test-{os.getpid()}-lock"
    ring = rt.HostRing(64, 64, name)
    ctx = mp.get_context("fork")
    p = ctx.Process(target=lambda: None)
    p.start()
    p.join()
    with open("/dev/shm" + name, "r+b") as fh:  # the lock word (RingHeader.lock, offset 192)
        m = mmap.mmap(fh.fileno(), 4096)
        m[192:196] = np.array([p.pid], dtype=np.uint32).tobytes()
        m.close()
    assert ring.push(np.zeros(64, dtype=np.uint8)) == 1
    assert ring.stats()["stolen"] == 1 and ring.size == 1

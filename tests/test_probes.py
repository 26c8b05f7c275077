"""Probe sources: record layout shared with the ring / GPU decoder, and every catalogue
signal has a producer whose program names exist in its source."""

import os
import re
import shutil
import subprocess

import pytest

from llm_slo_ebpf_toolkit_amd.probes import EBPF_DIR, PROBES
from llm_slo_ebpf_toolkit_amd.signals import catalog


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs a host C compiler")
def test_bpf_record_layout_matches_event_dtype(tmp_path):
    exe = tmp_path / "layout_check"
    subprocess.run(["gcc", "-Wall", "-I", EBPF_DIR, "-o", str(exe), os.path.join(EBPF_DIR, "layout_check.c")],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    # the in-kernel fixed-point rule (mislo_milli) == records.milli_int
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector import records

    rows = [tuple(int(x) for x in ln.split()[1:]) for ln in out.stdout.splitlines() if ln.startswith("milli ")]
    assert len(rows) == 52
    t, v, m = (np.array(c, dtype=np.uint64) for c in zip(*rows))
    shift = records.milli_shift_table()[t.astype(np.int64)]
    np.testing.assert_array_equal(records.milli_int(v, shift), m.astype(np.uint32))
    lines = out.stdout.splitlines()
    const = [int(x) for x in next(ln for ln in lines if ln.startswith("const ")).split()[1:]]
    assert const == [records.DEF_FIRST, records.DEF_TRACE, records.DEF_CTX, records.KERNEL_CTX_LIMIT,
                     records.KERNEL_TRACE_LIMIT]
    for ln in lines:
        if ln.startswith("conn32 "):
            k, c = (int(x) for x in ln.split()[1:])
            assert records.conn32(k) == c, ln
        if ln.startswith("trace "):
            f, v = (int(x) for x in ln.split()[1:])
            assert v == f % (records.KERNEL_TRACE_LIMIT - 1) + 1, ln


HOST_DIR = os.path.join(EBPF_DIR, "host")


@pytest.fixture(scope="module")
def probe_host(tmp_path_factory):
    """mislo_probe.h compiled for the host against in-process maps (probes/ebpf/host)."""
    if shutil.which("gcc") is None:
        pytest.skip("needs a host C compiler")
    exe = tmp_path_factory.mktemp("probe_host") / "probe_host"
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", HOST_DIR, "-I", EBPF_DIR, "-o", str(exe),
                    os.path.join(HOST_DIR, "probe_host.c")], check=True)
    return str(exe)


def _run_host(exe, tmp_path, events, *args):
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    events.tofile(fin)
    r = subprocess.run([exe, str(fin), str(fout), *map(str, args)], capture_output=True, text=True, check=True)
    import numpy as np

    stats = dict(zip(r.stdout.split()[::2], (int(x) for x in r.stdout.split()[1::2])))
    return np.fromfile(fout, dtype=np.uint32).reshape(-1, 4), stats


def _probe_events(n=3000, seed=5):
    """Replay events plus hand-made ones: explicit connection hashes, port-derived
    connections, traces shared across pods, zero timestamps, values under a floor."""
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

    w = ReplayGenerator(ReplayConfig(scenario="full", events_per_window=n, spans_per_window=64, n_services=8,
                                     seed=seed)).next_window()
    ev = np.ascontiguousarray(w.events)
    extra = np.zeros(64, dtype=records.EVENT)
    rng = np.random.default_rng(seed)
    extra["ts_ns"] = int(w.t0_ns) + rng.integers(0, 10**9, 64)
    extra["ts_ns"][::9] = 0
    extra["signal_type"] = rng.choice([1, 2, 4, 9], 64)
    extra["value"] = rng.integers(0, 5_000_000, 64)
    extra["pod_id"] = rng.integers(0, 4, 64)
    extra["pid"] = rng.integers(0, 3, 64)
    extra["src_port"] = rng.integers(0, 3, 64) * 40000
    extra["dst_port"] = 443
    extra["dst_ip"] = 0x0A000001
    extra["conn_h"][::5] = 0xDEADBEEF00000001
    extra["trace_h"][::2] = rng.choice(np.array([0x1111, 0x2222, 0xFFFFFFFFFFFFFFFF], dtype=np.uint64), 32)
    return np.concatenate([ev, extra])


def _probesim_records(events, cuts, cfg):
    """ProbeSim.encode over ``events`` with the epoch published at each (index, value) cut."""
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    rb = rt.Ringbuf.create_shm(f"/mislo-ph-{os.getpid()}-{len(events)}", 1 << 16)
    for i, v in cfg.items():
        rb.cfg_set(i, v)
    sim = rt.ProbeSim(rb, records.milli_shift_table(), 1 << 20)
    out, lo = [], 0
    for idx, val in list(cuts) + [(len(events), None)]:
        if idx > lo:
            out.append(sim.encode(np.ascontiguousarray(events[lo:idx])).reshape(-1, 4))
            lo = idx
        if val is not None:
            rb.cfg_set(124, val)
    return np.concatenate(out), rb


def test_probe_c_plumbing_matches_probesim(probe_host, tmp_path):
    """The BPF C that runs in the kernel (mislo_probe.h mislo_emit -> mislo_submit, compiled
    for the host) writes the same ring records as ProbeSim (the producer model the replay,
    the bench and the GPU tests drive): definitions ahead of first uses, context / trace ids,
    epoch offsets and tags across cuts, floors, and both id spaces' wrap / exhaustion."""
    import numpy as np

    ev = _probe_events()
    t0 = int(ev["ts_ns"][ev["ts_ns"] > 0].min())
    cuts = [(0, (t0 - 10**6) & ~3 | 1), (1000, (t0 + 3 * 10**8) & ~3 | 2), (2500, (t0 + 6 * 10**8) & ~3 | 3)]
    floors = {2 + 9: 2_000_000}  # syscall_latency below 2 ms stays in the kernel
    for trace_next, ctx_next in ((0, 0), ((1 << 24) - 40, (1 << 23) - 30)):
        args = ["--trace-next", trace_next, "--ctx-next", ctx_next, "--floor", "9:2000000"]
        for idx, val in cuts:
            args += ["--epoch-at", f"{idx}:{val}"]
        got, stats = _run_host(probe_host, tmp_path, ev, *args)
        ref, rb = _probesim_records(ev, cuts, {125: trace_next, 126: ctx_next, **floors})
        np.testing.assert_array_equal(got, ref)
        assert stats["trace_next"] == rb.cfg_get(125) and stats["ctx_next"] == rb.cfg_get(126)
        types = got[:, 1] & 0xFF
        assert (types == 0xFE).any() and (types == 0xFD).any()
        if ctx_next:  # the context space ran out: later new contexts carry id 0
            assert stats["ctx_next"] > (1 << 23) and ((got[:, 1] >> 8)[types < 0xF0] == 0).any()
            assert ((got[:, 0][types == 0xFD]) < 100).any()  # trace ids wrapped to the bottom


def test_probe_c_full_ring_matches_probesim(probe_host, tmp_path):
    """Ring full: bpf_ringbuf_output fails from the same record on in the C and in ProbeSim
    (a definition that does not fit leaves its id unassigned; the counters still advance)."""
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.runtime import load

    ev = _probe_events(n=600, seed=9)
    epoch = int(ev["ts_ns"][ev["ts_ns"] > 0].min()) & ~3
    rt = load()
    rb = rt.Ringbuf.create_shm(f"/mislo-phf-{os.getpid()}", 1 << 12)
    rb.cfg_set(124, epoch)
    RS = records.REC_STRIDE
    cap = rb.size // RS  # batch records
    got, stats = _run_host(probe_host, tmp_path, ev, "--epoch-at", f"0:{epoch}", "--ring-cap", cap)
    sim = rt.ProbeSim(rb, records.milli_shift_table(), 1 << 20)
    sim.submit(ev)
    n = rb.producer_pos // RS
    assert n == cap == len(got) // records.BATCH_SLOTS and sim.dropped > 0
    ring = rb.data_view()[: n * RS].view(np.uint32).reshape(-1, RS // 4)
    np.testing.assert_array_equal(ring[:, 2:].reshape(-1, 4), got)
    assert stats["trace_next"] == rb.cfg_get(125) and stats["ctx_next"] == rb.cfg_get(126)


def test_record_enum_matches_catalogue():
    src = open(os.path.join(EBPF_DIR, "mislo_record.h")).read()
    enum = {int(v): k for k, v in re.findall(r"MISLO_(\w+) = (\d+)", src)}
    for s in catalog.SIGNALS:
        assert s.kernel_type in enum, s.name
    assert catalog.HELLO_TYPE in enum


def test_every_signal_has_a_producer():
    for s in catalog.SIGNALS:
        assert s.name in PROBES, s.name
    for sig, (kind, obj, progs) in PROBES.items():
        if "bpf" not in kind:
            continue
        src = open(os.path.join(EBPF_DIR, obj + ".bpf.c")).read()
        for p in progs:
            assert re.search(rf"\b{p}\b\s*[(,)]", src), (sig, obj, p)
        assert 'SEC("license")' in src


def _resolve(rows):
    """Ring records -> the events they mean, ids resolved through the definitions ahead of them
    (what the GPU's k_ring_defs + decode recover): (ts_off, tag, type, value_milli, pod, pid,
    conn32, trace hash) per event, in ring order."""
    ctx, tr, out = {}, {}, []
    for a, tag_id, b, c in rows.tolist():
        t = tag_id & 0xFF
        if t == 0xFE:
            ctx[tag_id >> 8] = (b, c, a)
        elif t == 0xFD:
            tr[a] = b | (c << 32)
        elif t == 0xFC:  # a pad: the unused slot of a batch flushed before it filled
            continue
        else:
            pod, pid, c32 = ctx.get(tag_id >> 8, (0, 0, 0))
            tid = c & ((1 << 30) - 1)
            out.append((a, c >> 30, t, b, pod, pid, c32, tr.get(tid, 0) if tid else 0))
    return out


def test_probe_c_split_rings_route_every_record_with_its_definitions(probe_host, tmp_path):
    """Split rings (agent --gpus N): with mislo_shards routing pods to rings 1..3, every record
    goes to its pod's ring and each ring carries the context and trace definitions its own
    records use -- the same events, ring by ring, as a ProbeSim per ring fed its shard's records
    (what the replay producer and the bench drive)."""
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.runtime import load

    ev = _probe_events(n=2000, seed=13)
    t0 = int(ev["ts_ns"][ev["ts_ns"] > 0].min())
    epoch = (t0 - 10**6) & ~3 | 1
    pods = sorted(set(ev["pod_id"].tolist()) - {0})
    shard = {p: (i % 4) for i, p in enumerate(pods)}  # pod -> ring 0..3 (pod 0: unrouted -> 0)
    args = ["--epoch-at", f"0:{epoch}"]
    for p, s in shard.items():
        args += ["--shard", f"{p}:{s}"]
    got0, _ = _run_host(probe_host, tmp_path, ev, *args)
    rt = load()
    sh = np.array([shard.get(int(p), 0) for p in ev["pod_id"].tolist()])
    for s in range(4):
        got = got0 if s == 0 else np.fromfile(tmp_path / f"out.bin.{s}", dtype=np.uint32).reshape(-1, 4)
        rb = rt.Ringbuf.create_shm(f"/mislo-phs-{os.getpid()}-{s}", 1 << 18)
        rb.cfg_set(124, epoch)
        sim = rt.ProbeSim(rb, records.milli_shift_table(), 1 << 20)
        ref = sim.encode(np.ascontiguousarray(ev[sh == s])).reshape(-1, 4)
        a, b = _resolve(got), _resolve(ref)
        assert len(a) == int((sh == s).sum()) > 0 and a == b, s


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs a host C compiler")
def test_hip_and_rocr_wait_accounting_c_matches_its_rules(tmp_path):
    """gpu_kfd.bpf.c's uprobes on hipMemcpy(Async) (entry + return) and on ROCr's
    hsa_signal_wait_scacquire / _relaxed time the calls per process (mislo_gpu_act.h, compiled
    for the host as the kernel runs it): nested calls of different kinds each count, the same
    kind re-entered on a thread keeps the outer start, a return without an entry is ignored,
    threads of one process add up."""
    import random

    exe = tmp_path / "gpu_act_host"
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", EBPF_DIR, "-o", str(exe),
                    os.path.join(HOST_DIR, "gpu_act_host.c")], check=True)
    rng = random.Random(3)
    lines, now = [], 1000
    model = {}  # tgid -> [launches, copies, last, sync_ns, syncs, copy_ns, wait_ns, waits]
    open_ = {}  # (tgid, tid, kind) -> start
    for _ in range(3000):
        now += rng.randint(1, 5000)
        tgid, tid = rng.choice([(7, 70), (7, 71), (9, 90)])
        op = rng.random()
        m = model.setdefault(tgid, [0] * 8)
        if op < 0.2:
            copy = rng.randint(0, 1)
            lines.append(f"SUBMIT {copy} {tgid} {tid} {now}")
            m[1 if copy else 0] += 1
            m[2] = now
        elif op < 0.6:
            kind = rng.randint(0, 2)
            lines.append(f"ENTER {kind} {tgid} {tid} {now}")
            open_.setdefault((tgid, tid, kind), now)  # BPF_NOEXIST: the outer call's start stays
        else:
            kind = rng.randint(0, 2)
            lines.append(f"EXIT {kind} {tgid} {tid} {now}")
            t0 = open_.pop((tgid, tid, kind), None)
            if t0 is None:
                continue  # no entry seen
            dt = now - t0
            if kind == 0:
                m[3] += dt
                m[4] += 1
            elif kind == 1:
                m[5] += dt
            else:
                m[6] += dt
                m[7] += 1
    out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True).stdout
    got = {int(r.split()[0]): [int(x) for x in r.split()[1:]] for r in out.strip().splitlines()}
    want = {t: v for t, v in model.items() if any(v)}
    assert got == want

"""The native unprivileged sampler (runtime/csrc/procsampler.cpp) against its Python model
(collector/procfs.py SchedstatSampler), on fake /proc and cgroup trees: run-queue delay per
timeslice, the CPU the process waited for (cpu_steal_pct), CFS bandwidth throttling of the quota
group (cgroup v2 and v1), PSI memory stall, shedding masks and the pause switch, and the records
it pushes into a user ring."""

import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector import procfs
from llm_slo_ebpf_toolkit_amd.collector import records as R
from llm_slo_ebpf_toolkit_amd.runtime import load

T0 = 1_760_000_000 * 10**9
M0 = 5 * 10**9


def schedstat(root, pid, tid, run, wait, slices):
    d = root / str(pid) / "task" / str(tid)
    d.mkdir(parents=True, exist_ok=True)
    (d / "schedstat").write_text(f"{run} {wait} {slices}\n")


def psi(path, total_us):
    path.write_text(f"some avg10=0.00 avg60=0.00 avg300=0.00 total={total_us}\nfull avg10=0.00 avg60=0.00 avg300=0.00 total=0\n")


def world(tmp_path, v1=False):
    """Two pods: pod 7's process (pid 100, two threads, NSpid 17) sits in a quota group; pod 9's
    (pid 200) in a group without one."""
    proc, cg = tmp_path / "proc", tmp_path / "cg"
    (proc / "pressure").mkdir(parents=True)
    psi(proc / "pressure" / "memory", 0)
    schedstat(proc, 100, 100, 10, 1_000, 1)
    schedstat(proc, 100, 101, 10, 1_000, 1)
    schedstat(proc, 200, 200, 10, 0, 1)
    (proc / "100" / "status").write_text("Name:\tpython\nNSpid:\t100\t17\n")
    (proc / "200" / "status").write_text("Name:\tsh\nNSpid:\t200\n")
    if v1:
        q = cg / "cpu,cpuacct" / "kubepods" / "pod7"
        (q / "c1").mkdir(parents=True)
        (q / "cpu.cfs_quota_us").write_text("50000\n")
        (q / "c1" / "cpu.cfs_quota_us").write_text("-1\n")
        (q / "cpu.stat").write_text("nr_periods 1\nnr_throttled 0\nthrottled_time 0\n")
        (proc / "100" / "cgroup").write_text("5:memory:/kubepods/pod7/c1\n3:cpu,cpuacct:/kubepods/pod7/c1\n")
        (proc / "200" / "cgroup").write_text("3:cpu,cpuacct:/other\n")
        (cg / "cpu,cpuacct" / "other").mkdir(parents=True)
    else:
        q = cg / "kubepods" / "pod7"
        (q / "c1").mkdir(parents=True)
        (q / "cpu.max").write_text("50000 100000\n")
        (q / "c1" / "cpu.max").write_text("max 100000\n")
        (q / "cpu.stat").write_text("usage_usec 5\nnr_throttled 0\nthrottled_usec 0\n")
        psi(q / "c1" / "memory.pressure", 0)
        psi(q / "c1" / "cpu.pressure", 0)
        (proc / "100" / "cgroup").write_text("0::/kubepods/pod7/c1\n")
        (cg / "other").mkdir()
        (proc / "200" / "cgroup").write_text("0::/other\n")
    return proc, cg, q


def advance(proc, q, v1=False):
    # pid 100: thread 100 waited 30 ms over 10 slices (3 ms each), thread 101 40 us over 2 slices
    schedstat(proc, 100, 100, 20, 1_000 + 30_000_000, 11)
    schedstat(proc, 100, 101, 20, 1_000 + 40_000, 3)
    schedstat(proc, 200, 200, 90, 0, 5)  # ran, never waited
    if v1:
        (q / "cpu.stat").write_text("nr_periods 2\nnr_throttled 1\nthrottled_time 45000000\n")
    else:
        (q / "cpu.stat").write_text("usage_usec 9\nnr_throttled 1\nthrottled_usec 45000\n")
        psi(q / "c1" / "memory.pressure", 2_500)
        psi(q / "c1" / "cpu.pressure", 60_000)
    psi(proc / "pressure" / "memory", 900)


def model(proc, cg, targets, steal_sustain=1, **kw):
    return procfs.SchedstatSampler(lambda: dict(targets), lambda u: len(u), proc_root=str(proc), cgroup_root=str(cg),
                                   node_id=5, steal_sustain=steal_sustain, **kw)


def native(proc, cg, targets, ring=None, cpu_psi=False, steal_sustain=1):
    rt = load()
    s = rt.ProcSampler(ring, 5, str(proc), str(cg), cpu_psi, steal_sustain=steal_sustain)
    s.set_targets(dict(targets))
    return s


def nat_sample(s, now, mono):
    return np.frombuffer(s.tick(now, mono), dtype=R.EVENT)


@pytest.mark.parametrize("v1", [False, True])
def test_native_sampler_matches_the_model(tmp_path, v1):
    proc, cg, q = world(tmp_path, v1)
    targets = {100: 7, 200: 9}
    m, n = model(proc, cg, targets), native(proc, cg, targets)
    a, b = m.sample(T0, M0), nat_sample(n, T0, M0)
    assert len(a) == len(b) == 0  # first look primes every counter
    advance(proc, q, v1)
    a, b = m.sample(T0 + 10**8, M0 + 10**8), nat_sample(n, T0 + 10**8, M0 + 10**8)
    assert a.tobytes() == b.tobytes()
    got = {int(e["signal_type"]): (int(e["value"]), int(e["pid"]), int(e["tid"]), int(e["pod_id"]))
           for e in a if int(e["pod_id"]) == 7}
    # run-queue: only thread 100's waits reach the 100 us floor per slice -> 3 ms per slice
    assert got[procfs.RUNQUEUE_TYPE] == (3_000_000, 17, 100, 7)
    # steal: 30.04 ms of waiting over a 100 ms interval = 30.04 % of one CPU (milli-percent)
    assert got[procfs.STEAL_TYPE] == (30_040, 17, 100, 7)
    # CFS: the quota group (the pod, not the container) throttled 45 ms
    assert got[procfs.CFS_TYPE] == (45_000_000, 17, 100, 7)
    if v1:  # node PSI (v1 groups have no memory.pressure)
        assert got[procfs.MEM_RECLAIM_TYPE] == (900_000, 17, 100, 7)
    else:   # the container group's PSI wins over the node's
        assert got[procfs.MEM_RECLAIM_TYPE] == (2_500_000, 17, 100, 7)
    # pod 9 ran unhindered: only the node's memory stall (its group has no PSI file of its own)
    assert [(int(e["signal_type"]), int(e["value"])) for e in a if int(e["pod_id"]) == 9] == \
        [(procfs.MEM_RECLAIM_TYPE, 900_000)]
    assert (a["ts_ns"] == T0 + 10**8).all() and (a["node_id"] == 5).all()
    # a third interval with no change: nothing
    a, b = m.sample(T0 + 2 * 10**8, M0 + 2 * 10**8), nat_sample(n, T0 + 2 * 10**8, M0 + 2 * 10**8)
    assert len(a) == len(b) == 0
    st = n.stats()
    assert st["ticks"] == 3 and st["cfs_groups"] == 1 and st["runqueue_delay_ms"] == 1 and st["cpu_steal_pct"] == 1


def test_pod_cpu_pressure_raises_steal_when_enabled(tmp_path):
    proc, cg, q = world(tmp_path)
    targets = {100: 7}
    m, n = model(proc, cg, targets, cpu_psi=True), native(proc, cg, targets, cpu_psi=True)
    m.sample(T0, M0), nat_sample(n, T0, M0)
    advance(proc, q)
    a, b = m.sample(T0 + 10**8, M0 + 10**8), nat_sample(n, T0 + 10**8, M0 + 10**8)
    assert a.tobytes() == b.tobytes()
    steal = a[a["signal_type"] == procfs.STEAL_TYPE]
    assert int(steal["value"][0]) == 60_000  # the group stalled 60 ms of 100: above the process's own 30 %


def test_steal_needs_a_sustained_wait_share(tmp_path):
    """cpu_steal_pct comes out only once the wait share has held the floor for steal_sustain
    intervals in a row (a healthy service's threads cross it now and then, one interval at a
    time); an interval below the floor starts the count again. Model and native agree."""
    proc, cg, q = world(tmp_path)
    targets = {100: 7}
    m, n = model(proc, cg, targets, steal_sustain=3), native(proc, cg, targets, steal_sustain=3)
    m.sample(T0, M0), nat_sample(n, T0, M0)
    wait = [1_000]
    got = []
    for i, waited_ms in enumerate([30, 30, 0, 30, 30, 30, 40], start=1):
        wait[0] += waited_ms * 1_000_000
        schedstat(proc, 100, 100, 20, wait[0], 11 + i)
        t, mo = T0 + i * 10**8, M0 + i * 10**8
        a, b = m.sample(t, mo), nat_sample(n, t, mo)
        assert a.tobytes() == b.tobytes(), i
        got.append([int(e["value"]) for e in a if int(e["signal_type"]) == procfs.STEAL_TYPE])
    assert got == [[], [], [], [], [], [30_000], [40_000]], got


def test_shedding_mask_and_pause(tmp_path):
    proc, cg, q = world(tmp_path)
    targets = {100: 7}
    m, n = model(proc, cg, targets), native(proc, cg, targets)
    keep = procfs.ALL_MASK & ~(1 << procfs.STEAL_TYPE) & ~(1 << procfs.RUNQUEUE_TYPE)
    m.mask = n.mask = keep
    m.sample(T0, M0), nat_sample(n, T0, M0)
    advance(proc, q)
    a, b = m.sample(T0 + 10**8, M0 + 10**8), nat_sample(n, T0 + 10**8, M0 + 10**8)
    assert a.tobytes() == b.tobytes()
    assert sorted(int(t) for t in a["signal_type"]) == [procfs.MEM_RECLAIM_TYPE, procfs.CFS_TYPE]
    n.paused = True
    assert n.paused and n.mask == keep


@pytest.mark.parametrize("rec", [24, 32, 64])
def test_native_sampler_pushes_the_rings_record_format(tmp_path, rec):
    proc, cg, q = world(tmp_path)
    rt = load()
    ring = rt.HostRing(1024, rec, "", False)
    n = native(proc, cg, {100: 7}, ring=ring)
    nat_sample(n, T0, M0)
    advance(proc, q)
    ev = nat_sample(n, T0 + 10**8, M0 + 10**8)
    assert ring.size == len(ev) == 4
    raw = np.asarray(ring.records_view())[: len(ev) * rec].copy()
    want = R.to_user(ev.copy(), rec)
    assert raw.tobytes() == want.tobytes()
    assert n.stats()["emitted"] == 4


def test_native_sampler_thread_reads_this_process():
    """The sampler thread over the live /proc: this process with a thread kept runnable next to
    the main one reports without error; stop() joins."""
    import threading
    import time

    rt = load()
    ring = rt.HostRing(1 << 12, 24, "", False)
    s = procfs.NativeSampler(ring, lambda: {os.getpid(): 1}, refresh_s=0.05)
    s.start(0.01)
    stop = threading.Event()
    t = threading.Thread(target=lambda: [sum(range(1000)) for _ in iter(stop.is_set, True)])
    t.start()
    time.sleep(0.3)
    stop.set()
    t.join()
    s.stop()
    st = s.stats()
    assert st["ticks"] >= 5 and st["targets"] == 1 and st["dropped"] == 0
    assert st["max_tick_ns"] < 50_000_000  # a tick over one process is far below its interval


def test_ring_drop_mask_is_shared_with_attached_producers():
    rt = load()
    name = f"/mislo-dm-{os.getpid()}"
    owner = rt.HostRing(1024, 24, name, False)
    try:
        peer = rt.HostRing(0, 24, name, True)
        assert owner.drop_mask == 0
        owner.drop_mask = 1 << 13
        assert peer.drop_mask == 1 << 13
    finally:
        del owner


def test_steal_counts_only_while_neighbours_hold_the_pods_cpus(tmp_path):
    """A pod pinned to CPUs 0-1: a wait share at the floor counts only while other processes kept
    those CPUs busy (/proc/stat busy time less the pod's own on-CPU time, schedstat field 1): after
    a CPU fault, a pod working off its backlog waits behind its own threads (profiles/r4_config3_rerun:
    6 of 8 recovery windows read cpu_throttle). A pod on a large CPU set is not gated. Model and
    native agree record for record."""
    proc, cg, q = world(tmp_path)
    tck = os.sysconf("SC_CLK_TCK")
    (proc / "100" / "status").write_text("Name:\tpython\nNSpid:\t100\t17\nCpus_allowed_list:\t0-1\n")
    (proc / "200" / "status").write_text("Name:\tsh\nNSpid:\t200\nCpus_allowed_list:\t0-63\n")
    busy = [0] * 64

    def stat():
        lines = ["cpu  0 0 0 0 0 0 0 0 0 0"] + [f"cpu{c} {busy[c]} 0 0 1000 0 0 0 0 0 0" for c in range(64)]
        (proc / "stat").write_text("\n".join(lines) + "\nintr 0\n")

    stat()
    targets = {100: 7, 200: 9}
    m, n = model(proc, cg, targets), native(proc, cg, targets)
    m.sample(T0, M0), nat_sample(n, T0, M0)
    run, wait, run2, wait2 = 10, 1_000, 10, 0
    got = []
    # (pod 7's own on-CPU ms, CPU 0-1 busy ms each): neighbours held 70 %; then the pod alone
    for i, (own_ms, cpu_ms) in enumerate([(60, 100), (60, 100), (190, 100), (195, 100)], start=1):
        run += own_ms * 1_000_000
        wait += 30_000_000  # 30 % of one CPU waited every interval
        run2 += 1_000_000
        wait2 += 50_000_000  # pod 9 (64 CPUs): never gated
        schedstat(proc, 100, 100, run, wait, 10 * i + 1)
        schedstat(proc, 200, 200, run2, wait2, 10 * i + 1)
        for c in (0, 1):
            busy[c] += cpu_ms * tck // 1000
        stat()
        t, mo = T0 + i * 10**8, M0 + i * 10**8
        a, b = m.sample(t, mo), nat_sample(n, t, mo)
        assert a.tobytes() == b.tobytes(), i
        got.append({int(e["pod_id"]): int(e["value"]) for e in a if int(e["signal_type"]) == procfs.STEAL_TYPE})
    # /proc/stat is read only while a pinned pod waits at the floor: its first such interval has no
    # busy-time delta yet (unconfirmed), the second shows the neighbours, the last two only itself
    assert got == [{9: 50_000}, {7: 30_000, 9: 50_000}, {9: 50_000}, {9: 50_000}], got
    assert m.steal_gated == n.stats()["steal_gated"] == 3

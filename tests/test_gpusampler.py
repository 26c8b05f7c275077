"""The agent's native KFD sampler (runtime/csrc/gpusampler.h): other processes' wave occupancy of a
pod's GPU and the pod's queue evictions, read from a scripted /sys/class/kfd/kfd/proc tree, become
gpu_queue_delay_ms records of that pod. No GPU needed: the tree is plain files."""

import os

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.collector import records
from llm_slo_ebpf_toolkit_amd.runtime import load

rt = load()
DT = 500_000_000  # decision interval (ns)


class Kfd:
    """A KFD proc tree: kfd/<pid>/stats_<gpu>/{cu_occupancy,evicted_ms}, and /proc/<pid>/status
    with the process's pid in its own namespace."""

    def __init__(self, root):
        self.root = root
        self.kfd = str(root / "kfd")
        self.proc = str(root / "proc")
        os.makedirs(self.kfd, exist_ok=True)

    def proc_on(self, pid, gpus, ns_pid=None):
        for g in gpus:
            os.makedirs(f"{self.kfd}/{pid}/stats_{g}", exist_ok=True)
            self.occ(pid, g, 0)
            self.evicted(pid, g, 0)
        os.makedirs(f"{self.proc}/{pid}", exist_ok=True)
        with open(f"{self.proc}/{pid}/status", "w") as fh:
            fh.write(f"Name:\tpython\nPid:\t{pid}\nNSpid:\t{pid}" + (f"\t{ns_pid}" if ns_pid else "") + "\n")

    def occ(self, pid, gpu, v):
        with open(f"{self.kfd}/{pid}/stats_{gpu}/cu_occupancy", "w") as fh:
            fh.write(f"{v}\n")

    def evicted(self, pid, gpu, ms):
        with open(f"{self.kfd}/{pid}/stats_{gpu}/evicted_ms", "w") as fh:
            fh.write(f"{ms}\n")


def sampler(k, ring=None, **kw):
    return rt.GpuSampler(ring, node_id=3, kfd_proc=k.kfd, proc_root=k.proc, **kw)


def recs(raw):
    return np.frombuffer(raw, dtype=records.EVENT)


def test_other_processes_occupancy_of_the_pods_gpu_is_its_queue_delay(tmp_path):
    k = Kfd(tmp_path)
    k.proc_on(100, [7], ns_pid=12)      # the watched pod's process (pid 12 in its container)
    k.proc_on(200, [7])                 # another tenant on the same GPU
    k.proc_on(300, [9])                 # a process on another GPU: not the pod's contention
    s = sampler(k)
    s.set_target_list([(100, 5)])
    assert recs(s.decide(1_000_000_000, 10 * DT)).size == 0  # first decision: no interval yet
    k.occ(300, 9, 256)
    for i in range(10):
        k.occ(200, 7, 32 if i < 6 else 0)
        k.occ(100, 7, 4 if i % 2 else 0)   # the pod's own decode kernels, now and then
        s.sample()
    r = recs(s.decide(2_000_000_000, 11 * DT))
    assert r.size == 1
    e = r[0]
    assert (e["signal_type"], e["pod_id"], e["pid"], e["tid"], e["node_id"]) == (13, 5, 12, 100, 3)
    assert e["value"] == int(0.6 * DT) and e["flags"] == 1 << 8
    assert e["ts_ns"] == 2_000_000_000 - DT // 2
    (sh,) = s.shares()
    assert (sh["pod"], sh["gpu_id"], sh["samples"], sh["hot"], sh["own_hot"]) == (5, 7, 10, 6, 5)
    assert sh["foreign_mean"] == pytest.approx(32 * 6 / 10)
    st = s.stats()
    assert st["samples"] == 10 and st["decisions"] == 1 and st["emitted"] == 1


def test_an_idle_pod_is_not_contended_unless_its_hip_runtime_submitted_work(tmp_path):
    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    s = sampler(k)
    s.set_target_list([(100, 5)])
    s.set_hip_activity(100, launches=10)
    s.decide(0, DT)
    k.occ(200, 7, 64)
    for _ in range(5):
        s.sample()  # the pod's own occupancy reads 0 throughout (microsecond kernels between readings)
    assert recs(s.decide(0, 2 * DT)).size == 0 and not s.shares()[0]["active"]
    for _ in range(5):
        s.sample()
    s.set_hip_activity(100, launches=250, copies=3)  # hipLaunchKernel uprobes: it did run kernels
    r = recs(s.decide(0, 3 * DT))
    assert r.size == 1 and r[0]["value"] == DT and s.shares()[0]["active"]


def test_an_intervals_delay_is_stamped_over_its_sub_intervals(tmp_path):
    """``stamps``: the contended interval's delay split evenly over records at the sub-intervals'
    middles (a span's pod+pid join reaches 100 ms from its start); the floor still gates on the
    whole interval's share, so a neighbour's short burst adds no record."""
    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    s = sampler(k, stamps=5)
    s.set_target_list([(100, 5)])
    s.decide(0, DT)
    for i in range(10):
        k.occ(100, 7, 4)
        k.occ(200, 7, 64 if i < 6 else 0)
        s.sample()
    r = recs(s.decide(10 * DT, 2 * DT))
    assert r.size == 5
    assert r["ts_ns"].tolist() == [10 * DT - DT + (2 * i + 1) * DT // 10 for i in range(5)]
    assert (r["value"] == int(0.6 * DT) // 5).all() and int(s.shares()[0]["delay_ns"]) == int(0.6 * DT)
    for i in range(20):  # 1 of 20 readings hot: 5 % < the 10 % floor, no records
        k.occ(200, 7, 64 if i == 0 else 0)
        s.sample()
    assert recs(s.decide(11 * DT, 3 * DT)).size == 0


def test_a_pod_starved_by_a_neighbour_stays_active_for_the_hold(tmp_path):
    """A pod's kernels queued behind a neighbour that fills every CU hold no waves, so its own
    cu_occupancy reads 0 exactly while it is delayed most (the MI355X run of the real-driver test
    below: 3 of 9 contended intervals had a reading of its own). A pod active last interval stays
    active while the neighbour holds the GPU in >= starved_pct % of the readings, for at most
    starved_hold intervals; a neighbour below that share does not extend it."""
    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    s = sampler(k, starved_hold=2, starved_pct=90)
    s.set_target_list([(100, 5)])
    s.decide(0, DT)
    k.occ(100, 7, 4)
    k.occ(200, 7, 64)
    for _ in range(5):
        s.sample()
    assert recs(s.decide(0, 2 * DT)).size == 1 and not s.shares()[0]["starved"]
    k.occ(100, 7, 0)  # starved from here on
    got = []
    for i in range(4):
        for _ in range(5):
            s.sample()
        r = recs(s.decide(0, (3 + i) * DT))
        sh = s.shares()[0]
        got.append((r.size, sh["active"], sh["starved"]))
    assert got == [(1, True, True), (1, True, True), (0, False, False), (0, False, False)]
    # a neighbour holding the GPU in 60 % of the readings is contention, not starvation
    k.occ(100, 7, 4)
    for _ in range(5):
        s.sample()
    assert recs(s.decide(0, 7 * DT)).size == 1
    k.occ(100, 7, 0)
    for i in range(5):
        k.occ(200, 7, 64 if i < 3 else 0)
        s.sample()
    assert recs(s.decide(0, 8 * DT)).size == 0 and not s.shares()[0]["active"]


def test_processes_of_the_same_pod_are_its_own_load_and_other_pods_are_foreign(tmp_path):
    k = Kfd(tmp_path)
    for pid in (100, 101, 200):
        k.proc_on(pid, [7])
    s = sampler(k)
    s.set_target_list([(100, 5), (101, 5), (200, 6)])
    s.decide(0, DT)
    k.occ(100, 7, 8)
    k.occ(101, 7, 16)  # a second worker of pod 5
    for _ in range(4):
        s.sample()
    r = recs(s.decide(0, 2 * DT))
    # pod 5 sees pod 6 idle (no foreign load); pod 6 is idle itself, so no record although pod 5 holds waves
    assert r.size == 0
    by_pod = {x["pod"]: x for x in s.shares()}
    assert by_pod[5]["hot"] == 0 and by_pod[5]["own_hot"] == 4 and by_pod[6]["hot"] == 4 and not by_pod[6]["active"]
    k.occ(200, 7, 2)  # pod 6 starts running: each pod is the other's contention
    for _ in range(4):
        s.sample()
    r = recs(s.decide(0, 3 * DT))
    assert sorted(r["pod_id"].tolist()) == [5, 6] and (r["value"] == DT).all()


def test_floor_and_minimum_readings(tmp_path):
    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    s = sampler(k, floor_pct=25, min_samples=4)
    s.set_target_list([(100, 5)])
    s.decide(0, DT)
    k.occ(100, 7, 1)
    for i in range(3):
        k.occ(200, 7, 10)
        s.sample()
    assert recs(s.decide(0, 2 * DT)).size == 0 and s.shares() == []  # 3 readings < 4: undecided
    for i in range(5):
        k.occ(200, 7, 10 if i == 0 else 0)
        s.sample()
    assert recs(s.decide(0, 3 * DT)).size == 0 and s.shares()[0]["share"] == pytest.approx(0.2)


def test_queue_evictions_are_queue_delay_of_the_evicted_process(tmp_path):
    k = Kfd(tmp_path)
    k.proc_on(100, [7, 8], ns_pid=40)
    k.evicted(100, 8, 120)  # before the first reading: primes, not a record
    s = sampler(k)
    s.set_target_list([(100, 5)])
    assert recs(s.decide(0, DT)).size == 0
    k.evicted(100, 8, 127)
    r = recs(s.decide(0, 2 * DT))
    assert r.size == 1 and (r[0]["pod_id"], r[0]["pid"], r[0]["value"]) == (5, 40, 7_000_000)
    assert s.stats()["evictions"] == 1
    # with the BPF kprobes loaded the agent turns these off (no double counting)
    s2 = sampler(k, evictions=False)
    s2.set_target_list([(100, 5)])
    s2.decide(0, DT)
    k.evicted(100, 8, 150)
    assert recs(s2.decide(0, 2 * DT)).size == 0 and s2.stats()["evictions"] == 1


@pytest.mark.parametrize("rec", [24, 16])
def test_records_reach_the_user_ring_and_the_guard_mask_sheds_them(tmp_path, rec):
    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    ring = rt.HostRing(1 << 10, rec, "")
    s = sampler(k, ring=ring)
    s.set_target_list([(100, 5)])
    s.set_hip_activity(100, launches=1)
    s.decide(1 << 40, DT)
    s.set_hip_activity(100, launches=2)
    k.occ(200, 7, 3)
    for _ in range(3):
        s.sample()
    s.decide(1 << 40, 2 * DT)
    segs = ring.peek(16)
    assert sum(c for _, _, c in segs) == 1
    u = np.frombuffer(ring.records_view()[:rec].tobytes(), dtype=records.USER24 if rec == 24 else records.USER16)[0]
    assert (u["pid_sig"] >> 22) & 0x7F == 13 and (u["pod_ts"] & 0xFFFFF) == 5 and (u["pid_sig"] >> 30) & 1
    assert not (u["pid_sig"] >> 31) & 1  # no trace: one slot
    s.mask = 0  # the overhead guard shed gpu_queue_delay_ms: no readings, no records
    for _ in range(3):
        s.sample()
    assert recs(s.decide(1 << 40, 3 * DT)).size == 0 and s.stats()["samples"] == 3


def test_sampler_thread_runs_and_stops(tmp_path):
    import time

    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    k.occ(100, 7, 1)
    k.occ(200, 7, 5)
    ring = rt.HostRing(1 << 10, 64, "")
    s = sampler(k, ring=ring)
    s.set_target_list([(100, 5)])
    s.start(0.005, 0.05)
    time.sleep(0.4)
    s.stop()
    st = s.stats()
    assert st["samples"] >= 20 and st["emitted"] >= 3, st


def test_shedding_ladder_stops_the_kfd_sampler_at_its_gpu_rung(tmp_path):
    """The ladder's sampler rung walks the procfs signals and leaves the KFD sampler running;
    its GPU rung sets gpu_queue_delay_ms in every worker ring's drop mask, which the native
    sampler obeys: no readings, no records."""
    from llm_slo_ebpf_toolkit_amd.collector import kfd, procfs
    from llm_slo_ebpf_toolkit_amd.safety import ShedLadder
    from llm_slo_ebpf_toolkit_amd.signals import catalog

    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    k.occ(100, 7, 1)
    k.occ(200, 7, 9)
    rings = [rt.HostRing(1 << 10, 24, "") for _ in range(2)]
    ks = [kfd.KfdSampler(r, lambda: {100: 5}, kfd_proc=k.kfd, proc_root=k.proc) for r in rings]
    for s in ks:
        s.refresh()

    class Proc:
        mask, paused = procfs.ALL_MASK, False

    multi = procfs.MultiSampler([Proc()] + ks)
    lad = ShedLadder(catalog.DISABLE_ORDER, sampler=multi, user_ring=rings)
    steps = [lad.step() for _ in range(4)]
    assert all(w.startswith("sampler:") for w in steps), steps
    for s in ks:
        s.native.sample()
    assert ks[0].native.stats()["samples"] == 1  # still reading after the procfs signals were shed
    while True:
        w = lad.step()
        if w is None or w == "gpu:gpu_queue_delay_ms":
            break
    assert w == "gpu:gpu_queue_delay_ms" and all(int(r.drop_mask) >> 13 & 1 for r in rings)
    for s in ks:
        s.native.sample()
        assert s.native.stats()["samples"] <= 1


VICTIM = r"""
import sys, time, torch
w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
v = torch.randn(1, 4096, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
print("ready", flush=True)
end = time.time() + float(sys.argv[1])
while time.time() < end:  # an LLM decode step's shape: microsecond GEMVs and norms
    h = v
    for _ in range(64):
        h = torch.nn.functional.silu(h @ w) * 0.01 + h
        h = h / (h.float().pow(2).mean().sqrt().to(h.dtype) + 1)
    torch.cuda.synchronize()
    time.sleep(0.005)
"""

BURNER = r"""
import sys, time, torch
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
print("burning", time.time_ns(), flush=True)
end = time.time() + float(sys.argv[1])
while time.time() < end:
    for _ in range(8):
        a = (a @ a).clamp_(-1, 1)
    torch.cuda.synchronize()
"""


@pytest.mark.gpu
def test_kfd_sampler_on_the_real_driver_sees_another_process_on_the_pods_gpu():
    """The native KFD sampler against /sys/class/kfd on an MI355X box. The box runs us in a pid
    namespace, so the victim's KFD entry (named by host pid) is found as the entry that appears
    when it starts; the agent's DaemonSet (hostPID) gets it from the pod's cgroup instead."""
    import subprocess
    import sys
    import time

    if not os.path.isdir("/sys/class/kfd/kfd/proc"):
        pytest.skip("no KFD")
    from test_rocprof_tool import _require_quiet_gpu

    _require_quiet_gpu()  # "alone" must mean alone: another workload on the GPU is a precondition failure
    before = set(os.listdir("/sys/class/kfd/kfd/proc"))
    v = subprocess.Popen([sys.executable, "-c", VICTIM, "14"], stdout=subprocess.PIPE, text=True)
    b = None
    try:
        assert v.stdout.readline().startswith("ready")
        new = sorted(int(p) for p in set(os.listdir("/sys/class/kfd/kfd/proc")) - before if p.isdigit())
        assert new, "the victim's KFD entry did not appear"
        ring = rt.HostRing(1 << 12, 64, "")
        s = rt.GpuSampler(ring, node_id=1)
        s.set_target_list([(p, 1) for p in new])
        s.start(0.01, 0.5)
        time.sleep(4.0)
        b = subprocess.Popen([sys.executable, "-c", BURNER, "8"], stdout=subprocess.PIPE, text=True)
        t_b = int(b.stdout.readline().split()[1])
        time.sleep(5.0)
        s.stop()
        st = s.stats()
    finally:
        for p in (b, v):
            if p is not None and p.poll() is None:
                p.kill()
                p.wait(10)
    segs = ring.peek(1 << 12)
    r = np.concatenate([np.frombuffer(ring.records_view()[i * 64:(i + c) * 64].tobytes(), dtype=records.EVENT)
                        for _, i, c in segs]) if segs else np.zeros(0, records.EVENT)
    q = r[r["signal_type"] == 13]
    alone = int((q["ts_ns"] < t_b - 500_000_000).sum())
    shared = q[q["ts_ns"] > t_b + 500_000_000]
    res = {"victim_entries": new, "records_alone": alone, "records_shared": int(shared.size),
           "shared_value_ms": (shared["value"] / 1e6).round(1).tolist()[:10], "stats": dict(st),
           "sample_us_mean": st["sample_ns"] / max(st["samples"], 1) / 1e3}
    print(res)
    assert alone <= 1, res
    assert shared.size >= 5 and np.median(shared["value"]) >= 0.5 * 500_000_000, res


def test_without_a_procfs_sampler_the_ladder_never_pauses_the_kfd_samplers(tmp_path):
    """the agent hands the ladder only the procfs sampler (KFD samplers obey the rings'
    drop mask, the GPU rung). With no procfs sampler the first step must not be
    "sampler:paused" -- the KFD samplers keep reading until the GPU rung drops their signal."""
    from llm_slo_ebpf_toolkit_amd.collector import kfd
    from llm_slo_ebpf_toolkit_amd.safety import ShedLadder
    from llm_slo_ebpf_toolkit_amd.signals import catalog

    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    k.occ(100, 7, 1)
    k.occ(200, 7, 9)
    ring = rt.HostRing(1 << 10, 24, "")
    ks = kfd.KfdSampler(ring, lambda: {100: 5}, kfd_proc=k.kfd, proc_root=k.proc)
    ks.refresh()
    lad = ShedLadder(catalog.DISABLE_ORDER, sampler=None, user_ring=[ring])
    first = lad.step()
    assert first is not None and not first.startswith("sampler"), first
    ks.native.sample()
    assert ks.native.stats()["samples"] == (0 if first == "gpu:gpu_queue_delay_ms" else 1)


def test_a_pods_measured_gpu_wait_is_the_delay_other_processes_held_it(tmp_path):
    """the HIP / ROCr uprobes' per-process wait time (gpu_kfd.bpf.c: ROCr
    hsa_signal_wait_*, else hip*Synchronize + hipMemcpy call time) becomes gpu_queue_delay_ms
    evidence: the share of the pod's GPU wait other processes held the GPU."""
    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    s = sampler(k)
    s.set_target_list([(100, 5)])
    s.set_hip_activity(100, launches=1)
    s.decide(0, DT)
    k.occ(200, 7, 64)  # another process holds waves at every reading
    for _ in range(5):
        s.sample()
    # the pod launched nothing new, but its threads waited 0.3 of the interval on ROCr signals
    s.set_hip_activity(100, launches=1, wait_ns=int(0.3 * DT), waits=40)
    r = recs(s.decide(0, 2 * DT))
    sh = s.shares()[0]
    assert sh["active"] and sh["gpu_wait_ns"] == int(0.3 * DT)
    assert r.size == 1 and r[0]["value"] == int(0.3 * DT) == sh["delay_ns"]
    # no ROCr uprobes: the synchronize and copy call time stand in for the wait
    for _ in range(5):
        s.sample()
    s.set_hip_activity(100, launches=1, wait_ns=int(0.3 * DT), waits=40, sync_ns=int(0.1 * DT), syncs=3,
                       copy_ns=int(0.05 * DT))
    r = recs(s.decide(0, 3 * DT))
    assert r.size == 1 and r[0]["value"] == int(0.15 * DT)


def test_an_active_pod_that_did_not_wait_gets_no_delay(tmp_path):
    """with the uprobes reporting, a pod that launched work but never blocked on the GPU
    this interval has a measured wait of 0 -- its delay is 0 (share x 0), not the whole interval
    (the fallback for pods without the uprobes)."""
    k = Kfd(tmp_path)
    k.proc_on(100, [7])
    k.proc_on(200, [7])
    s = sampler(k)
    s.set_target_list([(100, 5)])
    s.set_hip_activity(100, launches=1, waits=4, wait_ns=1000)
    s.decide(0, DT)
    k.occ(200, 7, 64)
    for _ in range(5):
        s.sample()
    s.set_hip_activity(100, launches=9, waits=4, wait_ns=1000)  # launched more, waited no more
    r = recs(s.decide(0, 2 * DT))
    sh = s.shares()[0]
    assert sh["active"] and sh["wait_reported"] and sh["gpu_wait_ns"] == 0
    assert r.size == 0 or int(r[0]["value"]) == 0
    # a pod whose uprobes never fired (no HIP runtime hooks): the interval's share, as before
    k2 = Kfd(tmp_path / "b")
    k2.proc_on(100, [7])
    k2.proc_on(200, [7])
    s2 = sampler(k2)
    s2.set_target_list([(100, 5)])
    s2.decide(0, DT)
    k2.occ(100, 7, 1)
    k2.occ(200, 7, 64)
    for _ in range(5):
        s2.sample()
    r2 = recs(s2.decide(0, 2 * DT))
    assert not s2.shares()[0]["wait_reported"]
    assert r2.size == 1 and int(r2[0]["value"]) > 0

"""Config-3 pieces (BASELINE.json config 3, "demo/rag-service + vectordb"): the vector-DB stub,
the RAG service's keep-alive connection tuple on its spans, the unprivileged schedstat sampler and
record-level fault injection into an agent's emulated BPF ring."""

import json
import os
import threading
import urllib.request

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.cli import faultinject
from llm_slo_ebpf_toolkit_amd.collector import procfs
from llm_slo_ebpf_toolkit_amd.collector import records as R
from llm_slo_ebpf_toolkit_amd.collector.otlp import _ipv4


def write_schedstat(root, pid, tid, run, wait, slices):
    d = root / str(pid) / "task" / str(tid)
    d.mkdir(parents=True, exist_ok=True)
    (d / "schedstat").write_text(f"{run} {wait} {slices}\n")


def test_schedstat_sampler_emits_mean_wait_per_slice_above_the_floor(tmp_path):
    write_schedstat(tmp_path, 100, 100, 5_000_000, 1_000_000, 10)
    write_schedstat(tmp_path, 100, 101, 5_000_000, 1_000_000, 10)
    write_schedstat(tmp_path, 200, 200, 1, 1, 1)
    pushed = []
    s = procfs.SchedstatSampler(lambda: {100: 7, 200: 9}, lambda u: pushed.append(u) or len(u), rec=24,
                                proc_root=str(tmp_path), node_id=3, steal_floor_milli=1000,  # 1 %: see the steal record
                                steal_sustain=1)
    assert len(s.sample(10**18)) == 0  # first look: no deltas yet
    write_schedstat(tmp_path, 100, 100, 9_000_000, 1_000_000 + 4 * 2_000_000, 14)  # 2 ms per slice
    write_schedstat(tmp_path, 100, 101, 9_000_000, 1_000_000 + 4 * 50_000, 14)     # 50 us per slice: below
    write_schedstat(tmp_path, 200, 200, 2, 1, 2)                                     # ran, never waited
    ev = s.sample(10**18 + 100_000_000)
    # per process: the wait over the timeslices of its threads above the floor, then the CPU it
    # waited for over the interval (8.2 ms of 100 ms: 8.2 % of one CPU, in milli-percent)
    assert len(ev) == 2
    e = ev[0]
    assert (int(e["signal_type"]), int(e["value"]), int(e["pid"]), int(e["tid"]), int(e["pod_id"]),
            int(e["node_id"])) == (procfs.RUNQUEUE_TYPE, 2_000_000, 100, 100, 7, 3)
    assert (int(ev[1]["signal_type"]), int(ev[1]["value"]), int(ev[1]["pod_id"])) == (procfs.STEAL_TYPE, 8200, 7)
    write_schedstat(tmp_path, 100, 100, 9_500_000, 9_000_000 + 3_000_000, 15)
    assert s.tick(10**18 + 200_000_000) == 2 and s.emitted == 2 and pushed[0].dtype.itemsize == 24
    # an exited thread is forgotten
    os.remove(tmp_path / "100" / "task" / "101" / "schedstat")
    s.sample()
    assert (100, 101) not in s._prev


def test_sampler_records_carry_the_pid_the_pod_sees(tmp_path):
    """A containerised process: the agent watches it as host pid 4242, the pod's spans and its
    rocprofiler records say pid 17 (NSpid's innermost field). The run-queue record joins them on
    the pod + pid tier only if it carries 17 -- as the BPF probes do (mislo_ns_tgid). A process
    in the agent's own namespace keeps its pid."""
    for pid in (4242, 500):
        write_schedstat(tmp_path, pid, pid, 1, 1, 1)
    (tmp_path / "4242" / "status").write_text("Name:\tpython\nTgid:\t4242\nNSpid:\t4242\t17\n")
    (tmp_path / "500" / "status").write_text("Name:\tsh\nNSpid:\t500\n")
    s = procfs.SchedstatSampler(lambda: {4242: 7, 500: 8}, lambda u: len(u), proc_root=str(tmp_path))
    s.sample(10**18)
    for pid in (4242, 500):
        write_schedstat(tmp_path, pid, pid, 2, 1 + 3_000_000, 2)
    ev = s.sample(10**18 + 10**8)
    ev = ev[ev["signal_type"] == procfs.RUNQUEUE_TYPE]
    got = sorted((int(e["pod_id"]), int(e["pid"]), int(e["tid"])) for e in ev)
    assert got == [(7, 17, 4242), (8, 500, 500)]
    assert procfs.ns_pid(999, str(tmp_path)) == 999  # gone / unreadable: as given


def test_schedstat_sampler_reads_this_process():
    me = os.getpid()
    s = procfs.SchedstatSampler(lambda: {me: 1}, lambda u: len(u), floor_ns=0)
    s.sample()
    busy = threading.Thread(target=lambda: sum(range(2_000_000)))
    busy.start()
    busy.join()
    assert s.sample() is not None and s.samples == 2


def test_pod_lists(tmp_path):
    assert procfs.parse_pod_list("12:aaa, 13:bbb,") == {12: "aaa", 13: "bbb"}
    uid = "0f0e0d0c-0b0a-0908-0706-050403020100"
    d = tmp_path / "kubepods.slice" / f"kubepods-burstable-pod{uid.replace('-', '_')}.slice" / "cri-containerd-x.scope"
    d.mkdir(parents=True)
    (d / "cgroup.procs").write_text("41\n42\n")
    (tmp_path / "system.slice").mkdir()
    (tmp_path / "system.slice" / "cgroup.procs").write_text("1\n")
    assert procfs.pod_processes(str(tmp_path)) == {41: uid, 42: uid}
    # the probes' cgroup map: systemd (kubepods-...-pod<uid_>.slice) and cgroupfs (pod<uid>) names
    from llm_slo_ebpf_toolkit_amd.collector import bpf

    uid2 = "aaaaaaaa-bbbb-cccc-dddd-eeeeeeeeeeee"
    (tmp_path / "kubepods" / f"pod{uid2}").mkdir(parents=True)
    found = {u for _id, u in bpf.discover_pods(str(tmp_path)).values()}
    assert found == {uid, uid2}


def test_vectordb_search_over_http_keeps_the_connection():
    from llm_slo_ebpf_toolkit_amd.demo import vectordb
    from llm_slo_ebpf_toolkit_amd.demo.rag_service import VectorDBClient

    db = vectordb.VectorDB(replicas=4)
    hits = db.search("retrieval augmented generation", 3)
    assert len(hits) == 3 and hits[0]["score"] >= hits[-1]["score"]
    httpd = db.serve("127.0.0.1:0")
    try:
        port = httpd.server_address[1]
        cli = VectorDBClient(f"http://127.0.0.1:{port}")
        r1, a1 = cli.search("gpu kernels", 2)
        r2, a2 = cli.search("network latency", 2)
        assert len(r1) == 2 and len(r2) == 2
        assert a1["server.port"] == port and a1["server.address"] == "127.0.0.1"
        assert a1["client.port"] == a2["client.port"] > 0  # one keep-alive connection per thread
        assert db.searches == 3  # one direct, two over HTTP
    finally:
        httpd.shutdown()


def test_faultinject_emit_ring_writes_probe_records_for_the_connection():
    from llm_slo_ebpf_toolkit_amd.collector import bpf
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    prefix = f"/mislo-fi-{os.getpid()}"
    names = bpf.RingNames.of(prefix)
    ring, user, spans = bpf.create_rings(names, 1 << 16, 1024, 1024)
    t0 = 1_700_000_000_000_000_000
    ring.cfg_set(rt.CFG_EPOCH, t0 & ~3)
    rc = faultinject.main(["--emit-ring", prefix, "--signal", "tcp_retransmits_total", "--pod-id", "5",
                           "--conn", "51000:6333:127.0.0.1", "--rate", "2000", "--duration", "0.01"])
    assert rc == 0
    ev, defs, disc, busy = R.unframe(ring.data_view()[:ring.producer_pos].copy())
    assert not disc and not busy and len(ev) == 20
    c = R.conn32(R.conn_hash(51000, 6333, _ipv4("127.0.0.1")))
    raw = defs.view(np.uint32).reshape(-1, 4)
    ctx = [r for r in raw if (r[1] & 0xFF) == R.DEF_CTX]
    assert len(ctx) == 1 and (ctx[0][0], ctx[0][2], ctx[0][3]) == (c, 5, 0)
    rows = ev.view(np.uint32).reshape(-1, 4)
    assert (rows[:, 1] & 0xFF == 2).all() and (rows[:, 1] >> 8 == ctx[0][1] >> 8).all()
    # cumulative retransmits of the connection: 1, 2, ... (decoded milli-units rise)
    assert (np.diff(rows[:, 2].astype(np.int64)) > 0).all()


def test_faultinject_rejects_non_kernel_signal(capsys):
    assert faultinject.main(["--emit-ring", "/x", "--signal", "not_a_signal"]) == 2


def test_psi_memory_stall_becomes_reclaim_records(tmp_path):
    """Memory stall time (PSI) growth per interval -> mem_reclaim_latency_ms records of the
    watched processes; the pod's cgroup v2 file wins over the node's."""
    (tmp_path / "pressure").mkdir()
    node = tmp_path / "pressure" / "memory"
    node.write_text("some avg10=0.00 avg60=0.00 avg300=0.00 total=1000\nfull avg10=0.00 avg60=0.00 avg300=0.00 total=0\n")
    write_schedstat(tmp_path, 100, 100, 1, 1, 1)
    (tmp_path / "100" / "cgroup").write_text("0::/\n")
    s = procfs.SchedstatSampler(lambda: {100: 4}, lambda u: len(u), proc_root=str(tmp_path),
                                cgroup_root=str(tmp_path / "cg"))
    assert procfs.psi_available(str(tmp_path))
    assert len(s.sample()) == 0
    node.write_text("some avg10=1.00 avg60=0.00 avg300=0.00 total=6000\nfull avg10=0.00 avg60=0.00 avg300=0.00 total=0\n")
    ev = s.sample()
    assert len(ev) == 1 and int(ev[0]["signal_type"]) == procfs.MEM_RECLAIM_TYPE
    assert (int(ev[0]["value"]), int(ev[0]["pid"]), int(ev[0]["pod_id"])) == (5_000_000, 100, 4)
    assert len(s.sample()) == 0  # no growth, no record
    cg = tmp_path / "cg" / "kubepods" / "podx"
    cg.mkdir(parents=True)
    (cg / "memory.pressure").write_text("some avg10=0.00 avg60=0.00 avg300=0.00 total=7\n")
    (tmp_path / "100" / "cgroup").write_text("0::/kubepods/podx\n")
    assert procfs.psi_path(100, str(tmp_path), str(tmp_path / "cg")) == str(cg / "memory.pressure")
    assert procfs.read_psi_total_us(str(cg / "memory.pressure")) == 7


def test_faultinject_fault_profile_emits_every_kernel_signal_of_the_fault():
    from llm_slo_ebpf_toolkit_amd.collector import bpf
    from llm_slo_ebpf_toolkit_amd.runtime import load
    from llm_slo_ebpf_toolkit_amd.signals import catalog
    from llm_slo_ebpf_toolkit_amd.signals.generator import FAULT_OVERRIDES

    rt = load()
    prefix = f"/mislo-fp-{os.getpid()}"
    ring, _u, _s = bpf.create_rings(bpf.RingNames.of(prefix), 1 << 16, 1024, 1024)
    ring.cfg_set(rt.CFG_EPOCH, (1_700_000_000_000_000_000) & ~3)
    assert faultinject.main(["--emit-ring", prefix, "--fault", "network_partition", "--pod-id", "3", "--conn",
                             "51000:6333:127.0.0.1,51002:6333:127.0.0.1", "--rate", "1000", "--duration", "0.01"]) == 0
    ev, defs, _d, _b = R.unframe(ring.data_view()[:ring.producer_pos].copy())
    types = ev.view(np.uint32).reshape(-1, 4)[:, 1] & 0xFF
    want = {catalog.BY_NAME[n].kernel_type for n in FAULT_OVERRIDES["network_partition"]}
    assert set(types.tolist()) == want and len(ev) == 10 * len(want)
    ctx = [r for r in defs.view(np.uint32).reshape(-1, 4) if (r[1] & 0xFF) == R.DEF_CTX]
    assert {int(r[0]) for r in ctx} == {R.conn32(R.conn_hash(p, 6333, _ipv4("127.0.0.1"))) for p in (51000, 51002)}
    assert faultinject.main(["--emit-ring", prefix, "--fault", "no_such_fault"]) == 2

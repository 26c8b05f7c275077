"""Distributed path on CPU (gloo, world_size 2, 127.0.0.1): node sharding + trace-event
all-gather + packet all-reduce must reproduce the single-process window exactly."""

import os
import socket

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.models.bayes import NaiveBayes
from llm_slo_ebpf_toolkit_amd.parallel import exchange, shard
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.cpu import CpuWindowEngine
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

WORLD = 2


def global_window(seed=3):
    cfg = ReplayConfig(scenario="full", n_nodes=4, pods_per_node=4, n_services=8, events_per_window=6000,
                       spans_per_window=400, seed=seed)
    w = ReplayGenerator(cfg).next_window()
    ev = w.events.copy()
    rng = np.random.default_rng(seed)
    # move a third of the trace-tagged events to pods on other nodes: cross-node traces
    idx = np.nonzero(ev["trace_h"] != 0)[0]
    mv = rng.choice(idx, size=len(idx) // 3, replace=False)
    donors = rng.integers(0, len(ev), size=len(mv))
    for f in ("pod_id", "node_id", "svc_id", "pid"):
        ev[f][mv] = ev[f][donors]
    # unique timestamps so top-3 tie-breaks never depend on array order
    ev["ts_ns"] = ev["ts_ns"] + np.arange(len(ev), dtype=np.int64) % 7 * 0 + rng.permutation(len(ev)) * 3
    return ev, w.spans.copy(), w.n_groups, w.group_labels.copy()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ev, sp, G, labels = global_window()
        ev_l, sp_l = shard.shard(ev, sp, rank, world)
        merged, n_local = exchange.with_remote_trace_events(ev_l)
        eng = CpuWindowEngine(NaiveBayes.ref())

        def reduce_groups(gsum, gcnt):
            gs, gc = torch.from_numpy(gsum.copy()), torch.from_numpy(gcnt.copy())
            dist.all_reduce(gs)
            dist.all_reduce(gc)
            return gs.numpy(), gc.numpy()

        owned = labels.copy()
        owned[np.arange(G) % world != rank] = -1  # each incident group is scored once node-wide
        res = eng.run(merged, sp_l, G, owned, n_local=n_local, learn=True, reduce_groups=reduce_groups)
        pk = torch.from_numpy(res.packet.copy())
        dist.all_reduce(pk)
        gs, gc = reduce_groups(res.join.gsum, res.join.gcnt)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), span_h=sp_l["span_h"], attrs=res.join.attrs,
                 conf=res.join.conf, cnt=res.join.cnt, packet=pk.numpy(), gsum=gs, gcnt=gc,
                 n_local=n_local, n_merged=merged.shape[0])
    finally:
        dist.destroy_process_group()


def test_sharding_covers_every_record_once():
    ev, sp, _, _ = global_window()
    parts = [shard.shard(ev, sp, r, 3) for r in range(3)]
    assert sum(p[0].shape[0] for p in parts) == ev.shape[0]
    assert sum(p[1].shape[0] for p in parts) == sp.shape[0]


def test_halo_carries_recent_events():
    ev, sp, G, _ = global_window()
    order = np.argsort(ev["ts_ns"])
    first, second = ev[order[: len(ev) // 2]], ev[order[len(ev) // 2:]]
    h = exchange.Halo(outer_ns=2_000_000_000)
    m1, n1 = h.extend(first, sp)
    assert n1 == m1.shape[0] == first.shape[0]
    m2, n2 = h.extend(second, sp)
    assert n2 == second.shape[0] and m2.shape[0] > n2
    assert (m2["ts_ns"][n2:] >= int(sp["ts_ns"].min()) - 2_000_000_000).all()


@pytest.mark.timeout(300)
def test_gloo_two_ranks_match_single_process(tmp_path):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    ev, sp, G, labels = global_window()
    ref = CpuWindowEngine(NaiveBayes.ref()).run(ev, sp, G, labels, learn=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(WORLD)]
    # per-span enrichment identical to the global batch (trace tier crosses the shards)
    pos = {int(h): i for i, h in enumerate(sp["span_h"])}
    for part in r:
        for j, h in enumerate(part["span_h"]):
            i = pos[int(h)]
            np.testing.assert_array_equal(part["attrs"][j], ref.join.attrs[i])
            assert part["conf"][j] == ref.join.conf[i] and part["cnt"][j] == ref.join.cnt[i]
    assert any(p["n_merged"] > p["n_local"] for p in r)  # remote trace events were imported
    # incident features and the packed window statistics all-reduce to the global values
    np.testing.assert_array_equal(r[0]["gcnt"], ref.join.gcnt)
    np.testing.assert_allclose(r[0]["gsum"], ref.join.gsum, rtol=1e-12)
    pk, gp = r[0]["packet"], ref.packet
    lay = np.cumsum((0,) + tuple(oracle_layout()))
    for k, name in enumerate(("hist", "status", "misc", "dbg", "confusion")):
        np.testing.assert_array_equal(pk[lay[k]:lay[k + 1]], gp[lay[k]:lay[k + 1]], err_msg=name)
    np.testing.assert_allclose(pk[lay[5]:], gp[lay[5]:], rtol=1e-9, atol=1e-9)


def oracle_layout():
    from llm_slo_ebpf_toolkit_amd.pipeline.window import PACKET_LAYOUT

    return PACKET_LAYOUT


def test_numa_cpulist_and_affinity_choice(tmp_path):
    from llm_slo_ebpf_toolkit_amd.parallel import numa

    assert numa.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa.pci_bdf(0, 0x75, 0) == "0000:75:00.0"
    dev = tmp_path / "0000:75:00.0"
    dev.mkdir()
    (dev / "numa_node").write_text("1\n")
    (dev / "local_cpulist").write_text("48-95\n")
    local = numa.local_cpus_of_pci("0000:75:00.0", str(tmp_path))
    assert local == set(range(48, 96))
    assert numa.choose_affinity(range(96), local) == set(range(48, 96))
    assert numa.choose_affinity(range(48), local) is None          # cpuset excludes the GPU's socket
    assert numa.choose_affinity(range(48, 96), local) is None      # already local: nothing to do
    (dev / "numa_node").write_text("-1\n")                         # VMs: topology unknown
    assert numa.local_cpus_of_pci("0000:75:00.0", str(tmp_path)) is None
    assert numa.local_cpus_of_pci("0000:00:99.0", str(tmp_path)) is None

"""Distributed path on CPU (gloo, world_size 2 / 4 / 8, 127.0.0.1): the engine's multi-GPU window
protocol (parallel/exchange.py, the CPU model of ops/csrc/exchange.hip) over a real process
group -- node-sharded streams, the halo carried across window cuts, warn-level trace rows
exchanged as 24-byte XRec blocks and imported one window later, the packet all-reduce."""

import os
import socket

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.parallel import exchange, shard
from llm_slo_ebpf_toolkit_amd.pipeline import oracle
from llm_slo_ebpf_toolkit_amd.pipeline.replay import ReplayConfig, ReplayGenerator

WORLD = 2
HALO_MS, ICAP, XCAP = 2000.0, 20000, 4000


def global_windows(n_win=3, seed=3, n_nodes=4):
    """Consecutive windows of an ``n_nodes``-node cluster; a third of the trace-tagged events moved
    to pods on other nodes, so traces cross the node shards."""
    cfg = ReplayConfig(scenario="full", n_nodes=n_nodes, pods_per_node=4, n_services=8,
                       events_per_window=1500 * n_nodes, spans_per_window=100 * n_nodes, seed=seed)
    g = ReplayGenerator(cfg)
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_win):
        w = g.next_window()
        ev = w.events.copy()
        idx = np.nonzero(ev["trace_h"] != 0)[0]
        mv = rng.choice(idx, size=len(idx) // 3, replace=False)
        donors = rng.integers(0, len(ev), size=len(mv))
        for f in ("pod_id", "node_id", "svc_id", "pid"):
            ev[f][mv] = ev[f][donors]
        out.append((ev, w.spans.copy(), w.n_groups))
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_rank(rank, wins, allgather, xchg=XCAP, world=WORLD):
    m = exchange.ExchangeModel(rank, world, HALO_MS, ICAP, xchg, allgather)
    out = []
    for ev, sp, G in wins:
        ev_l, sp_l = shard.shard(ev, sp, rank, world)
        d = oracle.decode_events(ev_l)
        res = m.window(d, sp_l, G)
        out.append(dict(feat=res.feat, cnt=res.cnt, gsum=res.gsum, gcnt=res.gcnt, hist=oracle.histograms(d),
                        n_rows=res.n_rows, n_loc=len(d.ts), sent=m.sent))
    return out


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _run_rank(rank, global_windows(n_nodes=max(4, 2 * world)), exchange.torch_allgather(), world=world)
        hist = torch.from_numpy(np.stack([r["hist"] for r in res]))
        dist.all_reduce(hist)  # the packet all-reduce: node-wide counters
        np.savez(os.path.join(outdir, f"r{rank}.npz"), hist=hist.numpy(),
                 **{f"{k}{j}": r[k] for j, r in enumerate(res) for k in ("feat", "cnt", "gsum", "gcnt")},
                 n_rows=[r["n_rows"] for r in res], n_loc=[r["n_loc"] for r in res], sent=[r["sent"] for r in res])
    finally:
        dist.destroy_process_group()


def _in_memory(wins, xchg=XCAP, world=WORLD, icap=ICAP, models=None):
    """Every rank in one process, the all-gather done by hand (same blocks)."""
    ms = [exchange.ExchangeModel(r, world, HALO_MS, icap, xchg) for r in range(world)]
    if models is not None:
        models.extend(ms)
    out = [[] for _ in range(world)]
    for ev, sp, G in wins:
        loc = [shard.shard(ev, sp, r, world) for r in range(world)]
        ds = [oracle.decode_events(e) for e, _ in loc]
        blocks = [m.block(d) for m, d in zip(ms, ds)]
        for r, m in enumerate(ms):
            out[r].append(m.join(ds[r], loc[r][1], G, blocks if xchg else None))
    return out


def test_sharding_covers_every_record_once():
    ev, sp, _ = global_windows(1)[0]
    parts = [shard.shard(ev, sp, r, 3) for r in range(3)]
    assert sum(p[0].shape[0] for p in parts) == ev.shape[0]
    assert sum(p[1].shape[0] for p in parts) == sp.shape[0]


def test_halo_carries_the_previous_windows_tail():
    wins = global_windows()
    m = exchange.ExchangeModel(0, 1, HALO_MS, ICAP, 0)
    n_imp = []
    for ev, sp, G in wins:
        d = oracle.decode_events(ev)
        res = m.window(d, sp, G)
        n_imp.append(res.n_rows - len(d.ts))
        tmax = oracle.window_tmax(d, len(d.ts))
        assert (m.halo().ts >= tmax - int(HALO_MS * 1e6)).all()
    assert n_imp[0] == 0 and all(n > 0 for n in n_imp[1:])


def test_resident_generations_are_the_nested_halo_selections():
    """The engine keeps earlier windows' rows resident and filters them by per-age cut-offs
    (exchange.hip k_gen_begin); that is row for row, in the same order, what selecting each
    window's halo from [its rows | the halo it joined] (oracle.halo_rows) and carrying it forward
    would import -- so the join's tie-breaks by row order are unchanged too."""
    wins = global_windows()
    m = exchange.ExchangeModel(0, 1, HALO_MS, ICAP, 0, halo_windows=3)
    nested = oracle.empty_rows()
    seen = remote_seen = 0
    for j, (ev, sp, G) in enumerate(wins):
        d = oracle.decode_events(ev)
        # other GPUs' rows of this window (identity-free), joined after the halo
        tr = oracle.trace_rows(d, len(d.ts))
        remote = oracle.take(oracle.remote_rows(tr), np.arange(len(tr.ts)) % 7 == j % 7)
        h = m.halo()
        for f in oracle.Decoded.__dataclass_fields__:
            np.testing.assert_array_equal(getattr(h, f), getattr(nested, f), err_msg=f"window {j}: {f}")
        seen += len(h.ts)
        remote_seen += int((h.pod == 0).sum())
        m.injected = remote
        m.window(d, sp, G)
        nested = oracle.halo_rows(oracle.concat(oracle.concat(d, nested), remote), len(d.ts), int(HALO_MS * 1e6))
    assert seen > 0 and remote_seen > 0


def test_exchange_block_roundtrip():
    d = oracle.decode_events(global_windows(1)[0][0])
    rows = oracle.trace_rows(d, len(d.ts))
    back = exchange.parse_block(oracle.exchange_blocks([rows], 100000))
    np.testing.assert_array_equal(back.ts, rows.ts)
    np.testing.assert_array_equal(back.trace, rows.trace)
    np.testing.assert_array_equal(back.val, rows.val)
    assert (back.pod == 0).all() and (back.conn == 0).all() and (rows.status >= 1).all()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_ranks_run_the_device_protocol(tmp_path, world):
    """2, 4 and 8 gloo ranks (the node sizes bench.py --gpus runs) reproduce the single-process
    model of the same ranks exactly: features, candidates and group counts per rank and window."""
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    wins = global_windows(n_nodes=max(4, 2 * world))
    ref = _in_memory(wins, world=world)
    solo = _in_memory(wins, xchg=0, world=world)  # the same ranks without the exchange
    got = [np.load(tmp_path / f"r{k}.npz") for k in range(world)]
    for r in range(world):
        for j in range(len(wins)):
            np.testing.assert_array_equal(got[r][f"feat{j}"], ref[r][j].feat)
            np.testing.assert_array_equal(got[r][f"cnt{j}"], ref[r][j].cnt)
            np.testing.assert_array_equal(got[r][f"gcnt{j}"], ref[r][j].gcnt)
        if got[r]["n_loc"].sum():  # a rank the node hash gave no node has nothing to send
            assert (got[r]["sent"] > 0).all() and (got[r]["n_rows"] > got[r]["n_loc"]).all()
        else:  # but it still imports the others' rows
            assert (got[r]["n_rows"] > 0).all()
    assert sum(int(got[r]["n_loc"].sum() > 0) for r in range(world)) >= world - 1
    # cross-node traces: the exchange adds the other shard's elevated signals to the spans'
    # candidates in the same window
    for j in range(len(wins)):
        extra = sum(int(ref[r][j].cnt.sum() - solo[r][j].cnt.sum()) for r in range(world))
        assert extra > 0, j
    # node-wide counters: the all-reduced per-rank histograms are the global histograms
    for j, (ev, _, _) in enumerate(wins):
        np.testing.assert_array_equal(got[0]["hist"][j], oracle.histograms(oracle.decode_events(ev)))


def test_exchange_losses_are_counted_not_silent():
    """Rows over the exchange capacity (a rank selected more than its block holds) and over the
    import capacity (more peer rows than the window imports) are counted -- the packet's dbg[5] /
    dbg[6], llm_slo_agent_dropped_events_total{reason="xchg_cap"|"import_cap"} -- and the rows kept
    are the first ones, in rank order."""
    wins = global_windows(2, n_nodes=8)
    ms = []
    _in_memory(wins, xchg=50, world=8, icap=200, models=ms)
    full = []
    _in_memory(wins, xchg=100000, world=8, icap=10 ** 7, models=full)
    for m, f in zip(ms, full):
        assert m.sent == min(50, f.sent) and m.xchg_dropped == max(0, f.sent - 50)
        assert m.import_dropped > 0  # 7 peers x up to 50 rows > 200
    assert sum(m.xchg_dropped for m in ms) > 0
    assert all(f.xchg_dropped == 0 and f.import_dropped == 0 for f in full)


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
